// head.h -- per-sample records of the classifier head (head.hip) and their batch reduction
// (run inside lbt_step_reduce, batched.hip).
#pragma once
#include "dfxp_device.h"

#define LBT_HD __host__ __device__ inline

namespace lbt {

// Records of the N samples in scratch, TRANSPOSED so the batch reduction takes four samples per
// v_dot4 (NP = N rounded up to 16 bytes; bytes of samples >= N are never read as data: masked):
//   pqT[C][NP] int8 (Dense_q X codes) | gqT[64][NP] int8 (Dense_q grad codes, rows < K used) |
//   term[N] double (each sample's loss term)
LBT_HD int head_np(int N) { return (N + 15) & ~15; }
LBT_HD int64_t head_gq_off(int N, int C) { return (int64_t)C * head_np(N); }
LBT_HD int64_t head_term_off(int N, int C) { return (int64_t)(C + 64) * head_np(N); }
LBT_HD int64_t head_scratch_bytes(int N, int C) { return head_term_off(N, C) + 8 * (int64_t)N; }

constexpr int kHeadT = 256;
constexpr int kHeadLds = 4112;  // the step_reduce workgroup's LDS (rjob_block's 4112 B; head_reduce uses its own)

// One 256-thread workgroup: dw = dequant(sum_n pq[n]^T gq[n]) + wd2 * w (wgrad_reduce's formula)
// and loss[0] = (float)(sum of the terms in softmax_xent_kernel's order / loss_n). Thread (c, kq) owns
// channel c's outputs k = kq * kpt .. + kpt - 1 and sums them over the samples 4 at a time (v_dot4 on
// the transposed records, 16 samples per load): exact integers, so the order is free. With an exchange
// buffer (x.buf, lbt_step_reduce_x) the integer sums go to x.buf[(dw - gbase) + ...] instead, and the
// loss-term sum, in 2^-32 fixed point, to x.buf[loss_off]. u.w != NULL (lbt_step_reduce_update):
// MomentumOptimizer on each dw element as it is formed.
LBT_DEV void head_reduce(const lbt_head& h, const lbt_xchg& x, uint8_t* lds, const lbt_update& u) {
  (void)lds;
  __shared__ double s_red[kHeadT];
  const int t = threadIdx.x, C = h.C, K = h.K, N = h.N, NP = head_np(N);
  const int G = kHeadT / C, c = t % C, kq = t / C;  // threads t >= G * C idle (C <= 256)
  const int kpt = (K + G - 1) / G, k0 = kq * kpt;
  const int nk = kq < G ? (K - k0 < kpt ? (K - k0 > 0 ? K - k0 : 0) : kpt) : 0;
  const uint8_t* scr = reinterpret_cast<const uint8_t*>(h.scratch);
  const uint4* pr = reinterpret_cast<const uint4*>(scr + (int64_t)c * NP);
  const uint8_t* gbase = scr + head_gq_off(N, C);
  const double* term = reinterpret_cast<const double*>(scr + head_term_off(N, C));
  const float wscale = ldexpf(1.0f, -(frac_exp(h.qx) + frac_exp(h.qg)));
  // the loss terms: thread t sums rows t, t + 256, ... in order (softmax_xent_kernel's order), issued first
  double part = 0.0;
  for (int r = t; r < N; r += kHeadT) part += term[r];
  const int64_t ob = u.w ? h.dw - u.g : 0;
  for (int kb = k0; kb < k0 + nk; kb += 4) {  // 4 outputs per pass, in registers
    const int n4 = k0 + nk - kb < 4 ? k0 + nk - kb : 4;
    int acc[4] = {0, 0, 0, 0};
    for (int m = 0; m < NP / 16; ++m) {
      uint4 a = pr[m];
      const int valid = N - 16 * m;  // samples of this 16-byte group that exist
      if (valid < 16) {              // the last group: bytes of samples >= N masked (pads are not written)
        uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int nv = valid - 4 * q;
          w[q] = nv >= 4 ? w[q] : (nv <= 0 ? 0u : w[q] & ((1u << (8 * nv)) - 1u));
        }
        a = make_uint4(w[0], w[1], w[2], w[3]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i >= n4) break;
        const uint4 g = reinterpret_cast<const uint4*>(gbase + (int64_t)(kb + i) * NP)[m];
        int v = acc[i];
        v = __builtin_amdgcn_sdot4((int)a.x, (int)g.x, v, false);
        v = __builtin_amdgcn_sdot4((int)a.y, (int)g.y, v, false);
        v = __builtin_amdgcn_sdot4((int)a.z, (int)g.z, v, false);
        v = __builtin_amdgcn_sdot4((int)a.w, (int)g.w, v, false);
        acc[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= n4) break;
      const int e = c * K + kb + i;
      if (x.buf) {
        x.buf[(h.dw - x.gbase) + e] = (long long)acc[i];
        continue;
      }
      const float a = (float)(long long)acc[i] * wscale;
      const float b = h.wd2 * h.w[e];
      const float gv = a + b;
      h.dw[e] = gv;
      if (u.w) {  // sgd_momentum_elem's arithmetic (gscale 1)
        const float tm = u.mu * u.a[ob + e];
        const float an = tm + gv;
        LBT_ST_TAIL(u.a + ob + e, an);
        const float stp = u.lr * an;
        LBT_ST_TAIL(u.w + ob + e, h.w[e] - stp);
      }
    }
  }
  // the loss terms' tree sum s[t] += s[t + o], o = 128, 64, ..., 1: the two upper levels through LDS,
  // the six within wave 0 as shuffles (lane t < o adds lane t + o: the same additions in the same
  // order as the LDS tree, without its six barriers)
  static_assert(kHeadT == 256, "tree levels");
  s_red[t] = part;
  __syncthreads();
  if (t < 128) s_red[t] += s_red[t + 128];
  __syncthreads();
  if (t < 64) {
    double v = s_red[t] + s_red[t + 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if (t == 0) {
      h.loss[0] = (float)(v / (double)(h.loss_n > 0 ? h.loss_n : N));
      if (x.buf) x.buf[x.loss_off] = (long long)llrint(v * 4294967296.0);
    }
  }
}

}  // namespace lbt

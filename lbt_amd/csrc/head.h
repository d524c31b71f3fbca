// head.h -- per-sample records of the classifier head (head.hip) and their batch reduction
// (run inside lbt_step_reduce, batched.hip).
//
// Record of sample n at scratch + n * (C + kHeadRecPad) bytes:
//   pq[C] (Dense_q X codes) | gq[64] (Dense_q grad codes, K used) | loss term (double)
#pragma once
#include "dfxp_device.h"

namespace lbt {

constexpr int kHeadRecPad = 72;
constexpr int kHeadT = 256;
constexpr int kHeadRecBytes = 24576;                        // records staged per pass
constexpr int kHeadLds = kHeadRecBytes + kHeadT * 16 * 4;   // + per-thread partials

// One 256-thread workgroup: dw = dequant(sum_n pq[n]^T gq[n]) + wd2 * w (wgrad_reduce's formula)
// and loss[0] = (float)(sum of the terms in softmax_xent_kernel's order / loss_n). lds: kHeadLds
// bytes. With an exchange buffer (x.buf, lbt_step_reduce_x) the integer sums go to
// x.buf[(dw - gbase) + ...] instead, and the loss-term sum, in 2^-32 fixed point, to x.buf[loss_off].
// u.w != NULL (lbt_step_reduce_update): MomentumOptimizer on each dw element as it is formed.
LBT_DEV void head_reduce(const lbt_head& h, const lbt_xchg& x, uint8_t* lds, const lbt_update& u) {
  uint32_t* s_rec = reinterpret_cast<uint32_t*>(lds);
  int(*s_acc)[16] = reinterpret_cast<int(*)[16]>(lds + kHeadRecBytes);
  __shared__ double s_red[kHeadT];
  const int t = threadIdx.x, C = h.C, K = h.K, N = h.N;
  const int rs = C + kHeadRecPad, words = rs / 4;
  const int chunk = (kHeadRecBytes / 4) / words;  // samples per pass
  const int G = kHeadT / C, c = t % C, g = t / C;  // thread (c, g): channel c, samples g, g+G, ...
  const uint8_t* scr = reinterpret_cast<const uint8_t*>(h.scratch);
  const float wscale = ldexpf(1.0f, -(frac_exp(h.qx) + frac_exp(h.qg)));
  double part = 0.0;
  for (int kb = 0; kb < K; kb += 16) {
    float wf[16 * 256 / kHeadT];  // this pass's fp32 weights (decay term), loaded ahead
    float af[16 * 256 / kHeadT];  // ... and their momentum accumulators (u.w)
    const int64_t ob = u.w ? h.dw - u.g : 0;
#pragma unroll
    for (int j = 0; j < 16 * 256 / kHeadT; ++j) {
      const int o = t + j * kHeadT, oc = o >> 4, ok = kb + (o & 15);
      const int e = (oc < C && ok < K) ? oc * K + ok : 0;
      wf[j] = h.w[e];
      af[j] = u.w ? u.a[ob + e] : 0.f;
    }
    int sacc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) sacc[j] = 0;
    for (int n0 = 0; n0 < N; n0 += chunk) {
      const int nn = N - n0 < chunk ? N - n0 : chunk;
      __syncthreads();
      {  // every load in flight before the first LDS write (clamped addresses, no branches)
        const uint32_t* src = reinterpret_cast<const uint32_t*>(scr + (int64_t)n0 * rs);
        const int lim = nn * words;
        uint32_t v[kHeadRecBytes / 4 / kHeadT];
#pragma unroll
        for (int j = 0; j < kHeadRecBytes / 4 / kHeadT; ++j) {
          const int i = t + j * kHeadT;
          v[j] = src[i < lim ? i : 0];
        }
#pragma unroll
        for (int j = 0; j < kHeadRecBytes / 4 / kHeadT; ++j) s_rec[t + j * kHeadT] = v[j];
      }
      __syncthreads();
      const uint8_t* r8 = reinterpret_cast<const uint8_t*>(s_rec);
      if (g < G) {
#pragma unroll 4
        for (int r = g; r < nn; r += G) {
          const int x = (int)(int8_t)r8[r * rs + c];
          const uint32_t* gw = s_rec + r * words + C / 4 + kb / 4;  // 4-byte aligned only
          const uint32_t gv[4] = {gw[0], gw[1], gw[2], gw[3]};
#pragma unroll
          for (int w4 = 0; w4 < 4; ++w4)
#pragma unroll
            for (int b = 0; b < 4; ++b) sacc[4 * w4 + b] += x * (int)(int8_t)(gv[w4] >> (8 * b));
        }
      }
      if (kb == 0) {  // loss terms: thread t sums rows t, t + 256, ... in order (softmax_xent_kernel)
        for (int r = (t - n0 % kHeadT + kHeadT) % kHeadT; r < nn; r += kHeadT) {
          const uint32_t* tw = s_rec + r * words + C / 4 + 16;
          part += __longlong_as_double((long long)((uint64_t)tw[0] | ((uint64_t)tw[1] << 32)));
        }
      }
    }
    __syncthreads();
    if (g < G) {
#pragma unroll
      for (int j = 0; j < 16; ++j) s_acc[g * C + c][j] = sacc[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16 * 256 / kHeadT; ++j) {
      const int o = t + j * kHeadT, oc = o >> 4, ok = kb + (o & 15);
      if (oc < C && ok < K) {
        int sum = 0;
        for (int gg = 0; gg < G; ++gg) sum += s_acc[gg * C + oc][o & 15];
        if (x.buf) {
          x.buf[(h.dw - x.gbase) + oc * K + ok] = (long long)sum;
          continue;
        }
        const float a = (float)(long long)sum * wscale;
        const float b = h.wd2 * wf[j];
        const float gv = a + b;
        h.dw[oc * K + ok] = gv;
        if (u.w) {  // sgd_momentum_elem's arithmetic (gscale 1)
          const float tm = u.mu * af[j];
          const float an = tm + gv;
          LBT_ST_TAIL(u.a + ob + oc * K + ok, an);
          const float stp = u.lr * an;
          LBT_ST_TAIL(u.w + ob + oc * K + ok, wf[j] - stp);
        }
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

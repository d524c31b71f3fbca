// head.hip -- the classifier head of CIFAR10_Resnet20 (AvgPool_q -> Dense_q -> softmax
// cross-entropy, and back) per sample in ONE launch, one workgroup per sample: pool, quantise,
// logits, softmax, dz, quantise, dgrad, un-pool, and a record (pq, gq, loss term) from which
// lbt_step_reduce forms the batch reductions (Dense_q dW, mean loss; head.h).
//
// Replaces seven launches of ~5 us each whose work is a few KB; every value is computed by the
// same operations, in the same order, as those kernels (misc.hip avgpool / softmax_xent,
// quantize.hip quant1, conv_generic.hip fwd / dgrad), so the results are bit-identical
// (tests/test_gpu_parity.py::test_head_kernel_equals_launch_sequence).
//
// Latency, not bandwidth, is what a per-sample workgroup pays, so every global load is issued
// at the top (branch-free), and every loop over channels / classes is spread over the
// workgroup's 256 threads (integer partial sums are exact in any order; the fp32 sums keep the
// reference order).
//
// Reference: AvgPool_q dynamic_fixed_point.py:1009-1022, Dense_q :319-395 / :441-466,
// loss models.py:30-32.
#include "head.h"

namespace lbt {
namespace {

constexpr int kT = kHeadT;
constexpr int kXChunk = 16384;   // bytes of x staged per pass (pixels x C floats)
constexpr int kMaxW = 256 * 64;  // Dense_q weight codes C x K

// The noise of index i (< n) of a quantiser: its table when it has one, else Philox inline --
// branch-free (both formed, the table read from a clamped address) so that no wait for the
// load is forced at a control-flow join.
LBT_DEV float head_noise(const lbt_qdesc& q, const QState& s, int i, int n) {
  const bool tab = q.noise != nullptr;
  const float tv = (tab ? q.noise : zf())[tab ? (i < n ? i : n - 1) : 0];
  const float pv = noise1((uint64_t)i, q.qid, s.step, q.seed);
  return (s.active && q.stochastic) ? (tab ? tv : pv) : 0.f;
}

__global__ __launch_bounds__(kT) void head_kernel(lbt_head h) {
  __shared__ __attribute__((aligned(16))) float s_x[kXChunk / 4];
  __shared__ __attribute__((aligned(16))) int8_t s_w[kMaxW];
  __shared__ int s_pq[256], s_gq[64], s_part[16][16];
  __shared__ float s_z[64], s_dp[256];
  __shared__ int sh_cnt[2 * 2 * (kT / 64)];
  const int n = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int C = h.C, K = h.K, HW = h.HW, N = h.N;
  LBT_TS(0);
  const QState sx = qstate(h.qx), sg = qstate(h.qg);
  int ovx1 = 0, ovx2 = 0, ovg1 = 0, ovg2 = 0;  // wave totals (quant_w)

  // ---- every global load, issued together: Dense_q weight codes, label, noise, first x chunk
  const int nw = C * K / 4;
  uint32_t wv[kMaxW / 4 / kT];
#pragma unroll
  for (int j = 0; j < kMaxW / 4 / kT; ++j) {
    const int i = t + j * kT;
    wv[j] = reinterpret_cast<const uint32_t*>(h.wq)[i < nw ? i : 0];
  }
  const int y = h.labels[n];
  const float ux = head_noise(h.qx, sx, t, C);
  const float ug = head_noise(h.qg, sg, lane, K);
  const int P = (kXChunk / 4) / C;  // pixels per chunk
  constexpr int kV = kXChunk / 16 / kT;
  float4 v[kV];
#define LBT_HEAD_LOAD_CHUNK(p0_)                                                                 \
  do {                                                                                          \
    const int np_ = HW - (p0_) < P ? HW - (p0_) : P;                                             \
    const int nq_ = np_ * C / 4;                                                                 \
    const float4* src_ = reinterpret_cast<const float4*>(h.x + ((int64_t)n * HW + (p0_)) * C);   \
    _Pragma("unroll") for (int j = 0; j < kV; ++j) {                                             \
      const int i_ = t + j * kT;                                                                 \
      v[j] = src_[i_ < nq_ ? i_ : 0];                                                            \
    }                                                                                            \
  } while (0)
  LBT_HEAD_LOAD_CHUNK(0);

  // ---- AvgPool_q: channel t, the HW pixels summed in order (avgpool_fwd_kernel), from LDS
  float acc = 0.f;
  for (int p0 = 0;;) {
    // unconditional: slots past the chunk receive a harmless copy (loads stay un-predicated)
#pragma unroll
    for (int j = 0; j < kV; ++j) reinterpret_cast<float4*>(s_x)[t + j * kT] = v[j];
    if (p0 == 0) {
#pragma unroll
      for (int j = 0; j < kMaxW / 4 / kT; ++j) reinterpret_cast<uint32_t*>(s_w)[t + j * kT] = wv[j];
    }
    __syncthreads();
    const int np = HW - p0 < P ? HW - p0 : P;
    if (t < C) {
      int p = 0;
      for (; p + 8 <= np; p += 8) {  // 8 LDS reads in flight, adds in order
        float r[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = s_x[(p + q) * C + t];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = acc + r[q];
      }
      for (; p < np; ++p) acc = acc + s_x[p * C + t];
    }
    p0 += P;
    if (p0 >= HW) break;
    __syncthreads();
    LBT_HEAD_LOAD_CHUNK(p0);
  }
#undef LBT_HEAD_LOAD_CHUNK
  LBT_TS(1);
  if (t < C) {
    const float pooled = acc * (1.0f / (float)HW);
    if (h.pooled) h.pooled[(int64_t)n * C + t] = pooled;
    // Dense_q X quantiser (:385 stochastic_identity), noise index = channel (X.shape[1:] = [C])
    const int q = sx.active ? quant_w<-1>(sx, h.qx.stochastic, pooled, ux, ovx1, ovx2) : 0;
    s_pq[t] = q;
    if (h.pq) h.pq[(int64_t)n * C + t] = (int8_t)q;
  }
  __syncthreads();

  // ---- Dense_q forward: z[k] = (float)(sum_c pq[c] * wq[c][k]) * 2^-(ex + ew); thread
  // (k & 15, group t >> 4) sums channels c = group, group + 16, ... (exact integers)
  const float sxw = ldexpf(1.0f, -(frac_exp(h.qx) + frac_exp(h.qw)));
  for (int kb = 0; kb < K; kb += 16) {
    const int k = kb + (t & 15), grp = t >> 4;
    int a = 0;
    if (k < K) {
#pragma unroll 4
      for (int c = grp; c < C; c += 16) a += s_pq[c] * (int)s_w[c * K + k];
    }
    s_part[grp][t & 15] = a;
    __syncthreads();
    if (t < 16 && kb + t < K) {
      int z = 0;
#pragma unroll
      for (int gg = 0; gg < 16; ++gg) z += s_part[gg][t];
      const float zf_ = (float)z * sxw;
      s_z[kb + t] = zf_;
      h.logits[(int64_t)n * K + kb + t] = zf_;
    }
    __syncthreads();
  }

  // ---- softmax cross-entropy in wave 0, lane k = class (softmax_xent_kernel's arithmetic:
  // max, then s = sum of expf(z - m) in class order, p = expf(z - m) / s)
  if (wave == 0) {
    const float zk = lane < K ? s_z[lane] : 0.f;
    float m = s_z[0];
    for (int k = 1; k < K; ++k) m = s_z[k] > m ? s_z[k] : m;
    const float e = expf(zk - m);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = s + __shfl(e, k, 64);
    if (lane < K) {
      const float p = e / s;
      const float dz = (p - (lane == y ? 1.f : 0.f)) / (float)(h.loss_n > 0 ? h.loss_n : N);
      h.dz[(int64_t)n * K + lane] = dz;
      // Dense_q grad quantiser (:454), noise index = class
      const int q = sg.active ? quant_w<-1>(sg, h.qg.stochastic, dz, ug, ovg1, ovg2) : 0;
      s_gq[lane] = q;
      if (h.gq) h.gq[(int64_t)n * K + lane] = (int8_t)q;
    }
    if (lane == 0) {
      const float lse = logf(s) + m;
      const double term = (double)(lse - s_z[y]);
      uint8_t* rec = reinterpret_cast<uint8_t*>(h.scratch) + (int64_t)n * (C + kHeadRecPad);
      *reinterpret_cast<double*>(rec + C + 64) = term;  // 8-byte aligned: C % 8 == 0
    }
  }
  counts_stage_w(0, 2, ovx1, ovx2, sh_cnt);
  counts_stage_w(1, 2, ovg1, ovg2, sh_cnt);
  __syncthreads();
  counts_publish(0, 2, h.qx, sh_cnt);
  counts_publish(1, 2, h.qg, sh_cnt);

  // ---- the record's codes: pq[C] | gq[64]
  {
    uint32_t* rec = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(h.scratch) + (int64_t)n * (C + kHeadRecPad));
    if (t < C / 4) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) w |= (uint32_t)(s_pq[4 * t + b] & 255) << (8 * b);
      rec[t] = w;
    } else if (t >= 64 && t < 80) {
      const int j = t - 64;
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) w |= (uint32_t)((4 * j + b < K ? s_gq[4 * j + b] : 0) & 255) << (8 * b);
      rec[C / 4 + j] = w;
    }
  }

  // ---- Dense_q dgrad + AvgPool_q backward: gx[n][p][c] = ((float)(sum_k gq[k] wq[c][k]) * s) * (1/HW)
  if (t < C) {
    int a = 0;
    int k = 0;
    for (; k + 8 <= K; k += 8) {
#pragma unroll
      for (int q = 0; q < 8; ++q) a += s_gq[k + q] * (int)s_w[t * K + k + q];
    }
    for (; k < K; ++k) a += s_gq[k] * (int)s_w[t * K + k];
    s_dp[t] = (float)a * ldexpf(1.0f, -(frac_exp(h.qg) + frac_exp(h.qw)));
  }
  __syncthreads();
  {
    const float inv = 1.0f / (float)HW;
    float4* gx = reinterpret_cast<float4*>(h.gx + (int64_t)n * HW * C);
    const int nq = HW * C / 4;  // C % 4 == 0
    for (int i = t; i < nq; i += kT) {
      const int c = (4 * i) % C;
      gx[i] = make_float4(s_dp[c] * inv, s_dp[c + 1] * inv, s_dp[c + 2] * inv, s_dp[c + 3] * inv);
    }
  }
  LBT_TS(2);
}

}  // namespace
}  // namespace lbt

using namespace lbt;

LBT_TRACE_SETTER(head)

extern "C" int lbt_head_scratch_bytes(int32_t N, int32_t C, int32_t K) {
  (void)K;
  return N * (C + kHeadRecPad);
}

extern "C" int lbt_head_fwd_bwd(const lbt_head* h, void* stream) {
  if (!h || h->N <= 0 || h->HW <= 0 || h->C <= 0 || h->C > 256 || h->C % 8 || h->K <= 0 || h->K > 64) return LBT_EINVAL;
  if (!h->x || !h->wq || !h->labels || !h->logits || !h->dz || !h->gx || !h->scratch) return LBT_EINVAL;
  if ((int64_t)h->N * (h->C + kHeadRecPad) >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if ((reinterpret_cast<uintptr_t>(h->wq) & 3) || (reinterpret_cast<uintptr_t>(h->x) & 15) ||
      (reinterpret_cast<uintptr_t>(h->scratch) & 7))
    return LBT_EINVAL;
  hipLaunchKernelGGL(head_kernel, dim3((unsigned)h->N), dim3(kT), 0, (hipStream_t)stream, *h);
  return (int)hipGetLastError();
}

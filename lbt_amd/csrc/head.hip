// head.hip -- the classifier head of CIFAR10_Resnet20 (AvgPool_q -> Dense_q -> softmax
// cross-entropy, and back) as ONE launch: a workgroup per sample does everything per-sample
// (pool, quantise, logits, softmax, dz, quantise, dgrad, un-pool), and the workgroup that
// arrives last does the two batch reductions (the Dense_q weight gradient and the mean loss).
//
// Replaces eight launches of ~5 us each whose work is a few KB; every value is computed by the
// same operations, in the same order, as those kernels (misc.hip avgpool / softmax_xent,
// quantize.hip quant1, conv_generic.hip fwd / dgrad, conv_mfma.hip wgrad_reduce), so the
// results are bit-identical (tests/test_gpu_parity.py::test_head_kernel_equals_launch_sequence).
//
// Reference: AvgPool_q dynamic_fixed_point.py:1009-1022, Dense_q :319-395 / :441-466,
// loss models.py:30-32.
#include "dfxp_device.h"

namespace lbt {
namespace {

constexpr int kT = 256;
constexpr int kRecPad = 72;  // per-sample scratch record: pq[C] | gq[64] | loss term (double)
constexpr int kXChunk = 16384;   // bytes of x staged per pass (pixels x C floats)
constexpr int kRecBytes = 24576; // last workgroup: sample records per pass
constexpr int kBig = kRecBytes + kT * 16 * 4;
constexpr int kMaxW = 256 * 64;  // Dense_q weight codes C x K
static_assert(kXChunk <= kBig, "x chunk fits the staging area");

LBT_DEV uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// write-through store with no implied wait (the compiler's relaxed atomic store waits for every
// older memory op first); the arrival below drains them with one s_waitcnt
LBT_DEV void st_wt(uint32_t* p, uint32_t v) { asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory"); }

// The noise of index i (< n) of a quantiser: its table when it has one, else Philox inline --
// branch-free (both computed, the table read from a clamped address) so that no wait for the
// load is forced at a control-flow join.
LBT_DEV float head_noise(const lbt_qdesc& q, const QState& s, int i, int n) {
  const bool tab = q.noise != nullptr;
  const float tv = (tab ? q.noise : zf())[tab ? (i < n ? i : n - 1) : 0];
#ifdef LBT_EXP_NOPHILOX
  const float pv = 0.f;
#else
  const float pv = noise1((uint64_t)i, q.qid, s.step, q.seed);
#endif
  return (s.active && q.stochastic) ? (tab ? tv : pv) : 0.f;
}

__global__ __launch_bounds__(kT) void head_kernel(lbt_head h) {
  __shared__ float s_z[64];
  __shared__ int s_pq[256], s_gq[64];
  __shared__ float s_dp[256];
  __shared__ float s_ms[2];
  __shared__ double s_term;
  __shared__ int sh_cnt[2 * 2 * (kT / 64)];
  __shared__ unsigned s_last;
  __shared__ double s_red[kT];
  // phase-shared staging: x pixel chunks first; in the last workgroup sample records + partials
  __shared__ __attribute__((aligned(16))) uint8_t s_big[kBig];
  __shared__ __attribute__((aligned(16))) int8_t s_w[kMaxW];
  float* s_x = reinterpret_cast<float*>(s_big);
  uint32_t* s_rec = reinterpret_cast<uint32_t*>(s_big);
  int(*s_acc)[16] = reinterpret_cast<int(*)[16]>(s_big + kRecBytes);
  const int n = blockIdx.x, t = threadIdx.x;
  const int C = h.C, K = h.K, HW = h.HW, N = h.N;
  const QState sx = qstate(h.qx), sg = qstate(h.qg);
  int ovx1 = 0, ovx2 = 0, ovg1 = 0, ovg2 = 0;  // wave totals (quant_w)

  // ---- every global load this workgroup needs, issued together: the first x chunk (coalesced
  // 16-B loads), the Dense_q weight codes, the label and both quantisers' noise
  LBT_TS(0);
  const int P = (kXChunk / 4) / C;  // pixels per chunk
  constexpr int kV = kXChunk / 16 / kT;
  float4 v[kV];
#define LBT_HEAD_LOAD_CHUNK(p0_)                                                                       \
  do {                                                                                                \
    const int np_ = HW - (p0_) < P ? HW - (p0_) : P;                                                   \
    const int nq_ = np_ * C / 4;                                                                       \
    const float4* src_ = reinterpret_cast<const float4*>(h.x + ((int64_t)n * HW + (p0_)) * C);         \
    _Pragma("unroll") for (int j = 0; j < kV; ++j) {                                                   \
      const int i_ = t + j * kT;                                                                       \
      v[j] = src_[i_ < nq_ ? i_ : 0];                                                                  \
    }                                                                                                  \
  } while (0)
  const int nw = C * K / 4;
  uint32_t wv[kMaxW / 4 / kT];
#pragma unroll
  for (int j = 0; j < kMaxW / 4 / kT; ++j) {
    const int i = t + j * kT;
    wv[j] = reinterpret_cast<const uint32_t*>(h.wq)[i < nw ? i : 0];
  }
  const int y = h.labels[n];
  const float ux = head_noise(h.qx, sx, t, C);
  const float ug = head_noise(h.qg, sg, t, K);
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
    if (p0 == 0) LBT_TS(5);
    const int np = HW - p0 < P ? HW - p0 : P;
    if (t < C)
      for (int p = 0; p < np; ++p) acc = acc + s_x[p * C + t];
    p0 += P;
    if (p0 >= HW) break;
    __syncthreads();
    LBT_HEAD_LOAD_CHUNK(p0);
  }
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

  LBT_TS(6);
  // ---- Dense_q forward: z[k] = (float)(sum_c pq[c] * wq[c][k]) * 2^-(ex + ew)
  if (t < K) {
    int a = 0;
    for (int c = 0; c < C; ++c) a += s_pq[c] * (int)s_w[c * K + t];
    const float z = (float)a * ldexpf(1.0f, -(frac_exp(h.qx) + frac_exp(h.qw)));
    s_z[t] = z;
    h.logits[(int64_t)n * K + t] = z;
  }
  __syncthreads();

  // ---- softmax cross-entropy (softmax_xent_kernel's per-row arithmetic)
  if (t == 0) {
    float m = s_z[0];
    for (int k = 1; k < K; ++k) m = s_z[k] > m ? s_z[k] : m;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = s + expf(s_z[k] - m);
    s_ms[0] = m;
    s_ms[1] = s;
    const float lse = logf(s) + m;
    s_term = (double)(lse - s_z[y]);
  }
  __syncthreads();
  if (t < K) {
    const float m = s_ms[0], s = s_ms[1];
    const float p = expf(s_z[t] - m) / s;
    const float dz = (p - (t == y ? 1.f : 0.f)) / (float)N;
    h.dz[(int64_t)n * K + t] = dz;
    // Dense_q grad quantiser (:454), noise index = class
    const int q = sg.active ? quant_w<-1>(sg, h.qg.stochastic, dz, ug, ovg1, ovg2) : 0;
    s_gq[t] = q;
    if (h.gq) h.gq[(int64_t)n * K + t] = (int8_t)q;
  }
  counts_stage_w(0, 2, ovx1, ovx2, sh_cnt);
  counts_stage_w(1, 2, ovg1, ovg2, sh_cnt);
  __syncthreads();

  // ---- this sample's record for the batch reductions (one write-through word per lane):
  // pq[C] | gq[16 words] | loss term
  const int rs = C + kRecPad;
  uint8_t* scr = reinterpret_cast<uint8_t*>(h.scratch);
  if (t < rs / 4) {
    uint32_t v = 0;
    if (t < C / 4) {
#pragma unroll
      for (int b = 0; b < 4; ++b) v |= (uint32_t)(s_pq[4 * t + b] & 255) << (8 * b);
    } else if (t < C / 4 + 16) {
      const int j = t - C / 4;
#pragma unroll
      for (int b = 0; b < 4; ++b) v |= (uint32_t)((4 * j + b < K ? s_gq[4 * j + b] : 0) & 255) << (8 * b);
    } else {
      const uint64_t bits = (uint64_t)__double_as_longlong(s_term);
      v = t == C / 4 + 16 ? (uint32_t)bits : (uint32_t)(bits >> 32);
    }
    st_wt(reinterpret_cast<uint32_t*>(scr + (int64_t)n * rs) + t, v);
  }
  counts_publish(0, 2, h.qx, sh_cnt);
  counts_publish(1, 2, h.qg, sh_cnt);

  // ---- Dense_q dgrad + AvgPool_q backward: gx[n][p][c] = ((float)(sum_k gq[k] wq[c][k]) * s) * (1/HW)
  if (t < C) {
    int a = 0;
    for (int k = 0; k < K; ++k) a += s_gq[k] * (int)s_w[t * K + k];
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
  // ---- arrive: every storing wave drains its stores, then one lane takes a ticket
  LBT_TS(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) s_last = __hip_atomic_fetch_add(h.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)N - 1;
  __syncthreads();
  LBT_TS(3);
  if (!s_last) return;

  // ---- last workgroup: dW = dequant(sum_n pq[n]^T gq[n]) + wd2 * w, and the mean loss.
  // Thread (c, g) = (t % C, t / C) accumulates channel c against 16 classes over samples g, g+G, ...
  const int words = rs / 4;
  const int chunk = (kRecBytes / 4) / words;  // samples per LDS chunk
  const int G = kT / C, c = t % C, g = t / C;
  const float wscale = ldexpf(1.0f, -(frac_exp(h.qx) + frac_exp(h.qg)));
  double part = 0.0;
  for (int kb = 0; kb < K; kb += 16) {
    // this pass's fp32 weights (decay term), loaded ahead of the sample loop
    float wf[16 * 256 / kT];
#pragma unroll
    for (int j = 0; j < 16 * 256 / kT; ++j) {
      const int o = t + j * kT, oc = o >> 4, ok = kb + (o & 15);
      wf[j] = h.w[(oc < C && ok < K) ? oc * K + ok : 0];
    }
    int sacc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) sacc[j] = 0;
    for (int n0 = 0; n0 < N; n0 += chunk) {
      const int nn = N - n0 < chunk ? N - n0 : chunk;
      __syncthreads();
      const uint32_t* src = reinterpret_cast<const uint32_t*>(scr + (int64_t)n0 * rs);
      {  // every load in flight before the first LDS write (clamped addresses, no branches)
        const int lim = nn * words;
        uint32_t v[kRecBytes / 4 / kT];
#pragma unroll
        for (int j = 0; j < kRecBytes / 4 / kT; ++j) {
          const int i = t + j * kT;
          v[j] = ld_sc1(src + (i < lim ? i : 0));
        }
#pragma unroll
        for (int j = 0; j < kRecBytes / 4 / kT; ++j) s_rec[t + j * kT] = v[j];
      }
      __syncthreads();
      const uint8_t* r8 = reinterpret_cast<const uint8_t*>(s_rec);
      if (g < G) {
        for (int r = g; r < nn; r += G) {
          const int x = (int)(int8_t)r8[r * rs + c];
          const uint32_t* gw = s_rec + r * words + C / 4 + kb / 4;
#pragma unroll
          for (int w4 = 0; w4 < 4; ++w4) {
            const uint32_t v = gw[w4];
#pragma unroll
            for (int b = 0; b < 4; ++b) sacc[4 * w4 + b] += x * (int)(int8_t)(v >> (8 * b));
          }
        }
      }
      if (kb == 0) {  // loss terms: thread t sums rows t, t + 256, ... in order (softmax_xent_kernel)
        for (int r = 0; r < nn; ++r)
          if (((n0 + r) & (kT - 1)) == t) {
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
    for (int j = 0; j < 16 * 256 / kT; ++j) {
      const int o = t + j * kT, oc = o >> 4, ok = kb + (o & 15);
      if (oc < C && ok < K) {
        int sum = 0;
        for (int gg = 0; gg < G; ++gg) sum += s_acc[gg * C + oc][o & 15];
        const float a = (float)(long long)sum * wscale;
        const float b = h.wd2 * wf[j];
        h.dw[oc * K + ok] = a + b;
      }
    }
  }
  s_red[t] = part;
  __syncthreads();
  for (int o = kT / 2; o > 0; o >>= 1) {
    if (t < o) s_red[t] += s_red[t + o];
    __syncthreads();
  }
  if (t == 0) {
    h.loss[0] = (float)(s_red[0] / (double)N);
    LBT_TS(4);
    __hip_atomic_store(h.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace
}  // namespace lbt

using namespace lbt;

LBT_TRACE_SETTER(head)

extern "C" int lbt_head_scratch_bytes(int32_t N, int32_t C, int32_t K) {
  (void)K;
  return N * (C + kRecPad);
}

extern "C" int lbt_head_fwd_bwd(const lbt_head* h, void* stream) {
  if (!h || h->N <= 0 || h->HW <= 0 || h->C <= 0 || h->C > 256 || h->C % 4 || h->K <= 0 || h->K > 64) return LBT_EINVAL;
  if (!h->x || !h->wq || !h->labels || !h->logits || !h->loss || !h->dz || !h->w || !h->dw || !h->gx || !h->scratch ||
      !h->ticket)
    return LBT_EINVAL;
  if ((int64_t)h->N * (h->C + kRecPad) >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if ((int64_t)h->N * 128 * 128 >= ((int64_t)1 << 31)) return LBT_EINVAL;  // int32 dW sums
  if ((h->C + kRecPad) > kRecBytes || h->C * h->K > kMaxW || (reinterpret_cast<uintptr_t>(h->wq) & 3) ||
      (reinterpret_cast<uintptr_t>(h->x) & 15))
    return LBT_EINVAL;
  hipLaunchKernelGGL(head_kernel, dim3((unsigned)h->N), dim3(kT), 0, (hipStream_t)stream, *h);
  return (int)hipGetLastError();
}

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
#include "bn_moments.h"
#include "head.h"
#include "pk2.h"

namespace lbt {
namespace {

constexpr int kT = kHeadT;
// Phase stamps (scratch -DLBT_TRACE builds); -DLBT_HEADSTUDY: 1 = loads issued, 2 = end chain done, 3 = pool,
// 4 = logits, 5 = softmax + counters
#ifdef LBT_HEADSTUDY
#define LBT_HSS(i) LBT_TS(i)
#define LBT_HTS(i) do { if ((i) == 1) LBT_TS(3); else if ((i) == 2) LBT_TS(4); else if ((i) == 3) LBT_TS(5); } while (0)
#else
#define LBT_HSS(i) do { } while (0)
#define LBT_HTS(i) LBT_TS(i)
#endif
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

// lane k's value of v (k wave-uniform)
LBT_DEV float lane_f(float v, int k) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
}

// Pass A (bn.hip chain_bwd_a_kernel<1, kAFB | kAStoch | kAYMask | kAGmask>'s arithmetic, element for
// element) of sample n's gradient g[p][c] = s_dp[c] * (1/HW), the value the un-pool writes: ReLU
// mask from y_mask, gmask_out, the Rescale_q gradient quantiser (sums G2*R, G2), times gamma_q, the
// Normalization_q gradient quantiser (codes to gout, sums G, G*q), overflow counters. Thread t owns
// the channel quad c0 = 4t mod C of quads t, t + 256, ... (C | 1024). Every thread calls it.
// Sample n's pass-A operands of the first kPaPre quad passes (y mask, R / qn codes, the two noise
// tables' values when the quantisers have tables), loaded at the top of head_kernel so that their
// latency hides behind the pooling / logits / softmax instead of following them. Clamped
// addresses, no branches (the values are selected where they are used).
constexpr int kPaPre = 4;
struct HeadPaPre {
  float4 ym[kPaPre], nr[kPaPre], nn[kPaPre];
  int R[kPaPre], qn[kPaPre];
};
LBT_DEV bool head_pa_prefetchable(int HW, int C) { return HW * C / 4 <= kPaPre * kT; }
LBT_DEV void head_pa_prefetch(const lbt_chain_bwd_a& a, int n, int HW, int C, int q0, int q1, HeadPaPre& p,
                              bool operands = true) {
  const lbt_bwd_branch& B = a.b1;
  const int t = threadIdx.x;
  const int64_t base = (int64_t)n * HW * C;
  const float* tr = B.qrg.noise ? B.qrg.noise : zf();
  const float* tn = B.qng.noise ? B.qng.noise : zf();
  const uint32_t mr = B.qrg.noise ? 0xffffffffu : 0u, mn = B.qng.noise ? 0xffffffffu : 0u;
#pragma unroll
  for (int it = 0; it < kPaPre; ++it) {
    const int q = q0 + t + it * kT, qq = q < q1 ? q : q0;
    const int64_t e = base + 4 * (int64_t)qq;
    if (operands) {  // else the caller's end chain supplies them (lbt_head.chain)
      p.ym[it] = *reinterpret_cast<const float4*>(a.y_mask + e);
      p.R[it] = *reinterpret_cast<const int*>(B.R + e);
      p.qn[it] = *reinterpret_cast<const int*>(B.qn_codes + e);
    }
    p.nr[it] = *reinterpret_cast<const float4*>(tr + ((4u * (uint32_t)qq) & mr));
    p.nn[it] = *reinterpret_cast<const float4*>(tn + ((4u * (uint32_t)qq) & mn));
  }
}

// use_pre: pre holds head_pa_prefetch's operands (HW * C / 4 <= kPaPre * kT); else loaded here
// (quads [q0, q1) of the sample: the workgroup's share, q0 % (C / 4) == 0)
LBT_DEV void head_pass_a(const lbt_chain_bwd_a& a, int n, int HW, int C, int q0, int q1, const float* s_dp,
                         int* sh_cnt, const HeadPaPre& pre, bool use_pre) {
  __shared__ int s_sum[kT / 64][4 * 256];  // per wave: [sum][channel] (|.| < 2^19)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const lbt_bwd_branch& B = a.b1;
  const QState qrg = qstate(B.qrg), qng = qstate(B.qng);
  const int c0 = (4 * t) % C;
  const int64_t base = (int64_t)n * HW * C;
  const float inv = 1.0f / (float)HW;
  float gam[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) gam[k] = B.gb[c0 + k];
  int ov[2][2] = {{0, 0}, {0, 0}};
  int acc[4][4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[s][k] = 0;
  const bool sr = qrg.active && B.qrg.stochastic, sn = qng.active && B.qng.stochastic;
  // one quad pass (C % 4 == 0, so c0 is this thread's quad in every pass)
  auto pass = [&](int q, const float4& ym4, int Rw, int qw, const Noise4& nrg, const Noise4& nng) {
    const int64_t e = base + 4 * (int64_t)q;
    const float ym[4] = {ym4.x, ym4.y, ym4.z, ym4.w};
    float gv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float g = s_dp[c0 + k] * inv;
      gv[k] = ym[k] > 0.f ? g : 0.f;
    }
    if (a.gmask_out) st_out16(a.gmask_out + e, make_float4(gv[0], gv[1], gv[2], gv[3]));
    int G[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int R = (int)(int8_t)(Rw >> (8 * k)), qn = (int)(int8_t)(qw >> (8 * k));
      const int G2 = quant_w<1>(qrg, 1, gv[k], nrg.u[k], ov[0][0], ov[0][1]);
      acc[0][k] += G2 * R;
      acc[1][k] += G2;
      const float gh = (float)G2 * qrg.inv_m;
      const float d = gh * gam[k];
      G[k] = quant_w<1>(qng, 1, d, nng.u[k], ov[1][0], ov[1][1]);
      acc[2][k] += G[k];
      acc[3][k] += G[k] * qn;
    }
    st_out(B.gout + e,
           (int)((uint32_t)(G[0] & 255) | ((uint32_t)(G[1] & 255) << 8) | ((uint32_t)(G[2] & 255) << 16) | ((uint32_t)G[3] << 24)));
  };
  const Noise4 z4 = {{0.f, 0.f, 0.f, 0.f}};
  if (use_pre) {  // uniform
#pragma unroll
    for (int it = 0; it < kPaPre; ++it) {
      const int q = q0 + t + it * kT;
      if (q >= q1) break;
      const Noise4 nrg = !sr ? z4 : B.qrg.noise ? Noise4{{pre.nr[it].x, pre.nr[it].y, pre.nr[it].z, pre.nr[it].w}}
                                                : qnoise4(B.qrg, qrg.step, (uint64_t)q);
      const Noise4 nng = !sn ? z4 : B.qng.noise ? Noise4{{pre.nn[it].x, pre.nn[it].y, pre.nn[it].z, pre.nn[it].w}}
                                                : qnoise4(B.qng, qng.step, (uint64_t)q);
      pass(q, pre.ym[it], pre.R[it], pre.qn[it], nrg, nng);
    }
  } else {
    for (int q = q0 + t; q < q1; q += kT) {
      const int64_t e = base + 4 * (int64_t)q;
      const float4 ym4 = *reinterpret_cast<const float4*>(a.y_mask + e);
      const int Rw = *reinterpret_cast<const int*>(B.R + e);
      const int qw = *reinterpret_cast<const int*>(B.qn_codes + e);
      const Noise4 nrg = sr ? qnoise4(B.qrg, qrg.step, (uint64_t)q) : z4;
      const Noise4 nng = sn ? qnoise4(B.qng, qng.step, (uint64_t)q) : z4;
      pass(q, ym4, Rw, qw, nrg, nng);
    }
  }
  // channel sums: the lanes sharing a quad (t = c0/4 mod C/4) meet by shuffles within the wave, the
  // waves in LDS; one int64 atomic per (sum, channel) into this sample's shard
  const int per = C / 4;  // lanes l, l + per, ... share a quad (per | 64)
  if (chan_scatter_ok(per)) {  // uniform: row lane >> 4 ends with channel c0 + (lane >> 4)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int v = chan_scatter4(acc[s], per);
      if (chan_scatter_owner(per)) s_sum[wave][s * C + c0 + (lane >> 4)] = v;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int v = acc[s][k];
        for (int o = per; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
        if (lane < per) s_sum[wave][s * C + c0 + k] = v;
      }
  }
  counts_stage_w(2, 5, ov[0][0], ov[0][1], sh_cnt);
  counts_stage_w(3, 5, ov[1][0], ov[1][1], sh_cnt);
  __syncthreads();
  if (qrg.active) counts_publish(2, 5, B.qrg, sh_cnt);
  if (qng.active) counts_publish(3, 5, B.qng, sh_cnt);
  if (B.sums) {
    int64_t* dst = B.sums + (int64_t)shard_id() * 4 * C;
    for (int i = t; i < 4 * C; i += kT) {
      long long v = 0;
#pragma unroll
      for (int w = 0; w < kT / 64; ++w) v += s_sum[w][i];
      if (v) LBT_GADD((unsigned long long*)&dst[i], (unsigned long long)v);
    }
  }
}

// 64-bit sum over the four 16-lane rows of a wave (v_permlane16 / 32 swaps on both halves)
LBT_DEV long long head_rows_total64(long long v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)((unsigned long long)v >> 32);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  v = (long long)(((unsigned long long)b[0] << 32) | a[0]) + (long long)(((unsigned long long)b[1] << 32) | a[1]);
  const uint32_t lo2 = (uint32_t)v, hi2 = (uint32_t)((unsigned long long)v >> 32);
  const auto c = __builtin_amdgcn_permlane32_swap(lo2, lo2, false, false);
  const auto d = __builtin_amdgcn_permlane32_swap(hi2, hi2, false, false);
  return (long long)(((unsigned long long)d[0] << 32) | c[0]) + (long long)(((unsigned long long)d[1] << 32) | c[1]);
}

// The end chain's Normalization_q moment sums (the chain's sharded [32][2C] channel sums), issued as
// the launch's FIRST loads: wave w owns channels 16 w .. 16 w + 15 (C <= 64), lane l channel
// 16 w + (l & 15) of shards 8 (l >> 4) .. + 7 -- each load instruction covers 4 shards x 16 channels.
// (bn_moments had threads c < 2C issue all 32 shard loads each behind the launch's other loads.)
struct HeadStat {
  long long v[8][2];
};
LBT_DEV void head_stat_load(const lbt_bn_norm& b, int C, HeadStat& hs) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = wave * 16 + (lane & 15);
  const int64_t* cs = b.chsum + (int64_t)(8 * (lane >> 4)) * 2 * C + (c < C ? c : 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    hs.v[i][0] = cs[(int64_t)i * 2 * C];
    hs.v[i][1] = cs[(int64_t)i * 2 * C + C];
  }
}
// bn_moments' arithmetic on the loaded sums -> mu / sigma in LDS (and ms / running stats from workgroup 0)
LBT_DEV void head_stat_finish(const lbt_bn_norm& b, int C, const HeadStat& hs, float* mu, float* sg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  long long S1 = 0, S2 = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    S1 += hs.v[i][0];
    S2 += hs.v[i][1];
  }
  S1 = head_rows_total64(S1);
  S2 = head_rows_total64(S2);
  const int c = wave * 16 + (lane & 15);
  if (lane < 16 && c < C) {
    const double s = ldexp(1.0, -frac_exp(b.qn));
    const double mean_d = (double)S1 * s / (double)b.n;
    const double var_d = (double)S2 * (s * s) / (double)b.n - mean_d * mean_d;
    const float m = (float)mean_d, v = (float)var_d;
    const float sigma = sqrtf(v + b.eps);
    mu[c] = m;
    sg[c] = sigma;
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      if (b.ms) { b.ms[c] = m; b.ms[C + c] = sigma; }
      if (b.run_mean) {
        b.run_mean[c] = b.momentum * b.run_mean[c] + b.one_minus_momentum * m;
        b.run_var[c] = b.momentum * b.run_var[c] + b.one_minus_momentum * v;
      }
    }
  }
}

// ---- the last block's end chain inside the head (lbt_head.chain): bn.hip chain_fwd_kernel<1, kFQ |
// kFRes | kFRelu | kFStoch>'s arithmetic, element for element, over the whole sample (kChainSlots
// channel quads per thread; the pooling needs every pixel). Slot j < own covers this workgroup's pass-A
// quads q0 + t + j * kT (the only ones whose Rescale_q overflows it counts), the rest the sample's other
// quads in order, so pass A finds its y mask / R / qn codes in slots 0 .. own - 1.
constexpr int kChainSlots = 4;  // HW * C == 4 * kT * 4 (host check)
struct ChainIn {
  int q[kChainSlots];
  float4 r[kChainSlots], u[kChainSlots];
};
struct ChainOut {
  float4 y[kChainSlots];
  int R[kChainSlots];
};
LBT_DEV int chain_quad(int j, int own, int q0, int Q, int t) {
  return j < own ? q0 + t + j * kT : (q0 + Q / kChainSlots * own + t + (j - own) * kT) % Q;
}
LBT_DEV void chain_load(const lbt_chain_fwd& a, int n, int q0, int own, ChainIn& in) {
  const lbt_chain_branch& B = a.b1;
  const int t = threadIdx.x, Q = (int)(a.inner >> 2);
  const int64_t base = (int64_t)n * a.inner;
#pragma unroll
  for (int j = 0; j < kChainSlots; ++j) {
    const int qd = chain_quad(j, own, q0, Q, t);
    in.q[j] = *reinterpret_cast<const int*>(B.nrm.q + base + 4 * (int64_t)qd);
    in.r[j] = *reinterpret_cast<const float4*>(a.res + base + 4 * (int64_t)qd);
    in.u[j] = *reinterpret_cast<const float4*>(B.qr.noise + 4 * qd);
  }
}
// mu / sigma / gamma_q / beta_q per channel into P[4C] (LDS), then the chain; own slots count qr's
// overflows into ov1 / ov2 (wave totals, quant_w2)
LBT_DEV void chain_eval(const lbt_chain_fwd& a, int own, const ChainIn& in, float* P, long long* tmp, ChainOut& out,
                        int& ov1, int& ov2, const HeadStat& hs, bool hstat) {
  const lbt_chain_branch& B = a.b1;
  const int C = a.C, t = threadIdx.x;
  if (hstat)  // uniform: the sums loaded at the top of the launch
    head_stat_finish(B.nrm, C, hs, P, P + C);
  else
    bn_moments(B.nrm, C, P, P + C, tmp);
  for (int c = t; c < C; c += kT) { P[2 * C + c] = B.gb[c]; P[3 * C + c] = B.gb[C + c]; }
  __syncthreads();
  const int c0 = (4 * t) % C;
  const QState qr = qstate(B.qr);
  const float sn = qscale(B.nrm.qn);
  pf2 pm[2], psy[2], psr[2], pg[2], pb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const Recip r0 = recip(P[C + c0 + 2 * h]), r1 = recip(P[C + c0 + 2 * h + 1]);
    pm[h] = pk(P[c0 + 2 * h], P[c0 + 2 * h + 1]);
    psy[h] = pk(r0.y, r1.y);
    psr[h] = pk(r0.rc, r1.rc);
    pg[h] = pk(P[2 * C + c0 + 2 * h], P[2 * C + c0 + 2 * h + 1]);
    pb[h] = pk(P[3 * C + c0 + 2 * h], P[3 * C + c0 + 2 * h + 1]);
  }
#pragma unroll
  for (int j = 0; j < kChainSlots; ++j) {
    int z1 = 0, z2 = 0;  // the other workgroups' quads: their owner counts them
    const int q[4] = {(int)(int8_t)(in.q[j] & 255), (int)(int8_t)((in.q[j] >> 8) & 255),
                      (int)(int8_t)((in.q[j] >> 16) & 255), (int)(int8_t)(in.q[j] >> 24)};
    const float uu[4] = {in.u[j].x, in.u[j].y, in.u[j].z, in.u[j].w};
    const float rr[4] = {in.r[j].x, in.r[j].y, in.r[j].z, in.r[j].w};
    int R[4];
    float v[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const pf2 x1 = pcvt(q[2 * h], q[2 * h + 1]) * pk(sn, sn);
      const pf2 x2 = x1 - pm[h];
      const pf2 tt = pdiv_nz(x2, psy[h], psr[h]);  // == x2 / sigma (never -0: pk2.h pdiv_nz)
      if (j < own) quant_w2<1>(qr, 1, tt, pk(uu[2 * h], uu[2 * h + 1]), ov1, ov2, R[2 * h], R[2 * h + 1]);
      else quant_w2<1>(qr, 1, tt, pk(uu[2 * h], uu[2 * h + 1]), z1, z2, R[2 * h], R[2 * h + 1]);
      const pf2 xr = pcvt(R[2 * h], R[2 * h + 1]) * pk(qr.inv_m, qr.inv_m);
      const pf2 m1 = xr * pg[h];
      const pf2 t2 = m1 + pb[h];
      const pf2 y2 = t2 + pk(rr[2 * h], rr[2 * h + 1]);
      v[2 * h] = y2.x;
      v[2 * h + 1] = y2.y;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
    out.y[j] = make_float4(v[0], v[1], v[2], v[3]);
    out.R[j] = (int)((uint32_t)(R[0] & 255) | ((uint32_t)(R[1] & 255) << 8) | ((uint32_t)(R[2] & 255) << 16) |
                     ((uint32_t)R[3] << 24));
  }
}

// S workgroups per sample (grid N * S): each one pools, quantises, takes the logits, softmax and
// dgrad of its sample (the same operations on the same operands: identical values, a few KB from
// L2), and runs pass A / the un-pool over its 1/S of the sample's pixels; workgroup s == 0 alone
// writes the sample's outputs and counts its Dense_q quantisers.
// FAST (CHAIN, Dense_q weights <= 1 KB, noise tables for both Dense_q quantisers -- the ResNet-20 step): one
// weight word per thread instead of the kMaxW-sized clamped sweep, the tables read without the branch-free
// Philox twin, and the loads the dense layer needs issued AFTER the end chain's operands (vmcnt waits are
// in issue order: the chain no longer waits for the weights)
template <bool CHAIN, bool FAST = false>
__global__ __launch_bounds__(kT) void head_kernel(lbt_head h, lbt_chain_bwd_a pa, lbt_chain_fwd ch, int S) {
  static_assert(!FAST || CHAIN, "the fast head is the chain head");
  __shared__ __attribute__((aligned(16))) float s_x[kXChunk / 4];
  __shared__ __attribute__((aligned(16))) int8_t s_w[kMaxW];
  __shared__ int s_pq[256], s_gq[64], s_part[16][16];
  __shared__ float s_z[64], s_dp[256];
  __shared__ int sh_cnt[5 * 2 * (kT / 64)];  // counters: qx, qg (+ pass A's qrg, qng) (+ the chain's qr)
  const int n = (int)blockIdx.x / S, split = (int)blockIdx.x - n * S, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const bool lead = split == 0;
  const int C = h.C, K = h.K, HW = h.HW, N = h.N;
  const int q0 = split * (HW / S) * C / 4, q1 = q0 + (HW / S) * C / 4;  // host: HW % S == 0
  LBT_TS(0);
  // the end chain's moment sums before anything else (they gate the chain)
  HeadStat hs;
  const bool hstat = CHAIN && ch.C <= 4 * 16;  // uniform: one 16-channel group per wave
  if (hstat) head_stat_load(ch.b1.nrm, ch.C, hs);
  const QState sx = qstate(h.qx), sg = qstate(h.qg);
  int ovx1 = 0, ovx2 = 0, ovg1 = 0, ovg2 = 0;  // wave totals (quant_w)

  // ---- every global load, issued together: Dense_q weight codes, label, noise, first x chunk
  const int nw = C * K / 4;
  constexpr int kWv = FAST ? 1 : kMaxW / 4 / kT;
  uint32_t wv[kWv];
  int y;
  float ux, ug;
  auto load_dense = [&]() {
#pragma unroll
    for (int j = 0; j < kWv; ++j) {
      const int i = t + j * kT;
      wv[j] = reinterpret_cast<const uint32_t*>(h.wq)[i < nw ? i : 0];
    }
    y = h.labels[n];
    if constexpr (FAST) {  // both quantisers stochastic with tables (host check)
      ux = h.qx.noise[t < C ? t : C - 1];
      ug = h.qg.noise[lane < K ? lane : K - 1];
    } else {
      ux = head_noise(h.qx, sx, t, C);
      ug = head_noise(h.qg, sg, lane, K);
    }
  };
  if constexpr (!FAST) load_dense();
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
  // chain mode: the end chain's operands instead of the block output (the whole sample in one chunk)
  ChainIn cin;
  const int own = kChainSlots / S;
  if constexpr (CHAIN) chain_load(ch, n, q0, own, cin);
  else LBT_HEAD_LOAD_CHUNK(0);
  // the fused pass A's operands, in flight from here
  HeadPaPre pre;
  const bool pre_ok = h.pa && head_pa_prefetchable(HW / S, C);  // uniform
  if (pre_ok) head_pa_prefetch(pa, n, HW, C, q0, q1, pre, !CHAIN);
  if constexpr (FAST) load_dense();
  LBT_HSS(1);  // every load of the top issued
  int ovr1 = 0, ovr2 = 0;
  if constexpr (CHAIN) {
    // the chain's block output into s_x (pooling) and, for this workgroup's quads, pass A's operands
    // (y mask, R codes, and the qn codes: the chain's input)
    __shared__ float s_P[4 * 256];
    __shared__ long long s_t[2 * 256];
    ChainOut co;
    chain_eval(ch, own, cin, s_P, s_t, co, ovr1, ovr2, hs, hstat);
    LBT_HSS(2);  // moments + the end chain done
    const int Q = HW * C / 4;
#pragma unroll
    for (int j = 0; j < kChainSlots; ++j) reinterpret_cast<float4*>(s_x)[chain_quad(j, own, q0, Q, t)] = co.y[j];
#pragma unroll
    for (int j = 0; j < kPaPre; ++j)
      if (j < own) {
        pre.ym[j] = co.y[j];
        pre.R[j] = co.R[j];
        pre.qn[j] = cin.q[j];
      }
  }

  // ---- AvgPool_q: channel t, the HW pixels summed in order (avgpool_fwd_kernel), from LDS
  float acc = 0.f;
  for (int p0 = 0;;) {
    // unconditional: slots past the chunk receive a harmless copy (loads stay un-predicated)
    if constexpr (!CHAIN) {
#pragma unroll
      for (int j = 0; j < kV; ++j) reinterpret_cast<float4*>(s_x)[t + j * kT] = v[j];
    }
    if (p0 == 0) {
#pragma unroll
      for (int j = 0; j < kWv; ++j) reinterpret_cast<uint32_t*>(s_w)[t + j * kT] = wv[j];
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
    if constexpr (!CHAIN) LBT_HEAD_LOAD_CHUNK(p0);
  }
#undef LBT_HEAD_LOAD_CHUNK
  LBT_HTS(1);
  if (t < C) {
    const float pooled = acc * (1.0f / (float)HW);
    if (h.pooled && lead) h.pooled[(int64_t)n * C + t] = pooled;
    // Dense_q X quantiser (:385 stochastic_identity), noise index = channel (X.shape[1:] = [C])
    const int q = sx.active ? quant_w<-1>(sx, h.qx.stochastic, pooled, ux, ovx1, ovx2) : 0;
    s_pq[t] = q;
    if (h.pq && lead) h.pq[(int64_t)n * C + t] = (int8_t)q;
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
      if (lead) h.logits[(int64_t)n * K + kb + t] = zf_;
    }
    __syncthreads();
  }

  LBT_HTS(2);
  // ---- softmax cross-entropy in wave 0, lane k = class (softmax_xent_kernel's arithmetic:
  // max, then s = sum of expf(z - m) in class order, p = expf(z - m) / s)
  if (wave == 0) {
    // the class loops read lane k's value with v_readlane (no LDS / ds_bpermute round trip per
    // class; same values, same order)
    const float zk = lane < K ? s_z[lane] : 0.f;
    float m = lane_f(zk, 0);
    for (int k = 1; k < K; ++k) {
      const float zc = lane_f(zk, k);
      m = zc > m ? zc : m;
    }
    const float e = expf(zk - m);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = s + lane_f(e, k);
    if (lane < K) {
      const float p = e / s;
      const float dz = (p - (lane == y ? 1.f : 0.f)) / (float)(h.loss_n > 0 ? h.loss_n : N);
      if (lead) h.dz[(int64_t)n * K + lane] = dz;
      // Dense_q grad quantiser (:454), noise index = class
      const int q = sg.active ? quant_w<-1>(sg, h.qg.stochastic, dz, ug, ovg1, ovg2) : 0;
      s_gq[lane] = q;
      if (h.gq && lead) h.gq[(int64_t)n * K + lane] = (int8_t)q;
    }
    if (lane == 0 && lead) {
      const float lse = logf(s) + m;
      const double term = (double)(lse - s_z[y]);
      reinterpret_cast<double*>(reinterpret_cast<uint8_t*>(h.scratch) + head_term_off(N, C))[n] = term;
    }
  }
  counts_stage_w(0, 5, ovx1, ovx2, sh_cnt);
  counts_stage_w(1, 5, ovg1, ovg2, sh_cnt);
  if constexpr (CHAIN) counts_stage_w(4, 5, ovr1, ovr2, sh_cnt);
  __syncthreads();
  if (lead) {
    counts_publish(0, 5, h.qx, sh_cnt);
    counts_publish(1, 5, h.qg, sh_cnt);
  }
  if constexpr (CHAIN) counts_publish(4, 5, ch.b1.qr, sh_cnt);

  LBT_HTS(3);
  // ---- the sample's column of the transposed records (head.h): pqT[c][n], gqT[k][n]
  if (lead) {
    uint8_t* scr = reinterpret_cast<uint8_t*>(h.scratch);
    const int NP = head_np(N);
    if (t < C) scr[(int64_t)t * NP + n] = (uint8_t)s_pq[t];
    if (t < K) scr[head_gq_off(N, C) + (int64_t)t * NP + n] = (uint8_t)s_gq[t];
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
  LBT_HTS(4);
  if (h.pa) {  // uniform (the descriptor itself travels by value in pa)
    head_pass_a(pa, n, HW, C, q0, q1, s_dp, sh_cnt, pre, pre_ok);
    LBT_HTS(5);
    return;
  }
  {
    const float inv = 1.0f / (float)HW;
    float4* gx = reinterpret_cast<float4*>(h.gx + (int64_t)n * HW * C);
    for (int i = q0 + t; i < q1; i += kT) {  // C % 4 == 0
      const int c = (4 * i) % C;
      gx[i] = make_float4(s_dp[c] * inv, s_dp[c + 1] * inv, s_dp[c + 2] * inv, s_dp[c + 3] * inv);
    }
  }
  LBT_HTS(5);
}

}  // namespace
}  // namespace lbt

using namespace lbt;

LBT_TRACE_SETTER(head)

extern "C" int lbt_head_scratch_bytes(int32_t N, int32_t C, int32_t K) {
  (void)K;
  return (int)head_scratch_bytes(N, C);
}

extern "C" int lbt_head_fwd_bwd(const lbt_head* h, void* stream) {
  if (!h || h->N <= 0 || h->HW <= 0 || h->C <= 0 || h->C > 256 || h->C % 8 || h->K <= 0 || h->K > 64) return LBT_EINVAL;
  if ((!h->x && !h->chain) || !h->wq || !h->labels || !h->logits || !h->dz || (!h->gx && !h->pa) || !h->scratch)
    return LBT_EINVAL;
  lbt_chain_fwd ch{};
  if (h->chain) {  // the end chain's configuration (see the header); it rides on the fused pass A
    ch = *h->chain;
    const lbt_chain_branch& B = ch.b1;
    if (!h->pa || ch.has_b2 || ch.C != h->C || ch.rows != h->N || ch.inner != (int64_t)h->HW * h->C ||
        ch.inner != 4 * kT * kChainSlots || !B.nrm.q || B.nrm.frozen || !B.nrm.chsum || !B.gb || B.qr.bits <= 0 ||
        !B.qr.stochastic || !B.qr.noise || !ch.res || !ch.relu || (ch.o1 && ch.qo1.bits > 0) ||
        (ch.o2 && ch.qo2.bits > 0) || (reinterpret_cast<uintptr_t>(ch.res) & 15) ||
        (reinterpret_cast<uintptr_t>(B.qr.noise) & 15))
      return LBT_EINVAL;
  }
  if (h->pa) {  // the fused pass A: one branch, y mask, stochastic quantisers, C | 1024, C <= 256
    const lbt_chain_bwd_a& a = *h->pa;
    if (a.has_b2 || !a.y_mask || a.C != h->C || a.rows != h->N || a.inner != (int64_t)h->HW * h->C ||
        (1024 % h->C) || !a.b1.R || !a.b1.qn_codes || !a.b1.gout || !a.b1.gb || a.b1.qrg.bits <= 0 ||
        a.b1.qng.bits <= 0 || !a.b1.qrg.stochastic || !a.b1.qng.stochastic)
      return LBT_EINVAL;
  }
  if (head_scratch_bytes(h->N, h->C) >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if ((reinterpret_cast<uintptr_t>(h->wq) & 3) || (reinterpret_cast<uintptr_t>(h->x) & 15) ||
      (reinterpret_cast<uintptr_t>(h->scratch) & 7))
    return LBT_EINVAL;
  lbt_chain_bwd_a pa{};
  if (h->pa) pa = *h->pa;
  // workgroups per sample: the pass A / un-pool split over up to LBT_HEAD_SPLIT pixel ranges (default 2;
  // 4 when 2 per sample leave the launch with fewer workgroups than CUs -- small per-GPU batches:
  // 17.0 -> 15.6 us at B=16)
  static const int senv = [] {
    const char* e = getenv("LBT_HEAD_SPLIT");
    return e ? atoi(e) : 0;
  }();
  const int smax = senv > 0 ? senv : (h->N * 2 < 256 ? 4 : 2);
  int S = smax;
  while (S > 1 && (h->HW % S || (int64_t)h->N * S > 0x7fffffff || (h->chain && kChainSlots % S))) --S;
  const bool fast = h->chain && h->C * h->K <= 4 * kT && h->qx.noise && h->qg.noise && h->qx.bits > 0 && h->qg.bits > 0 &&
                    h->qx.stochastic && h->qg.stochastic;
  if (fast)
    hipLaunchKernelGGL((head_kernel<true, true>), dim3((unsigned)(h->N * S)), dim3(kT), 0, (hipStream_t)stream, *h, pa, ch, S);
  else if (h->chain)
    hipLaunchKernelGGL(head_kernel<true>, dim3((unsigned)(h->N * S)), dim3(kT), 0, (hipStream_t)stream, *h, pa, ch, S);
  else
    hipLaunchKernelGGL(head_kernel<false>, dim3((unsigned)(h->N * S)), dim3(kT), 0, (hipStream_t)stream, *h, pa, ch, S);
  return (int)hipGetLastError();
}

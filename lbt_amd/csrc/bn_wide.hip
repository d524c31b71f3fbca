// bn_wide.hip -- BN backward (Rescale_q :686-691, Normalization_q :620-623) for 9..16-bit
// gradient quantisers: the arithmetic of bn.hip's chain_bwd_a /
// chain_bwd_b element for element, with int16 gradient codes and int64 channel sums (int16 x
// int8 products summed over a channel overflow int32).
//
// Layout: workgroup = 64 channels (16 channel quads) x 16 pixel positions, over a run of spb
// samples; grid = (ceil(C/64), ceil(HW/16), ceil(N/spb)). A thread owns ONE position of the sample
// (pixel hw, channels c0..c0+3) and walks it through its samples: the stochastic-rounding noise
// (dynamic_fixed_point.py:32-38: over x.shape[1:], broadcast over the batch) depends on the
// position only, so its Philox call is made once per thread, not once per element (that call
// was what bounded these passes: ~4 quarter-rate 32-bit multiplies per round). A wave reads
// 4 pixels x 64 consecutive channels of one sample (coalesced), keeps its channel sums in
// registers, and the 16 pixel lanes meet (shuffles, then LDS) before one atomic per
// (channel, sum) into a shard.
#include <cstdlib>
#include "dfxp_device.h"
#include "pk2.h"

namespace {

using namespace lbt;

constexpr int kT = 256, kCB = 64, kRL = 4;

struct WideA {
  const float* g;        // [rows][C] incoming gradient (fp32)
  lbt_qdesc qrg;         // rescale grad quantiser (bits 0: no rescale part)
  const int8_t* R;       // rescale input codes
  const float* gamma_q;  // quantised gamma (fp32) [C]
  lbt_qdesc qng;         // norm grad quantiser (bits 0: no norm part -> dout)
  const int8_t* qn;      // norm input codes
  int16_t* gout;         // norm grad codes
  float* dout;           // fp32 output when there is no norm part
  int64_t* sums;         // [NSHARD][4C]: S(G2 R), S(G2), S(G), S(G qn)
  int64_t rows, inner;
  int C, spb;            // samples per workgroup
  int64_t hw, samples;   // positions per sample (inner / C), samples (rows / hw)
  // ReLU mask on the incoming gradient (ReLU_q backward): from the forward output y_mask > 0, or
  // (mask_r) recomputed from the R codes as the forward chain's pre-ReLU value
  // ((float)R * s_r) * gb[c] + gb[C + c] > 0; the masked gradient optionally out (gmask_out).
  const float* y_mask;
  int mask_r;
  lbt_qdesc qr;          // the R codes' quantiser (mask_r)
  const float* gb;       // [gamma_q | beta_q] (mask_r)
  float* gmask_out;
  const float* g2;       // optional second summand of the incoming gradient: g + g2 (ResidualBlock_q
                         // .backward's add of the two branch gradients, :865-869, done here)
  const uint8_t* y_bits; // the y_mask > 0 mask as one byte per channel quad (lbt_chain_fwd.ybits)
};

// Thread = 4 consecutive channels (one Philox4x32 call covers their 4 noise values) x one pixel.
constexpr int kCQ = 16;        // channel quads per workgroup (64 channels)
constexpr int kRL4 = kT / kCQ; // 16 pixel lanes

// Per-thread channel sums run in int32: a thread sees at most kRowsA samples (|G| <= 2^15 codes
// times |R|, |qn| <= 2^7 gives |product| <= 2^22, so 2^8 of them stay below 2^31) and the workgroup
// widens to int64 when it folds its lanes. YM: the y_mask / g2 operands exist (ResidualBottleneck_q's last BN
// and its shortcut BN); the mask_r and plain forms carry no registers for them.
constexpr int kRowsA = 256;

#ifndef LBT_BNA_WPE
#define LBT_BNA_WPE 4  // waves per SIMD the register allocation targets
#endif
template <bool YM>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(LBT_BNA_WPE))) void bn_bwd_a_wide_kernel(WideA a) {
  __shared__ long long red[kT / 64][4][kCB];
  __shared__ int sh_cnt[2 * 2 * (kT / 64)];
  const int cq = threadIdx.x % kCQ, pl = threadIdx.x / kCQ;
  const int c0 = blockIdx.x * kCB + 4 * cq;
  const int64_t hw = (int64_t)blockIdx.y * kRL4 + pl;
  // C % 4 == 0: the quad is whole. A wave's lane 0 has the smallest pixel and channel of the wave,
  // so an invalid lane 0 means an idle wave (the wave-total counters below read lane 0)
  const bool cv = c0 < a.C && hw < a.hw;
  const QState srg = qstate(a.qrg), sng = qstate(a.qng);
  const int64_t n0 = (int64_t)blockIdx.z * a.spb;
  const int64_t n1 = n0 + a.spb < a.samples ? n0 + a.spb : a.samples;
  const int64_t pos = hw * a.C + c0;  // offset inside a sample: the noise position
  float gam[4], bet[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    gam[k] = (cv && a.gamma_q) ? a.gamma_q[c0 + k] : 0.f;
    bet[k] = (cv && a.mask_r) ? a.gb[a.C + c0 + k] : 0.f;
  }
  const float sr = a.mask_r ? qstate(a.qr).inv_m : 0.f;
  const float* __restrict__ gp = a.g;
  const float* __restrict__ g2p = YM ? a.g2 : nullptr;
  const float* __restrict__ ymp = YM ? a.y_mask : nullptr;
  const uint8_t* __restrict__ ybp = YM ? a.y_bits : nullptr;
  const int8_t* __restrict__ Rp = a.R;
  const int8_t* __restrict__ qnp = a.qn;
  const bool needR = a.mask_r || srg.active;
  int s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0}, s3[4] = {0, 0, 0, 0};
  int o1 = 0, o2 = 0, p1 = 0, p2 = 0;  // wave totals (quant_w)
  constexpr int U = 2;  // samples in flight per thread: every load of both issued before any use
  if (cv) {
    const uint64_t blk = (uint64_t)pos >> 2;
    const Noise4 z{{0.f, 0.f, 0.f, 0.f}};
    const Noise4 nz1 = (srg.active && a.qrg.stochastic) ? qnoise4(a.qrg, srg.step, blk) : z;
    const Noise4 nz2 = (sng.active && a.qng.stochastic) ? qnoise4(a.qng, sng.step, blk) : z;
    // channel pairs for the packed math (pk2.h)
    const pf2 u1[2] = {pk(nz1.u[0], nz1.u[1]), pk(nz1.u[2], nz1.u[3])};
    const pf2 u2[2] = {pk(nz2.u[0], nz2.u[1]), pk(nz2.u[2], nz2.u[3])};
    const pf2 gam2[2] = {pk(gam[0], gam[1]), pk(gam[2], gam[3])};
    const pf2 bet2[2] = {pk(bet[0], bet[1]), pk(bet[2], bet[3])};
    for (int64_t nb = n0; nb < n1; nb += U) {
      float4 gv[U], g2v[YM ? U : 1], ym[YM ? U : 1];
      char4 rv[U], qv[U];
      uint32_t yb[YM ? U : 1];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t n = nb + u < n1 ? nb + u : nb;
        const int64_t e = n * a.inner + pos;
        gv[u] = *reinterpret_cast<const float4*>(gp + e);
        if (YM && g2p) g2v[u] = *reinterpret_cast<const float4*>(g2p + e);
        if (YM && ymp) ym[u] = *reinterpret_cast<const float4*>(ymp + e);
        if (YM && ybp) yb[u] = ybp[e >> 2];
        if (needR) rv[u] = *reinterpret_cast<const char4*>(Rp + e);
        if (sng.active) qv[u] = *reinterpret_cast<const char4*>(qnp + e);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (nb + u >= n1) break;
        const int64_t e = (nb + u) * a.inner + pos;
        pf2 d2[2] = {pk(gv[u].x, gv[u].y), pk(gv[u].z, gv[u].w)};
        if (YM && g2p) {
          d2[0] = d2[0] + pk(g2v[u].x, g2v[u].y);
          d2[1] = d2[1] + pk(g2v[u].z, g2v[u].w);
        }
        const int R[4] = {needR ? rv[u].x : 0, needR ? rv[u].y : 0, needR ? rv[u].z : 0, needR ? rv[u].w : 0};
        if (YM && ymp) {
          d2[0].x = ym[u].x > 0.f ? d2[0].x : 0.f;
          d2[0].y = ym[u].y > 0.f ? d2[0].y : 0.f;
          d2[1].x = ym[u].z > 0.f ? d2[1].x : 0.f;
          d2[1].y = ym[u].w > 0.f ? d2[1].y : 0.f;
        } else if (YM && ybp) {
          d2[0].x = (yb[u] & 1u) ? d2[0].x : 0.f;
          d2[0].y = (yb[u] & 2u) ? d2[0].y : 0.f;
          d2[1].x = (yb[u] & 4u) ? d2[1].x : 0.f;
          d2[1].y = (yb[u] & 8u) ? d2[1].y : 0.f;
        } else if (a.mask_r) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // bn.hip chain_bwd_a's recomputation, op for op
            const pf2 xr = pcvt(R[2 * h], R[2 * h + 1]) * pk(sr, sr);
            const pf2 m1 = xr * gam2[h];
            const pf2 yv = m1 + bet2[h];
            d2[h].x = yv.x > 0.f ? d2[h].x : 0.f;
            d2[h].y = yv.y > 0.f ? d2[h].y : 0.f;
          }
        }
        if (a.gmask_out) *reinterpret_cast<float4*>(a.gmask_out + e) = make_float4(d2[0].x, d2[0].y, d2[1].x, d2[1].y);
        if (srg.active) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            int G2[2];
            quant_w2<-1>(srg, a.qrg.stochastic, d2[h], u1[h], o1, o2, G2[0], G2[1]);
            s0[2 * h] += G2[0] * R[2 * h];
            s0[2 * h + 1] += G2[1] * R[2 * h + 1];
            s1[2 * h] += G2[0];
            s1[2 * h + 1] += G2[1];
            const pf2 gh = pcvt(G2[0], G2[1]) * pk(srg.inv_m, srg.inv_m);
            d2[h] = gh * gam2[h];
          }
        }
        if (sng.active) {
          const int qn[4] = {qv[u].x, qv[u].y, qv[u].z, qv[u].w};
          int G[4];
#pragma unroll
          for (int h = 0; h < 2; ++h) quant_w2<-1>(sng, a.qng.stochastic, d2[h], u2[h], p1, p2, G[2 * h], G[2 * h + 1]);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            s2[k] += G[k];
            s3[k] += G[k] * qn[k];
          }
          short4 o;
          o.x = (short)G[0]; o.y = (short)G[1]; o.z = (short)G[2]; o.w = (short)G[3];
          *reinterpret_cast<short4*>(a.gout + e) = o;
        } else if (a.dout) {
          *reinterpret_cast<float4*>(a.dout + e) = make_float4(d2[0].x, d2[0].y, d2[1].x, d2[1].y);
        }
      }
    }
  }
  // the 4 pixel lanes of a wave hold the same channels (lanes cq, cq + 16, cq + 32, cq + 48): fold
  // them with shuffles (in int64 from here), then one LDS row per wave
  long long t0[4], t1[4], t2[4], t3[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t0[k] = s0[k]; t1[k] = s1[k]; t2[k] = s2[k]; t3[k] = s3[k];
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      t0[k] += __shfl_xor(t0[k], o, 64);
      t1[k] += __shfl_xor(t1[k], o, 64);
      t2[k] += __shfl_xor(t2[k], o, 64);
      t3[k] += __shfl_xor(t3[k], o, 64);
    }
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < kCQ) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[wv][0][4 * cq + k] = t0[k];
      red[wv][1][4 * cq + k] = t1[k];
      red[wv][2][4 * cq + k] = t2[k];
      red[wv][3][4 * cq + k] = t3[k];
    }
  }
  // per-thread counters -> wave totals -> LDS (one barrier publishes counters and sums)
  counts_stage_w(0, 2, o1, o2, sh_cnt);
  counts_stage_w(1, 2, p1, p2, sh_cnt);
  __syncthreads();
  if (srg.active) counts_publish(0, 2, a.qrg, sh_cnt);
  if (sng.active) counts_publish(1, 2, a.qng, sh_cnt);
  if (a.sums) {
    int64_t* dst = a.sums + (int64_t)shard_id() * 4 * a.C;
    for (int i = threadIdx.x; i < 4 * kCB; i += kT) {
      const int sidx = i / kCB, cl = i - sidx * kCB, c = blockIdx.x * kCB + cl;
      if (c >= a.C) continue;
      long long v = 0;
      for (int l = 0; l < kT / 64; ++l) v += red[l][sidx][cl];
      if (v) atomicAdd((unsigned long long*)&dst[sidx * a.C + c], (unsigned long long)v);
    }
  }
}

struct WideB {
  const int16_t* G;      // norm grad codes
  lbt_qdesc qng;
  const int8_t* qn;      // norm input codes
  lbt_qdesc qn_q;
  const float* ms;       // [2C] mu, sigma (forward)
  const int64_t* sums;   // [NSHARD][4C] from pass A (S(G) at 2C, S(G qn) at 3C)
  int64_t n;             // elements per channel
  float* dx;
  int64_t rows;
  int C, spb;            // samples per workgroup (pass A's layout)
  int64_t hw, samples;
  // optional: the consuming conv's gradient quantiser applied to dx (int16 codes, Conv2d_q
  // :299-300 at 9..16 bits) instead of storing dx; inner = per-sample elements (noise period)
  int16_t* gq;
  lbt_qdesc qo;
  int64_t inner;
};

#ifndef LBT_BWDB_U
#define LBT_BWDB_U 2
#endif
__global__ __launch_bounds__(kT) void bn_bwd_b_wide_kernel(WideB b) {
  __shared__ float s_mg[kCB], s_mgx[kCB];
  __shared__ long long s_part[2][kT / kCB][kCB];
  __shared__ int sh_cnt[2 * (kT / 64)];
  const int cq = threadIdx.x % kCQ;
  const int c0 = blockIdx.x * kCB + 4 * cq;
  const QState sgq = qstate(b.qng), sn = qstate(b.qn_q), so = qstate(b.qo);
  const bool quant = b.gq != nullptr;
  {  // the pass-A shard sums of this workgroup's channels: every thread folds 32 / (kT / kCB) shards
    constexpr int kParts = kT / kCB, kPer = LBT_NSHARD / kParts;
    const int cl = threadIdx.x % kCB, part = threadIdx.x / kCB, c = blockIdx.x * kCB + cl;
    long long SG = 0, SGQ = 0;
    if (c < b.C) {
#pragma unroll
      for (int k = part * kPer; k < (part + 1) * kPer; ++k) {
        SG += b.sums[(int64_t)k * 4 * b.C + 2 * b.C + c];
        SGQ += b.sums[(int64_t)k * 4 * b.C + 3 * b.C + c];
      }
    }
    s_part[0][part][cl] = SG;
    s_part[1][part][cl] = SGQ;
  }
  __syncthreads();
  if (threadIdx.x < kCB && blockIdx.x * kCB + (int)threadIdx.x < b.C) {
    // bn.hip chain_bwd_b's moment prologue, for this workgroup's channels
    const int c = blockIdx.x * kCB + threadIdx.x;
    long long SG = 0, SGQ = 0;
#pragma unroll
    for (int k = 0; k < kT / kCB; ++k) {
      SG += s_part[0][k][threadIdx.x];
      SGQ += s_part[1][k][threadIdx.x];
    }
    const double s = (double)sn.inv_m, gsc = (double)sgq.inv_m, n = (double)b.n;
    const float m = b.ms[c], sig = b.ms[b.C + c];
    s_mg[threadIdx.x] = (float)(gsc * (double)SG / n);
    s_mgx[threadIdx.x] = (float)(gsc * (s * (double)SGQ - (double)m * (double)SG) / (n * (double)sig));
  }
  __syncthreads();
  int o1 = 0, o2 = 0;  // wave totals (quant_w)
  const int64_t hw = (int64_t)blockIdx.y * kRL4 + threadIdx.x / kCQ;
  // as in pass A: an invalid lane 0 means an idle wave. No early exit: every thread reaches the
  // barriers of the counter flush the same number of times
  if (c0 < b.C && hw < b.hw) {
    float mu[4], mg[4], mgx[4];
    Recip rs[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mu[k] = b.ms[c0 + k];
      rs[k] = recip(b.ms[b.C + c0 + k]);
      mg[k] = s_mg[4 * cq + k];
      mgx[k] = s_mgx[4 * cq + k];
    }
    // channel pairs (0, 1), (2, 3) for the packed math (pk2.h)
    pf2 mu2[2], mg2[2], mgx2[2], rsy[2], rsr[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      mu2[h] = pk(mu[2 * h], mu[2 * h + 1]);
      mg2[h] = pk(mg[2 * h], mg[2 * h + 1]);
      mgx2[h] = pk(mgx[2 * h], mgx[2 * h + 1]);
      rsy[h] = pk(rs[2 * h].y, rs[2 * h + 1].y);
      rsr[h] = pk(rs[2 * h].rc, rs[2 * h + 1].rc);
    }
    const pf2 sn2 = pk(sn.inv_m, sn.inv_m), sg2 = pk(sgq.inv_m, sgq.inv_m);
    const int64_t n0 = (int64_t)blockIdx.z * b.spb;
    const int64_t n1 = n0 + b.spb < b.samples ? n0 + b.spb : b.samples;
    const int64_t pos = hw * b.C + c0, inner = b.hw * b.C;
    const Noise4 nz = (quant && b.qo.stochastic) ? qnoise4(b.qo, so.step, (uint64_t)pos >> 2)
                                                 : Noise4{{0.f, 0.f, 0.f, 0.f}};
    const int8_t* __restrict__ qnp = b.qn;
    const int16_t* __restrict__ Gp = b.G;
    constexpr int U = LBT_BWDB_U;  // samples in flight per thread (2: ~6 MB in flight on the chip, 46 % of HBM)
    // a uniform 64-bit sample-batch base + 32-bit lane offsets (u * inner + pos < 2^31, host-checked)
    const uint32_t inner32 = (uint32_t)inner, pos32 = (uint32_t)pos;
    for (int64_t nb = n0; nb < n1; nb += U) {
      const int64_t eb = nb * inner;
      char4 qva[U];
      short4 gva[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t o = (uint32_t)(nb + u < n1 ? u : 0) * inner32 + pos32;
        qva[u] = *reinterpret_cast<const char4*>(qnp + eb + o);
        gva[u] = *reinterpret_cast<const short4*>(Gp + eb + o);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
      if (nb + u >= n1) break;
      const int64_t e = eb + (int64_t)((uint32_t)u * inner32 + pos32);
      const char4 qv = qva[u];
      const short4 gv = gva[u];
      const int q[4] = {qv.x, qv.y, qv.z, qv.w}, G[4] = {gv.x, gv.y, gv.z, gv.w};
      pf2 o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const pf2 x1 = pcvt(q[2 * h], q[2 * h + 1]) * sn2;
        const pf2 x2 = x1 - mu2[h];
        const pf2 xh = pdiv_nz(x2, rsy[h], rsr[h]);  // == x2 / sigma (never -0: pk2.h pdiv_nz)
        const pf2 gh = pcvt(G[2 * h], G[2 * h + 1]) * sg2;
        const pf2 t1 = gh - mg2[h];
        const pf2 t2 = xh * mgx2[h];
        o[h] = pdiv_nz(t1 - t2, rsy[h], rsr[h]);  // == (t1 - t2) / sigma (t1 = G s - mg is never -0, so neither is t1 - t2)
      }
      if (quant) {
        int c[4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
          quant_w2<-1>(so, b.qo.stochastic, o[h], pk(nz.u[2 * h], nz.u[2 * h + 1]), o1, o2, c[2 * h], c[2 * h + 1]);
        short4 v;
        v.x = (short)c[0]; v.y = (short)c[1]; v.z = (short)c[2]; v.w = (short)c[3];
        *reinterpret_cast<short4*>(b.gq + e) = v;
      } else {
        *reinterpret_cast<float4*>(b.dx + e) = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
      }
      __builtin_amdgcn_sched_barrier(0);  // one sample at a time (interleaved, the batch costs ~8 VGPRs a sample)
      }
    }
  }
  if (quant) block_flush_counts_w(b.qo, o1, o2, sh_cnt);
}

// Samples per workgroup: up to 16 (one noise call per 16 elements of a thread's position) while
// the grid keeps ~1024+ workgroups.
int samples_per_block(int64_t xy, int64_t samples) {
  static const int64_t target = [] {  // workgroups aimed for (LBT_BWD_WGS; default 1024)
    const char* e = getenv("LBT_BWD_WGS");
    const int v = e ? atoi(e) : 0;
    return (int64_t)(v > 0 ? v : 1024);
  }();
  int64_t s = samples * xy / target;
  if (s > 16) s = 16;
  if (s < 1) s = 1;
  if ((samples + s - 1) / s > 65535) s = (samples + 65534) / 65535;  // grid.z limit
  return (int)s;
}

int launch_b(WideB b, int cb, hipStream_t st) {
  if (b.inner * (LBT_BWDB_U + 1) >= ((int64_t)1 << 31)) return LBT_EINVAL;  // 32-bit lane offsets
  b.hw = b.inner / b.C;
  if (b.rows % b.hw) return LBT_EINVAL;
  b.samples = b.rows / b.hw;
  const int64_t yb = (b.hw + kRL4 - 1) / kRL4;
  b.spb = samples_per_block((int64_t)cb * yb, b.samples);
  const int64_t zb = (b.samples + b.spb - 1) / b.spb;
  if (yb > 65535 || zb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_bwd_b_wide_kernel, dim3((unsigned)cb, (unsigned)yb, (unsigned)zb), dim3(kT), 0, st, b);
  return (int)hipGetLastError();
}

int launch_a(WideA a, int cb, hipStream_t st) {
  if (a.qrg.bits > 16 || a.qng.bits > 16) return LBT_EINVAL;  // the int32 lane sums assume <= 16-bit codes
  a.hw = a.inner / a.C;
  if (a.rows % a.hw) return LBT_EINVAL;
  a.samples = a.rows / a.hw;
  const int64_t yb = (a.hw + kRL4 - 1) / kRL4;
  a.spb = samples_per_block((int64_t)cb * yb, a.samples);
  const int64_t zb = (a.samples + a.spb - 1) / a.spb;
  if (yb > 65535 || zb > 65535 || a.spb > kRowsA) return LBT_EINVAL;
  const dim3 grid((unsigned)cb, (unsigned)yb, (unsigned)zb);
  if (a.y_mask || a.y_bits || a.g2)
    hipLaunchKernelGGL(bn_bwd_a_wide_kernel<true>, grid, dim3(kT), 0, st, a);
  else
    hipLaunchKernelGGL(bn_bwd_a_wide_kernel<false>, grid, dim3(kT), 0, st, a);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int lbt_bn_bwd_a_wide(const float* g, lbt_qdesc qrg, const int8_t* R, const float* gamma_q, lbt_qdesc qng,
                                 const int8_t* qn, int16_t* gout, float* dout, int64_t* sums, int64_t rows,
                                 int64_t inner, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || inner <= 0 || inner % C) return LBT_EINVAL;
  if ((qrg.bits > 0 && (!R || !gamma_q)) || (qng.bits > 0 && (!qn || !gout))) return LBT_EINVAL;
  WideA a{g, qrg, R, gamma_q, qng, qn, gout, dout, sums, rows, inner, C, 0, 0, 0, nullptr, 0, lbt_qdesc{}, nullptr,
          nullptr, nullptr, nullptr};
  return launch_a(a, (C + kCB - 1) / kCB, (hipStream_t)stream);
}

extern "C" int lbt_bn_bwd_b_wide(const int16_t* G, lbt_qdesc qng, const int8_t* qn, lbt_qdesc qn_q, const float* ms,
                                 const int64_t* sums, int64_t n, float* dx, int64_t rows, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || !G || !qn || !ms || !sums || !dx) return LBT_EINVAL;
  int64_t hw = 1024;  // no quantiser, so no noise period: any split of the rows into "samples" of hw pixels
  while (rows % hw) hw >>= 1;
  WideB b{G, qng, qn, qn_q, ms, sums, n, dx, rows, C, 0, 0, 0, nullptr, lbt_qdesc{}, hw * C};
  return launch_b(b, (C + kCB - 1) / kCB, (hipStream_t)stream);
}

// Pass A with the ReLU mask folded in (y_mask, or mask_r: recomputed from R with qr and
// gb = [gamma_q | beta_q]) and the masked gradient optionally stored (gmask_out).
extern "C" int lbt_bn_bwd_a_wide_masked(const float* g, const float* g2, const float* y_mask, const uint8_t* y_bits,
                                        int32_t mask_r, lbt_qdesc qr,
                                        const float* gb, float* gmask_out, lbt_qdesc qrg, const int8_t* R,
                                        lbt_qdesc qng, const int8_t* qn, int16_t* gout, float* dout, int64_t* sums,
                                        int64_t rows, int64_t inner, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || inner <= 0 || inner % C) return LBT_EINVAL;
  if ((qrg.bits > 0 && (!R || !gb)) || (qng.bits > 0 && (!qn || !gout))) return LBT_EINVAL;
  if (mask_r && (y_mask || y_bits || !R || !gb || qr.bits <= 0)) return LBT_EINVAL;
  if (y_mask && y_bits) return LBT_EINVAL;
  WideA a{g, qrg, R, gb, qng, qn, gout, dout, sums, rows, inner, C, 0, 0, 0, y_mask, mask_r, qr, gb, gmask_out, g2,
          y_bits};
  return launch_a(a, (C + kCB - 1) / kCB, (hipStream_t)stream);
}

// Pass B whose dx goes straight into the consuming conv's 9..16-bit gradient quantiser: gq int16
// codes [rows][C] + that quantiser's overflow counters (noise period inner), no fp32 dx.
extern "C" int lbt_bn_bwd_b_wide_q(const int16_t* G, lbt_qdesc qng, const int8_t* qn, lbt_qdesc qn_q, const float* ms,
                                   const int64_t* sums, int64_t n, int16_t* gq, lbt_qdesc qo, int64_t rows,
                                   int64_t inner, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || !G || !qn || !ms || !sums || !gq || inner <= 0 || inner % C) return LBT_EINVAL;
  if (qo.bits <= 0 || qo.bits > 16 || (qo.stochastic && !qo.step && !qo.noise)) return LBT_EINVAL;
  WideB b{G, qng, qn, qn_q, ms, sums, n, nullptr, rows, C, 0, 0, 0, gq, qo, inner};
  return launch_b(b, (C + kCB - 1) / kCB, (hipStream_t)stream);
}

// bn_wide.hip -- BN backward (Rescale_q :686-691, Normalization_q :620-623) for 9..16-bit
// gradient quantisers: the arithmetic of bn.hip's chain_bwd_a /
// chain_bwd_b element for element, with int16 gradient codes and int64 channel sums (int16 x
// int8 products summed over a channel overflow int32).
//
// Layout: workgroup = 64 channels x 4 row lanes; grid = (ceil(C/64), row splits). A thread walks
// rows r = lane_r, lane_r + 4, ... of its split for one channel (a wave reads 64 consecutive
// channels of a row: coalesced), keeps its channel sums in registers, and the 4 row lanes meet in
// LDS before one atomic per (channel, sum) into shard (blockIdx.y mod LBT_NSHARD).
#include "dfxp_device.h"

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
  int C, rpb;            // rows per workgroup
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
};

// Thread = 4 consecutive channels (one Philox4x32 call covers their 4 noise values) x one row lane.
constexpr int kCQ = 16;        // channel quads per workgroup (64 channels)
constexpr int kRL4 = kT / kCQ; // 16 row lanes

__global__ __launch_bounds__(kT) void bn_bwd_a_wide_kernel(WideA a) {
  __shared__ long long red[kT / 64][4][kCB];
  __shared__ int sh_cnt[2 * 2 * (kT / 64)];
  const int cq = threadIdx.x % kCQ, rl = threadIdx.x / kCQ;
  const int c0 = blockIdx.x * kCB + 4 * cq;
  const bool cv = c0 < a.C;  // C % 4 == 0: the quad is whole
  const QState srg = qstate(a.qrg), sng = qstate(a.qng);
  const int64_t r0 = (int64_t)blockIdx.y * a.rpb;
  const int64_t r1 = r0 + a.rpb < a.rows ? r0 + a.rpb : a.rows;
  float gam[4], bet[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    gam[k] = (cv && a.gamma_q) ? a.gamma_q[c0 + k] : 0.f;
    bet[k] = (cv && a.mask_r) ? a.gb[a.C + c0 + k] : 0.f;
  }
  const float sr = a.mask_r ? qstate(a.qr).inv_m : 0.f;
  const float* __restrict__ gp = a.g;
  const float* __restrict__ g2p = a.g2;
  const float* __restrict__ ymp = a.y_mask;
  const int8_t* __restrict__ Rp = a.R;
  const int8_t* __restrict__ qnp = a.qn;
  const bool needR = a.mask_r || srg.active;
  long long s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0}, s3[4] = {0, 0, 0, 0};
  int o1 = 0, o2 = 0, p1 = 0, p2 = 0;
  constexpr int U = 2;  // rows in flight per thread: every load of both issued before any use
  if (cv) {
    for (int64_t rb = r0 + rl; rb < r1; rb += U * kRL4) {
      float4 gv[U], g2v[U], ym[U];
      char4 rv[U], qv[U];
      bool live[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = rb + u * kRL4;
        live[u] = r < r1;
        const int64_t e = (live[u] ? r : rb) * a.C + c0;
        gv[u] = *reinterpret_cast<const float4*>(gp + e);
        if (g2p) g2v[u] = *reinterpret_cast<const float4*>(g2p + e);
        if (ymp) ym[u] = *reinterpret_cast<const float4*>(ymp + e);
        if (needR) rv[u] = *reinterpret_cast<const char4*>(Rp + e);
        if (sng.active) qv[u] = *reinterpret_cast<const char4*>(qnp + e);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!live[u]) break;
        const int64_t e = (rb + u * kRL4) * a.C + c0;
        const uint64_t blk = (uint64_t)(e % a.inner) >> 2;  // inner % 4 == 0
        float d[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
        if (g2p) {
          d[0] = d[0] + g2v[u].x; d[1] = d[1] + g2v[u].y; d[2] = d[2] + g2v[u].z; d[3] = d[3] + g2v[u].w;
        }
        const int R[4] = {needR ? rv[u].x : 0, needR ? rv[u].y : 0, needR ? rv[u].z : 0, needR ? rv[u].w : 0};
        if (ymp) {
          const float m[4] = {ym[u].x, ym[u].y, ym[u].z, ym[u].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) d[k] = m[k] > 0.f ? d[k] : 0.f;
        } else if (a.mask_r) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {  // bn.hip chain_bwd_a's recomputation, op for op
            const float xr = (float)R[k] * sr;
            const float m1 = xr * gam[k];
            const float yv = m1 + bet[k];
            d[k] = yv > 0.f ? d[k] : 0.f;
          }
        }
        if (a.gmask_out) *reinterpret_cast<float4*>(a.gmask_out + e) = make_float4(d[0], d[1], d[2], d[3]);
        if (srg.active) {
          const Noise4 nz = a.qrg.stochastic ? qnoise4(a.qrg, srg.step, blk) : Noise4{{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int G2 = quant1(srg, a.qrg.stochastic, d[k], nz.u[k], o1, o2);
            s0[k] += (long long)G2 * R[k];
            s1[k] += G2;
            const float gh = (float)G2 * srg.inv_m;
            d[k] = gh * gam[k];
          }
        }
        if (sng.active) {
          const Noise4 nz = a.qng.stochastic ? qnoise4(a.qng, sng.step, blk) : Noise4{{0.f, 0.f, 0.f, 0.f}};
          const int qn[4] = {qv[u].x, qv[u].y, qv[u].z, qv[u].w};
          int G[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            G[k] = quant1(sng, a.qng.stochastic, d[k], nz.u[k], p1, p2);
            s2[k] += G[k];
            s3[k] += (long long)G[k] * qn[k];
          }
          short4 o;
          o.x = (short)G[0]; o.y = (short)G[1]; o.z = (short)G[2]; o.w = (short)G[3];
          *reinterpret_cast<short4*>(a.gout + e) = o;
        } else if (a.dout) {
          *reinterpret_cast<float4*>(a.dout + e) = make_float4(d[0], d[1], d[2], d[3]);
        }
      }
    }
  }
  // the 4 row lanes of a wave hold the same channels (lanes cq, cq + 16, cq + 32, cq + 48): fold
  // them with shuffles, then one LDS row per wave
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      s0[k] += __shfl_xor(s0[k], o, 64);
      s1[k] += __shfl_xor(s1[k], o, 64);
      s2[k] += __shfl_xor(s2[k], o, 64);
      s3[k] += __shfl_xor(s3[k], o, 64);
    }
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < kCQ) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[wv][0][4 * cq + k] = s0[k];
      red[wv][1][4 * cq + k] = s1[k];
      red[wv][2][4 * cq + k] = s2[k];
      red[wv][3][4 * cq + k] = s3[k];
    }
  }
  // per-thread counters -> wave totals -> LDS (one barrier publishes counters and sums)
  counts_stage(0, 2, o1, o2, sh_cnt);
  counts_stage(1, 2, p1, p2, sh_cnt);
  __syncthreads();
  if (srg.active) counts_publish(0, 2, a.qrg, sh_cnt);
  if (sng.active) counts_publish(1, 2, a.qng, sh_cnt);
  if (a.sums) {
    int64_t* dst = a.sums + (int64_t)(blockIdx.y % LBT_NSHARD) * 4 * a.C;
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
  int C, rpb;
  // optional: the consuming conv's gradient quantiser applied to dx (int16 codes, Conv2d_q
  // :299-300 at 9..16 bits) instead of storing dx; inner = per-sample elements (noise period)
  int16_t* gq;
  lbt_qdesc qo;
  int64_t inner;
};

__global__ __launch_bounds__(kT) void bn_bwd_b_wide_kernel(WideB b) {
  __shared__ float s_mg[kCB], s_mgx[kCB];
  __shared__ int sh_cnt[2 * (kT / 64)];
  const int cq = threadIdx.x % kCQ, rl = threadIdx.x / kCQ;
  const int c0 = blockIdx.x * kCB + 4 * cq;
  const QState sgq = qstate(b.qng), sn = qstate(b.qn_q), so = qstate(b.qo);
  const bool quant = b.gq != nullptr;
  if (threadIdx.x < kCB && blockIdx.x * kCB + (int)threadIdx.x < b.C) {
    // bn.hip chain_bwd_b's moment prologue, for this workgroup's channels
    const int c = blockIdx.x * kCB + threadIdx.x;
    long long SG = 0, SGQ = 0;
    for (int k = 0; k < LBT_NSHARD; ++k) {
      SG += b.sums[(int64_t)k * 4 * b.C + 2 * b.C + c];
      SGQ += b.sums[(int64_t)k * 4 * b.C + 3 * b.C + c];
    }
    const double s = (double)sn.inv_m, gsc = (double)sgq.inv_m, n = (double)b.n;
    const float m = b.ms[c], sig = b.ms[b.C + c];
    s_mg[threadIdx.x] = (float)(gsc * (double)SG / n);
    s_mgx[threadIdx.x] = (float)(gsc * (s * (double)SGQ - (double)m * (double)SG) / (n * (double)sig));
  }
  __syncthreads();
  int o1 = 0, o2 = 0;
  if (c0 >= b.C) {
    if (quant) block_flush_counts(b.qo, o1, o2, sh_cnt);  // every thread takes part in the flush
    return;
  }
  float mu[4], sig[4], mg[4], mgx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    mu[k] = b.ms[c0 + k];
    sig[k] = b.ms[b.C + c0 + k];
    mg[k] = s_mg[4 * cq + k];
    mgx[k] = s_mgx[4 * cq + k];
  }
  const int64_t r0 = (int64_t)blockIdx.y * b.rpb;
  const int64_t r1 = r0 + b.rpb < b.rows ? r0 + b.rpb : b.rows;
  const int8_t* __restrict__ qnp = b.qn;
  const int16_t* __restrict__ Gp = b.G;
  constexpr int U = 2;  // rows in flight per thread
  for (int64_t rb = r0 + rl; rb < r1; rb += U * kRL4) {
    char4 qva[U];
    short4 gva[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + u * kRL4 < r1 ? rb + u * kRL4 : rb;
      qva[u] = *reinterpret_cast<const char4*>(qnp + r * b.C + c0);
      gva[u] = *reinterpret_cast<const short4*>(Gp + r * b.C + c0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
    if (rb + u * kRL4 >= r1) break;
    const int64_t e = (rb + u * kRL4) * b.C + c0;
    const char4 qv = qva[u];
    const short4 gv = gva[u];
    const int q[4] = {qv.x, qv.y, qv.z, qv.w}, G[4] = {gv.x, gv.y, gv.z, gv.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x1 = (float)q[k] * sn.inv_m;
      const float x2 = x1 - mu[k];
      const float xh = x2 / sig[k];
      const float gh = (float)G[k] * sgq.inv_m;
      const float t1 = gh - mg[k];
      const float t2 = xh * mgx[k];
      o[k] = (t1 - t2) / sig[k];
    }
    if (quant) {
      const uint64_t blk = (uint64_t)(e % b.inner) >> 2;  // inner % 4 == 0
      const Noise4 nz = b.qo.stochastic ? qnoise4(b.qo, so.step, blk) : Noise4{{0.f, 0.f, 0.f, 0.f}};
      short4 v;
      v.x = (short)quant1(so, b.qo.stochastic, o[0], nz.u[0], o1, o2);
      v.y = (short)quant1(so, b.qo.stochastic, o[1], nz.u[1], o1, o2);
      v.z = (short)quant1(so, b.qo.stochastic, o[2], nz.u[2], o1, o2);
      v.w = (short)quant1(so, b.qo.stochastic, o[3], nz.u[3], o1, o2);
      *reinterpret_cast<short4*>(b.gq + e) = v;
    } else {
      *reinterpret_cast<float4*>(b.dx + e) = make_float4(o[0], o[1], o[2], o[3]);
    }
    }
  }
  if (quant) block_flush_counts(b.qo, o1, o2, sh_cnt);
}

// ~2048 workgroups in all
int rows_per_block(int64_t rows, int cblocks) {
  int64_t splits = 2048 / (cblocks > 0 ? cblocks : 1);  // ~2048 workgroups: up to 8 per CU in flight
  if (splits < 1) splits = 1;
  int64_t rpb = (rows + splits - 1) / splits;
  if (rpb < kRL4) rpb = kRL4;
  return (int)rpb;
}

}  // namespace

extern "C" int lbt_bn_bwd_a_wide(const float* g, lbt_qdesc qrg, const int8_t* R, const float* gamma_q, lbt_qdesc qng,
                                 const int8_t* qn, int16_t* gout, float* dout, int64_t* sums, int64_t rows,
                                 int64_t inner, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || inner <= 0 || inner % C) return LBT_EINVAL;
  if ((qrg.bits > 0 && (!R || !gamma_q)) || (qng.bits > 0 && (!qn || !gout))) return LBT_EINVAL;
  WideA a{g, qrg, R, gamma_q, qng, qn, gout, dout, sums, rows, inner, C, 0, nullptr, 0, lbt_qdesc{}, nullptr, nullptr,
          nullptr};
  const int cb = (C + kCB - 1) / kCB;
  a.rpb = rows_per_block(rows, cb);
  const int64_t yb = (rows + a.rpb - 1) / a.rpb;
  if (yb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_bwd_a_wide_kernel, dim3((unsigned)cb, (unsigned)yb), dim3(kT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_bwd_b_wide(const int16_t* G, lbt_qdesc qng, const int8_t* qn, lbt_qdesc qn_q, const float* ms,
                                 const int64_t* sums, int64_t n, float* dx, int64_t rows, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || !G || !qn || !ms || !sums || !dx) return LBT_EINVAL;
  WideB b{G, qng, qn, qn_q, ms, sums, n, dx, rows, C, 0, nullptr, lbt_qdesc{}, 1};
  const int cb = (C + kCB - 1) / kCB;
  b.rpb = rows_per_block(rows, cb);
  const int64_t yb = (rows + b.rpb - 1) / b.rpb;
  if (yb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_bwd_b_wide_kernel, dim3((unsigned)cb, (unsigned)yb), dim3(kT), 0, (hipStream_t)stream, b);
  return (int)hipGetLastError();
}

// Pass A with the ReLU mask folded in (y_mask, or mask_r: recomputed from R with qr and
// gb = [gamma_q | beta_q]) and the masked gradient optionally stored (gmask_out).
extern "C" int lbt_bn_bwd_a_wide_masked(const float* g, const float* g2, const float* y_mask, int32_t mask_r, lbt_qdesc qr,
                                        const float* gb, float* gmask_out, lbt_qdesc qrg, const int8_t* R,
                                        lbt_qdesc qng, const int8_t* qn, int16_t* gout, float* dout, int64_t* sums,
                                        int64_t rows, int64_t inner, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || inner <= 0 || inner % C) return LBT_EINVAL;
  if ((qrg.bits > 0 && (!R || !gb)) || (qng.bits > 0 && (!qn || !gout))) return LBT_EINVAL;
  if (mask_r && (y_mask || !R || !gb || qr.bits <= 0)) return LBT_EINVAL;
  WideA a{g, qrg, R, gb, qng, qn, gout, dout, sums, rows, inner, C, 0, y_mask, mask_r, qr, gb, gmask_out, g2};
  const int cb = (C + kCB - 1) / kCB;
  a.rpb = rows_per_block(rows, cb);
  const int64_t yb = (rows + a.rpb - 1) / a.rpb;
  if (yb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_bwd_a_wide_kernel, dim3((unsigned)cb, (unsigned)yb), dim3(kT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// Pass B whose dx goes straight into the consuming conv's 9..16-bit gradient quantiser: gq int16
// codes [rows][C] + that quantiser's overflow counters (noise period inner), no fp32 dx.
extern "C" int lbt_bn_bwd_b_wide_q(const int16_t* G, lbt_qdesc qng, const int8_t* qn, lbt_qdesc qn_q, const float* ms,
                                   const int64_t* sums, int64_t n, int16_t* gq, lbt_qdesc qo, int64_t rows,
                                   int64_t inner, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || C % 4 || !G || !qn || !ms || !sums || !gq || inner <= 0 || inner % C) return LBT_EINVAL;
  if (qo.bits <= 0 || qo.bits > 16 || (qo.stochastic && !qo.step && !qo.noise)) return LBT_EINVAL;
  WideB b{G, qng, qn, qn_q, ms, sums, n, nullptr, rows, C, 0, gq, qo, inner};
  const int cb = (C + kCB - 1) / kCB;
  b.rpb = rows_per_block(rows, cb);
  const int64_t yb = (rows + b.rpb - 1) / b.rpb;
  if (yb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_bwd_b_wide_kernel, dim3((unsigned)cb, (unsigned)yb), dim3(kT), 0, (hipStream_t)stream, b);
  return (int)hipGetLastError();
}

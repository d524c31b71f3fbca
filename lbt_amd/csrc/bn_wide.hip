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
};

__global__ __launch_bounds__(kT) void bn_bwd_a_wide_kernel(WideA a) {
  __shared__ long long red[kRL][4][kCB];
  __shared__ int sh_cnt[2 * 2 * (kT / 64)];
  const int cl = threadIdx.x & (kCB - 1), rl = threadIdx.x / kCB;
  const int c = blockIdx.x * kCB + cl;
  const bool cv = c < a.C;
  const QState srg = qstate(a.qrg), sng = qstate(a.qng);
  const int64_t r0 = (int64_t)blockIdx.y * a.rpb;
  const int64_t r1 = r0 + a.rpb < a.rows ? r0 + a.rpb : a.rows;
  const float gam = (cv && a.gamma_q) ? a.gamma_q[c] : 0.f;
  long long s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int o1 = 0, o2 = 0, p1 = 0, p2 = 0;
  if (cv) {
    for (int64_t r = r0 + rl; r < r1; r += kRL) {
      const int64_t e = r * a.C + c;
      const uint64_t ni = (uint64_t)(e % a.inner);
      float d = a.g[e];
      if (srg.active) {
        const float u = a.qrg.stochastic ? qnoise1(a.qrg, srg.step, ni) : 0.f;
        const int G2 = quant1(srg, a.qrg.stochastic, d, u, o1, o2);
        s0 += (long long)G2 * a.R[e];
        s1 += G2;
        const float gh = (float)G2 * srg.inv_m;
        d = gh * gam;
      }
      if (sng.active) {
        const float u = a.qng.stochastic ? qnoise1(a.qng, sng.step, ni) : 0.f;
        const int G = quant1(sng, a.qng.stochastic, d, u, p1, p2);
        s2 += G;
        s3 += (long long)G * a.qn[e];
        a.gout[e] = (int16_t)G;
      } else if (a.dout) {
        a.dout[e] = d;
      }
    }
  }
  red[rl][0][cl] = s0;
  red[rl][1][cl] = s1;
  red[rl][2][cl] = s2;
  red[rl][3][cl] = s3;
  // per-thread counters -> wave totals -> LDS (one barrier publishes counters and sums)
  counts_stage(0, 2, o1, o2, sh_cnt);
  counts_stage(1, 2, p1, p2, sh_cnt);
  __syncthreads();
  if (srg.active) counts_publish(0, 2, a.qrg, sh_cnt);
  if (sng.active) counts_publish(1, 2, a.qng, sh_cnt);
  if (a.sums && threadIdx.x < kCB && cv) {
    int64_t* dst = a.sums + (int64_t)(blockIdx.y % LBT_NSHARD) * 4 * a.C;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const long long v = red[0][s][cl] + red[1][s][cl] + red[2][s][cl] + red[3][s][cl];
      if (v) atomicAdd((unsigned long long*)&dst[s * a.C + c], (unsigned long long)v);
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
};

__global__ __launch_bounds__(kT) void bn_bwd_b_wide_kernel(WideB b) {
  __shared__ float s_mg[kCB], s_mgx[kCB];
  const int cl = threadIdx.x & (kCB - 1), rl = threadIdx.x / kCB;
  const int c = blockIdx.x * kCB + cl;
  const bool cv = c < b.C;
  const QState sgq = qstate(b.qng), sn = qstate(b.qn_q);
  if (rl == 0 && cv) {  // bn.hip chain_bwd_b's moment prologue, for this workgroup's channels
    long long SG = 0, SGQ = 0;
    for (int k = 0; k < LBT_NSHARD; ++k) {
      SG += b.sums[(int64_t)k * 4 * b.C + 2 * b.C + c];
      SGQ += b.sums[(int64_t)k * 4 * b.C + 3 * b.C + c];
    }
    const double s = (double)sn.inv_m, gsc = (double)sgq.inv_m, n = (double)b.n;
    const float m = b.ms[c], sig = b.ms[b.C + c];
    s_mg[cl] = (float)(gsc * (double)SG / n);
    s_mgx[cl] = (float)(gsc * (s * (double)SGQ - (double)m * (double)SG) / (n * (double)sig));
  }
  __syncthreads();
  if (!cv) return;
  const float mu = b.ms[c], sig = b.ms[b.C + c], mg = s_mg[cl], mgx = s_mgx[cl];
  const int64_t r0 = (int64_t)blockIdx.y * b.rpb;
  const int64_t r1 = r0 + b.rpb < b.rows ? r0 + b.rpb : b.rows;
  for (int64_t r = r0 + rl; r < r1; r += kRL) {
    const int64_t e = r * b.C + c;
    const float x1 = (float)b.qn[e] * sn.inv_m;
    const float x2 = x1 - mu;
    const float xh = x2 / sig;
    const float gh = (float)b.G[e] * sgq.inv_m;
    const float t1 = gh - mg;
    const float t2 = xh * mgx;
    b.dx[e] = (t1 - t2) / sig;
  }
}

// ~512 workgroups in all
int rows_per_block(int64_t rows, int cblocks) {
  int64_t splits = 512 / (cblocks > 0 ? cblocks : 1);
  if (splits < 1) splits = 1;
  int64_t rpb = (rows + splits - 1) / splits;
  if (rpb < kRL) rpb = kRL;
  return (int)rpb;
}

}  // namespace

extern "C" int lbt_bn_bwd_a_wide(const float* g, lbt_qdesc qrg, const int8_t* R, const float* gamma_q, lbt_qdesc qng,
                                 const int8_t* qn, int16_t* gout, float* dout, int64_t* sums, int64_t rows,
                                 int64_t inner, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || inner <= 0 || inner % C) return LBT_EINVAL;
  if ((qrg.bits > 0 && (!R || !gamma_q)) || (qng.bits > 0 && (!qn || !gout))) return LBT_EINVAL;
  WideA a{g, qrg, R, gamma_q, qng, qn, gout, dout, sums, rows, inner, C, 0};
  const int cb = (C + kCB - 1) / kCB;
  a.rpb = rows_per_block(rows, cb);
  const int64_t yb = (rows + a.rpb - 1) / a.rpb;
  if (yb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_bwd_a_wide_kernel, dim3((unsigned)cb, (unsigned)yb), dim3(kT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_bwd_b_wide(const int16_t* G, lbt_qdesc qng, const int8_t* qn, lbt_qdesc qn_q, const float* ms,
                                 const int64_t* sums, int64_t n, float* dx, int64_t rows, int32_t C, void* stream) {
  if (rows <= 0 || C <= 0 || !G || !qn || !ms || !sums || !dx) return LBT_EINVAL;
  WideB b{G, qng, qn, qn_q, ms, sums, n, dx, rows, C, 0};
  const int cb = (C + kCB - 1) / kCB;
  b.rpb = rows_per_block(rows, cb);
  const int64_t yb = (rows + b.rpb - 1) / b.rpb;
  if (yb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_bwd_b_wide_kernel, dim3((unsigned)cb, (unsigned)yb), dim3(kT), 0, (hipStream_t)stream, b);
  return (int)hipGetLastError();
}

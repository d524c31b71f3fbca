// stem_bwd.h -- the stem's whole backward (pass B of the stem BN + conv1's weight gradient) as a
// workgroup body over NH 256-pixel row blocks, shared by
//   stem.hip       stem_bwd_rows_kernel (NH = 1, 256 threads: lbt_conv_stem_bwd), and
//   conv_mfma.hip  conv_wgrad_many_stem_kernel (NH = 2, 512 threads: the tail blocks of the batched
//                  end-of-backward weight-gradient launch, lbt_conv_wgrad_many_stem_i8).
// Pass B (bn.hip chain_bwd_b_body's arithmetic, dynamic_fixed_point.py:620-623) is evaluated straight
// into the wgrad's LDS gradient image, then conv1's dW partials (:302) on v_mfma_f32_16x16x32_f16:
// fp16 holds every 9-bit image code and 8-bit gradient code exactly and every 64-pixel partial sum
// stays an integer below 2^24, so the fp32 accumulation is exact (stem.hip header). d loss / d image
// is never needed, so the gradient codes only go to memory when b.gq asks for them.
#pragma once
#include "conv_epilogue.h"

namespace {

typedef _Float16 sb_h8 __attribute__((ext_vector_type(8)));
typedef float sb_f4 __attribute__((ext_vector_type(4)));

constexpr int kSbPixels = 256;  // pixels per row block (64 per wave, 4 waves)
constexpr int kSbImg = 4096;    // staged image codes per row block: (256 / W + 2) * (W + 2) * Cin
constexpr int kSbWMax = 64, kSbCinMax = 4;

struct StemBwdArgs {
  lbt_chain_bwd_b b;
  const int16_t* x;
  lbt_conv_desc d;
  int K;
  int32_t* slab;
  int nshard;
};

template <int NH>
struct StemBwdShared {
  int red[NH][4][32][16];  // per-wave dW partials [k][co]; the statistics' long long sums before the MFMAs
  int16_t img[NH][kSbImg];
  __attribute__((aligned(16))) int8_t g[NH][kSbPixels * 16];
  float pb[NH][32];
  int cnt[2 * NH * 4];
};

LBT_DEV lbt::Noise4 sb_noise4(const lbt_qdesc& q, const lbt::QState& s, int64_t g) {
  lbt::Noise4 n = {{0.f, 0.f, 0.f, 0.f}};
  if (s.active && q.stochastic) n = lbt::qnoise4(q, s.step, (uint64_t)g);
  return n;
}

// Host check of lbt_conv_stem_bwd's shapes: stem_wgrad_rows_kernel's (3x3 / stride 1 / SAME, Cout 16,
// W | 64, whole 256-pixel row blocks) with the pass-B chain's (C 16, 8-bit codes, no dx / gcolsum).
inline bool stem_bwd_shape_ok(const lbt_chain_bwd_b* b, const lbt_conv_desc& d) {
  const int K = d.KH * d.KW * d.Cin;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  const bool shape = d.Cout == 16 && d.KH == 3 && d.KW == 3 && d.SH == 1 && d.SW == 1 && d.PT == 1 && d.PL == 1 &&
                     d.Ho == d.H && d.Wo == d.W && d.Cin >= 1 && d.Cin <= kSbCinMax && K <= 32 && d.W >= 8 &&
                     d.W <= kSbWMax && 64 % d.W == 0 && ((int64_t)d.H * d.W) % kSbPixels == 0 &&
                     (kSbPixels / d.W + 2) * (d.W + 2) * d.Cin <= kSbImg && M < ((int64_t)1 << 31);
  return shape && b->C == 16 && b->rows == d.N && b->inner == (int64_t)d.H * d.W * 16 && b->G && b->qn_codes &&
         b->ms && b->sums && !b->dx && !b->gcolsum && b->qo.bits > 0 && b->qo.bits <= 8;
}

// Row blocks blk*NH .. blk*NH + NH-1; threadIdx.x >> 8 picks the block, every thread of the workgroup
// reaches every barrier. Partials of the NH blocks are summed in LDS and added into shard blk % nshard.
template <int NH>
LBT_DEV void stem_bwd_body(const StemBwdArgs& p, uint32_t blk, StemBwdShared<NH>& sm) {
  using namespace lbt;
  constexpr int C = 16, NT = 256 * NH;
  const lbt_chain_bwd_b& a = p.b;
  const lbt_conv_desc& d = p.d;
  const int h = (int)(threadIdx.x >> 8), t = (int)(threadIdx.x & 255);
  const int lane = t & 63, wave = t >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int nkt = (p.K + 15) >> 4;
  const int W = d.W, Cin = d.Cin, HWp = d.H * d.W;
  const int64_t m0 = ((int64_t)blk * NH + h) * kSbPixels;  // host: HW % 256 == 0, 256 % W == 0
  const int n = (int)(m0 / HWp), oy0 = (int)(m0 - (int64_t)n * HWp) / W;
  const int NC = W + 2, E = (kSbPixels / W + 2) * NC * Cin;  // host: E <= kSbImg
  int16_t* s_img = sm.img[h];
  int8_t* s_g = sm.g[h];
  float* s_pb = sm.pb[h];
  // ---- loads: the pass-B statistics' 32 shards (threads < 2C of each block), this thread's 4 channel
  // quads of G / q codes and their noise, and the image rows of the wgrad
  // (each thread: one of the 2C sums over LBT_NSHARD / 8 shards; the 8 partials meet in LDS)
  static_assert(LBT_NSHARD % 8 == 0, "shard groups");
  constexpr int kSv = LBT_NSHARD / 8;
  long long sv[kSv];
  const int sc = t & 31, sg = t >> 5;
#pragma unroll
  for (int k = 0; k < kSv; ++k) sv[k] = a.sums[(int64_t)(sg * kSv + k) * 4 * C + 2 * C + sc];
  const int cq = (t & 3) * 4;
  int Gv[4], Qv[4];
  Noise4 nz[4];
  const QState sgq = qstate(a.qng), sn = qstate(a.qn), so = qstate(a.qo);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int lp = (t >> 2) + 64 * j;                     // local pixel
    const int64_t e = (m0 + lp) * C + cq;                  // element offset (NHWC, C = 16)
    Gv[j] = *reinterpret_cast<const int*>(a.G + e);
    Qv[j] = *reinterpret_cast<const int*>(a.qn_codes + e);
    const int64_t gl = ((m0 - (int64_t)n * HWp + lp) * C + cq) >> 2;  // noise block within the row
    nz[j] = sb_noise4(a.qo, so, gl);
  }
  {
    constexpr int kPer = kSbImg / 256;
    int16_t v[kPer];
    bool ok[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int e = t + q * 256;
      const int ci = e % Cin, pc = e / Cin, col = pc % NC, row = pc / NC;
      const int iy = oy0 - 1 + row, ix = col - 1;
      ok[q] = e < E && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)W;
      v[q] = p.x[ok[q] ? (((int64_t)n * d.H + iy) * W + ix) * Cin + ci : 0];
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int e = t + q * 256;
      if (e < E) s_img[e] = ok[q] ? v[q] : (int16_t)0;
    }
  }
  // ---- pass-B constants mg, mgx per channel, in double exactly as chain_bwd_b_body
  long long* tmp = reinterpret_cast<long long*>(&sm.red[h][0][0][0]);  // [8][2C], free until the MFMAs
  {
    long long s = 0;
#pragma unroll
    for (int k = 0; k < kSv; ++k) s += sv[k];
    tmp[sg * 2 * C + sc] = s;
  }
  __syncthreads();
  if (t < C) {
    const double s = (double)sn.inv_m, gsc = (double)sgq.inv_m, nn = (double)a.n;
    const float m = a.ms[t], sig = a.ms[C + t];
    long long sgi = 0, sgqi = 0;  // exact integer sums: any order
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sgi += tmp[k * 2 * C + t];
      sgqi += tmp[k * 2 * C + C + t];
    }
    const double SG = (double)sgi, SGQ = (double)sgqi;
    s_pb[t] = (float)(gsc * SG / nn);
    s_pb[C + t] = (float)(gsc * (s * SGQ - (double)m * SG) / (nn * (double)sig));
  }
  __syncthreads();
  float rmu[4], rmg[4], rmgx[4];
  Recip rsg[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rmu[k] = a.ms[cq + k];
    rsg[k] = recip(a.ms[C + cq + k]);
    rmg[k] = s_pb[cq + k];
    rmgx[k] = s_pb[C + cq + k];
  }
  int ov1 = 0, ov2 = 0;  // wave totals
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int G[4], q[4], c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      G[k] = (int8_t)((Gv[j] >> (8 * k)) & 0xff);
      q[k] = (int8_t)((Qv[j] >> (8 * k)) & 0xff);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x1 = (float)q[k] * sn.inv_m;
      const float x2 = x1 - rmu[k];
      const float xh = div_by(x2, rsg[k]);  // == x2 / sigma
      const float gh = (float)G[k] * sgq.inv_m;
      const float t1 = gh - rmg[k];
      const float t2 = xh * rmgx[k];
      const float dx = div_by(t1 - t2, rsg[k]);  // == (t1 - t2) / sigma
      c[k] = quant_w<-1>(so, a.qo.stochastic, dx, nz[j].u[k], ov1, ov2);
    }
    const int lp = (t >> 2) + 64 * j;
    const int w = (int)((uint32_t)(c[0] & 0xff) | ((uint32_t)(c[1] & 0xff) << 8) | ((uint32_t)(c[2] & 0xff) << 16) |
                        ((uint32_t)c[3] << 24));
    *reinterpret_cast<int*>(s_g + lp * 16 + cq) = w;
    if (a.gq) *reinterpret_cast<int*>(a.gq + (m0 + lp) * C + cq) = w;
  }
  if (a.qo.counts) counts_stage_w(0, 1, ov1, ov2, sm.cnt);  // slot per wave of the workgroup
  __syncthreads();
  sb_f4 acc[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) acc[kt] = sb_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    sb_h8 af[2], b;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int k = kt * 16 + r;
      const int tap = k / Cin, ci = k - tap * Cin, kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int lm = wave * 64 + 32 * s + 8 * kg + j, ly = lm / W, ox = lm - ly * W;
        const int v = (kt < nkt && k < p.K) ? (int)s_img[((ly + kh) * NC + ox + kw) * Cin + ci] : 0;
        af[kt][j] = (_Float16)(float)v;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = (_Float16)(float)(int)s_g[(wave * 64 + 32 * s + 8 * kg + j) * 16 + r];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
      if (kt < nkt) acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[kt], b, acc[kt], 0, 0, 0);
  }
  counts_publish(0, 1, a.qo, sm.cnt);  // sums every wave's slot (blockDim.x / 64 of them)
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (kt < nkt) sm.red[h][wave][kt * 16 + 4 * kg + i][r] = (int)acc[kt][i];
  __syncthreads();
  int32_t* out = p.slab + (int64_t)(blk % (uint32_t)p.nshard) * p.K * 16;
  for (int i = threadIdx.x; i < p.K * 16; i += NT) {
    const int k = i / 16, c = i - k * 16;
    int v = 0;
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) v += sm.red[hh][0][k][c] + sm.red[hh][1][k][c] + sm.red[hh][2][k][c] + sm.red[hh][3][k][c];
    if (v) LBT_GADD(&out[i], v);  // integer atomics: exact, order-independent
  }
}

}  // namespace

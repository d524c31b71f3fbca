// stem.hip -- the network's first convolution (conv1 of the CIFAR ResNets, models.py:387-391)
// on v_mfma_f32_16x16x32_f16.
//
// Its input is the image quantised to SIGNED bits+1 = 9-bit codes (dynamic_fixed_point.py:
// 287-289 with the conv input's extra bit), which int8 MFMA cannot take. fp16 holds every code
// with |x| <= 2048 and every weight / gradient code (|v| <= 128) exactly, their products are
// exact in the fp32 accumulator, and every partial sum stays an integer below 2^24 (fwd: K <= 32
// products; wgrad: runs of 64 pixels), so the fp32 accumulation is EXACT -- the results are the
// integer GEMM's, bit for bit, whatever order the hardware sums in.
//
// fp16 16x16x32 operand map (gfx950): lane l holds A[row l&15][k = 8*(l>>4) + j] and
// B[k = 8*(l>>4) + j][col l&15], j = 0..7; C/D: col = l&15, row = 4*(l>>4) + reg.
//
// fwd:   rows = output pixels, cols = Cout, k = patch index (kh, kw, ci) in HWIO order, K <= 32:
//        ONE MFMA per 16 x 16 output tile; epilogue = fp32 store or the shared quantising
//        epilogue (Normalization_q input quantiser + exact channel sums, conv_epilogue.h).
// wgrad: rows = patch index k, cols = Cout, k-dim = pixels: each wave sums 64 pixels (2 MFMAs
//        per 16x16 tile), the 4 waves of a workgroup are combined in LDS and each workgroup
//        adds its exact int32 partial into shard (wg % nshard) of a zeroed slab[nshard][K][Cout]
//        (integer atomics) for lbt_conv_wgrad_reduce(_many).
#include "conv_epilogue.h"
#include "stem_bwd.h"

#include <cstdlib>

using namespace lbt;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

namespace {

constexpr int kThreads = 256;
constexpr int kWgPixels = 256;  // stem wgrad pixels per workgroup (64 per wave)

struct StemFwdArgs {
  const int16_t* x;
  const int8_t* w;  // HWIO [K][Cout]
  lbt_conv_desc d;
  int K;
  lbt_qdesc qx, qw;
  float* y;
  QOut o;
};

// Offset of patch element k of output pixel (n, oy, ox) in the NHWC code image, or -1 outside
// it. Callers compute every offset of a fragment first and then issue all the loads, so the
// gathers of a lane are in flight together.
LBT_DEV int64_t patch_off(const lbt_conv_desc& d, int n, int oy, int ox, int k) {
  const int tap = k / d.Cin, ci = k - tap * d.Cin;
  const int kh = tap / d.KW, kw = tap - kh * d.KW;
  const int iy = oy * d.SH + kh - d.PT, ix = ox * d.SW + kw - d.PL;
  if ((unsigned)iy >= (unsigned)d.H || (unsigned)ix >= (unsigned)d.W) return -1;
  return (((int64_t)n * d.H + iy) * d.W + ix) * d.Cin + ci;
}

// 8 patch codes -> fp16 fragment (offsets < 0 read as 0)
LBT_DEV h8 gather8(const int16_t* __restrict__ x, const int64_t (&off)[8]) {
  int16_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = x[off[j] < 0 ? 0 : off[j]];
  h8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (_Float16)(float)(off[j] < 0 ? 0 : (int)v[j]);
  return a;
}

template <int NT>
__global__ __launch_bounds__(kThreads) void stem_fwd_kernel(StemFwdArgs p) {
  using G = EpiGeom<NT>;
  constexpr int NTW = G::NTW, WPM = G::WPM, MTB = G::MTB;
  __shared__ EpiShared<NT> sh;
  LBT_TS(0);
  const lbt_conv_desc& d = p.d;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int mt_local = wave / WPM;
  const int nt0 = (wave % WPM) * NTW;
  const int64_t mtile = (int64_t)blockIdx.x * MTB + mt_local;
  const int r = lane & 15, kg = lane >> 4;
  const int64_t M = p.o.M;
  const bool want_q = p.o.yq != nullptr;
  const QState qs = qstate(p.o.q);
  f4v acc[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) acc[j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int64_t m = mtile * 16 + r;
  int64_t off[8];
  {
    const uint32_t mu = (uint32_t)(m < M ? m : 0);
    const int ox = (int)(mu % (uint32_t)d.Wo);
    const uint32_t t = mu / (uint32_t)d.Wo;
    const int oy = (int)(t % (uint32_t)d.Ho), n = (int)(t / (uint32_t)d.Ho);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * kg + j;
      off[j] = (m < M && k < p.K) ? patch_off(d, n, oy, ox, k) : -1;
    }
  }
  const h8 a = gather8(p.x, off);
  h8 b[NTW];
  {
    int8_t wv[NTW][8];
#pragma unroll
    for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * kg + j;
        wv[jt][j] = p.w[(int64_t)(k < p.K ? k : 0) * d.Cout + (nt0 + jt) * 16 + r];
      }
#pragma unroll
    for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
      for (int j = 0; j < 8; ++j) b[jt][j] = (_Float16)(float)(8 * kg + j < p.K ? (int)wv[jt][j] : 0);
  }
  float u[NTW][4];
  if (want_q) epi_noise<NTW>(p.o, mtile, nt0, lane, u);
#pragma unroll
  for (int jt = 0; jt < NTW; ++jt) acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[jt], acc[jt], 0, 0, 0);
  LBT_TS(1);
  const float scale = ldexpf(1.0f, -(frac_exp(p.qx) + frac_exp(p.qw)));
  float v[NTW][4];
#pragma unroll
  for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
    for (int i = 0; i < 4; ++i) v[jt][i] = acc[jt][i] * scale;
  if (!want_q) {
#pragma unroll
    for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = mtile * 16 + kg * 4 + i;
        if (row < M) p.y[row * d.Cout + (nt0 + jt) * 16 + r] = v[jt][i];
      }
    return;
  }
  LBT_TS(2);
  epi_quant<NT>(p.o, qs, mtile, nt0, wave, lane, v, u, sh);
  LBT_TS(3);
}

// The same conv when a block's pixels are whole output rows of one image (3x3, stride 1, SAME, W | the
// block's MTB*16 pixels, Cin <= 4): the block first stages its input rows plus the one-row / one-column
// halo ([rows + 2][W + 2][Cin] int16, zeros outside the image) in LDS with one coalesced load per
// thread, and every lane gathers its 8 patch codes from there -- instead of 8 scattered 2-byte global
// loads per lane. Same fp16 fragments, same MFMA, same epilogue: bit-identical.
constexpr int kStemRowsMax = 4, kStemWMax = 64, kStemCinMax = 4;
template <int NT>
__global__ __launch_bounds__(kThreads) void stem_fwd_rows_kernel(StemFwdArgs p) {
  using G = EpiGeom<NT>;
  constexpr int NTW = G::NTW, WPM = G::WPM, MTB = G::MTB, PB = MTB * 16;
  __shared__ EpiShared<NT> sh;
  __shared__ int16_t s_img[kStemRowsMax * (kStemWMax + 2) * kStemCinMax];
  LBT_TS(0);
  const lbt_conv_desc& d = p.d;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int mt_local = wave / WPM;
  const int nt0 = (wave % WPM) * NTW;
  const int64_t mtile = (int64_t)blockIdx.x * MTB + mt_local;
  const int r = lane & 15, kg = lane >> 4;
  const int64_t M = p.o.M;
  const bool want_q = p.o.yq != nullptr;
  const QState qs = qstate(p.o.q);
  const int W = d.W, Cin = d.Cin, HWp = d.H * d.W;
  const int64_t m0 = (int64_t)blockIdx.x * PB;  // host: HW % PB == 0, PB % W == 0
  const int n = (int)(m0 / HWp), oy0 = (int)(m0 - (int64_t)n * HWp) / W;
  const int NR = PB / W + 2, NC = W + 2, E = NR * NC * Cin;
  // ---- stage: element t = ((row * NC) + col) * Cin + ci of rows oy0-1 .. oy0+PB/W, cols -1 .. W
  // (two elements per thread: E <= 2 * kThreads, host check; both loads issued before the stores)
  {
    int16_t v[2];
    bool ok[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int t = (int)threadIdx.x + h * kThreads;
      const int ci = t % Cin, pc = t / Cin, col = pc % NC, row = pc / NC;
      const int iy = oy0 - 1 + row, ix = col - 1;
      ok[h] = t < E && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)W;
      v[h] = p.x[ok[h] ? (((int64_t)n * d.H + iy) * W + ix) * Cin + ci : 0];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int t = (int)threadIdx.x + h * kThreads;
      if (t < E) s_img[t] = ok[h] ? v[h] : (int16_t)0;
    }
  }
  // ---- operands that do not need the image: weights, epilogue noise
  h8 b[NTW];
  {
    int8_t wv[NTW][8];
#pragma unroll
    for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * kg + j;
        wv[jt][j] = p.w[(int64_t)(k < p.K ? k : 0) * d.Cout + (nt0 + jt) * 16 + r];
      }
#pragma unroll
    for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
      for (int j = 0; j < 8; ++j) b[jt][j] = (_Float16)(float)(8 * kg + j < p.K ? (int)wv[jt][j] : 0);
  }
  float u[NTW][4];
  if (want_q) epi_noise<NTW>(p.o, mtile, nt0, lane, u);
  __syncthreads();
  // ---- this lane's 8 patch codes from LDS: pixel (oy0 + ly, ox), k = 8kg + j = (tap, ci)
  const int lm = (int)(mtile * 16 + r - m0), ly = lm / W, ox = lm - ly * W;
  h8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kg + j;
    const int tap = k / Cin, ci = k - tap * Cin, kh = tap / 3, kw = tap - kh * 3;
    const int v = k < p.K ? (int)s_img[((ly + kh) * NC + ox + kw) * Cin + ci] : 0;
    a[j] = (_Float16)(float)v;
  }
  f4v acc[NTW];
#pragma unroll
  for (int jt = 0; jt < NTW; ++jt) acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[jt], f4v{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  LBT_TS(1);
  const float scale = ldexpf(1.0f, -(frac_exp(p.qx) + frac_exp(p.qw)));
  float v[NTW][4];
#pragma unroll
  for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
    for (int i = 0; i < 4; ++i) v[jt][i] = acc[jt][i] * scale;
  if (!want_q) {
#pragma unroll
    for (int jt = 0; jt < NTW; ++jt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = mtile * 16 + kg * 4 + i;
        if (row < M) p.y[row * d.Cout + (nt0 + jt) * 16 + r] = v[jt][i];
      }
    return;
  }
  LBT_TS(2);
  epi_quant<NT>(p.o, qs, mtile, nt0, wave, lane, v, u, sh);
  LBT_TS(3);
}

// grid = nsplit workgroups of kWgPixels pixels; Cout <= 64 (ct tiles), K <= 32 (2 kt tiles)
__global__ __launch_bounds__(kThreads) void stem_wgrad_kernel(const int16_t* __restrict__ x,
                                                              const int8_t* __restrict__ gq, lbt_conv_desc d, int K,
                                                              int64_t M, int32_t* __restrict__ slab, int nshard) {
  __shared__ int red[4][32][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int nct = d.Cout >> 4;
  const int nkt = (K + 15) >> 4;
  f4v acc[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[kt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
  const int64_t p0 = (int64_t)blockIdx.x * kWgPixels + wave * 64;
  // operands of both 32-pixel steps first (one memory round trip), then the MFMAs
  h8 a[2][2], b[2][4];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    int pn[8], poy[8], pox[8];
    bool pv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t m = p0 + 32 * s + 8 * kg + j;
      pv[j] = m < M;
      const uint32_t mu = (uint32_t)(pv[j] ? m : 0);
      pox[j] = (int)(mu % (uint32_t)d.Wo);
      const uint32_t t = mu / (uint32_t)d.Wo;
      poy[j] = (int)(t % (uint32_t)d.Ho);
      pn[j] = (int)(t / (uint32_t)d.Ho);
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int k = kt * 16 + r;
      int64_t off[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) off[j] = (kt < nkt && k < K && pv[j]) ? patch_off(d, pn[j], poy[j], pox[j], k) : -1;
      a[s][kt] = gather8(x, off);
    }
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      if (ct >= nct) {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[s][ct][j] = (_Float16)0.f;
        continue;
      }
      const int c = ct * 16 + r;
      int8_t gv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t m = p0 + 32 * s + 8 * kg + j;
        gv[j] = gq[(pv[j] ? m : 0) * d.Cout + c];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) b[s][ct][j] = (_Float16)(float)(pv[j] ? (int)gv[j] : 0);
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        if (kt < nkt && ct < nct) acc[kt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[s][kt], b[s][ct], acc[kt][ct], 0, 0, 0);
  // D[row = k][col = c]: row = kt*16 + 4*kg + i, col = ct*16 + r
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (kt < nkt && ct < nct) red[wave][kt * 16 + 4 * kg + i][ct * 16 + r] = (int)acc[kt][ct][i];
  __syncthreads();
  int32_t* out = slab + (int64_t)(blockIdx.x % nshard) * K * d.Cout;
  for (int i = threadIdx.x; i < K * d.Cout; i += kThreads) {
    const int k = i / d.Cout, c = i - k * d.Cout;
    const int v = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
    if (v) LBT_GADD(&out[i], v);  // integer atomics: exact, order-independent
  }
}

// stem_wgrad_kernel's arithmetic when a block's 256 pixels are whole rows of one image (3x3 / stride
// 1 / SAME, W | 64, Cin <= 4, Cout == 16): the block stages its 256 // W input rows + halo and its
// [256][16] gradient codes in LDS (coalesced), and the lanes build the same fp16 fragments from there.
constexpr int kSWRows = 256 / 8 + 2;  // rows of the staged image for W >= 8
__global__ __launch_bounds__(kThreads) void stem_wgrad_rows_kernel(const int16_t* __restrict__ x,
                                                                   const int8_t* __restrict__ gq, lbt_conv_desc d,
                                                                   int K, int32_t* __restrict__ slab, int nshard) {
  __shared__ int red[4][32][64];
  __shared__ int16_t s_img[kSWRows * (kStemWMax + 2) * kStemCinMax > 4096 ? 4096 : kSWRows * (kStemWMax + 2) * kStemCinMax];
  __shared__ __attribute__((aligned(16))) int8_t s_g[kWgPixels * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, t = threadIdx.x;
  const int r = lane & 15, kg = lane >> 4;
  const int nkt = (K + 15) >> 4;
  const int W = d.W, Cin = d.Cin, HWp = d.H * d.W;
  const int64_t m0 = (int64_t)blockIdx.x * kWgPixels;  // host: HW % 256 == 0, 256 % W == 0
  const int n = (int)(m0 / HWp), oy0 = (int)(m0 - (int64_t)n * HWp) / W;
  const int NC = W + 2, E = (kWgPixels / W + 2) * NC * Cin;  // host: E <= 4096
  // ---- stage the image rows (up to 16 per thread, all loads before the stores) and the codes
  {
    const int4 gv = *reinterpret_cast<const int4*>(gq + m0 * 16 + t * 16);
    constexpr int kPer = 16;
    int16_t v[kPer];
    bool ok[kPer];
#pragma unroll
    for (int h = 0; h < kPer; ++h) {
      const int e = t + h * kThreads;
      const int ci = e % Cin, pc = e / Cin, col = pc % NC, row = pc / NC;
      const int iy = oy0 - 1 + row, ix = col - 1;
      ok[h] = e < E && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)W;
      v[h] = x[ok[h] ? (((int64_t)n * d.H + iy) * W + ix) * Cin + ci : 0];
    }
#pragma unroll
    for (int h = 0; h < kPer; ++h) {
      const int e = t + h * kThreads;
      if (e < E) s_img[e] = ok[h] ? v[h] : (int16_t)0;
    }
    *reinterpret_cast<int4*>(s_g + t * 16) = gv;
  }
  __syncthreads();
  f4v acc[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) acc[kt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    h8 a[2], b;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int k = kt * 16 + r;
      const int tap = k / Cin, ci = k - tap * Cin, kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int lm = wave * 64 + 32 * s + 8 * kg + j, ly = lm / W, ox = lm - ly * W;
        const int v = (kt < nkt && k < K) ? (int)s_img[((ly + kh) * NC + ox + kw) * Cin + ci] : 0;
        a[kt][j] = (_Float16)(float)v;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = (_Float16)(float)(int)s_g[(wave * 64 + 32 * s + 8 * kg + j) * 16 + r];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
      if (kt < nkt) acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[kt], b, acc[kt], 0, 0, 0);
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (kt < nkt) red[wave][kt * 16 + 4 * kg + i][r] = (int)acc[kt][i];
  __syncthreads();
  int32_t* out = slab + (int64_t)(blockIdx.x % nshard) * K * 16;
  for (int i = threadIdx.x; i < K * 16; i += kThreads) {
    const int k = i / 16, c = i - k * 16;
    const int v = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
    if (v) LBT_GADD(&out[i], v);  // integer atomics: exact, order-independent
  }
}

// ---- the stem's whole backward in one launch (lbt_conv_stem_bwd): stem_bwd.h's body over one
// 256-pixel row block per workgroup (pass B of the stem BN into the wgrad's LDS operand, conv1's dW).
__global__ __launch_bounds__(kThreads) void stem_bwd_rows_kernel(StemBwdArgs p) {
  __shared__ __attribute__((aligned(16))) StemBwdShared<1> sm;
  LBT_TS(0);
  stem_bwd_body<1>(p, blockIdx.x, sm);
  LBT_TS(3);
}


// The CIFAR stem (Cout 16, 3x3 / stride 1 / SAME, W == 32, Cin <= 4, quantising epilogue) on whole row
// bands: a 512-thread workgroup owns kSbRows output rows of one image (512 pixels = 32 16-row tiles, 4 per
// wave). The input rows + halo are staged in LDS once, each wave loads the weight fragment once and runs
// its 4 tiles' MFMAs and quantisers, the channel sums and overflow counters accumulate in registers over
// the tiles and leave once per workgroup. (stem_fwd_rows_kernel: 64-pixel blocks of 4 waves, 2048
// workgroups at B = 128, each repeating the weight / noise / descriptor loads and the publish barrier.)
// Per tile the same fp16 fragments, the same MFMA, the same quantiser and noise as stem_fwd_rows_kernel's
// epilogue (epi_quant): bit-identical codes; integer channel sums and counts (order-free).
constexpr int kSbRows = 16, kSbW = 32, kSbThreads = 512, kSbTiles = 4;
constexpr int kSbElems = (kSbRows + 2) * (kSbW + 2) * kStemCinMax, kSbIt = (kSbElems + kSbThreads - 1) / kSbThreads;
static_assert(kSbRows * kSbW == 16 * kSbTiles * (kSbThreads / 64), "a band is 4 tiles per wave");
__global__ __launch_bounds__(kSbThreads) void stem_fwd_band_kernel(StemFwdArgs p) {
  __shared__ int16_t s_img[kSbElems];
  __shared__ int s_part[kSbThreads / 64][2][16];
  __shared__ int s_cnt[2 * (kSbThreads / 64)];
  LBT_TS(0);
  const lbt_conv_desc& d = p.d;
  const int Cin = d.Cin, H = d.H, bands = H / kSbRows;
  const int n = (int)blockIdx.x / bands, oy0 = ((int)blockIdx.x - n * bands) * kSbRows;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, kg = lane >> 4;
  constexpr int NC = kSbW + 2;
  const int E = (kSbRows + 2) * NC * Cin;
  const int64_t HWo = p.o.HWo, m0 = (int64_t)n * HWo + (int64_t)oy0 * kSbW;  // the band's first pixel
  // ---- every load first: the band's input rows + halo (zeros outside the image), the weight fragment,
  // the 4 tiles' epilogue noise
  int16_t xv[kSbIt];
  bool xok[kSbIt];
#pragma unroll
  for (int h = 0; h < kSbIt; ++h) {
    const int t = tid + h * kSbThreads;
    const int ci = t % Cin, pc = t / Cin, col = pc % NC, row = pc / NC;
    const int iy = oy0 - 1 + row, ix = col - 1;
    xok[h] = t < E && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)kSbW;
    xv[h] = p.x[xok[h] ? (((int64_t)n * H + iy) * kSbW + ix) * Cin + ci : 0];
  }
  int8_t wv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kg + j;
    wv[j] = p.w[(int64_t)(k < p.K ? k : 0) * 16 + r];
  }
  const bool tab = p.o.q.stochastic && p.o.q.noise;  // else the quantiser ignores u: read zeros
  const float* nsrc = tab ? p.o.q.noise : zf();
  const uint32_t nmask = tab ? 0xffffffffu : 0u;
  float u[kSbTiles][4];
#pragma unroll
  for (int tt = 0; tt < kSbTiles; ++tt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t pix = (uint32_t)(oy0 * kSbW + (wave * kSbTiles + tt) * 16 + 4 * kg + i);  // < HWo
      u[tt][i] = nsrc[(pix * 16u + (uint32_t)r) & nmask];
    }
  const QState qs = qstate(p.o.q);
  const float scale = ldexpf(1.0f, -(frac_exp(p.qx) + frac_exp(p.qw)));
#pragma unroll
  for (int h = 0; h < kSbIt; ++h) {
    const int t = tid + h * kSbThreads;
    if (t < E) s_img[t] = xok[h] ? xv[h] : (int16_t)0;
  }
  h8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (_Float16)(float)(8 * kg + j < p.K ? (int)wv[j] : 0);
  __syncthreads();
  LBT_TS(1);
  // ---- the wave's 4 tiles: 8 patch codes per lane from LDS, one MFMA, the quantiser
  int ov1 = 0, ov2 = 0, s1 = 0, s2 = 0;
#pragma unroll
  for (int tt = 0; tt < kSbTiles; ++tt) {
    const int mt = wave * kSbTiles + tt;
    const int lm = mt * 16 + r, ly = lm / kSbW, ox = lm - ly * kSbW;
    h8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * kg + j;
      const int tap = k / Cin, ci = k - tap * Cin, kh = tap / 3, kw = tap - kh * 3;
      const int v = k < p.K ? (int)s_img[((ly + kh) * NC + ox + kw) * Cin + ci] : 0;
      a[j] = (_Float16)(float)v;
    }
    const f4v acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, f4v{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    int cc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = quant_w<-1>(qs, p.o.q.stochastic, acc[i] * scale, u[tt][i], ov1, ov2);
      cc[i] = c;
      s1 += c;
      s2 += c * c;
    }
    // the 4 lanes of a column quad swap codes so lane r stores row 4 kg + (r & 3)'s 4 columns (epi_quant)
    const uint32_t packed = quad_pack_codes(cc, r & 3);
    const int64_t rowp = m0 + mt * 16 + 4 * kg + (r & 3);
    st_out(p.o.yq + (uint32_t)rowp * 16u + (r & ~3), (int)packed);  // M * 16 < 2^31 (launcher)
  }
  LBT_TS(2);
  // ---- channel sums and counters of the band: one barrier, one atomic per (channel, sum)
  const int t2 = rows_scatter2(s1, s2);  // row 0: column r's S1, row 1: its S2
  if (kg < 2) s_part[wave][kg][r] = t2;
  if (p.o.q.counts) counts_stage_w(0, 1, ov1, ov2, s_cnt);  // wave totals (quant_w)
  __syncthreads();
  counts_publish(0, 1, p.o.q, s_cnt);
  if (p.o.chsum && tid < 32) {
    const int which = tid >> 4, col = tid & 15;
    long long tot = 0;
#pragma unroll
    for (int w = 0; w < kSbThreads / 64; ++w) tot += s_part[w][which][col];
    if (tot) LBT_GADD((unsigned long long*)&p.o.chsum[(int64_t)shard_id() * 32 + tid], (unsigned long long)tot);
  }
  LBT_TS(3);
}
}  // namespace

LBT_TRACE_SETTER(stem)

extern "C" int lbt_conv_stem_fwd(const int16_t* x, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw,
                                 float* y, int8_t* yq, lbt_qdesc qout, int64_t* ychsum, void* stream) {
  const int K = d.KH * d.KW * d.Cin;
  if (K <= 0 || K > 32 || d.Cout <= 0 || d.Cout % 16 || d.Cout > 128) return LBT_EINVAL;
  if ((y == nullptr) == (yq == nullptr)) return LBT_EINVAL;
  if (yq && (qout.bits > 8 || (qout.stochastic && !qout.noise))) return LBT_EINVAL;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (M <= 0) return LBT_OK;
  StemFwdArgs p;
  p.x = x; p.w = w_hwio; p.d = d; p.K = K; p.qx = qx; p.qw = qw; p.y = y;
  p.o = QOut{yq, qout, yq ? ychsum : nullptr, M, d.Cout, (int64_t)d.Ho * d.Wo};
  if (M * d.Cout >= (int64_t)1 << 31) return LBT_EINVAL;  // 32-bit element offsets
  hipStream_t st = (hipStream_t)stream;
  const int64_t mtiles = (M + 15) / 16;
  // whole-row bands of 16 rows (the CIFAR-10 stem of the fused plan) when they fill the chip: 10.5 vs 11.8 us
  // at B = 128 (256 bands), but 10.5 vs 5.6 us at B = 16 (32 bands: a band's serial 4-tile chain is the
  // launch), profiles/round6/stem_band.txt. LBT_STEM_BAND=0 / 1: never / always.
  static const int band_env = getenv("LBT_STEM_BAND") ? atoi(getenv("LBT_STEM_BAND")) : -1;
  const int64_t nband = (int64_t)d.N * (d.H / kSbRows);
  if ((band_env == 1 || (band_env < 0 && nband >= 256)) && yq && d.Cout == 16 && d.KH == 3 && d.KW == 3 &&
      d.SH == 1 && d.SW == 1 && d.PT == 1 && d.PL == 1 && d.Ho == d.H && d.Wo == d.W && d.W == kSbW &&
      d.H % kSbRows == 0 && d.Cin <= kStemCinMax) {
    hipLaunchKernelGGL(stem_fwd_band_kernel, dim3((unsigned)nband), dim3(kSbThreads), 0, st, p);
    return (int)hipGetLastError();
  }
  // whole-row blocks staged in LDS (CIFAR stems): 3x3 / stride 1 / SAME, block pixels = whole rows
  const int pb = d.Cout == 16 ? 64 : 32;  // EpiGeom<Cout/16>::MTB * 16 of the two row variants
  if ((d.Cout == 16 || d.Cout == 32) && d.KH == 3 && d.KW == 3 && d.SH == 1 && d.SW == 1 && d.PT == 1 &&
      d.PL == 1 && d.Ho == d.H && d.Wo == d.W && d.Cin <= kStemCinMax && d.W <= kStemWMax && pb % d.W == 0 &&
      pb / d.W + 2 <= kStemRowsMax && ((int64_t)d.H * d.W) % pb == 0 &&
      (pb / d.W + 2) * (d.W + 2) * d.Cin <= 2 * kThreads &&
      getenv("LBT_STEM_GATHER") == nullptr) {
    const unsigned blocks = (unsigned)(M / pb);
    switch (d.Cout / 16) {
      case 1: hipLaunchKernelGGL(stem_fwd_rows_kernel<1>, dim3(blocks), dim3(kThreads), 0, st, p); break;
      case 2: hipLaunchKernelGGL(stem_fwd_rows_kernel<2>, dim3(blocks), dim3(kThreads), 0, st, p); break;
      default: return LBT_EINVAL;
    }
    return (int)hipGetLastError();
  }
  switch (d.Cout / 16) {
    case 1: hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3((unsigned)((mtiles + 3) / 4)), dim3(kThreads), 0, st, p); break;
    case 2: hipLaunchKernelGGL(stem_fwd_kernel<2>, dim3((unsigned)((mtiles + 1) / 2)), dim3(kThreads), 0, st, p); break;
    case 4: hipLaunchKernelGGL(stem_fwd_kernel<4>, dim3((unsigned)mtiles), dim3(kThreads), 0, st, p); break;
    case 8: hipLaunchKernelGGL(stem_fwd_kernel<8>, dim3((unsigned)mtiles), dim3(kThreads), 0, st, p); break;
    default: return LBT_EINVAL;
  }
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_stem_wgrad(const int16_t* x, const int8_t* gq, lbt_conv_desc d, int32_t* slab, int32_t nshard,
                                   void* stream) {
  const int K = d.KH * d.KW * d.Cin;
  if (K <= 0 || K > 32 || d.Cout <= 0 || d.Cout % 16 || d.Cout > 64 || nshard <= 0) return LBT_EINVAL;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (M <= 0) return LBT_OK;
  const int64_t blocks = (M + kWgPixels - 1) / kWgPixels;
  // int32 shard totals stay exact: <= ceil(blocks/nshard) * 256 pixels * 2048 * 128 < 2^31
  if ((blocks + nshard - 1) / nshard > 31 || M >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if (d.Cout == 16 && d.KH == 3 && d.KW == 3 && d.SH == 1 && d.SW == 1 && d.PT == 1 && d.PL == 1 && d.Ho == d.H &&
      d.Wo == d.W && d.Cin <= kStemCinMax && d.W >= 8 && d.W <= kStemWMax && 64 % d.W == 0 &&
      ((int64_t)d.H * d.W) % kWgPixels == 0 && (kWgPixels / d.W + 2) * (d.W + 2) * d.Cin <= 4096 &&
      (kWgPixels / d.W + 2) * (d.W + 2) * d.Cin <= 16 * kThreads && getenv("LBT_STEM_GATHER") == nullptr) {
    hipLaunchKernelGGL(stem_wgrad_rows_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, x, gq, d,
                       K, slab, (int)nshard);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, x, gq, d, K, M,
                     slab, (int)nshard);
  return (int)hipGetLastError();
}

// stem_bwd_rows_kernel's shapes: stem_wgrad_rows_kernel's (3x3 / stride 1 / SAME, Cout 16, W | 64,
// whole 256-pixel row blocks) with the pass-B chain's (C 16, 8-bit stochastic or nearest codes)
extern "C" int lbt_conv_stem_bwd(const lbt_chain_bwd_b* b, const int16_t* x, lbt_conv_desc d, int32_t* slab,
                                 int32_t nshard, void* stream) {
  if (!b || !x || !slab || nshard <= 0) return LBT_EINVAL;
  const int K = d.KH * d.KW * d.Cin;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (M <= 0) return LBT_OK;
  if (!stem_bwd_shape_ok(b, d)) return LBT_EINVAL;
  const int64_t blocks = M / kWgPixels;
  if ((blocks + nshard - 1) / nshard > 31) return LBT_EINVAL;  // int32 shard totals stay exact
  StemBwdArgs p;
  p.b = *b; p.x = x; p.d = d; p.K = K; p.slab = slab; p.nshard = nshard;
  hipLaunchKernelGGL(stem_bwd_rows_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

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
//        writes one int32 partial slab[wg][K][Cout] for lbt_conv_wgrad_reduce(_many).
#include "conv_epilogue.h"

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

// patch element k of output pixel (n, oy, ox) -> input code (0 outside the image)
LBT_DEV int patch_code(const int16_t* x, const lbt_conv_desc& d, int n, int oy, int ox, int k) {
  const int tap = k / d.Cin, ci = k - tap * d.Cin;
  const int kh = tap / d.KW, kw = tap - kh * d.KW;
  const int iy = oy * d.SH + kh - d.PT, ix = ox * d.SW + kw - d.PL;
  if ((unsigned)iy >= (unsigned)d.H || (unsigned)ix >= (unsigned)d.W) return 0;
  return x[(((int64_t)n * d.H + iy) * d.W + ix) * d.Cin + ci];
}

__global__ __launch_bounds__(kThreads) void stem_fwd_kernel(StemFwdArgs p) {
  __shared__ int sh_cnt[2 * kThreads / 64];
  __shared__ long long sh_sum[2 * 128];
  __shared__ float tile[4][16][33];
  LBT_TS(0);
  const lbt_conv_desc& d = p.d;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nt_total = d.Cout >> 4;
  const int wpm = nt_total < 4 ? nt_total : 4;  // waves per M-tile
  const int ntw = nt_total / wpm;               // n-tiles per wave (1 or 2)
  const int mtb = 4 / wpm;                      // M-tiles per block
  const int mt_local = wave / wpm;
  const int nt0 = (wave % wpm) * ntw;
  const int64_t mtile = (int64_t)blockIdx.x * mtb + mt_local;
  const bool wave_live = mt_local < mtb;
  const int r = lane & 15, kg = lane >> 4;
  const int64_t M = p.o.M;
  const bool want_q = p.o.yq != nullptr;
  const bool want_sum = want_q && p.o.chsum != nullptr;
  if (want_sum) {
    for (int i = threadIdx.x; i < 2 * d.Cout; i += kThreads) sh_sum[i] = 0;
    __syncthreads();
  }
  f4v acc[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
  if (wave_live) {
    const int64_t m = mtile * 16 + r;
    h8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (_Float16)0.f;
    if (m < M) {
      const int ox = (int)(m % d.Wo);
      const int64_t t = m / d.Wo;
      const int oy = (int)(t % d.Ho), n = (int)(t / d.Ho);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * kg + j;
        if (k < p.K) a[j] = (_Float16)(float)patch_code(p.x, d, n, oy, ox, k);
      }
    }
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      if (jt >= ntw) continue;
      const int col = (nt0 + jt) * 16 + r;
      h8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * kg + j;
        b[j] = (_Float16)(float)(k < p.K ? (int)p.w[(int64_t)k * d.Cout + col] : 0);
      }
      acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[jt], 0, 0, 0);
    }
  }
  LBT_TS(1);
  const float scale = ldexpf(1.0f, -(frac_exp(p.qx) + frac_exp(p.qw)));
  if (!want_q) {
    if (!wave_live) return;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      if (jt >= ntw) continue;
      const int col = (nt0 + jt) * 16 + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = mtile * 16 + kg * 4 + i;
        if (row < M) p.y[row * d.Cout + col] = acc[jt][i] * scale;
      }
    }
    return;
  }
  if (wave_live) {
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      if (jt >= ntw) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) tile[wave][kg * 4 + i][jt * 16 + r] = acc[jt][i] * scale;
    }
  }
  wave_lds_sync();
  LBT_TS(2);
  quant_epilogue(p.o, tile[wave], wave_live, mtile, nt0, ntw, sh_sum, sh_cnt);
  LBT_TS(3);
}

// grid = nsplit workgroups of kWgPixels pixels; Cout <= 64 (ct tiles), K <= 32 (2 kt tiles)
__global__ __launch_bounds__(kThreads) void stem_wgrad_kernel(const int16_t* __restrict__ x,
                                                              const int8_t* __restrict__ gq, lbt_conv_desc d, int K,
                                                              int64_t M, int32_t* __restrict__ slab) {
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
      const int64_t mm = pv[j] ? m : 0;
      pox[j] = (int)(mm % d.Wo);
      const int64_t t = mm / d.Wo;
      poy[j] = (int)(t % d.Ho);
      pn[j] = (int)(t / d.Ho);
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int k = kt * 16 + r;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        a[s][kt][j] = (_Float16)(float)((kt < nkt && k < K && pv[j]) ? patch_code(x, d, pn[j], poy[j], pox[j], k) : 0);
    }
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int c = ct * 16 + r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t m = p0 + 32 * s + 8 * kg + j;
        b[s][ct][j] = (_Float16)(float)((ct < nct && pv[j]) ? (int)gq[m * d.Cout + c] : 0);
      }
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
  int32_t* out = slab + (int64_t)blockIdx.x * K * d.Cout;
  for (int i = threadIdx.x; i < K * d.Cout; i += kThreads) {
    const int k = i / d.Cout, c = i - k * d.Cout;
    out[i] = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
  }
}

}  // namespace

LBT_TRACE_SETTER(stem)

extern "C" int lbt_conv_stem_fwd(const int16_t* x, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw,
                                 float* y, int8_t* yq, lbt_qdesc qout, int64_t* ychsum, void* stream) {
  const int K = d.KH * d.KW * d.Cin;
  if (K <= 0 || K > 32 || d.Cout <= 0 || d.Cout % 16 || d.Cout > 128) return LBT_EINVAL;
  if ((y == nullptr) == (yq == nullptr)) return LBT_EINVAL;
  if (yq && qout.bits > 8) return LBT_EINVAL;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (M <= 0) return LBT_OK;
  StemFwdArgs p;
  p.x = x; p.w = w_hwio; p.d = d; p.K = K; p.qx = qx; p.qw = qw; p.y = y;
  p.o = QOut{yq, qout, yq ? ychsum : nullptr, M, d.Cout, (int64_t)d.Ho * d.Wo};
  const int nt = d.Cout / 16, wpm = nt < 4 ? nt : 4, mtb = 4 / wpm;
  const int64_t blocks = ((M + 15) / 16 + mtb - 1) / mtb;
  if (blocks > 0x7fffffff) return LBT_EINVAL;
  hipLaunchKernelGGL(stem_fwd_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_stem_wgrad(const int16_t* x, const int8_t* gq, lbt_conv_desc d, int32_t* slab, int32_t nsplit,
                                   void* stream) {
  const int K = d.KH * d.KW * d.Cin;
  if (K <= 0 || K > 32 || d.Cout <= 0 || d.Cout % 16 || d.Cout > 64) return LBT_EINVAL;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (nsplit != (int32_t)((M + kWgPixels - 1) / kWgPixels)) return LBT_EINVAL;
  if (M <= 0) return LBT_OK;
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3((unsigned)nsplit), dim3(kThreads), 0, (hipStream_t)stream, x, gq, d, K, M,
                     slab);
  return (int)hipGetLastError();
}

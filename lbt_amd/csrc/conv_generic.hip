// conv_generic.hip -- any-shape integer convolution on the VALU (int32 accumulation).
//
// Used where the MFMA implicit GEMM does not apply:
//   * signed 9-bit inputs (ResNet conv1 reads the image, quantised at bits+1 = 9 bits,
//     dynamic_fixed_point.py:287-288 -- int8 MFMA is signed x signed 8-bit);
//   * channel counts that are not multiples of 16 (conv1 Cin=3, Dense_q 64->10 run as a
//     1x1 conv on [B,1,1,C], custom.py's MNIST convs).
// Exact integer arithmetic, so results are bit-identical to the MFMA path and the oracle.
#include "dfxp_device.h"

using namespace lbt;

namespace {

template <typename TX>
__global__ __launch_bounds__(256) void conv_fwd_generic_kernel(const TX* __restrict__ x, const int8_t* __restrict__ w,
                                                              lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw,
                                                              float* __restrict__ y) {
  const float scale = ldexpf(1.0f, -(frac_exp(qx) + frac_exp(qw)));
  const int64_t total = (int64_t)d.N * d.Ho * d.Wo * d.Cout;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint32_t iu = (uint32_t)i;  // total < 2^31 (launcher)
  const int co = (int)(iu % (uint32_t)d.Cout);
  uint32_t m = iu / (uint32_t)d.Cout;
  const int ow = (int)(m % (uint32_t)d.Wo);
  m /= (uint32_t)d.Wo;
  const int oh = (int)(m % (uint32_t)d.Ho);
  const int n = (int)(m / (uint32_t)d.Ho);
  int acc = 0;
  for (int kh = 0; kh < d.KH; ++kh) {
    const int ih = oh * d.SH + kh - d.PT;
    if ((unsigned)ih >= (unsigned)d.H) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int iw = ow * d.SW + kw - d.PL;
      if ((unsigned)iw >= (unsigned)d.W) continue;
      const TX* xp = x + (((int64_t)n * d.H + ih) * d.W + iw) * d.Cin;
      const int8_t* wp = w + ((int64_t)(kh * d.KW + kw) * d.Cin) * d.Cout + co;
      for (int ci = 0; ci < d.Cin; ++ci) acc += (int)xp[ci] * (int)wp[(int64_t)ci * d.Cout];
    }
  }
  y[i] = (float)acc * scale;
}

// TG = int16_t with TACC = int64: 9..16-bit gradient codes (config 4), whose products with 8-bit
// weights overflow an int32 sum.
template <typename TG, typename TACC>
__global__ __launch_bounds__(256) void conv_dgrad_generic_kernel(const TG* __restrict__ g,
                                                                const int8_t* __restrict__ w, lbt_conv_desc d,
                                                                lbt_qdesc qg, lbt_qdesc qw, float* __restrict__ dx,
                                                                const float* __restrict__ add_src) {
  const float scale = ldexpf(1.0f, -(frac_exp(qg) + frac_exp(qw)));
  const int64_t total = (int64_t)d.N * d.H * d.W * d.Cin;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint32_t iu = (uint32_t)i;  // total < 2^31 (launcher)
  const int ci = (int)(iu % (uint32_t)d.Cin);
  uint32_t m = iu / (uint32_t)d.Cin;
  const int iw = (int)(m % (uint32_t)d.W);
  m /= (uint32_t)d.W;
  const int ih = (int)(m % (uint32_t)d.H);
  const int n = (int)(m / (uint32_t)d.H);
  TACC acc = 0;
  for (int kh = 0; kh < d.KH; ++kh) {
    const int ny = ih + d.PT - kh;
    if (ny < 0 || ny % d.SH) continue;
    const int oh = ny / d.SH;
    if (oh >= d.Ho) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int nx = iw + d.PL - kw;
      if (nx < 0 || nx % d.SW) continue;
      const int ow = nx / d.SW;
      if (ow >= d.Wo) continue;
      const TG* gp = g + (((int64_t)n * d.Ho + oh) * d.Wo + ow) * d.Cout;
      const int8_t* wp = w + ((int64_t)(kh * d.KW + kw) * d.Cin + ci) * d.Cout;
      for (int co = 0; co < d.Cout; ++co) acc += (TACC)((int)gp[co] * (int)wp[co]);
    }
  }
  const float v = (float)acc * scale;
  dx[i] = add_src ? v + add_src[i] : v;
}

// grid = (nsplit, output tiles of kMaxOut*256); block (b, t) reduces pixels [b*per, (b+1)*per)
// for outputs [t*kTile, (t+1)*kTile) in chunks of kChunk pixels staged in LDS (the im2col
// patch columns k in [klo, khi) that tile needs, and the G rows), each thread owning <= 16 outputs.
constexpr int kMaxChunk = 32;  // pixels per LDS pass (fewer when Cout is large: the G rows must fit)
constexpr int kMaxOut = 16;
constexpr int kTile = kMaxOut * 256;
template <typename TX, typename TG, typename TACC>
__global__ __launch_bounds__(256) void conv_wgrad_generic_kernel(const TX* __restrict__ x, const TG* __restrict__ g,
                                                                lbt_conv_desc d, TACC* __restrict__ slab,
                                                                int64_t P, int nsplit, int kChunk) {
  extern __shared__ int16_t sh[];
  const int K = d.KH * d.KW * d.Cin;
  const int nout = K * d.Cout;
  const int o0 = blockIdx.y * kTile;
  const int o1 = o0 + kTile < nout ? o0 + kTile : nout;
  const int klo = o0 / d.Cout, khi = (o1 - 1) / d.Cout + 1;
  const int KS = khi - klo;
  int16_t* Xs = sh;                 // [kChunk][KS]
  int16_t* Gs = sh + kChunk * KS;   // [kChunk][Cout]
  const int64_t per = (P + nsplit - 1) / nsplit;
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = p0 + per < P ? p0 + per : P;
  TACC acc[kMaxOut];
#pragma unroll
  for (int j = 0; j < kMaxOut; ++j) acc[j] = 0;
  const int64_t HWo = (int64_t)d.Ho * d.Wo;
  for (int64_t c0 = p0; c0 < p1; c0 += kChunk) {
    const int cn = (int)(p1 - c0 < kChunk ? p1 - c0 : kChunk);
    for (int t = threadIdx.x; t < kChunk * KS; t += blockDim.x) {
      const int pl = t / KS, k = klo + (t - pl * KS);
      int v = 0;
      if (pl < cn) {
        const uint32_t p = (uint32_t)(c0 + pl);  // P < 2^31 (launcher)
        const uint32_t n = p / (uint32_t)HWo;
        const uint32_t rem = p - n * (uint32_t)HWo;
        const int oh = (int)(rem / (uint32_t)d.Wo), ow = (int)(rem - (uint32_t)oh * (uint32_t)d.Wo);
        const int tap = k / d.Cin, ci = k - tap * d.Cin;
        const int kh = tap / d.KW, kw = tap - kh * d.KW;
        const int ih = oh * d.SH + kh - d.PT, iw = ow * d.SW + kw - d.PL;
        if ((unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W)
          v = (int)x[(((int64_t)n * d.H + ih) * d.W + iw) * d.Cin + ci];
      }
      Xs[t] = (int16_t)v;
    }
    for (int t = threadIdx.x; t < kChunk * d.Cout; t += blockDim.x) {
      const int pl = t / d.Cout, co = t - pl * d.Cout;
      Gs[t] = pl < cn ? (int16_t)g[(c0 + pl) * d.Cout + co] : (int16_t)0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kMaxOut; ++j) {
      const int o = o0 + threadIdx.x + j * blockDim.x;
      if (o < o1) {
        const int k = o / d.Cout, co = o - k * d.Cout;
        TACC a = acc[j];
        for (int pl = 0; pl < kChunk; ++pl) a += (TACC)((int)Xs[pl * KS + (k - klo)] * (int)Gs[pl * d.Cout + co]);
        acc[j] = a;
      }
    }
    __syncthreads();
  }
  TACC* dst = slab + (int64_t)blockIdx.x * nout;
#pragma unroll
  for (int j = 0; j < kMaxOut; ++j) {
    const int o = o0 + threadIdx.x + j * blockDim.x;
    if (o < o1) dst[o] = acc[j];
  }
}

bool desc_ok(const lbt_conv_desc& d) {
  return d.N > 0 && d.H > 0 && d.W > 0 && d.KH > 0 && d.KW > 0 && d.SH > 0 && d.SW > 0 && d.Ho > 0 &&
         d.Wo > 0 && d.Cin > 0 && d.Cout > 0;
}

}  // namespace

extern "C" int lbt_conv_fwd_generic(const void* xq, int32_t x_i16, const int8_t* w_hwio, lbt_conv_desc d,
                                    lbt_qdesc qx, lbt_qdesc qw, float* y, void* stream) {
  if (!desc_ok(d)) return LBT_EINVAL;
  const int64_t total = (int64_t)d.N * d.Ho * d.Wo * d.Cout;
  if (total >= ((int64_t)1 << 31)) return LBT_EINVAL;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  if (x_i16)
    hipLaunchKernelGGL(conv_fwd_generic_kernel<int16_t>, dim3(blocks), dim3(256), 0, st, (const int16_t*)xq, w_hwio, d,
                       qx, qw, y);
  else
    hipLaunchKernelGGL(conv_fwd_generic_kernel<int8_t>, dim3(blocks), dim3(256), 0, st, (const int8_t*)xq, w_hwio, d,
                       qx, qw, y);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_dgrad_generic(const int8_t* gq, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qg,
                                      lbt_qdesc qw, float* dx, const float* add_src, void* stream) {
  if (!desc_ok(d)) return LBT_EINVAL;
  const int64_t total = (int64_t)d.N * d.H * d.W * d.Cin;
  if (total >= ((int64_t)1 << 31)) return LBT_EINVAL;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL((conv_dgrad_generic_kernel<int8_t, int>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, gq,
                     w_hwio, d, qg, qw, dx, add_src);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_dgrad_generic16(const int16_t* gq, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qg,
                                        lbt_qdesc qw, float* dx, const float* add_src, void* stream) {
  if (!desc_ok(d)) return LBT_EINVAL;
  const int64_t total = (int64_t)d.N * d.H * d.W * d.Cin;
  if (total >= ((int64_t)1 << 31)) return LBT_EINVAL;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL((conv_dgrad_generic_kernel<int16_t, long long>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     gq, w_hwio, d, qg, qw, dx, add_src);
  return (int)hipGetLastError();
}

namespace {

// shared geometry of the generic wgrad launches; false = shape not supported
bool wgrad_geom(const lbt_conv_desc& d, int nsplit, dim3& grid, int& chunk, size_t& shm, int64_t& P) {
  if (!desc_ok(d) || nsplit <= 0) return false;
  const int64_t K = (int64_t)d.KH * d.KW * d.Cin;
  const int64_t nout = K * d.Cout;
  const int64_t tiles = (nout + kTile - 1) / kTile;
  if (tiles > 65535) return false;
  P = (int64_t)d.N * d.Ho * d.Wo;
  if (P >= ((int64_t)1 << 31)) return false;
  const int64_t ks_max = (kTile + d.Cout - 1) / d.Cout + 1 < K ? (kTile + d.Cout - 1) / d.Cout + 1 : K;
  chunk = (int)((64 * 1024) / (sizeof(int16_t) * (ks_max + d.Cout)));
  if (chunk > kMaxChunk) chunk = kMaxChunk;
  if (chunk < 1) return false;
  shm = sizeof(int16_t) * chunk * (ks_max + d.Cout);
  grid = dim3(nsplit, (unsigned)tiles);
  return true;
}

template <typename TACC>
__global__ __launch_bounds__(256) void wgrad_reduce_generic_kernel(const TACC* __restrict__ slab, int nsplit, int64_t total,
                                                                  lbt_qdesc qx, lbt_qdesc qg, const float* __restrict__ w,
                                                                  float wd2, float* __restrict__ dw,
                                                                  long long* __restrict__ num) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  long long s = 0;
  for (int b = 0; b < nsplit; ++b) s += (long long)slab[(int64_t)b * total + i];
  if (num) {  // the exact exchange: the numerator, dequantised after the all-reduce
    num[i] = s;
    return;
  }
  const float scale = ldexpf(1.0f, -(frac_exp(qx) + frac_exp(qg)));
  const float a = (float)s * scale;
  const float b = wd2 * w[i];
  dw[i] = a + b;
}

// Many splits (the wide wgrad kernels' stored partials): 64 outputs x 4 split groups per block,
// each group summing every 4th split; groups meet in LDS. Same exact int64 total, same epilogue.
__global__ __launch_bounds__(256) void wgrad_reduce64_split_kernel(const long long* __restrict__ slab, int nsplit,
                                                                   int64_t total, lbt_qdesc qx, lbt_qdesc qg,
                                                                   const float* __restrict__ w, float wd2,
                                                                   float* __restrict__ dw, long long* __restrict__ num) {
  __shared__ long long red[4][64];
  const int lo = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lo;
  long long s = 0;
  if (i < total) {
#pragma unroll 4
    for (int b = sg; b < nsplit; b += 4) s += slab[(int64_t)b * total + i];
  }
  red[sg][lo] = s;
  __syncthreads();
  if (sg != 0 || i >= total) return;
  s = red[0][lo] + red[1][lo] + red[2][lo] + red[3][lo];
  if (num) {
    num[i] = s;
    return;
  }
  const float scale = ldexpf(1.0f, -(frac_exp(qx) + frac_exp(qg)));
  const float a = (float)s * scale;
  const float b = wd2 * w[i];
  dw[i] = a + b;
}

// lbt_conv_wgrad_reduce64_many: wgrad_reduce64_split_kernel's block (64 outputs x 4 split groups) for the
// job owning the block -- the last job whose first_block <= blockIdx.x (uniform scalar loads of the small
// job array). The int64 totals are exact in any order, so every output equals the single-job launch's.
__global__ __launch_bounds__(256) void wgrad_reduce64_many_kernel(const lbt_r64job* __restrict__ jobs, int njobs) {
  __shared__ long long red[4][64];
  const int b = (int)blockIdx.x;
  int jb = 0;
  for (int k = 1; k < njobs; ++k)
    if (jobs[k].first_block <= b) jb = k;
  const lbt_r64job& J = jobs[jb];
  const int64_t total = (int64_t)J.K * J.Cout;
  const int lo = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int64_t i = (int64_t)(b - J.first_block) * 64 + lo;
  const long long* slab = reinterpret_cast<const long long*>(J.slab);
  long long s = 0;
  if (i < total) {
#pragma unroll 4
    for (int k = sg; k < J.nsplit; k += 4) s += slab[(int64_t)k * total + i];
  }
  red[sg][lo] = s;
  __syncthreads();
  if (sg != 0 || i >= total) return;
  s = red[0][lo] + red[1][lo] + red[2][lo] + red[3][lo];
  const float scale = ldexpf(1.0f, -(frac_exp(J.qx) + frac_exp(J.qg)));
  const float a = (float)s * scale;
  const float c = J.wd2 * J.w[i];
  J.dw[i] = a + c;
}

}  // namespace

extern "C" int lbt_conv_wgrad_reduce64_many(const lbt_r64job* jobs, int32_t njobs, int32_t nblocks, void* stream) {
  if (njobs < 0 || nblocks < 0 || (njobs > 0 && (!jobs || nblocks <= 0))) return LBT_EINVAL;
  if (njobs == 0) return LBT_OK;
  hipLaunchKernelGGL(wgrad_reduce64_many_kernel, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, jobs,
                     njobs);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_wgrad_generic(const void* xq, int32_t x_i16, const int8_t* gq, lbt_conv_desc d,
                                      int32_t* slab, int32_t nsplit, void* stream) {
  dim3 grid;
  int chunk;
  size_t shm;
  int64_t P;
  if (!wgrad_geom(d, nsplit, grid, chunk, shm, P)) return LBT_EINVAL;
  if ((P + nsplit - 1) / nsplit > 8192) return LBT_EINVAL;  // int32 partial bound for 9-bit x 8-bit
  hipStream_t st = (hipStream_t)stream;
  if (x_i16)
    hipLaunchKernelGGL((conv_wgrad_generic_kernel<int16_t, int8_t, int32_t>), grid, dim3(256), shm, st,
                       (const int16_t*)xq, gq, d, slab, P, nsplit, chunk);
  else
    hipLaunchKernelGGL((conv_wgrad_generic_kernel<int8_t, int8_t, int32_t>), grid, dim3(256), shm, st,
                       (const int8_t*)xq, gq, d, slab, P, nsplit, chunk);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_wgrad_generic16(const void* xq, int32_t x_i16, const int16_t* gq, lbt_conv_desc d,
                                        int64_t* slab, int32_t nsplit, void* stream) {
  dim3 grid;
  int chunk;
  size_t shm;
  int64_t P;
  if (!wgrad_geom(d, nsplit, grid, chunk, shm, P)) return LBT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (x_i16)
    hipLaunchKernelGGL((conv_wgrad_generic_kernel<int16_t, int16_t, long long>), grid, dim3(256), shm, st,
                       (const int16_t*)xq, gq, d, (long long*)slab, P, nsplit, chunk);
  else
    hipLaunchKernelGGL((conv_wgrad_generic_kernel<int8_t, int16_t, long long>), grid, dim3(256), shm, st,
                       (const int8_t*)xq, gq, d, (long long*)slab, P, nsplit, chunk);
  return (int)hipGetLastError();
}

static int reduce64_launch(const int64_t* slab, int32_t nsplit, int32_t K, int32_t Cout, lbt_qdesc qx, lbt_qdesc qg,
                           const float* w, float wd2, float* dw, int64_t* num, void* stream) {
  if (nsplit <= 0 || K <= 0 || Cout <= 0) return LBT_EINVAL;
  const int64_t total = (int64_t)K * Cout;
  if (nsplit > 8)
    hipLaunchKernelGGL(wgrad_reduce64_split_kernel, dim3((unsigned)((total + 63) / 64)), dim3(256), 0,
                       (hipStream_t)stream, (const long long*)slab, nsplit, total, qx, qg, w, wd2, dw, (long long*)num);
  else
    hipLaunchKernelGGL((wgrad_reduce_generic_kernel<long long>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const long long*)slab, nsplit, total, qx, qg, w, wd2, dw, (long long*)num);
  return (int)hipGetLastError();
}
extern "C" int lbt_conv_wgrad_reduce64(const int64_t* slab, int32_t nsplit, int32_t K, int32_t Cout, lbt_qdesc qx,
                                       lbt_qdesc qg, const float* w, float wd2, float* dw, void* stream) {
  return reduce64_launch(slab, nsplit, K, Cout, qx, qg, w, wd2, dw, nullptr, stream);
}
extern "C" int lbt_conv_wgrad_reduce64_x(const int64_t* slab, int32_t nsplit, int32_t K, int32_t Cout, int64_t* num,
                                         void* stream) {
  if (!num) return LBT_EINVAL;
  return reduce64_launch(slab, nsplit, K, Cout, lbt_qdesc{}, lbt_qdesc{}, nullptr, 0.f, nullptr, num, stream);
}

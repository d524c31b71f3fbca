// pool.hip -- MaxPool_q (dynamic_fixed_point.py:993-1006, tf.nn.max_pool) forward and backward.
//
// Forward: thread per output, the window scanned in (kh, kw) order with a strict '>' so the FIRST
// maximum wins; padding positions (TF SAME pads with -inf) are skipped. The winning window
// position is kept as one byte per output for the backward.
// Backward (TF MaxPoolGrad): each output's gradient goes to its argmax input; thread per INPUT
// element sums the gradients of the windows that chose it in ascending output order (oh, ow) --
// the order TF's CPU kernel accumulates them in -- starting from 0.
#include "dfxp_device.h"

namespace {

constexpr int kT = 256;

__global__ __launch_bounds__(kT) void maxpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                         uint8_t* __restrict__ amax, lbt_conv_desc d) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int64_t total = (int64_t)d.N * d.Ho * d.Wo * d.Cin;
  if (e >= total) return;
  const int c = (int)(e % d.Cin);
  int64_t m = e / d.Cin;
  const int ow = (int)(m % d.Wo);
  m /= d.Wo;
  const int oh = (int)(m % d.Ho);
  const int n = (int)(m / d.Ho);
  float best = -INFINITY;
  int bi = 0;
  for (int kh = 0; kh < d.KH; ++kh) {
    const int ih = oh * d.SH + kh - d.PT;
    if ((unsigned)ih >= (unsigned)d.H) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int iw = ow * d.SW + kw - d.PL;
      if ((unsigned)iw >= (unsigned)d.W) continue;
      const float v = x[(((int64_t)n * d.H + ih) * d.W + iw) * d.Cin + c];
      if (v > best) {
        best = v;
        bi = kh * d.KW + kw;
      }
    }
  }
  y[e] = best;
  amax[e] = (uint8_t)bi;
}

__global__ __launch_bounds__(kT) void maxpool_bwd_kernel(const float* __restrict__ g, const uint8_t* __restrict__ amax,
                                                         float* __restrict__ dx, lbt_conv_desc d) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int64_t total = (int64_t)d.N * d.H * d.W * d.Cin;
  if (e >= total) return;
  const int c = (int)(e % d.Cin);
  int64_t m = e / d.Cin;
  const int iw = (int)(m % d.W);
  m /= d.W;
  const int ih = (int)(m % d.H);
  const int n = (int)(m / d.H);
  // outputs whose window covers ih: oh*SH - PT <= ih <= oh*SH - PT + KH - 1
  const int ylo = ih + d.PT - d.KH + 1, yhi = ih + d.PT;
  const int xlo = iw + d.PL - d.KW + 1, xhi = iw + d.PL;
  int oh0 = ylo <= 0 ? 0 : (ylo + d.SH - 1) / d.SH, oh1 = yhi < 0 ? -1 : yhi / d.SH;
  int ow0 = xlo <= 0 ? 0 : (xlo + d.SW - 1) / d.SW, ow1 = xhi < 0 ? -1 : xhi / d.SW;
  if (oh1 >= d.Ho) oh1 = d.Ho - 1;
  if (ow1 >= d.Wo) ow1 = d.Wo - 1;
  float s = 0.f;
  for (int oh = oh0; oh <= oh1; ++oh)
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int64_t o = (((int64_t)n * d.Ho + oh) * d.Wo + ow) * d.Cin + c;
      const int pos = (ih - (oh * d.SH - d.PT)) * d.KW + (iw - (ow * d.SW - d.PL));
      if ((int)amax[o] == pos) s = s + g[o];
    }
  dx[e] = s;
}

constexpr int kNoRoute = 255;  // argmax code of a relu pool window that routes no gradient

// maxpool_fwd_kernel for 4 channels per thread (C % 4 == 0): the same scan and strict '>' per
// channel, 16-byte loads, one 4-byte argmax store.
// relu != 0: the pool of the preceding ReLU_q's output computed from its INPUT: max(relu(a), ...) =
// relu(max(a, ...)), so y is bit-identical. The argmax differs only where the window's max is <= 0
// (the reference's first zero vs the first raw maximum): there y = 0, the fused backward
// (maxpool_relu_bwd) routes nothing, and the code is kNoRoute -- the ReLU mask travels in the argmax,
// so the backward need not read y.
__global__ __launch_bounds__(kT) void maxpool_fwd4_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                          uint8_t* __restrict__ amax, lbt_conv_desc d, int relu) {
  const int64_t e4 = ((int64_t)blockIdx.x * kT + threadIdx.x) * 4;
  const int64_t total = (int64_t)d.N * d.Ho * d.Wo * d.Cin;
  if (e4 >= total) return;
  const int c = (int)(e4 % d.Cin);
  int64_t m = e4 / d.Cin;
  const int ow = (int)(m % d.Wo);
  m /= d.Wo;
  const int oh = (int)(m % d.Ho);
  const int n = (int)(m / d.Ho);
  float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int bi[4] = {0, 0, 0, 0};
  for (int kh = 0; kh < d.KH; ++kh) {
    const int ih = oh * d.SH + kh - d.PT;
    if ((unsigned)ih >= (unsigned)d.H) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int iw = ow * d.SW + kw - d.PL;
      if ((unsigned)iw >= (unsigned)d.W) continue;
      const float4 v4 = *reinterpret_cast<const float4*>(x + (((int64_t)n * d.H + ih) * d.W + iw) * d.Cin + c);
      const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (v[j] > best[j]) {
          best[j] = v[j];
          bi[j] = kh * d.KW + kw;
        }
    }
  }
  if (relu) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // the ReLU mask rides in the argmax: a window whose max is <= 0 (y = 0) routes no gradient, so
      // its code is kNoRoute, which no window position equals (KH*KW <= 255, launcher)
      if (!(best[j] > 0.f)) bi[j] = kNoRoute;
      best[j] = best[j] > 0.f ? best[j] : 0.f;
    }
  }
  *reinterpret_cast<float4*>(y + e4) = make_float4(best[0], best[1], best[2], best[3]);
  *reinterpret_cast<uchar4*>(amax + e4) = make_uchar4((uint8_t)bi[0], (uint8_t)bi[1], (uint8_t)bi[2], (uint8_t)bi[3]);
}

// The same gradient routing for 4 channels per thread (C % 4 == 0: 16-byte g / y and 4-byte amax
// loads), optionally with the preceding ReLU_q's backward folded in (ymask = this pool's forward
// output): the mask x > 0 of an input element is needed only where some window routes gradient to
// it, i.e. where it is that window's maximum, and then relu(x) = y[o] (the pool input is the ReLU
// output), so x > 0 <=> y[o] > 0 -- the mask costs one 16-byte load per window instead of a pass
// over the ReLU input, and dx is the exact value relu_bwd(maxpool_bwd(g)) stores (sum or +0).
// IT: the index type of the element -> (n, ih, iw, c) decomposition -- uint32_t when the tensor has < 2^31
// elements (ResNet-50's pool: 205 M), whose divisions are a few VALU ops where int64's are a software
// routine per division (three per thread); the same indices, so the same sums.
template <typename IT>
__global__ __launch_bounds__(kT) void maxpool_bwd4_kernel(const float* __restrict__ g, const uint8_t* __restrict__ amax,
                                                          const float* __restrict__ ymask, float* __restrict__ dx,
                                                          lbt_conv_desc d) {
  const int64_t e4 = ((int64_t)blockIdx.x * kT + threadIdx.x) * 4;
  const int64_t total = (int64_t)d.N * d.H * d.W * d.Cin;
  if (e4 >= total) return;
  const IT ei = (IT)e4;
  const int c = (int)(ei % (IT)d.Cin);
  IT m = ei / (IT)d.Cin;
  const int iw = (int)(m % (IT)d.W);
  m /= (IT)d.W;
  const int ih = (int)(m % (IT)d.H);
  const int n = (int)(m / (IT)d.H);
  const int ylo = ih + d.PT - d.KH + 1, yhi = ih + d.PT;
  const int xlo = iw + d.PL - d.KW + 1, xhi = iw + d.PL;
  int oh0 = ylo <= 0 ? 0 : (ylo + d.SH - 1) / d.SH, oh1 = yhi < 0 ? -1 : yhi / d.SH;
  int ow0 = xlo <= 0 ? 0 : (xlo + d.SW - 1) / d.SW, ow1 = xhi < 0 ? -1 : xhi / d.SW;
  if (oh1 >= d.Ho) oh1 = d.Ho - 1;
  if (ow1 >= d.Wo) ow1 = d.Wo - 1;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int oh = oh0; oh <= oh1; ++oh)
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int64_t o = (((int64_t)n * d.Ho + oh) * d.Wo + ow) * d.Cin + c;
      const int pos = (ih - (oh * d.SH - d.PT)) * d.KW + (iw - (ow * d.SW - d.PL));
      const uchar4 a = *reinterpret_cast<const uchar4*>(amax + o);
      const float4 gv = *reinterpret_cast<const float4*>(g + o);
      float4 yv = make_float4(1.f, 1.f, 1.f, 1.f);
      if (ymask) yv = *reinterpret_cast<const float4*>(ymask + o);
      if ((int)a.x == pos && yv.x > 0.f) s[0] = s[0] + gv.x;
      if ((int)a.y == pos && yv.y > 0.f) s[1] = s[1] + gv.y;
      if ((int)a.z == pos && yv.z > 0.f) s[2] = s[2] + gv.z;
      if ((int)a.w == pos && yv.w > 0.f) s[3] = s[3] + gv.w;
    }
  *reinterpret_cast<float4*>(dx + e4) = make_float4(s[0], s[1], s[2], s[3]);
}

void launch_bwd4(const float* g, const uint8_t* amax, const float* y, float* dx, const lbt_conv_desc& d, int64_t n,
                 hipStream_t st) {
  const dim3 grid((unsigned)((n / 4 + kT - 1) / kT));
  if (n < ((int64_t)1 << 31))
    hipLaunchKernelGGL(maxpool_bwd4_kernel<uint32_t>, grid, dim3(kT), 0, st, g, amax, y, dx, d);
  else
    hipLaunchKernelGGL(maxpool_bwd4_kernel<int64_t>, grid, dim3(kT), 0, st, g, amax, y, dx, d);
}

bool pool_desc_ok(const lbt_conv_desc& d) {
  return d.N > 0 && d.H > 0 && d.W > 0 && d.Cin > 0 && d.KH > 0 && d.KW > 0 && d.SH > 0 && d.SW > 0 && d.Ho > 0 &&
         d.Wo > 0;
}

}  // namespace

// d: N, H, W, Cin (= C), KH, KW, SH, SW, PT, PL, Ho, Wo (Cout, PB, PR unused)
extern "C" int lbt_maxpool_fwd(const float* x, float* y, uint8_t* amax, lbt_conv_desc d, void* stream) {
  if (d.N <= 0 || d.H <= 0 || d.W <= 0 || d.Cin <= 0 || d.KH <= 0 || d.KW <= 0 || d.KH * d.KW > 256 || d.SH <= 0 ||
      d.SW <= 0 || d.Ho <= 0 || d.Wo <= 0)
    return LBT_EINVAL;
  const int64_t n = (int64_t)d.N * d.Ho * d.Wo * d.Cin;
  if (d.Cin % 4 == 0)
    hipLaunchKernelGGL(maxpool_fwd4_kernel, dim3((unsigned)((n / 4 + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream,
                       x, y, amax, d, 0);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream, x,
                       y, amax, d);
  return (int)hipGetLastError();
}

extern "C" int lbt_maxpool_bwd(const float* g, const uint8_t* amax, float* dx, lbt_conv_desc d, void* stream) {
  if (d.N <= 0 || d.H <= 0 || d.W <= 0 || d.Cin <= 0 || d.KH <= 0 || d.KW <= 0 || d.SH <= 0 || d.SW <= 0 ||
      d.Ho <= 0 || d.Wo <= 0)
    return LBT_EINVAL;
  const int64_t n = (int64_t)d.N * d.H * d.W * d.Cin;
  if (d.Cin % 4 == 0)
    launch_bwd4(g, amax, nullptr, dx, d, n, (hipStream_t)stream);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream, g,
                       amax, dx, d);
  return (int)hipGetLastError();
}

// ReLU_q (forward) of the pool's input folded into the pool: x = the ReLU's input, y = pool(relu(x)).
// Only for use with lbt_maxpool_relu_bwd (see maxpool_fwd4_kernel). C % 4 == 0.
extern "C" int lbt_maxpool_relu_fwd(const float* x, float* y, uint8_t* amax, lbt_conv_desc d, void* stream) {
  if (!pool_desc_ok(d) || d.Cin % 4 || d.KH * d.KW > kNoRoute) return LBT_EINVAL;
  const int64_t n = (int64_t)d.N * d.Ho * d.Wo * d.Cin;
  hipLaunchKernelGGL(maxpool_fwd4_kernel, dim3((unsigned)((n / 4 + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream,
                     x, y, amax, d, 1);
  return (int)hipGetLastError();
}

// ReLU_q backward of the pool's input folded into the pool backward (y = this pool's forward
// output): dx = relu_bwd(maxpool_bwd(g)) in one pass. C % 4 == 0. y == NULL: amax comes from
// lbt_maxpool_relu_fwd and carries the mask (kNoRoute), so y is not read (16 of 36 bytes per window).
extern "C" int lbt_maxpool_relu_bwd(const float* g, const uint8_t* amax, const float* y, float* dx, lbt_conv_desc d,
                                    void* stream) {
  if (!pool_desc_ok(d) || d.Cin % 4) return LBT_EINVAL;
  const int64_t n = (int64_t)d.N * d.H * d.W * d.Cin;
  launch_bwd4(g, amax, y, dx, d, n, (hipStream_t)stream);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- AvgPool_q, any window
// dynamic_fixed_point.py:1009-1022 (tf.nn.avg_pool): y = (sum of the window's valid inputs in (kh, kw)
// order, fp32) / count, count = the number of valid (non-padding) positions -- TF SAME excludes the
// padding from the mean. Backward (TF AvgPoolGrad): each output spreads g / count over its window;
// a thread per INPUT adds the shares of the windows holding it in ascending output order.
namespace {

LBT_DEV int avg_count(const lbt_conv_desc& d, int oh, int ow) {
  int ch = 0, cw = 0;
  for (int kh = 0; kh < d.KH; ++kh) ch += (unsigned)(oh * d.SH + kh - d.PT) < (unsigned)d.H;
  for (int kw = 0; kw < d.KW; ++kw) cw += (unsigned)(ow * d.SW + kw - d.PL) < (unsigned)d.W;
  return ch * cw;
}

__global__ __launch_bounds__(kT) void avgpool_gen_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             lbt_conv_desc d) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int64_t total = (int64_t)d.N * d.Ho * d.Wo * d.Cin;
  if (e >= total) return;
  const int c = (int)(e % d.Cin);
  int64_t m = e / d.Cin;
  const int ow = (int)(m % d.Wo);
  m /= d.Wo;
  const int oh = (int)(m % d.Ho);
  const int n = (int)(m / d.Ho);
  float acc = 0.f;
  for (int kh = 0; kh < d.KH; ++kh) {
    const int ih = oh * d.SH + kh - d.PT;
    if ((unsigned)ih >= (unsigned)d.H) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int iw = ow * d.SW + kw - d.PL;
      if ((unsigned)iw >= (unsigned)d.W) continue;
      acc = acc + x[(((int64_t)n * d.H + ih) * d.W + iw) * d.Cin + c];
    }
  }
  y[e] = acc / (float)avg_count(d, oh, ow);
}

__global__ __launch_bounds__(kT) void avgpool_gen_bwd_kernel(const float* __restrict__ g, float* __restrict__ dx,
                                                             lbt_conv_desc d) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int64_t total = (int64_t)d.N * d.H * d.W * d.Cin;
  if (e >= total) return;
  const int c = (int)(e % d.Cin);
  int64_t m = e / d.Cin;
  const int iw = (int)(m % d.W);
  m /= d.W;
  const int ih = (int)(m % d.H);
  const int n = (int)(m / d.H);
  // outputs whose window holds (ih, iw): oh*SH - PT <= ih < oh*SH - PT + KH
  const int oh_lo = max(0, (ih + d.PT - d.KH + d.SH) / d.SH), oh_hi = min(d.Ho - 1, (ih + d.PT) / d.SH);
  const int ow_lo = max(0, (iw + d.PL - d.KW + d.SW) / d.SW), ow_hi = min(d.Wo - 1, (iw + d.PL) / d.SW);
  float acc = 0.f;
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int r = ih + d.PT - oh * d.SH;
    if (r < 0 || r >= d.KH) continue;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int q = iw + d.PL - ow * d.SW;
      if (q < 0 || q >= d.KW) continue;
      const float share = g[(((int64_t)n * d.Ho + oh) * d.Wo + ow) * d.Cin + c] / (float)avg_count(d, oh, ow);
      acc = acc + share;
    }
  }
  dx[e] = acc;
}

}  // namespace

extern "C" int lbt_avgpool_gen_fwd(const float* x, float* y, lbt_conv_desc d, void* stream) {
  if (!pool_desc_ok(d)) return LBT_EINVAL;
  const int64_t n = (int64_t)d.N * d.Ho * d.Wo * d.Cin;
  hipLaunchKernelGGL(avgpool_gen_fwd_kernel, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream, x,
                     y, d);
  return (int)hipGetLastError();
}

extern "C" int lbt_avgpool_gen_bwd(const float* g, float* dx, lbt_conv_desc d, void* stream) {
  if (!pool_desc_ok(d)) return LBT_EINVAL;
  const int64_t n = (int64_t)d.N * d.H * d.W * d.Cin;
  hipLaunchKernelGGL(avgpool_gen_bwd_kernel, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream, g,
                     dx, d);
  return (int)hipGetLastError();
}

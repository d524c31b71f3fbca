// fp32.hip -- the full-width end of the reference's bit-width domain (weight_quantization asserts
// 1 <= bits <= 32, dynamic_fixed_point.py:21-23): quantisers of 17..31 bits produce fake-quantised
// fp32 values whose integer codes no longer fit the int8 / int16 GEMM paths, and bits == 32 is the
// full-precision bypass. Layers at those widths run their contractions and BatchNorm statistics on
// these fp32 kernels, exactly as TF computes them on the fake-quantised tensors (fp32 operands),
// with every reduction accumulated in double in a fixed order (deterministic; within ~1 ulp of an
// exact sum). Not the hot path: straightforward VALU loops.
//
//  lbt_conv_fwd_f32 / _dgrad_f32 / _wgrad_f32 (+ _wgrad_reduce_f32)   Conv2d_q :287-305, Dense_q :388-460
//  lbt_chan_sums_f32                                                 per-channel sums (moments, dgamma)
//  lbt_bn_f32_fwd / lbt_bn_f32_bwd                                   Normalization_q :584-623
//  lbt_affine_f32 / lbt_affine_grads_f32                             Rescale_q :677-691
#include "dfxp_device.h"

namespace {

constexpr int kT = 256;

__global__ __launch_bounds__(kT) void conv_fwd_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          lbt_conv_desc d, float* __restrict__ y) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (e >= (int64_t)d.N * d.Ho * d.Wo * d.Cout) return;
  const int co = (int)(e % d.Cout);
  int64_t m = e / d.Cout;
  const int ow = (int)(m % d.Wo);
  m /= d.Wo;
  const int oh = (int)(m % d.Ho);
  const int n = (int)(m / d.Ho);
  double acc = 0.0;
  for (int kh = 0; kh < d.KH; ++kh) {
    const int ih = oh * d.SH + kh - d.PT;
    if ((unsigned)ih >= (unsigned)d.H) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int iw = ow * d.SW + kw - d.PL;
      if ((unsigned)iw >= (unsigned)d.W) continue;
      const float* xp = x + (((int64_t)n * d.H + ih) * d.W + iw) * d.Cin;
      const float* wp = w + ((int64_t)(kh * d.KW + kw) * d.Cin) * d.Cout + co;
      for (int ci = 0; ci < d.Cin; ++ci) acc += (double)xp[ci] * (double)wp[(int64_t)ci * d.Cout];
    }
  }
  y[e] = (float)acc;
}

__global__ __launch_bounds__(kT) void conv_dgrad_f32_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                            lbt_conv_desc d, float* __restrict__ dx,
                                                            const float* __restrict__ add) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (e >= (int64_t)d.N * d.H * d.W * d.Cin) return;
  const int ci = (int)(e % d.Cin);
  int64_t m = e / d.Cin;
  const int iw = (int)(m % d.W);
  m /= d.W;
  const int ih = (int)(m % d.H);
  const int n = (int)(m / d.H);
  double acc = 0.0;
  for (int kh = 0; kh < d.KH; ++kh) {
    const int ty = ih + d.PT - kh;
    if (ty < 0 || ty % d.SH) continue;
    const int oh = ty / d.SH;
    if (oh >= d.Ho) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int tx = iw + d.PL - kw;
      if (tx < 0 || tx % d.SW) continue;
      const int ow = tx / d.SW;
      if (ow >= d.Wo) continue;
      const float* gp = g + (((int64_t)n * d.Ho + oh) * d.Wo + ow) * d.Cout;
      const float* wp = w + ((int64_t)(kh * d.KW + kw) * d.Cin + ci) * d.Cout;
      for (int co = 0; co < d.Cout; ++co) acc += (double)gp[co] * (double)wp[co];
    }
  }
  const float v = (float)acc;
  dx[e] = add ? v + add[e] : v;
}

// grid (splits, ceil(K*Cout / 256)): slab[split][k][co] = sum over the split's pixels of x_tap * g
__global__ __launch_bounds__(kT) void conv_wgrad_f32_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                            lbt_conv_desc d, double* __restrict__ slab, int nsplit) {
  const int64_t K = (int64_t)d.KH * d.KW * d.Cin;
  const int64_t o = (int64_t)blockIdx.y * kT + threadIdx.x;
  if (o >= K * d.Cout) return;
  const int co = (int)(o % d.Cout);
  const int64_t k = o / d.Cout;
  const int ci = (int)(k % d.Cin), tap = (int)(k / d.Cin);
  const int kh = tap / d.KW, kw = tap - kh * d.KW;
  const int64_t P = (int64_t)d.N * d.Ho * d.Wo;
  const int64_t per = (P + nsplit - 1) / nsplit, p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = p0 + per < P ? p0 + per : P;
  double acc = 0.0;
  for (int64_t p = p0; p < p1; ++p) {
    const int ow = (int)(p % d.Wo);
    const int64_t t = p / d.Wo;
    const int oh = (int)(t % d.Ho);
    const int n = (int)(t / d.Ho);
    const int ih = oh * d.SH + kh - d.PT, iw = ow * d.SW + kw - d.PL;
    if ((unsigned)ih >= (unsigned)d.H || (unsigned)iw >= (unsigned)d.W) continue;
    acc += (double)x[(((int64_t)n * d.H + ih) * d.W + iw) * d.Cin + ci] * (double)g[p * d.Cout + co];
  }
  slab[(int64_t)blockIdx.x * K * d.Cout + o] = acc;
}

__global__ __launch_bounds__(kT) void wgrad_reduce_f32_kernel(const double* __restrict__ slab, int nsplit, int64_t total,
                                                              const float* __restrict__ w, float wd2,
                                                              float* __restrict__ dw) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= total) return;
  double s = 0.0;
  for (int b = 0; b < nsplit; ++b) s += slab[(int64_t)b * total + i];
  const float a = (float)s;
  const float b = wd2 * w[i];
  dw[i] = a + b;
}

// grid (splits, ceil(C / 256)), thread = channel: part[split][c] = sum a, part[split][C + c] = sum a*b
// (b NULL: a*a) over the split's rows of a [rows][C] tensor.
__global__ __launch_bounds__(kT) void chan_sums_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           int64_t rows, int C, int nsplit, double* __restrict__ part) {
  const int c = blockIdx.y * kT + threadIdx.x;
  if (c >= C) return;
  const int64_t per = (rows + nsplit - 1) / nsplit, r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    const double v = a[r * C + c];
    s1 += v;
    s2 += v * (b ? (double)b[r * C + c] : v);
  }
  part[(int64_t)blockIdx.x * 2 * C + c] = s1;
  part[(int64_t)blockIdx.x * 2 * C + C + c] = s2;
}

LBT_DEV void chan_total(const double* part, int nsplit, int C, int c, double& s1, double& s2) {
  s1 = 0.0;
  s2 = 0.0;
  for (int b = 0; b < nsplit; ++b) {
    s1 += part[(int64_t)b * 2 * C + c];
    s2 += part[(int64_t)b * 2 * C + C + c];
  }
}

// Normalization_q on fp32 inputs: mu = (float)(S1/n), var = (float)(S2/n - mean^2) (biased, as
// tf.nn.moments), sigma = sqrtf(var + eps), y = (x - mu) / sigma; running averages as lbt_bn_norm;
// frozen: the running averages instead (testing mode). Every block finalises its channels in LDS.
__global__ __launch_bounds__(kT) void bn_f32_fwd_kernel(const float* __restrict__ x, const double* __restrict__ part,
                                                        int nsplit, int64_t rows, int C, float eps, float mom,
                                                        float omm, float* ms, float* run_mean, float* run_var,
                                                        int frozen, float* __restrict__ y) {
  extern __shared__ float sh[];  // mu[C], sigma[C]
  const bool writer = blockIdx.x == 0;
  for (int c = threadIdx.x; c < C; c += kT) {
    float m, v;
    if (frozen) {
      m = run_mean[c];
      v = run_var[c];
    } else {
      double s1, s2;
      chan_total(part, nsplit, C, c, s1, s2);
      const double md = s1 / (double)rows;
      m = (float)md;
      v = (float)(s2 / (double)rows - md * md);
    }
    const float sig = sqrtf(v + eps);
    sh[c] = m;
    sh[C + c] = sig;
    if (writer) {
      ms[c] = m;
      ms[C + c] = sig;
      if (!frozen && run_mean) {
        run_mean[c] = mom * run_mean[c] + omm * m;
        run_var[c] = mom * run_var[c] + omm * v;
      }
    }
  }
  __syncthreads();
  const int64_t n = rows * C;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
    const int c = (int)(i % C);
    const float t = x[i] - sh[c];
    y[i] = t / sh[C + c];
  }
}

// Normalization_q backward on fp32 gradients g (the grad quantiser's fake-quantised values):
// part = chan sums (sum g, sum g*x); mg = (float)(Sg/n), mgx = (float)((Sgx - mu*Sg) / (n*sigma));
// dx = ((g - mg) - xhat*mgx) / sigma, xhat = (x - mu) / sigma -- the integer path's formula.
// frozen: mean and var are constants, dx = g / sigma.
__global__ __launch_bounds__(kT) void bn_f32_bwd_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                        const float* __restrict__ ms, const double* __restrict__ part,
                                                        int nsplit, int64_t rows, int C, int frozen,
                                                        float* __restrict__ dx) {
  extern __shared__ float sh[];  // mg[C], mgx[C]
  for (int c = threadIdx.x; c < C; c += kT) {
    if (frozen) {
      sh[c] = 0.f;
      sh[C + c] = 0.f;
      continue;
    }
    double sg, sgx;
    chan_total(part, nsplit, C, c, sg, sgx);
    sh[c] = (float)(sg / (double)rows);
    sh[C + c] = (float)((sgx - (double)ms[c] * sg) / ((double)rows * (double)ms[C + c]));
  }
  __syncthreads();
  const int64_t n = rows * C;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
    const int c = (int)(i % C);
    const float sig = ms[C + c];
    if (frozen) {
      dx[i] = g[i] / sig;
      continue;
    }
    const float xh = (x[i] - ms[c]) / sig;
    const float t1 = g[i] - sh[c];
    const float t2 = xh * sh[C + c];
    dx[i] = (t1 - t2) / sig;
  }
}

// Rescale_q: y = x * gb[c] + gb[C + c] (gb = [gamma_q | beta_q]); with g != NULL the backward dx = g * gamma_q.
__global__ __launch_bounds__(kT) void affine_f32_kernel(const float* __restrict__ x, const float* __restrict__ gb,
                                                        int64_t n, int C, int bwd, float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const float m = x[i] * gb[c];
  y[i] = bwd ? m : m + gb[C + c];
}

// dgamma = (float)(sum g*x) + wd2 * gamma, dbeta = (float)(sum g) from chan sums of (g, x).
__global__ void affine_grads_f32_kernel(const double* __restrict__ part, int nsplit, int C, const float* gamma,
                                        float wd2, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sg, sgx;
  chan_total(part, nsplit, C, c, sg, sgx);
  const float a = (float)sgx;
  const float b = wd2 * gamma[c];
  dgamma[c] = a + b;
  dbeta[c] = (float)sg;
}

bool desc_ok(const lbt_conv_desc& d) {
  return d.N > 0 && d.H > 0 && d.W > 0 && d.Cin > 0 && d.Cout > 0 && d.KH > 0 && d.KW > 0 && d.SH > 0 && d.SW > 0 &&
         d.Ho > 0 && d.Wo > 0;
}

unsigned nblk(int64_t n) { return (unsigned)((n + kT - 1) / kT); }

}  // namespace

extern "C" int lbt_conv_fwd_f32(const float* x, const float* w, lbt_conv_desc d, float* y, void* stream) {
  if (!desc_ok(d) || !x || !w || !y) return LBT_EINVAL;
  hipLaunchKernelGGL(conv_fwd_f32_kernel, dim3(nblk((int64_t)d.N * d.Ho * d.Wo * d.Cout)), dim3(kT), 0,
                     (hipStream_t)stream, x, w, d, y);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_dgrad_f32(const float* g, const float* w, lbt_conv_desc d, float* dx, const float* add_src,
                                  void* stream) {
  if (!desc_ok(d) || !g || !w || !dx) return LBT_EINVAL;
  hipLaunchKernelGGL(conv_dgrad_f32_kernel, dim3(nblk((int64_t)d.N * d.H * d.W * d.Cin)), dim3(kT), 0,
                     (hipStream_t)stream, g, w, d, dx, add_src);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_wgrad_f32(const float* x, const float* g, lbt_conv_desc d, double* slab, int32_t nsplit,
                                  void* stream) {
  if (!desc_ok(d) || nsplit <= 0 || nsplit > 65535 || !slab) return LBT_EINVAL;
  const int64_t K = (int64_t)d.KH * d.KW * d.Cin;
  const int64_t yb = (K * d.Cout + kT - 1) / kT;
  if (yb > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(conv_wgrad_f32_kernel, dim3((unsigned)nsplit, (unsigned)yb), dim3(kT), 0, (hipStream_t)stream, x,
                     g, d, slab, nsplit);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_wgrad_reduce_f32(const double* slab, int32_t nsplit, int64_t total, const float* w, float wd2,
                                         float* dw, void* stream) {
  if (nsplit <= 0 || total <= 0) return LBT_EINVAL;
  hipLaunchKernelGGL(wgrad_reduce_f32_kernel, dim3(nblk(total)), dim3(kT), 0, (hipStream_t)stream, slab, nsplit, total,
                     w, wd2, dw);
  return (int)hipGetLastError();
}

extern "C" int lbt_chan_sums_f32(const float* a, const float* b, int64_t rows, int32_t C, int32_t nsplit, double* part,
                                 void* stream) {
  if (rows <= 0 || C <= 0 || nsplit <= 0 || nsplit > 65535 || !a || !part) return LBT_EINVAL;
  hipLaunchKernelGGL(chan_sums_f32_kernel, dim3((unsigned)nsplit, (unsigned)((C + kT - 1) / kT)), dim3(kT), 0,
                     (hipStream_t)stream, a, b, rows, C, nsplit, part);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_f32_fwd(const float* x, const double* part, int32_t nsplit, int64_t rows, int32_t C, float eps,
                              float momentum, float one_minus_momentum, float* ms, float* run_mean, float* run_var,
                              int32_t frozen, float* y, void* stream) {
  if (rows <= 0 || C <= 0 || C > 8192 || !ms || (!frozen && (!part || nsplit <= 0))) return LBT_EINVAL;
  const int64_t blocks = std::min<int64_t>(1024, (rows * C + kT - 1) / kT);
  hipLaunchKernelGGL(bn_f32_fwd_kernel, dim3((unsigned)blocks), dim3(kT), 2 * C * sizeof(float), (hipStream_t)stream, x,
                     part, nsplit, rows, C, eps, momentum, one_minus_momentum, ms, run_mean, run_var, frozen, y);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_f32_bwd(const float* g, const float* x, const float* ms, const double* part, int32_t nsplit,
                              int64_t rows, int32_t C, int32_t frozen, float* dx, void* stream) {
  if (rows <= 0 || C <= 0 || C > 8192 || !ms || (!frozen && (!part || nsplit <= 0))) return LBT_EINVAL;
  const int64_t blocks = std::min<int64_t>(1024, (rows * C + kT - 1) / kT);
  hipLaunchKernelGGL(bn_f32_bwd_kernel, dim3((unsigned)blocks), dim3(kT), 2 * C * sizeof(float), (hipStream_t)stream, g,
                     x, ms, part, nsplit, rows, C, frozen, dx);
  return (int)hipGetLastError();
}

extern "C" int lbt_affine_f32(const float* x, const float* gb, int64_t n, int32_t C, int32_t bwd, float* y,
                              void* stream) {
  if (n <= 0 || C <= 0) return LBT_EINVAL;
  hipLaunchKernelGGL(affine_f32_kernel, dim3(nblk(n)), dim3(kT), 0, (hipStream_t)stream, x, gb, n, C, bwd, y);
  return (int)hipGetLastError();
}

extern "C" int lbt_affine_grads_f32(const double* part, int32_t nsplit, int32_t C, const float* gamma, float wd2,
                                    float* dgamma, float* dbeta, void* stream) {
  if (C <= 0 || nsplit <= 0) return LBT_EINVAL;
  hipLaunchKernelGGL(affine_grads_f32_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, part, nsplit, C,
                     gamma, wd2, dgamma, dbeta);
  return (int)hipGetLastError();
}

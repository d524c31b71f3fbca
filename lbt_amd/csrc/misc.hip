// misc.hip -- the unquantised fp32 glue of the ResNet-20 DFXP step and its optimiser:
//   ReLU_q (dynamic_fixed_point.py:983-990), residual add (:862, :869), AvgPool_q (:1009-1022),
//   mean sparse softmax cross-entropy (models.py:30-32) and MomentumOptimizer (trainer.py:81-82).
// All HBM-bound elementwise passes with 16-byte vector accesses where the shape allows.
#include "dfxp_device.h"

using namespace lbt;

namespace {

__global__ void relu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    float4 v = *reinterpret_cast<const float4*>(x + i);
    v.x = v.x > 0.f ? v.x : 0.f; v.y = v.y > 0.f ? v.y : 0.f;
    v.z = v.z > 0.f ? v.z : 0.f; v.w = v.w > 0.f ? v.w : 0.f;
    *reinterpret_cast<float4*>(y + i) = v;
  } else {
    for (int64_t k = i; k < n; ++k) y[k] = x[k] > 0.f ? x[k] : 0.f;
  }
}

__global__ void relu_bwd_kernel(const float* __restrict__ g, const float* __restrict__ x, float* __restrict__ dx,
                                int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 gv = *reinterpret_cast<const float4*>(g + i);
    const float4 xv = *reinterpret_cast<const float4*>(x + i);
    float4 o;
    o.x = xv.x > 0.f ? gv.x : 0.f; o.y = xv.y > 0.f ? gv.y : 0.f;
    o.z = xv.z > 0.f ? gv.z : 0.f; o.w = xv.w > 0.f ? gv.w : 0.f;
    *reinterpret_cast<float4*>(dx + i) = o;
  } else {
    for (int64_t k = i; k < n; ++k) dx[k] = x[k] > 0.f ? g[k] : 0.f;
  }
}

__global__ void add_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ y, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 av = *reinterpret_cast<const float4*>(a + i);
    const float4 bv = *reinterpret_cast<const float4*>(b + i);
    *reinterpret_cast<float4*>(y + i) = make_float4(av.x + bv.x, av.y + bv.y, av.z + bv.z, av.w + bv.w);
  } else {
    for (int64_t k = i; k < n; ++k) y[k] = a[k] + b[k];
  }
}

__global__ void avgpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int HW, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C;
  const float* p = x + (int64_t)n * HW * C + c;
  float acc = 0.f;
  // same sequential order as before (bit-exact), but 16 loads in flight per round trip
  for (int k0 = 0; k0 < HW; k0 += 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = p[(int64_t)(k0 + k < HW ? k0 + k : k0) * C];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k0 + k < HW) acc = acc + v[k];
  }
  y[i] = acc * (1.0f / (float)HW);
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ g, float* __restrict__ dx, int N, int HW, int C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * HW * C) return;
  const int c = (int)(i % C);
  const int n = (int)(i / ((int64_t)HW * C));
  dx[i] = g[n * C + c] * (1.0f / (float)HW);
}

// one block; rows strided over threads; loss = mean over rows
// norm: the batch the mean is over (N; the GLOBAL batch for a data-parallel shard); loss_fx: the
// ordered double sum of the loss terms in 2^-32 fixed point (the exact exchange's loss slot)
__global__ void softmax_xent_kernel(const float* __restrict__ z, const int32_t* __restrict__ labels, int N, int K,
                                    float* __restrict__ loss, float* __restrict__ dz, int norm, long long* loss_fx) {
  __shared__ double red[256];
  double part = 0.0;
  for (int r = threadIdx.x; r < N; r += blockDim.x) {
    const float* zr = z + (int64_t)r * K;
    float m = zr[0];
    for (int k = 1; k < K; ++k) m = zr[k] > m ? zr[k] : m;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = s + expf(zr[k] - m);
    const int y = labels[r];
    for (int k = 0; k < K; ++k) {
      const float p = expf(zr[k] - m) / s;
      dz[(int64_t)r * K + k] = (p - (k == y ? 1.f : 0.f)) / (float)norm;
    }
    const float lse = logf(s) + m;
    part += (double)(lse - zr[y]);
  }
  red[threadIdx.x] = part;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = (float)(red[0] / (double)norm);
    if (loss_fx) *loss_fx = (long long)llrint(red[0] * 4294967296.0);
  }
}

__global__ void sgd_momentum_kernel(float* __restrict__ w, float* __restrict__ a, const float* __restrict__ g,
                                    int64_t n, float lr, float mu, float gscale) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sgd_momentum_elem(w, a, g, i, lr, mu, gscale);
}

__global__ void bias_add_kernel(float* __restrict__ y, const float* __restrict__ b, int64_t n, int C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = y[i] + b[i % C];
}

// db[c] = (float)(sum_shards S1[c]) * 2^-eg : the bias gradient of Conv2d_q / Dense_q
// (dynamic_fixed_point.py:209,459) from the grad quantiser's exact per-channel code sums.
__global__ void bias_grad_kernel(const int64_t* __restrict__ chsum, int C, lbt_qdesc qg, float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  long long s = 0;
  for (int k = 0; k < LBT_NSHARD; ++k) s += chsum[(int64_t)k * 2 * C + c];
  db[c] = (float)((double)s * ldexp(1.0, -frac_exp(qg)));
}

unsigned blocks4(int64_t n) { return (unsigned)(((n + 3) / 4 + 255) / 256); }

// bitwise comparison of div_by(x, recip(y)) with the compiler's correctly rounded x / y
__global__ void selftest_div_kernel(const float* __restrict__ x, const float* __restrict__ y, int64_t n,
                                    int32_t* __restrict__ bad, float* __restrict__ qa, float* __restrict__ qb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = x[i] / y[i];
  const float b = div_by(x[i], recip(y[i]));
  if (__float_as_uint(a) != __float_as_uint(b)) atomicAdd(bad, 1);
  if (qa) { qa[i] = a; qb[i] = b; }
}

}  // namespace

extern "C" int lbt_relu_fwd(const float* x, float* y, int64_t n, void* stream) {
  if (n <= 0) return LBT_OK;
  hipLaunchKernelGGL(relu_fwd_kernel, dim3(blocks4(n)), dim3(256), 0, (hipStream_t)stream, x, y, n);
  return (int)hipGetLastError();
}
extern "C" int lbt_relu_bwd(const float* g, const float* x, float* dx, int64_t n, void* stream) {
  if (n <= 0) return LBT_OK;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(blocks4(n)), dim3(256), 0, (hipStream_t)stream, g, x, dx, n);
  return (int)hipGetLastError();
}
extern "C" int lbt_add(const float* a, const float* b, float* y, int64_t n, void* stream) {
  if (n <= 0) return LBT_OK;
  hipLaunchKernelGGL(add_kernel, dim3(blocks4(n)), dim3(256), 0, (hipStream_t)stream, a, b, y, n);
  return (int)hipGetLastError();
}
extern "C" int lbt_avgpool_fwd(const float* x, float* y, int32_t N, int32_t HW, int32_t C, void* stream) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((N * C + 63) / 64), dim3(64), 0, (hipStream_t)stream, x, y, N, HW, C);
  return (int)hipGetLastError();
}
extern "C" int lbt_avgpool_bwd(const float* g, float* dx, int32_t N, int32_t HW, int32_t C, void* stream) {
  const int64_t n = (int64_t)N * HW * C;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, g, dx, N,
                     HW, C);
  return (int)hipGetLastError();
}
extern "C" int lbt_softmax_xent(const float* z, const int32_t* labels, int32_t N, int32_t K, float* loss, float* dz,
                                void* stream) {
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, z, labels, N, K, loss, dz, N,
                     nullptr);
  return (int)hipGetLastError();
}
extern "C" int lbt_softmax_xent_n(const float* z, const int32_t* labels, int32_t N, int32_t K, int32_t norm, float* loss,
                                  float* dz, int64_t* loss_fx, void* stream) {
  if (N <= 0 || K <= 0 || norm < N) return LBT_EINVAL;
  if (K > 64) return lbt_softmax_xent_wide_n(z, labels, N, K, norm, loss, dz, loss_fx, stream);
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, z, labels, N, K, loss, dz, norm,
                     (long long*)loss_fx);
  return (int)hipGetLastError();
}
extern "C" int lbt_sgd_momentum(float* w, float* a, const float* g, int64_t n, float lr, float mu, float gscale,
                                void* stream) {
  if (n <= 0) return LBT_OK;
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w, a,
                     g, n, lr, mu, gscale);
  return (int)hipGetLastError();
}
extern "C" int lbt_bias_add(float* y, const float* b, int64_t n, int32_t C, void* stream) {
  if (n <= 0) return LBT_OK;
  hipLaunchKernelGGL(bias_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, y, b, n, C);
  return (int)hipGetLastError();
}
extern "C" int lbt_bias_grad(const int64_t* chsum, int32_t C, lbt_qdesc qg, float* db, void* stream) {
  hipLaunchKernelGGL(bias_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, chsum, C, qg, db);
  return (int)hipGetLastError();
}

extern "C" int lbt_selftest_div(const float* x, const float* y, int64_t n, int32_t* bad, float* qa, float* qb,
                                void* stream) {
  if (n <= 0) return LBT_OK;
  hipLaunchKernelGGL(selftest_div_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, y,
                     n, bad, qa, qb);
  return (int)hipGetLastError();
}

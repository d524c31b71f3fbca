// bn_moments.h -- Normalization_q's batch moments from the exact integer channel sums
// (dynamic_fixed_point.py:584-612), shared by the element-chain kernels (bn.hip) and the fused
// head (head.hip), which evaluates the last block's end chain itself.
#pragma once
#include "dfxp_device.h"

namespace lbt {

// Sum a sharded [LBT_NSHARD][stride] int64 buffer's first n entries into LDS tmp[n].
LBT_DEV void sum_shards(const int64_t* src, int n, int stride, long long* tmp) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    long long v[LBT_NSHARD];  // every shard's load in flight at once
#pragma unroll
    for (int k = 0; k < LBT_NSHARD; ++k) v[k] = src[(int64_t)k * stride + i];
    long long s = 0;
#pragma unroll
    for (int k = 0; k < LBT_NSHARD; ++k) s += v[k];
    tmp[i] = s;
  }
}

// Normalization_q moments from the exact integer sums -> mu / sigma in LDS (and ms / running
// stats from the first workgroup).
LBT_DEV void bn_moments(const lbt_bn_norm& b, int C, float* mu, float* sg, long long* tmp) {
  const bool writer = blockIdx.x == 0 && blockIdx.y == 0;
  if (b.frozen) {  // testing mode: the running averages, no update
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float m = b.run_mean[c], sigma = sqrtf(b.run_var[c] + b.eps);
      mu[c] = m;
      sg[c] = sigma;
      if (writer && b.ms) { b.ms[c] = m; b.ms[C + c] = sigma; }
    }
    return;
  }
  sum_shards(b.chsum, 2 * C, 2 * C, tmp);
  __syncthreads();
  const double s = ldexp(1.0, -frac_exp(b.qn));
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const double mean_d = (double)tmp[c] * s / (double)b.n;
    const double var_d = (double)tmp[C + c] * (s * s) / (double)b.n - mean_d * mean_d;
    const float m = (float)mean_d, v = (float)var_d;
    const float sigma = sqrtf(v + b.eps);
    mu[c] = m;
    sg[c] = sigma;
    if (writer) {
      if (b.ms) { b.ms[c] = m; b.ms[C + c] = sigma; }
      if (b.run_mean) {
        b.run_mean[c] = b.momentum * b.run_mean[c] + b.one_minus_momentum * m;
        b.run_var[c] = b.momentum * b.run_var[c] + b.one_minus_momentum * v;
      }
    }
  }
}

}  // namespace lbt

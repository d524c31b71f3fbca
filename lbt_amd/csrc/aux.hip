// aux.hip -- the components either side of the hot path, as kernels:
//
//   lbt_grad_buffer_bwd     GradientBuffer_q.backward (dynamic_fixed_point.py:473-509): error-feedback
//                           gradient quantisation, total = pad(g) + buffer; gq = Q(total); buffer = total - gq
//   lbt_pre_dense           Dense_q._pre_dense_func (:397-439, dormant in the reference's trainer): the
//                           per-element small-gradient accumulator state machine
//   lbt_augment_flip_crop   trainer.py:24-28 preprocess_image: random left-right flip, zero pad, random crop
//
// All element-parallel (each element's state is its own), one thread per element / output.
#include "dfxp_device.h"

using namespace lbt;

namespace {

constexpr int kT = 256;

// ---------------------------------------------------------------- GradientBuffer_q.backward
__global__ __launch_bounds__(kT) void grad_buffer_bwd_kernel(const float* __restrict__ g, int64_t n_g,
                                                             float* __restrict__ buffer, int64_t n_buf, int64_t inner,
                                                             lbt_qdesc q, float* __restrict__ gq) {
  __shared__ int sh_cnt[2 * kT / 64];
  const QState s = qstate(q);
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  int ov1 = 0, ov2 = 0;
  if (i < n_buf) {
    // tf.pad(grad) + buffer: rows past the incoming batch are zero-padded (:497-500)
    const float total = (i < n_g ? g[i] : 0.f) + buffer[i];
    float v;
    if (q.bits >= 32) {
      v = total;  // weight_quantization's bits == 32 bypass (:21-23)
    } else {
      const float u = (s.active && q.stochastic) ? qnoise1(q, s.step, (uint64_t)(i % inner)) : 0.f;
      const int c = quant1(s, q.stochastic, total, u, ov1, ov2);
      v = (float)c * s.inv_m;
    }
    buffer[i] = total - v;  // update_buffer_op (:503)
    if (i < n_g) gq[i] = v; // gradq[:tf.shape(grad)[0]] (:506)
  }
  block_flush_counts(q, ov1, ov2, sh_cnt);
}

// ---------------------------------------------------------------- Dense_q._pre_dense_func
// eps = 1 / 2^(bits - grad_range) (:444); state arrays [in_units][units] indexed [i][j] for the
// grad's (i, j) (the reference loops over grad's shape, :408-410). eps is a power of two, so
// numpy's float floor division a // eps is exactly floorf(a / eps).
__global__ __launch_bounds__(kT) void pre_dense_kernel(float* __restrict__ grad, int rows, int cols, int state_cols,
                                                       lbt_qdesc qg, float* __restrict__ accu,
                                                       int32_t* __restrict__ init_flag, int32_t* __restrict__ rem_flag) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (e >= (int64_t)rows * cols) return;
  const int i = (int)(e / cols), j = (int)(e - (int64_t)i * cols);
  const int64_t sidx = (int64_t)i * state_cols + j;
  const float eps = ldexpf(1.0f, -(frac_exp(qg) + 1));
  float g = grad[e];
  float a = accu[sidx];
  int init = init_flag[sidx], rem = rem_flag[sidx];
  if (init == 1) {
    if (eps > fabsf(g)) {
      init = 0;
      a = rem == 1 ? a + g : g;
    }
  } else {
    a = a + g;
    if (fabsf(a) > eps) {
      init = 1;
      g = a;
      if (a > 0.f) {
        const float k = floorf(a / eps);
        a = a - k * eps;
      } else {
        const float k = floorf((-a) / eps);
        a = a + k * eps;
      }
      rem = 1;
    }
  }
  grad[e] = g;
  accu[sidx] = a;
  init_flag[sidx] = init;
  rem_flag[sidx] = rem;
}

// ---------------------------------------------------------------- preprocess_image
// Per sample n, one Philox4x32-10 draw r = philox(n, kAugStream, counter_lo, counter_hi; seed):
// flip = r.x & 1, oy = r.y % (2 pad + 1), ox = r.z % (2 pad + 1). Then
// y[n,i,j,c] = flipped[n, i + oy - pad, j + ox - pad, c] (0 outside), flipped[.,.,j] = x[.,.,W-1-j]:
// tf.image.random_flip_left_right -> pad_to_bounding_box(pad, pad, H+2pad, W+2pad) -> random_crop(H, W).
constexpr uint32_t kAugStream = 0x41554721u;  // "AUG!"

__global__ __launch_bounds__(kT) void augment_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int H,
                                                     int W, int C, int pad, uint64_t seed, uint64_t counter) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int64_t total = (int64_t)N * H * W * C;
  if (e >= total) return;
  const int c = (int)(e % C);
  int64_t m = e / C;
  const int j = (int)(m % W);
  m /= W;
  const int i = (int)(m % H);
  const int n = (int)(m / H);
  const U4 r = philox((uint32_t)n, kAugStream, (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)seed,
                      (uint32_t)(seed >> 32));
  const uint32_t span = 2u * (uint32_t)pad + 1u;
  const int flip = (int)(r.x & 1u), oy = (int)(r.y % span), ox = (int)(r.z % span);
  const int si = i + oy - pad, sj0 = j + ox - pad;
  float v = 0.f;
  if (si >= 0 && si < H && sj0 >= 0 && sj0 < W) {
    const int sj = flip ? W - 1 - sj0 : sj0;
    v = x[(((int64_t)n * H + si) * W + sj) * C + c];
  }
  y[e] = v;
}

// ---------------------------------------------------------------- 4-bit weight images
// dst[i] = (src[2i] & 15) | (src[2i+1] << 4): two signed 4-bit codes per byte, element order kept.
__global__ __launch_bounds__(kT) void pack_int4_kernel(const int8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       int64_t nbytes) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= nbytes) return;
  dst[i] = (uint8_t)((src[2 * i] & 15) | ((src[2 * i + 1] & 15) << 4));
}

}  // namespace

extern "C" int lbt_pack_int4(const int8_t* src, uint8_t* dst, int64_t n, void* stream) {
  if (n <= 0 || n % 2) return LBT_EINVAL;
  const int64_t nb = n / 2;
  hipLaunchKernelGGL(pack_int4_kernel, dim3((unsigned)((nb + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream, src, dst,
                     nb);
  return (int)hipGetLastError();
}

extern "C" int lbt_grad_buffer_bwd(const float* g, int64_t n_g, float* buffer, int64_t n_buf, int64_t inner,
                                   lbt_qdesc q, float* gq, void* stream) {
  if (n_buf <= 0 || n_g < 0 || n_g > n_buf || inner <= 0) return LBT_EINVAL;
  if (q.bits < 32 && (q.bits < 2 || q.bits > 16)) return LBT_EINVAL;
  hipLaunchKernelGGL(grad_buffer_bwd_kernel, dim3((unsigned)((n_buf + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream,
                     g, n_g, buffer, n_buf, inner, q, gq);
  return (int)hipGetLastError();
}

extern "C" int lbt_pre_dense(float* grad, int32_t rows, int32_t cols, int32_t state_rows, int32_t state_cols,
                             lbt_qdesc qg, float* accu, int32_t* init_flag, int32_t* rem_flag, void* stream) {
  // the reference indexes the [in_units][units] state with the grad's (i, j): out of range is an
  // IndexError there, LBT_EINVAL here
  if (rows <= 0 || cols <= 0 || rows > state_rows || cols > state_cols) return LBT_EINVAL;
  const int64_t n = (int64_t)rows * cols;
  hipLaunchKernelGGL(pre_dense_kernel, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream, grad, rows,
                     cols, state_cols, qg, accu, init_flag, rem_flag);
  return (int)hipGetLastError();
}

extern "C" int lbt_augment_flip_crop(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C, int32_t pad,
                                     uint64_t seed, uint64_t counter, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || pad < 0 || x == y) return LBT_EINVAL;
  const int64_t n = (int64_t)N * H * W * C;
  hipLaunchKernelGGL(augment_kernel, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, (hipStream_t)stream, x, y, N, H,
                     W, C, pad, seed, counter);
  return (int)hipGetLastError();
}

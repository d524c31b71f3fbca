// dense.hip -- Dense_q (dynamic_fixed_point.py:319-395, 441-466) for wide classifier heads
// (ResNet-50's 2048 -> 1000 fc) on int8 MFMA, plus the wide softmax-CE.
//
//   fwd   : y[n][u]  = sum_k x[n][k] * W[k][u]       (x int8 codes, W int8 codes)
//   dgrad : dx[n][k] = sum_u g[n][u] * W[k][u]       (g int8, or int16 for 9..16-bit gradients)
//   wgrad : dW[k][u] = sum_n x[n][k] * g[n][u] * 2^-e + fl(2 wd) * W[k][u]
//
// The GEMMs: rows = batch (few), k = the contraction, columns = the other side. B comes from
// packed images built by lbt_dense_pack from the quantiser's HWIO codes ([col][k], k contiguous,
// zero-padded to a multiple of 64). A workgroup owns one 16 x 16 output tile; its 4 waves split
// k, and their exact int32 partials meet in LDS. int16 gradient codes are split
// g = 256*hi + lo' + 128 (hi, lo' int8) into two int8 MFMA passes plus an all-ones pass for
// sum_k W, recombined exactly in int64 (the identity igemm.hip uses). wgrad's contraction is the
// batch (N <= a few hundred), so it runs on the VALU with int64 sums and finishes dW in place.
// Every result equals the generic kernels' exact integer arithmetic, bit for bit.
//
// MFMA 16x16x64_i8 map (probed): lane l holds A[row l&15][k = 16*(l>>4) .. +15],
// B[k = 16*(l>>4) .. +15][col l&15]; C/D: col = l&15, row = 4*(l>>4) + reg.
#include "dfxp_device.h"
#include "lds_tr.h"

using namespace lbt;

namespace {

constexpr int kThreads = 256;

// [W: IN x OUT] -> wf [OUT][KF] (k = in, zero beyond IN), wd [IN][UP] (k = out, zero beyond OUT)
__global__ void dense_pack_kernel(const int8_t* __restrict__ w, int IN, int OUT, int8_t* __restrict__ wf, int KF,
                                  int8_t* __restrict__ wd, int UP) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nf = (int64_t)OUT * KF, nd = (int64_t)IN * UP;
  if (i < nf) {
    const int u = (int)(i / KF), k = (int)(i - (int64_t)u * KF);
    wf[i] = k < IN ? w[(int64_t)k * OUT + u] : (int8_t)0;
  } else if (i < nf + nd) {
    const int64_t j = i - nf;
    const int k = (int)(j / UP), u = (int)(j - (int64_t)k * UP);
    wd[j] = u < OUT ? w[(int64_t)k * OUT + u] : (int8_t)0;
  }
}

// 16 codes of row `row` from k0 on (two 8-element halves, each either fully inside [0, kvalid) or
// zero; kvalid % 8 == 0), as int8 (A8) or the int16 codes' (hi, lo') split (A16).
template <bool A16>
LBT_DEV void load_frag(const void* a, int lda, int nrows, int kvalid, int row, int k0, v4i& f0, v4i& f1) {
  if constexpr (A16) {
    const int16_t* p = reinterpret_cast<const int16_t*>(a) + (int64_t)(row < nrows ? row : 0) * lda;
    v4i h[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = k0 + 8 * s;
      const bool ok = row < nrows && k < kvalid;
      const v4i v = *reinterpret_cast<const v4i*>(p + (ok ? k : 0));
      h[s] = ok ? v : v4i{0, 0, 0, 0};
    }
    // 16 int16 -> hi bytes (f0) and lo' = (g & 255) - 128 bytes (f1)
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t w0 = (uint32_t)h[q >> 1][(q & 1) * 2], w1 = (uint32_t)h[q >> 1][(q & 1) * 2 + 1];
      // w0 = (g1 << 16) | g0, w1 = (g3 << 16) | g2 (little endian)
      hi[q] = __builtin_amdgcn_perm(w1, w0, 0x07050301u);
      lo[q] = __builtin_amdgcn_perm(w1, w0, 0x06040200u) ^ 0x80808080u;
    }
    f0 = v4i{(int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    f1 = v4i{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3]};
  } else {
    const int8_t* p = reinterpret_cast<const int8_t*>(a) + (int64_t)(row < nrows ? row : 0) * lda;
    v2i h[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = k0 + 8 * s;
      const bool ok = row < nrows && k < kvalid;
      const v2i v = *reinterpret_cast<const v2i*>(p + (ok ? k : 0));
      h[s] = ok ? v : v2i{0, 0};
    }
    f0 = v4i{h[0].x, h[0].y, h[1].x, h[1].y};
    f1 = f0;
  }
}

// out[row][col] = (sum_k a[row][k] * b[col][k]) * 2^-(ea+eb); grid (ceil(ncols/16), ceil(nrows/16))
template <bool A16>
__global__ __launch_bounds__(kThreads) void dense_gemm_kernel(const void* __restrict__ a, int lda, int kvalid,
                                                              const int8_t* __restrict__ b, int kb, int nrows,
                                                              int ncols, lbt_qdesc qa, lbt_qdesc qb,
                                                              float* __restrict__ out) {
  constexpr int NC = A16 ? 3 : 1;  // accumulators: (hi, lo', ones) or one
  __shared__ int red[4][NC][16][17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int row = blockIdx.y * 16 + r, col = blockIdx.x * 16 + r;
  const int8_t* bp = b + (int64_t)(col < ncols ? col : 0) * kb;
  const bool col_ok = col < ncols;
  v4i acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = v4i{0, 0, 0, 0};
  const int nks = kb / 64;
  for (int ks = wave; ks < nks; ks += 4) {
    const int k0 = ks * 64 + 16 * kg;
    v4i f0, f1;
    load_frag<A16>(a, lda, nrows, kvalid, row, k0, f0, f1);
    v4i bf = *reinterpret_cast<const v4i*>(bp + k0);
    if (!col_ok) bf = v4i{0, 0, 0, 0};
    acc[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f0, bf, acc[0], 0, 0, 0);
    if constexpr (A16) {
      acc[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f1, bf, acc[1], 0, 0, 0);
      const v4i ones = v4i{0x01010101, 0x01010101, 0x01010101, 0x01010101};
      acc[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, bf, acc[2], 0, 0, 0);
    }
  }
  // D: col = r, row = 4*kg + i
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][c][4 * kg + i][r] = acc[c][i];
  __syncthreads();
  if (threadIdx.x >= 256) return;
  const int orow = threadIdx.x >> 4, ocol = threadIdx.x & 15;
  long long s[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    s[c] = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) s[c] += red[w][c][orow][ocol];
  }
  long long total = s[0];
  if constexpr (A16) total = 256ll * s[0] + s[1] + 128ll * s[2];
  const int gr = blockIdx.y * 16 + orow, gc = blockIdx.x * 16 + ocol;
  if (gr < nrows && gc < ncols) {
    const float scale = ldexpf(1.0f, -(frac_exp(qa) + frac_exp(qb)));
    out[(int64_t)gr * ncols + gc] = (float)total * scale;
  }
}

// dW[k][u..u+3] = (float)(sum_n x[n][k] * g[n][u]) * 2^-(ex+eg) + wd2 * W[k][u]; thread = (k, 4 u)
template <typename TG>
__global__ __launch_bounds__(kThreads) void dense_wgrad_kernel(const int8_t* __restrict__ x, const TG* __restrict__ g,
                                                               int N, int IN, int OUT, lbt_qdesc qx, lbt_qdesc qg,
                                                               const float* __restrict__ w, float wd2,
                                                               float* __restrict__ dw, long long* __restrict__ num) {
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int uq = OUT / 4;
  if (t >= (int64_t)IN * uq) return;
  const int k = (int)(t / uq), u = (int)(t - (int64_t)k * uq) * 4;
  long long s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int n = 0; n < N; ++n) {
    const int xv = x[(int64_t)n * IN + k];
    const TG* gp = g + (int64_t)n * OUT + u;
    s0 += (long long)(xv * (int)gp[0]);
    s1 += (long long)(xv * (int)gp[1]);
    s2 += (long long)(xv * (int)gp[2]);
    s3 += (long long)(xv * (int)gp[3]);
  }
  const float scale = ldexpf(1.0f, -(frac_exp(qx) + frac_exp(qg)));
  const int64_t o = (int64_t)k * OUT + u;
  const long long sv[4] = {s0, s1, s2, s3};
  if (num) {  // the exact exchange: the numerators, dequantised after the all-reduce (lbt_step_finish)
#pragma unroll
    for (int j = 0; j < 4; ++j) num[o + j] = sv[j];
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float av = (float)sv[j] * scale;
    const float bv = wd2 * w[o + j];
    dw[o + j] = av + bv;
  }
}

constexpr int kSxReg = 16;  // logits per lane held in registers (K <= 1024)
// mean sparse softmax-CE over [N][K] logits for wide K (models.py:30-32): one wave per row
// (16 waves), the row's max / sum by wave reductions, per-row losses in double combined in a
// fixed order. Same per-element formulas as softmax_xent_kernel (misc.hip).
__global__ __launch_bounds__(1024) void softmax_xent_wide_kernel(const float* __restrict__ z,
                                                                 const int32_t* __restrict__ labels, int N, int K,
                                                                 float* __restrict__ loss, float* __restrict__ dz,
                                                                 int norm, long long* loss_fx) {
  __shared__ double part[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double acc = 0.0;
  // the row in registers (ImageNet's 1000 classes: 16 per lane) when K <= 1024, the wave's next row loaded
  // while this one is reduced (the looped form below made three dependent passes over global memory per row:
  // 205 us per ResNet-50 step at B = 256); each lane's max / sum run over its k in the same ascending order
  // and through the same shuffle tree, so every value is the loops' bit for bit
  const bool regs = K <= 64 * kSxReg;
  float v[kSxReg];
  auto load_row = [&](int rr, float (&dst)[kSxReg]) {
    const float* zr = z + (int64_t)rr * K;
#pragma unroll
    for (int i = 0; i < kSxReg; ++i) {
      const int k = lane + 64 * i;
      dst[i] = k < K ? zr[k] : -INFINITY;
    }
  };
  if (regs && wave < N) load_row(wave, v);
  for (int rr = wave; rr < N; rr += 16) {
    const float* zr = z + (int64_t)rr * K;
    if (regs) {
      float vn[kSxReg];
      if (rr + 16 < N) load_row(rr + 16, vn);
      float m = -INFINITY;
#pragma unroll
      for (int i = 0; i < kSxReg; ++i) m = fmaxf(m, v[i]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < kSxReg; ++i)
        if (lane + 64 * i < K) s = s + expf(v[i] - m);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s = s + __shfl_xor(s, o, 64);
      const int y = labels[rr];
#pragma unroll
      for (int i = 0; i < kSxReg; ++i) {
        const int k = lane + 64 * i;
        if (k < K) {
          const float p = expf(v[i] - m) / s;
          dz[(int64_t)rr * K + k] = (p - (k == y ? 1.f : 0.f)) / (float)norm;
        }
      }
      if (lane == 0) {
        const float lse = logf(s) + m;
        acc += (double)(lse - zr[y]);
      }
#pragma unroll
      for (int i = 0; i < kSxReg; ++i) v[i] = vn[i];
      continue;
    }
    float m = -INFINITY;
    for (int k = lane; k < K; k += 64) m = fmaxf(m, zr[k]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s = s + expf(zr[k] - m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s = s + __shfl_xor(s, o, 64);
    const int y = labels[rr];
    for (int k = lane; k < K; k += 64) {
      const float p = expf(zr[k] - m) / s;
      dz[(int64_t)rr * K + k] = (p - (k == y ? 1.f : 0.f)) / (float)norm;
    }
    if (lane == 0) {
      const float lse = logf(s) + m;
      acc += (double)(lse - zr[y]);
    }
  }
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += part[w];
    loss[0] = (float)(t / (double)norm);
    if (loss_fx) *loss_fx = (long long)llrint(t * 4294967296.0);
  }
}

}  // namespace

extern "C" int lbt_dense_pack(const int8_t* w_hwio, int32_t in_units, int32_t units, int8_t* wf, int32_t kf,
                              int8_t* wd, int32_t up, void* stream) {
  if (in_units <= 0 || units <= 0 || kf < in_units || up < units || kf % 64 || up % 64) return LBT_EINVAL;
  const int64_t n = (int64_t)units * kf + (int64_t)in_units * up;
  hipLaunchKernelGGL(dense_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w_hwio,
                     in_units, units, wf, kf, wd, up);
  return (int)hipGetLastError();
}

// out[rows][cols] = a[rows][kvalid] . b[cols][kb]^T, scaled; a int8 (a16 = 0) or int16 codes
extern "C" int lbt_dense_gemm(const void* a, int32_t a16, int32_t lda, int32_t kvalid, const int8_t* b, int32_t kb,
                              int32_t rows, int32_t cols, lbt_qdesc qa, lbt_qdesc qb, float* out, void* stream) {
  if (rows <= 0 || cols <= 0) return LBT_OK;
  if (kvalid <= 0 || kvalid % 8 || kb % 64 || kb < kvalid || lda < kvalid || lda % 8) return LBT_EINVAL;
  if ((int64_t)kb * 128 * 128 >= ((int64_t)1 << 31)) return LBT_EINVAL;  // int32 partials per accumulator
  dim3 grid((unsigned)((cols + 15) / 16), (unsigned)((rows + 15) / 16));
  hipStream_t st = (hipStream_t)stream;
  if (a16)
    hipLaunchKernelGGL(dense_gemm_kernel<true>, grid, dim3(kThreads), 0, st, a, lda, kvalid, b, kb, rows, cols, qa, qb, out);
  else
    hipLaunchKernelGGL(dense_gemm_kernel<false>, grid, dim3(kThreads), 0, st, a, lda, kvalid, b, kb, rows, cols, qa, qb, out);
  return (int)hipGetLastError();
}

static int dense_wgrad_launch(const int8_t* xq, const void* g, int32_t g16, int32_t N, int32_t in_units,
                              int32_t units, lbt_qdesc qx, lbt_qdesc qg, const float* w, float wd2, float* dw,
                              int64_t* num, void* stream) {
  if (N <= 0 || in_units <= 0 || units <= 0 || units % 4) return LBT_EINVAL;
  const int64_t threads = (int64_t)in_units * (units / 4);
  dim3 grid((unsigned)((threads + kThreads - 1) / kThreads));
  hipStream_t st = (hipStream_t)stream;
  if (g16)
    hipLaunchKernelGGL(dense_wgrad_kernel<int16_t>, grid, dim3(kThreads), 0, st, xq, (const int16_t*)g, N, in_units,
                       units, qx, qg, w, wd2, dw, (long long*)num);
  else
    hipLaunchKernelGGL(dense_wgrad_kernel<int8_t>, grid, dim3(kThreads), 0, st, xq, (const int8_t*)g, N, in_units,
                       units, qx, qg, w, wd2, dw, (long long*)num);
  return (int)hipGetLastError();
}

extern "C" int lbt_dense_wgrad(const int8_t* xq, const void* g, int32_t g16, int32_t N, int32_t in_units,
                               int32_t units, lbt_qdesc qx, lbt_qdesc qg, const float* w, float wd2, float* dw,
                               void* stream) {
  return dense_wgrad_launch(xq, g, g16, N, in_units, units, qx, qg, w, wd2, dw, nullptr, stream);
}
extern "C" int lbt_dense_wgrad_x(const int8_t* xq, const void* g, int32_t g16, int32_t N, int32_t in_units,
                                 int32_t units, int64_t* num, void* stream) {
  if (!num) return LBT_EINVAL;
  return dense_wgrad_launch(xq, g, g16, N, in_units, units, lbt_qdesc{}, lbt_qdesc{}, nullptr, 0.f, nullptr, num,
                            stream);
}

extern "C" int lbt_softmax_xent_wide_n(const float* z, const int32_t* labels, int32_t N, int32_t K, int32_t norm,
                                       float* loss, float* dz, int64_t* loss_fx, void* stream) {
  if (N <= 0 || K <= 0 || norm < N) return LBT_EINVAL;
  hipLaunchKernelGGL(softmax_xent_wide_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, z, labels, N, K, loss, dz,
                     norm, (long long*)loss_fx);
  return (int)hipGetLastError();
}

extern "C" int lbt_softmax_xent_wide(const float* z, const int32_t* labels, int32_t N, int32_t K, float* loss,
                                     float* dz, void* stream) {
  if (N <= 0 || K <= 0) return LBT_EINVAL;
  hipLaunchKernelGGL(softmax_xent_wide_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, z, labels, N, K, loss, dz,
                     N, nullptr);
  return (int)hipGetLastError();
}

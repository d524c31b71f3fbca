// quantize.hip -- DFXP quantiser, range controller and weight packing for gfx950.
//
//  lbt_dfxp_quantize        weight_quantization + overflow statistics (dynamic_fixed_point.py:4-67)
//  lbt_dfxp_range_update    update_range for every quantiser slot (dynamic_fixed_point.py:70-94)
//  lbt_dfxp_quantize_weight weight quantiser fused with the GEMM operand packing
//
// HBM-bound: the activation/gradient quantiser reads 4 B and writes 1 B per element. Each
// thread owns 4 consecutive noise indices (one Philox call, one float4 load per row) and
// walks `rpt` rows of the batch, so the noise -- shared across dim 0 by the reference's
// tf.random_uniform(X.shape[1:]) -- is generated once per thread, not once per element.
#include "dfxp_device.h"

using namespace lbt;

namespace {

constexpr int kThreads = 256;

// rows x inner, inner % 4 == 0: vectorised path.
__global__ __launch_bounds__(kThreads) void quantize_rows_kernel(
    const float* __restrict__ x, void* __restrict__ out, int out_kind, int64_t rows, int64_t inner,
    int rpt, lbt_qdesc q, int64_t* __restrict__ chsum, int C) {
  extern __shared__ long long sh_sum[];  // [2*C] when chsum
  __shared__ int sh_cnt[2 * kThreads / 64];
  const QState s = qstate(q);
  const int64_t groups = inner >> 2;
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * rpt;
  if (chsum) {
    for (int i = threadIdx.x; i < 2 * C; i += kThreads) sh_sum[i] = 0;
    __syncthreads();
  }
  int ov1 = 0, ov2 = 0;
  int s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (g < groups) {
    Noise4 n = {{0.f, 0.f, 0.f, 0.f}};
    if (q.stochastic) n = qnoise4(q, s.step, g);
    const int64_t rend = r0 + rpt < rows ? r0 + rpt : rows;
#pragma unroll 4
    for (int64_t r = r0; r < rend; ++r) {
      const int64_t base = r * inner + (g << 2);
      const float4 v = *reinterpret_cast<const float4*>(x + base);
      int c[4];
      c[0] = quant1(s, q.stochastic, v.x, n.u[0], ov1, ov2);
      c[1] = quant1(s, q.stochastic, v.y, n.u[1], ov1, ov2);
      c[2] = quant1(s, q.stochastic, v.z, n.u[2], ov1, ov2);
      c[3] = quant1(s, q.stochastic, v.w, n.u[3], ov1, ov2);
      if (out_kind == LBT_OUT_I8 || out_kind == LBT_OUT_U8OFF) {
        const int off = out_kind == LBT_OUT_U8OFF ? 128 : 0;
        char4 o;
        o.x = (int8_t)((out_kind == LBT_OUT_U8OFF && c[0] < 0 ? 0 : c[0]) - off);
        o.y = (int8_t)((out_kind == LBT_OUT_U8OFF && c[1] < 0 ? 0 : c[1]) - off);
        o.z = (int8_t)((out_kind == LBT_OUT_U8OFF && c[2] < 0 ? 0 : c[2]) - off);
        o.w = (int8_t)((out_kind == LBT_OUT_U8OFF && c[3] < 0 ? 0 : c[3]) - off);
        *reinterpret_cast<char4*>((int8_t*)out + base) = o;
      } else if (out_kind == LBT_OUT_I16) {
        short4 o;
        o.x = (short)c[0]; o.y = (short)c[1]; o.z = (short)c[2]; o.w = (short)c[3];
        *reinterpret_cast<short4*>((int16_t*)out + base) = o;
      } else {
        float4 o;
        o.x = (float)c[0] * s.inv_m; o.y = (float)c[1] * s.inv_m;
        o.z = (float)c[2] * s.inv_m; o.w = (float)c[3] * s.inv_m;
        *reinterpret_cast<float4*>((float*)out + base) = o;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) { s1[k] += c[k]; s2[k] += c[k] * c[k]; }
    }
  }
  if (chsum) {
    const int per = chan_period(C);
    const int ch = (int)((g << 2) % C);
    if (chan_scatter_ok(per)) {  // uniform: row lane >> 4 ends with channel ch + (lane >> 4)
      const int cr = ch + (int)((threadIdx.x & 63) >> 4);
      const int v1 = chan_scatter4(s1, per), v2 = chan_scatter4(s2, per);
      if (chan_scatter_owner(per)) {
        if (v1) atomicAdd((unsigned long long*)&sh_sum[cr], (unsigned long long)(long long)v1);
        if (v2) atomicAdd((unsigned long long*)&sh_sum[C + cr], (unsigned long long)(long long)v2);
      }
    } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) { s1[k] = wave_chan_reduce(s1[k], per); s2[k] = wave_chan_reduce(s2[k], per); }
    if (chan_owner(per)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (s1[k]) atomicAdd((unsigned long long*)&sh_sum[ch + k], (unsigned long long)(long long)s1[k]);
        if (s2[k]) atomicAdd((unsigned long long*)&sh_sum[C + ch + k], (unsigned long long)(long long)s2[k]);
      }
    }
    }
  }
  if (q.counts) counts_stage(0, 1, ov1, ov2, sh_cnt);
  if (!(chsum || q.counts)) return;
  __syncthreads();  // one barrier publishes counters and channel sums
  counts_publish(0, 1, q, sh_cnt);
  if (chsum) block_flush_sums(sh_sum, 2 * C, chsum, 2 * C);
}

// Any shape: one element per thread, per-element Philox (weights, gamma/beta, odd shapes).
__global__ __launch_bounds__(kThreads) void quantize_generic_kernel(
    const float* __restrict__ x, void* __restrict__ out, int out_kind, int64_t n, int64_t inner,
    lbt_qdesc q, int64_t* __restrict__ chsum, int C) {
  __shared__ int sh_cnt[2 * kThreads / 64];
  const QState s = qstate(q);
  int64_t* cs = chsum ? chsum + (int64_t)shard_id() * 2 * C : nullptr;
  int ov1 = 0, ov2 = 0;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const float u = q.stochastic ? qnoise1(q, s.step, i % inner) : 0.f;
    const int c = quant1(s, q.stochastic, x[i], u, ov1, ov2);
    store_code(out, out_kind, i, c, s.inv_m);
    if (cs) {
      const int ch = (int)(i % C);
      atomicAdd((unsigned long long*)&cs[ch], (unsigned long long)(long long)c);
      atomicAdd((unsigned long long*)&cs[C + ch], (unsigned long long)(long long)(c * c));
    }
  }
  block_flush_counts(q, ov1, ov2, sh_cnt);
}

// grid: one wave per slot (4 slots per 256-thread block)
__global__ void range_update_kernel(int32_t* exps, int32_t* counts, const int32_t* bits,
                                    const float* target, const float* nelem, int nslots,
                                    uint64_t* step) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i < nslots && nelem[i] > 0.f) {  // slots not fed this step keep their exponent
    int c1, c2;
    if (wave_shard_totals(counts, i, c1, c2)) range_apply(i, c1, c2, exps, bits, target, nelem);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) step[0] += 1ull;
}

// lbt_step_update: [sgd_blocks optimiser blocks][range-update blocks (4 slots each)]
__global__ __launch_bounds__(256) void step_update_kernel(float* __restrict__ w, float* __restrict__ a,
                                                          const float* __restrict__ g, int64_t n, float lr, float mu,
                                                          float gscale, int sgd_blocks, int32_t* exps, int32_t* counts,
                                                          const int32_t* bits, const float* target, const float* nelem,
                                                          int nslots, uint64_t* step, int vec) {
  if ((int)blockIdx.x < sgd_blocks) {
    // 4 consecutive parameters per thread (16-byte loads / stores when w, a, g are 16-byte aligned:
    // vec), each through sgd_momentum_elem's arithmetic
    const int64_t i = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
    if (vec && i + 4 <= n) {
      float4 wv = *reinterpret_cast<const float4*>(w + i);
      float4 av = *reinterpret_cast<const float4*>(a + i);
      const float4 gv = *reinterpret_cast<const float4*>(g + i);
      float* wp = &wv.x;
      float* ap = &av.x;
      const float* gp = &gv.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) sgd_momentum_elem(wp, ap, gp, k, lr, mu, gscale);
      *reinterpret_cast<float4*>(a + i) = av;
      *reinterpret_cast<float4*>(w + i) = wv;
    } else {
      for (int64_t k = i; k < i + 4 && k < n; ++k) sgd_momentum_elem(w, a, g, k, lr, mu, gscale);
    }
    return;
  }
  const int rb = (int)blockIdx.x - sgd_blocks;
  const int i = rb * 4 + (threadIdx.x >> 6);
  if (i < nslots && nelem[i] > 0.f) {
    int c1, c2;
    if (wave_shard_totals(counts, i, c1, c2)) range_apply(i, c1, c2, exps, bits, target, nelem);
  }
  if (rb == 0 && threadIdx.x == 0) step[0] += 1ull;
}

__global__ void counts_fold_kernel(int32_t* counts, int nslots, float* folded) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nslots) return;
  int c1, c2;
  if (wave_shard_totals(counts, i, c1, c2)) {
    folded[4 * i + 0] = (float)(c1 >> 12);
    folded[4 * i + 1] = (float)(c1 & 4095);
    folded[4 * i + 2] = (float)(c2 >> 12);
    folded[4 * i + 3] = (float)(c2 & 4095);
  }
}

__global__ void range_update_folded_kernel(int32_t* exps, const float* folded, const int32_t* bits,
                                           const float* target, const float* nelem, int nslots,
                                           uint64_t* step) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nslots && nelem[i] > 0.f) {
    const int c1 = (int)folded[4 * i + 0] * 4096 + (int)folded[4 * i + 1];
    const int c2 = (int)folded[4 * i + 2] * 4096 + (int)folded[4 * i + 3];
    range_apply(i, c1, c2, exps, bits, target, nelem);
  }
  if (i == 0) step[0] += 1ull;
}

// One block per output channel co: quantise W[:, :, :, co], write every packed layout and the
// column sum (no atomics -> no zeroing needed between steps).
__global__ __launch_bounds__(kThreads) void quantize_weight_kernel(
    const float* __restrict__ w, int KH, int KW, int Cin, int Cout, lbt_qdesc q,
    int8_t* __restrict__ w_hwio, int8_t* __restrict__ wf, int ksf, int8_t* __restrict__ wd, int ksd,
    int32_t* __restrict__ colsum) {
  __shared__ int red[kThreads / 64];
  __shared__ int sh_cnt[2 * kThreads / 64];
  const QState s = qstate(q);
  const int co = blockIdx.x;
  const int K = KH * KW * Cin;
  const int64_t inner = (int64_t)KW * Cin * Cout;
  const int cslices_in = (Cin + 15) / 16, cslices_out = (Cout + 15) / 16;
  int ov1 = 0, ov2 = 0, csum = 0;
  for (int k = threadIdx.x; k < K; k += kThreads) {
    const int tap = k / Cin, ci = k % Cin;
    const int64_t idx = (int64_t)k * Cout + co;  // HWIO flat index
    const float u = q.stochastic ? qnoise1(q, s.step, idx % inner) : 0.f;
    const int c = quant1(s, q.stochastic, w[idx], u, ov1, ov2);
    csum += c;
    if (w_hwio) w_hwio[idx] = (int8_t)c;
    if (wf) wf[((int64_t)co * ksf + tap * cslices_in + ci / 16) * 16 + (ci & 15)] = (int8_t)c;
    if (wd) wd[((int64_t)ci * ksd + tap * cslices_out + co / 16) * 16 + (co & 15)] = (int8_t)c;
  }
  block_flush_counts(q, ov1, ov2, sh_cnt);
  if (colsum) {
    csum = wave_sum_i32(csum);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = csum;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int i = 0; i < kThreads / 64; ++i) t += red[i];
      colsum[co] = t;
    }
  }
}

}  // namespace

extern "C" int lbt_dfxp_quantize(const float* x, void* out, int out_kind, int64_t rows, int64_t inner,
                                 lbt_qdesc q, int64_t* chsum, int32_t C, void* stream) {
  if (rows <= 0 || inner <= 0) return LBT_OK;
  // 1..16 bits: integer codes; 17..31 bits: fake-quantised fp32 values only (the codes exceed int16)
  if (q.bits < 1 || q.bits > 31 || (q.bits > 16 && out_kind != LBT_OUT_F32)) return LBT_EINVAL;
  if ((out_kind == LBT_OUT_I8 && q.bits > 8) || (out_kind == LBT_OUT_U8OFF && q.bits > 9)) return LBT_EINVAL;
  if (chsum && (C <= 0 || inner % C)) return LBT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = rows * inner;
  const bool vec = (inner % 4 == 0) && (reinterpret_cast<uintptr_t>(x) % 16 == 0) &&
                   (!chsum || C % 4 == 0) && (inner >= 64);
  if (vec) {
    const int64_t groups = inner / 4;
    const int64_t gblocks = (groups + kThreads - 1) / kThreads;
    // aim for ~512 fat workgroups: Philox and the per-channel reductions amortise over rpt rows
    int64_t rpt = (gblocks * rows) / 512;
    if (rpt < 1) rpt = 1;
    if (rpt > 64) rpt = 64;
    const int64_t yblocks = (rows + rpt - 1) / rpt;
    if (yblocks > 65535) return LBT_EINVAL;
    const size_t shm = chsum ? sizeof(long long) * 2 * C : 0;
    hipLaunchKernelGGL(quantize_rows_kernel, dim3((unsigned)gblocks, (unsigned)yblocks), dim3(kThreads), shm, st,
                       x, out, out_kind, rows, inner, (int)rpt, q, chsum, C);
  } else {
    int64_t blocks = (n + kThreads - 1) / kThreads;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(quantize_generic_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, st, x, out, out_kind, n,
                       inner, q, chsum, C);
  }
  return (int)hipGetLastError();
}

extern "C" int lbt_dfxp_range_update(int32_t* exps, int32_t* counts, const int32_t* bits, const float* target,
                                     const float* nelem, int32_t nslots, uint64_t* step, void* stream) {
  const int blocks = nslots > 0 ? (nslots + 3) / 4 : 1;
  hipLaunchKernelGGL(range_update_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, exps, counts, bits,
                     target, nelem, nslots, step);
  return (int)hipGetLastError();
}

extern "C" int lbt_step_update(float* w, float* a, const float* g, int64_t n, float lr, float mu, float gscale,
                               int32_t* exps, int32_t* counts, const int32_t* bits, const float* target,
                               const float* nelem, int32_t nslots, uint64_t* step, void* stream) {
  if (n < 0 || nslots < 0) return LBT_EINVAL;
  const int vec = (((uintptr_t)w | (uintptr_t)a | (uintptr_t)g) & 15) == 0;  // float4 access
  const int64_t sgd_blocks = (n + 1023) / 1024;
  const int rblocks = nslots > 0 ? (nslots + 3) / 4 : 1;
  if (sgd_blocks + rblocks >= ((int64_t)1 << 31)) return LBT_EINVAL;
  hipLaunchKernelGGL(step_update_kernel, dim3((unsigned)(sgd_blocks + rblocks)), dim3(256), 0, (hipStream_t)stream, w, a,
                     g, n, lr, mu, gscale, (int)sgd_blocks, exps, counts, bits, target, nelem, nslots, step, vec);
  return (int)hipGetLastError();
}

extern "C" int lbt_dfxp_counts_fold(int32_t* counts, int32_t nslots, float* folded, void* stream) {
  if (nslots <= 0) return LBT_OK;
  hipLaunchKernelGGL(counts_fold_kernel, dim3((nslots + 3) / 4), dim3(256), 0, (hipStream_t)stream, counts, nslots,
                     folded);
  return (int)hipGetLastError();
}

extern "C" int lbt_dfxp_range_update_folded(int32_t* exps, const float* folded, const int32_t* bits,
                                            const float* target, const float* nelem, int32_t nslots,
                                            uint64_t* step, void* stream) {
  const int blocks = nslots > 0 ? (nslots + 255) / 256 : 1;
  hipLaunchKernelGGL(range_update_folded_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, exps, folded,
                     bits, target, nelem, nslots, step);
  return (int)hipGetLastError();
}

extern "C" int lbt_dfxp_quantize_weight(const float* w, int32_t KH, int32_t KW, int32_t Cin, int32_t Cout,
                                        lbt_qdesc q, int8_t* w_hwio, int8_t* wf, int32_t ksf, int8_t* wd,
                                        int32_t ksd, int32_t* colsum, void* stream) {
  if (q.bits < 1 || q.bits > 8) return LBT_EINVAL;
  if (wf && ksf * 16 < KH * KW * ((Cin + 15) / 16) * 16) return LBT_EINVAL;
  if (wd && ksd * 16 < KH * KW * ((Cout + 15) / 16) * 16) return LBT_EINVAL;
  hipLaunchKernelGGL(quantize_weight_kernel, dim3(Cout), dim3(kThreads), 0, (hipStream_t)stream, w, KH, KW, Cin,
                     Cout, q, w_hwio, wf, ksf, wd, ksd, colsum);
  return (int)hipGetLastError();
}

extern "C" int lbt_abi_version(void) { return 21; }

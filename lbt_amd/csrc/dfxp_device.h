// dfxp_device.h -- device-side building blocks of the gfx950 DFXP path:
//   * Philox4x32-10 noise (the build's counter RNG; oracle/philox.py is its CPU twin)
//   * the DFXP quantiser of dynamic_fixed_point.py:26-38 on one element
//   * the overflow predicates of dynamic_fixed_point.py:60-66
//   * wave64 reductions
// Compiled with -ffp-contract=off: every fp32 op below rounds exactly like the numpy oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/lbt_dfxp.h"

#define LBT_DEV __device__ __forceinline__

// Global reduction flushes (counters, channel sums, weight-gradient shards). LBT_EXP_PLAINSTORE
// is a timing experiment only (scratch builds): plain stores instead of atomics, wrong results.
#ifdef LBT_EXP_PLAINSTORE
#define LBT_GADD(p, v) (*(p) = (v))
#else
#define LBT_GADD(p, v) atomicAdd((p), (v))
#endif

// Phase timestamps for kernel studies (scratch builds with -DLBT_TRACE only): LBT_TS(i) stores
// s_memrealtime (100 MHz) of workgroup thread 0 into trace[wg*8 + i]; slot 7 = XCC id.
#ifdef LBT_TRACE
static __device__ unsigned long long* lbt_trace_buf;
#define LBT_TS(i)                                                                                       \
  do {                                                                                                  \
    if (threadIdx.x == 0 && lbt_trace_buf) {                                                            \
      const size_t wg_ = (size_t)blockIdx.x + (size_t)blockIdx.y * gridDim.x;                           \
      lbt_trace_buf[wg_ * 8 + (i)] = __builtin_amdgcn_s_memrealtime();                                  \
      if ((i) == 0) {                                                                                   \
        unsigned x_;                                                                                    \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x_));                               \
        lbt_trace_buf[wg_ * 8 + 7] = x_;                                                                \
      }                                                                                                 \
    }                                                                                                   \
  } while (0)
// slot 6 = a role tag (workgroups of one launch doing different work: tools/trace_phases.py groups by it)
#define LBT_TROLE(v)                                                                                    \
  do {                                                                                                  \
    if (threadIdx.x == 0 && lbt_trace_buf)                                                              \
      lbt_trace_buf[((size_t)blockIdx.x + (size_t)blockIdx.y * gridDim.x) * 8 + 6] = (v);               \
  } while (0)
#define LBT_TRACE_SETTER(tu)                                                                            \
  extern "C" int lbt_trace_set_##tu(void* p) {                                                          \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(lbt_trace_buf), &p, sizeof(p));                            \
  }
#else
#define LBT_TS(i) \
  do {            \
  } while (0)
#define LBT_TROLE(v) \
  do {               \
  } while (0)
#define LBT_TRACE_SETTER(tu)
#endif

namespace lbt {

// Outputs that a LATER launch reads in the latency-bound ResNet-20 step (codes, block outputs,
// masked gradients of the fused conv kernels, the head, the step's prologue and tail): written
// through to memory (`global_store ... sc1`) instead of staying dirty in this
// XCD's L2 until the end-of-launch write-back, which the next dependent launch waits for (MI355X_
// MICROARCH "boundary": + B / 6 TB/s for B dirty bytes; tools/wt_probe.hip: a 4 / 12 MB writer + its
// reader 4.36 -> 4.09 / 6.38 -> 6.16 us with 16-B stores, 6.07 -> 5.27 us with 4-B stores). Seven in
// eight readers sit on another XCD, whose L2 never held the line. NOT for the streaming wide-layer
// kernels (ResNet-50: tens to hundreds of MB per launch): there the same stores cost 42.2 -> 47.9 ms
// per step (bn.hip, bn_wide.hip, igemm.hip, quantize.hip keep plain stores). 4- and 8-byte: a relaxed agent-
// scope atomic store (the compiler's own sc1 store); 16-byte: a raw buffer store with the sc1 bit.
// -DLBT_PLAIN_OUT (scratch A/B builds): plain stores.
#ifdef LBT_PLAIN_OUT
LBT_DEV void st_out(int* p, int v) { *p = v; }
#else
LBT_DEV void st_out(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
#endif
// 16-byte: base[i .. i+3] (i < 2^29, base uniform) by buffer_store_dwordx4 ... sc1 (a compiler-
// scheduled store: inline asm stores escaped its store-data hazard checks and corrupted results)
#if defined(LBT_PLAIN_OUT) || defined(LBT_PLAIN_OUT4)
LBT_DEV void st_out4(float* base, uint32_t i, float4 v) { *reinterpret_cast<float4*>(base + i) = v; }
#else
LBT_DEV void st_out4(float* base, uint32_t i, float4 v) {
  typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  const v4u_ x = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)(i * 4u), 0, 16 /* sc1 */);
}
#endif
LBT_DEV void st_out(int8_t* p, int v) { st_out(reinterpret_cast<int*>(p), v); }
LBT_DEV void st_out(float* p, float v) { st_out(reinterpret_cast<int*>(p), __float_as_int(v)); }
#ifdef LBT_PLAIN_OUT
LBT_DEV void st_out8(void* p, long long v) { *reinterpret_cast<long long*>(p) = v; }
#else
LBT_DEV void st_out8(void* p, long long v) {
  __hip_atomic_store(reinterpret_cast<long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#endif
// The step's tail (the optimiser's w / a / g) keeps plain stores: written through they cost 9 us per step
// (A/B, profiles/r04l_ab: the next step's prologue then reads the weights from memory, not L2).
// LBT_WT_TAIL (scratch A/B builds): write-through there too.
#ifdef LBT_WT_TAIL
#define LBT_ST_TAIL(p, v) st_out((p), (v))
#else
#define LBT_ST_TAIL(p, v) (void)(*(p) = (v))
#endif
// 16 bytes at any 64-bit address (two 8-byte write-through stores)
LBT_DEV void st_out16(float* p, float4 v) {
  st_out8(p, (long long)(((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x)));
  st_out8(p + 2, (long long)(((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z)));
}

constexpr int kEMax = 30;  // reference computes 2**e in int32: defined for 0 <= e <= 30

// ------------------------------------------------------------------ Philox4x32-10
struct U4 { uint32_t x, y, z, w; };

LBT_DEV U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return U4{c0, c1, c2, c3};
}

LBT_DEV float u24(uint32_t r) { return (float)(r >> 8) * 5.9604644775390625e-8f; }  // * 2^-24

// Noise for the 4 consecutive noise indices 4*blk .. 4*blk+3 of one quantiser at one step.
struct Noise4 { float u[4]; };
LBT_DEV Noise4 noise4(uint64_t blk, uint32_t qid, uint64_t step, uint64_t seed) {
  U4 r = philox((uint32_t)blk, qid, (uint32_t)step, (uint32_t)(step >> 32), (uint32_t)seed,
                (uint32_t)(seed >> 32));
  Noise4 n;
  n.u[0] = u24(r.x); n.u[1] = u24(r.y); n.u[2] = u24(r.z); n.u[3] = u24(r.w);
  return n;
}
// Noise of noise-block blk (indices 4blk..4blk+3) of quantiser q: from its per-step table if it
// has one (lbt_dfxp_noise_fill wrote the same Philox values), else Philox inline.
LBT_DEV Noise4 qnoise4(const lbt_qdesc& q, uint64_t step, uint64_t blk) {
  if (q.noise) {
    const float4 v = *reinterpret_cast<const float4*>(q.noise + 4 * blk);
    return Noise4{{v.x, v.y, v.z, v.w}};
  }
  return noise4(blk, q.qid, step, q.seed);
}
LBT_DEV float noise1(uint64_t idx, uint32_t qid, uint64_t step, uint64_t seed) {
  U4 r = philox((uint32_t)(idx >> 2), qid, (uint32_t)step, (uint32_t)(step >> 32), (uint32_t)seed,
                (uint32_t)(seed >> 32));
  const uint32_t k = (uint32_t)(idx & 3);
  return u24(k == 0 ? r.x : k == 1 ? r.y : k == 2 ? r.z : r.w);
}
LBT_DEV float qnoise1(const lbt_qdesc& q, uint64_t step, uint64_t idx) {
  return q.noise ? q.noise[idx] : noise1(idx, q.qid, step, q.seed);
}

// ------------------------------------------------------------------ branch-free operand loads
// A load whose value leaves a branch becomes a register copy that must wait for the load, which
// serialises a kernel's gathers. Optional operands therefore load from this zero block instead
// (index masked to 0) and out-of-range gathers from a clamped address, selected afterwards.
static __device__ __attribute__((aligned(16))) int32_t kZeroBlock[64];  // zero-initialised, never written
LBT_DEV const float* zf() { return reinterpret_cast<const float*>(kZeroBlock); }
LBT_DEV const int32_t* zi() { return kZeroBlock; }

// ------------------------------------------------------------------ quantiser state
// The per-call view of one quantiser: multiplier m = 2^e, limit L = 2^(bits-1).
struct QState {
  float m, inv_m, L, Lm1, Lh;
  int e;
  uint64_t step;
  int active;
};

LBT_DEV int frac_exp(const lbt_qdesc& q) {
  int e = q.bits - q.exps[q.slot] - 1;
  return e < 0 ? 0 : (e > kEMax ? kEMax : e);
}

// Branch-free: the exponent and step loads of every quantiser a kernel uses issue together (an
// inactive quantiser, or one without a step counter, reads the zero block), so a kernel's
// prologue pays one dependent scalar-memory round trip for all of them instead of one (or two)
// per quantiser.
LBT_DEV QState qstate(const lbt_qdesc& q) {
  QState s;
  s.active = q.bits > 0;
  const int32_t* ep = s.active ? q.exps + q.slot : zi();
  const uint64_t* sp = (s.active && q.step) ? q.step : reinterpret_cast<const uint64_t*>(zi());
  const int I = *ep;
  const uint64_t st = *sp;
  int e = q.bits - I - 1;
  e = e < 0 ? 0 : (e > kEMax ? kEMax : e);
  s.e = s.active ? e : 0;
  s.m = s.active ? ldexpf(1.0f, e) : 0.f;
  s.inv_m = s.active ? ldexpf(1.0f, -e) : 0.f;
  s.L = s.active ? ldexpf(1.0f, q.bits - 1) : 0.f;
  s.Lm1 = s.active ? s.L - 1.0f : 0.f;
  s.Lh = s.active ? ldexpf(1.0f, q.bits - 2) : 0.f;
  s.step = st;
  return s;
}

// dequant scale 2^-e of a quantiser (the exponent the codes were produced with)
LBT_DEV float qscale(const lbt_qdesc& q) { return ldexpf(1.0f, -frac_exp(q)); }

// the wave's index in its workgroup as a wave-uniform (scalar) value: threadIdx.x >> 6 is a per-lane
// VGPR value to the compiler, so everything derived from it -- chunk / tile indices, addresses, the
// branches on it -- was computed per lane on the VALU (divisions included)
LBT_DEV int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// One element: integer code + overflow predicates (on the UNquantised x, against I_t).
// stochastic: floor(clip(x*m + u, -L, L-1)); nearest: rint(clip(x*m, -L, L-1)) (half-even).
// The asymmetric predicate xm >= T or xm < -T (T = L, Lh: powers of two) is ONE compare on
// a = max(xm, -xm (1 - 2^-24)): for xm < 0 the product rounds to >= T exactly when -xm > T (the float
// below T is T (1 - 2^-24)); NaN compares false either way. Bit-identical counts, fewer VALU.
LBT_DEV float ovf_abs(float xm) { return fmaxf(xm, xm * -0x1.fffffep-1f); }
// (int)floorf(v) as one v_cvt_flr_i32_f32 (|v| < 2^31, not NaN: the quantisers' clipped operands)
LBT_DEV int floor_i(float v) {
  int r;
  asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}
LBT_DEV int quant1(const QState& s, int stochastic, float x, float u, int& ov1, int& ov2) {
  const float xm = x * s.m;  // exact: m is a power of two
  const float a = ovf_abs(xm);
  ov1 += a >= s.L;
  ov2 += a >= s.Lh;
  float v = stochastic ? (xm + u) : xm;
  v = fminf(fmaxf(v, -s.L), s.Lm1);
  v = stochastic ? floorf(v) : rintf(v);
  return (int)v;
}

// ------------------------------------------------------------------ division by a reused divisor
// The compiler's correctly rounded fp32 x / y is
//   ys = div_scale(y); r0 = rcp(ys); e = fma(-ys, r0, 1); rc = fma(e, r0, r0);
//   xs = div_scale(x); q = xs * rc; r = fma(-ys, q, xs); q1 = fma(r, rc, q); r1 = fma(-ys, q1, xs);
//   div_fixup(div_fmas(r1, rc, q1))
// where div_scale / div_fmas / div_fixup are identities unless an operand or the quotient is
// near the ends of the exponent range (|x|,|y| in [2^-60, 2^60] here: BN moments of DFXP codes).
// Recip holds the divisor-only part (once per channel); div_by runs the rest: the SAME operations,
// so the same bits as '/' (tests/test_gpu_parity.py hammers it against '/').
struct Recip { float y, rc; };
LBT_DEV Recip recip(float y) {
  const float r0 = __builtin_amdgcn_rcpf(y);
  const float e = fmaf(-y, r0, 1.0f);
  return Recip{y, fmaf(e, r0, r0)};
}
// y > 0. copysign restores what div_fixup does for x = -0 (the fma chain yields +0); for x != 0
// the quotient already carries x's sign.
LBT_DEV float div_by(float x, const Recip& d) {
  const float q = x * d.rc;
  const float r = fmaf(-d.y, q, x);
  const float q1 = fmaf(r, d.rc, q);
  const float r1 = fmaf(-d.y, q1, x);
  return copysignf(fmaf(r1, d.rc, q1), x);
}


// Same quantiser, overflow predicates counted per WAVE: the compares become lane masks and
// s_bcnt1 / s_add on the scalar unit accumulate them, so ov1w / ov2w are wave totals (identical in
// every lane) and cost no VALU beyond the compares. STOCH is the rounding mode when known.
template <int STOCH>  // 1 stochastic, 0 nearest, -1 from `stochastic`
LBT_DEV int quant_w(const QState& s, int stochastic, float x, float u, int& ov1w, int& ov2w) {
  const float xm = x * s.m;
  const float a = ovf_abs(xm);
  ov1w += __popcll(__ballot(a >= s.L));
  ov2w += __popcll(__ballot(a >= s.Lh));
  const bool st = STOCH < 0 ? stochastic != 0 : STOCH == 1;
  float v = st ? (xm + u) : xm;
  v = fminf(fmaxf(v, -s.L), s.Lm1);
  v = st ? floorf(v) : rintf(v);
  return (int)v;
}

// Wave-total counters (from quant_w) of quantiser i of nq into the block's LDS staging area.
// Lane 0 publishes: callers guarantee lane 0 was active in every quant_w call of the wave (their
// inactive lanes are trailing ones -- elements past the end -- so the lowest lane always has work
// when any lane does), hence its running totals are the wave's.
LBT_DEV void counts_stage_w(int i, int nq, int ov1w, int ov2w, int* sh) {
  if ((threadIdx.x & 63) == 0) {
    int* p = sh + (threadIdx.x >> 6) * 2 * nq + 2 * i;
    p[0] = ov1w;
    p[1] = ov2w;
  }
}

// Lane (jj + K) & 3's v, jj = this lane's slot in its 4-lane group (K = 0..3, compile time): a DPP quad
// permutation (a VALU move; __shfl would be an LDS ds_bpermute round trip)
template <int K>
LBT_DEV int quad_from(int v) {
  if constexpr (K == 0) return v;
  else if constexpr (K == 1) return __builtin_amdgcn_mov_dpp(v, 0x39, 0xf, 0xf, false);  // quad_perm [1,2,3,0]
  else if constexpr (K == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  else return __builtin_amdgcn_mov_dpp(v, 0x93, 0xf, 0xf, false);                        // quad_perm [3,0,1,2]
}
template <int K>
LBT_DEV float quad_from(float v) { return __int_as_float(quad_from<K>(__float_as_int(v))); }
// 4 lanes x 4 byte codes transposed: lane jj of a 4-lane group holding c[i] (its column, rows i < 4)
// returns row jj's codes of the group's 4 columns packed into a dword (column g*4 + b in byte b)
LBT_DEV uint32_t quad_pack_codes(const int (&c)[4], int jj) {
  uint32_t packed = 0;
  auto step = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int sc = (jj - k) & 3;
    const int send = sc == 0 ? c[0] : sc == 1 ? c[1] : sc == 2 ? c[2] : c[3];
    const int got = quad_from<k>(send);
    packed |= ((uint32_t)got & 0xFFu) << (8 * ((jj + k) & 3));
  };
  step(std::integral_constant<int, 0>{});
  step(std::integral_constant<int, 1>{});
  step(std::integral_constant<int, 2>{});
  step(std::integral_constant<int, 3>{});
  return packed;
}

// ------------------------------------------------------------------ reductions
LBT_DEV int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
LBT_DEV long long wave_sum_i64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

LBT_DEV int shard_id() {
  return (int)((blockIdx.x + blockIdx.y * 7u + blockIdx.z * 13u) % LBT_NSHARD);
}

// Overflow counts of nq quantisers flushed behind ONE barrier:
//   counts_stage(i, nq, ov1, ov2, sh)  every thread, before the barrier: wave totals -> LDS
//                                      (sh holds 2*nq ints per wave)
//   __syncthreads()
//   counts_publish(i, nq, q, sh)       every thread, after it: lanes 2i, 2i+1 add the workgroup
//                                      totals of quantiser i into this workgroup's shard
LBT_DEV void counts_stage(int i, int nq, int ov1, int ov2, int* sh) {
  ov1 = wave_sum_i32(ov1);
  ov2 = wave_sum_i32(ov2);
  if ((threadIdx.x & 63) == 0) {
    int* p = sh + (threadIdx.x >> 6) * 2 * nq + 2 * i;
    p[0] = ov1;
    p[1] = ov2;
  }
}
LBT_DEV void counts_publish(int i, int nq, const lbt_qdesc& q, const int* sh) {
  const int j = (int)threadIdx.x - 2 * i;
  if (!q.counts || j < 0 || j > 1) return;
  const int nw = (blockDim.x + 63) >> 6;
  int t = 0;
  for (int w = 0; w < nw; ++w) t += sh[w * 2 * nq + 2 * i + j];
  if (t) LBT_GADD(q.counts + ((int64_t)q.slot * LBT_NSHARD + shard_id()) * LBT_CSTRIDE + j, t);
}

// counts_publish for a block of NW waves (compile time), counter i published by lanes 0/1 of wave
// i % NW, so a kernel's counters go out from different waves in parallel (the generic form runs a
// blockDim-bounded loop in wave 0 for every counter, one after another, at the kernel's tail).
template <int NW>
LBT_DEV void counts_publish_nw(int i, int nq, const lbt_qdesc& q, const int* sh) {
  const int j = (int)threadIdx.x - 64 * (i % NW);
  if (!q.counts || j < 0 || j > 1) return;
  int t = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += sh[w * 2 * nq + 2 * i + j];
  if (t) LBT_GADD(q.counts + ((int64_t)q.slot * LBT_NSHARD + shard_id()) * LBT_CSTRIDE + j, t);
}

// Single-quantiser flush for kernels with nothing else to publish. EVERY thread of the block
// must call it (contains barriers). sh must hold 2 ints per wave.
LBT_DEV void block_flush_counts(const lbt_qdesc& q, int ov1, int ov2, int* sh) {
  if (!q.counts) return;  // uniform
  counts_stage(0, 1, ov1, ov2, sh);
  __syncthreads();
  counts_publish(0, 1, q, sh);
  __syncthreads();
}

// block_flush_counts with wave totals (quant_w): lane 0 of each wave holds its wave's counts.
LBT_DEV void block_flush_counts_w(const lbt_qdesc& q, int ov1w, int ov2w, int* sh) {
  if (!q.counts) return;  // uniform
  counts_stage_w(0, 1, ov1w, ov2w, sh);
  __syncthreads();
  counts_publish(0, 1, q, sh);
  __syncthreads();
}

// Add a block-local per-channel partial (LDS, long long[n]) into shard shard_id() of a
// sharded int64 buffer laid out [LBT_NSHARD][stride].
LBT_DEV void block_flush_sums(const long long* sh, int n, int64_t* dst, int stride) {
  int64_t* d = dst + (int64_t)shard_id() * stride;
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    if (sh[i]) LBT_GADD((unsigned long long*)&d[i], (unsigned long long)sh[i]);
}

// Per-channel partial sums of "channel-quad" threads: thread g owns elements 4g..4g+3 of a row,
// i.e. channels c0..c0+3 with c0 = 4g mod C, so lanes whose g differ by a multiple of C/4 hold the
// same channels. chan_period(C) = C/4 when that is a power of two <= 32 (then a xor-butterfly
// over offsets C/4 .. 32 leaves the wave total in lanes 0 .. C/4-1), else 0 (no pre-reduction).
LBT_DEV int chan_period(int C) {
  const int p = C >> 2;
  return (C % 4 == 0 && p > 0 && p <= 32 && (p & (p - 1)) == 0) ? p : 0;
}
// All 64 lanes must call it.
LBT_DEV int wave_chan_reduce(int v, int period) {
  if (period)
    for (int o = period; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// true if this lane should publish its (reduced) per-channel partials
LBT_DEV bool chan_owner(int period) { return period == 0 || (int)(threadIdx.x & 63) < period; }

// ---- reduce-scatter over the wave's four 16-lane rows, on VALU lane swaps (no LDS round trips).
// v_permlane16_swap(x, y) swaps x's odd rows with y's even rows, so the sum of its two results holds
// x's row-pair sums (rows 0+1, 2+3) in rows 0 / 2 and y's in rows 1 / 3; v_permlane32_swap(P, Q)
// swaps P's upper half with Q's lower half, so the sum of its results holds P's half totals in rows
// 0-1 and Q's in rows 2-3. Integer sums: exact in any order.
// rows_scatter4: row r (lanes 16r..16r+15) ends with v_r summed over the four rows at its lane
// position (three swaps for four values; a full butterfly spends two per value).
LBT_DEV int rows_scatter4(int v0, int v1, int v2, int v3) {
  const auto a = __builtin_amdgcn_permlane16_swap(v0, v1, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(v2, v3, false, false);
  const int p01 = (int)a[0] + (int)a[1], p23 = (int)b[0] + (int)b[1];
  const auto c = __builtin_amdgcn_permlane32_swap(p01, p23, false, false);
  return (int)c[0] + (int)c[1];
}
// rows_scatter2: rows 0 and 2 end with v0's four-row total, rows 1 and 3 with v1's
LBT_DEV int rows_scatter2(int v0, int v1) {
  const auto a = __builtin_amdgcn_permlane16_swap(v0, v1, false, false);
  const int p = (int)a[0] + (int)a[1];
  const auto c = __builtin_amdgcn_permlane32_swap(p, p, false, false);
  return (int)c[0] + (int)c[1];
}
// Channel-quad partials v[k] (channel c0 + k, lanes l, l + period, ... sharing c0; period a power of
// two <= 16): the wave total of channel c0 + (lane >> 4) lands in the lanes (lane & 15) < period of
// row lane >> 4 (chan_scatter_owner). The DPP steps add the row's period-spaced repeats.
LBT_DEV int chan_scatter4(const int v[4], int period) {
  int t = rows_scatter4(v[0], v[1], v[2], v[3]);
  if (period <= 8) t += __builtin_amdgcn_update_dpp(0, t, 0x128, 0xf, 0xf, false);  // row_ror:8
  if (period <= 4) t += __builtin_amdgcn_update_dpp(0, t, 0x124, 0xf, 0xf, false);  // row_ror:4
  if (period <= 2) t += __builtin_amdgcn_update_dpp(0, t, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  if (period <= 1) t += __builtin_amdgcn_update_dpp(0, t, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  return t;
}
LBT_DEV bool chan_scatter_ok(int period) { return period >= 1 && period <= 16; }
LBT_DEV bool chan_scatter_owner(int period) { return (int)(threadIdx.x & 15) < period; }

// MomentumOptimizer.apply_gradients (trainer.py:81-82) on element i: a = mu*a + g*gscale; w -= lr*a.
// update_range on one slot from its total counters (dynamic_fixed_point.py:70-94).
LBT_DEV void range_apply(int i, int c1, int c2, int32_t* exps, const int32_t* bits, const float* target,
                         const float* nelem) {
  if (bits[i] >= 32) return;  // the 32-bit bypass adds no update_range op (:22-23)
  const float r1 = (float)c1 / nelem[i];
  const float r2 = (float)c2 / nelem[i];
  const float t = target[i];
  const int delta = r1 > t ? 1 : (r2 <= t ? -1 : 0);
  int I = exps[i] + delta;
  const int hi = bits[i] - 1, lo = bits[i] - 1 - kEMax;
  I = I > hi ? hi : (I < lo ? lo : I);
  exps[i] = I;
}

// One wave per slot: lane k < LBT_NSHARD reads (and zeroes) shard k, a wave sum gives the totals.
LBT_DEV bool wave_shard_totals(int32_t* counts, int i, int& c1, int& c2) {
  const int lane = threadIdx.x & 63;
  int a = 0, b = 0;
  if (lane < LBT_NSHARD) {
    int32_t* c = counts + ((int64_t)i * LBT_NSHARD + lane) * LBT_CSTRIDE;
    a = c[0];
    b = c[1];
    c[0] = 0;
    c[1] = 0;
  }
  c1 = wave_sum_i32(a);
  c2 = wave_sum_i32(b);
  return lane == 0;
}

LBT_DEV void sgd_momentum_elem(float* w, float* a, const float* g, int64_t i, float lr, float mu, float gscale) {
  const float t = mu * a[i];
  const float gg = g[i] * gscale;
  const float an = t + gg;
  a[i] = an;
  const float step = lr * an;
  w[i] = w[i] - step;
}

// Store one code in the requested encoding.
LBT_DEV void store_code(void* out, int kind, int64_t i, int qv, float inv_m) {
  switch (kind) {
    case LBT_OUT_I8: ((int8_t*)out)[i] = (int8_t)qv; break;
    case LBT_OUT_U8OFF: ((int8_t*)out)[i] = (int8_t)((qv < 0 ? 0 : qv) - 128); break;
    case LBT_OUT_I16: ((int16_t*)out)[i] = (int16_t)qv; break;
    default: ((float*)out)[i] = (float)qv * inv_m; break;
  }
}

}  // namespace lbt

// batched.hip -- one launch for the per-layer "small" work of a training step:
//   weight quantisation + GEMM operand packing of every conv / dense (dynamic_fixed_point.py:289-290,386-387),
//   gamma / beta quantisation of every Rescale_q (:679-682), the split reduction + dequant + 2*wd*W of every
//   weight gradient (:302, :457) and every Rescale_q's dgamma / dbeta (:689-690).
// Each of these is a few KB of work whose cost as its own kernel is the ~2-4 us launch/latency floor; ~90
// such launches per ResNet-20 step become 4. Job descriptors are read from device memory (grid.y = job).
#include "dfxp_device.h"
#include "head.h"

using namespace lbt;

namespace {

constexpr int kThreads = 256;

LBT_DEV void quantize_weights_block(const lbt_wjob* __restrict__ jobs, int bx, int by) {
  __shared__ int red[kThreads / 64];
  __shared__ int sh_cnt[2 * kThreads / 64];
  const lbt_wjob j = jobs[by];
  const int co = bx;
  if (co >= j.Cout) return;  // uniform per block
  const QState s = qstate(j.q);
  const int K = j.KH * j.KW * j.Cin;
  const int64_t inner = (int64_t)j.KW * j.Cin * j.Cout;
  const int csi = (j.Cin + 15) / 16, cso = (j.Cout + 15) / 16;
  int ov1 = 0, ov2 = 0, csum = 0;
  for (int k = threadIdx.x; k < K; k += kThreads) {
    const int tap = k / j.Cin, ci = k % j.Cin;
    const int64_t idx = (int64_t)k * j.Cout + co;
    const float u = j.q.stochastic ? qnoise1(j.q, s.step, idx % inner) : 0.f;
    const int c = quant1(s, j.q.stochastic, j.w[idx], u, ov1, ov2);
    csum += c;
    if (j.w_hwio) j.w_hwio[idx] = (int8_t)c;
    if (j.wf) j.wf[((int64_t)co * j.ksf + tap * csi + ci / 16) * 16 + (ci & 15)] = (int8_t)c;
    if (j.wd) j.wd[((int64_t)ci * j.ksd + tap * cso + co / 16) * 16 + (co & 15)] = (int8_t)c;
  }
  block_flush_counts(j.q, ov1, ov2, sh_cnt);
  if (j.colsum) {
    csum = wave_sum_i32(csum);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = csum;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int i = 0; i < kThreads / 64; ++i) t += red[i];
      j.colsum[co] = t;
    }
  }
}

// The step prologue's weight quantiser: block bx of job `by` quantises output channels 4 bx .. 4 bx + 3
// for every k (float4 loads of a W row's 4 channels, one Philox call per 4 noise indices: idx % 4 == 0,
// inner % 4 == 0), every row's load issued before the arithmetic; the codes go out as char4 stores to
// w_hwio and the dgrad image (4 consecutive channels of one 16-channel group) and as bytes to the fwd
// image. quantize_weights_block took one channel per block (1 408 blocks, a Philox call and a
// Cout-strided 4-byte load per weight: ~5.6 us per block, the prologue's critical path). Jobs that are
// not 4-channel aligned (the Dense_q W of 10 classes) go channel by channel: bx, bx + nb, ... Same codes,
// counters and column sums.
LBT_DEV void quantize_weights_block4(const lbt_wjob* __restrict__ jobs, int bx, int by, int nb) {
  __shared__ int red4[4][kThreads / 64];
  __shared__ int sh_cnt4[2 * kThreads / 64];
  const lbt_wjob j = jobs[by];
  const bool quad = j.Cout % 4 == 0 && !(reinterpret_cast<uintptr_t>(j.w) & 15) &&
                    !(reinterpret_cast<uintptr_t>(j.w_hwio) & 3) && !(reinterpret_cast<uintptr_t>(j.wd) & 3);
  if (!quad) {  // uniform per block
    for (int co = bx; co < j.Cout; co += nb) quantize_weights_block(jobs, co, by);
    return;
  }
  const int co = 4 * bx;
  if (co >= j.Cout) return;  // uniform per block
  const QState s = qstate(j.q);
  const int st = j.q.stochastic;
  const int K = j.KH * j.KW * j.Cin;
  const int64_t inner = (int64_t)j.KW * j.Cin * j.Cout;
  const int csi = (j.Cin + 15) / 16, cso = (j.Cout + 15) / 16;
  int ov1 = 0, ov2 = 0, cs[4] = {0, 0, 0, 0};
  constexpr int kRows = 2;  // k rows per thread per pass: every load in flight before the Philox calls (2: the prologue stays at <= 64 VGPRs, 8 waves per SIMD -- one round for its ~1 300 workgroups)
  for (int k0 = 0; k0 < K; k0 += kRows * kThreads) {
    float4 wv[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int k = k0 + (int)threadIdx.x + r * kThreads;
      wv[r] = *reinterpret_cast<const float4*>(j.w + (int64_t)(k < K ? k : 0) * j.Cout + co);
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int k = k0 + (int)threadIdx.x + r * kThreads;
      if (k >= K) break;
      const int64_t idx = (int64_t)k * j.Cout + co;
      const Noise4 nz = st ? qnoise4(j.q, s.step, (uint64_t)((idx % inner) >> 2)) : Noise4{{0.f, 0.f, 0.f, 0.f}};
      const float w4[4] = {wv[r].x, wv[r].y, wv[r].z, wv[r].w};
      int c[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        c[e] = quant1(s, st, w4[e], nz.u[e], ov1, ov2);
        cs[e] += c[e];
      }
      const char4 cv = make_char4((char)c[0], (char)c[1], (char)c[2], (char)c[3]);
      const int tap = k / j.Cin, ci = k - tap * j.Cin;
      if (j.w_hwio) *reinterpret_cast<char4*>(j.w_hwio + idx) = cv;
      if (j.wf) {
#pragma unroll
        for (int e = 0; e < 4; ++e) j.wf[((int64_t)(co + e) * j.ksf + tap * csi + ci / 16) * 16 + (ci & 15)] = (int8_t)c[e];
      }
      if (j.wd) *reinterpret_cast<char4*>(j.wd + ((int64_t)ci * j.ksd + tap * cso + co / 16) * 16 + (co & 15)) = cv;
    }
  }
  block_flush_counts(j.q, ov1, ov2, sh_cnt4);
  if (j.colsum) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int v = wave_sum_i32(cs[e]);
      if ((threadIdx.x & 63) == 0) red4[e][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      int t = 0;
      for (int i = 0; i < kThreads / 64; ++i) t += red4[threadIdx.x][i];
      j.colsum[co + threadIdx.x] = t;
    }
  }
}

__global__ __launch_bounds__(kThreads) void quantize_weights_kernel(const lbt_wjob* __restrict__ jobs) {
  quantize_weights_block(jobs, blockIdx.x, blockIdx.y);
}

LBT_DEV void quantize_many_block(const lbt_qjob* __restrict__ jobs, int by) {
  __shared__ int sh_cnt[2 * kThreads / 64];
  const lbt_qjob j = jobs[by];
  const QState s = qstate(j.q);
  int ov1 = 0, ov2 = 0;
  for (int64_t i = threadIdx.x; i < j.n; i += kThreads) {
    const float u = j.q.stochastic ? qnoise1(j.q, s.step, i % j.inner) : 0.f;
    const int c = quant1(s, j.q.stochastic, j.x[i], u, ov1, ov2);
    store_code(j.out, j.out_kind, i, c, s.inv_m);
  }
  block_flush_counts(j.q, ov1, ov2, sh_cnt);
}

__global__ __launch_bounds__(kThreads) void quantize_many_kernel(const lbt_qjob* __restrict__ jobs) {
  quantize_many_block(jobs, blockIdx.y);
}

// MomentumOptimizer on one element whose parameter wv and accumulator am were loaded by the caller:
// sgd_momentum_elem's operations and order (gscale 1: g * 1.0f == g), so bit-identical to lbt_step_update
LBT_DEV void sgd_update(float wv, float am, float gv, const lbt_update& u, int64_t o) {
  const float t = u.mu * am;
  const float an = t + gv;
  LBT_ST_TAIL(u.a + o, an);
  const float step = u.lr * an;
  LBT_ST_TAIL(u.w + o, wv - step);
}

// Blocks are allotted to the jobs in order, lbt_rjob_blocks(K*Cout) = ceil(K*Cout / kRBlock) each (1-D
// grid); a block reduces kRBlock consecutive outputs (kRPer per thread, 256 apart: coalesced) over the
// slab's shards, with the offset correction 128 * sum_p g[co] (x_u8off) summed once per column into LDS.
// (256 outputs per block made ~1 060 blocks of a ResNet-20 step: dispatched over ~7 us, the launch's
// critical path. lds: >= 4 KB.)
#ifndef LBT_RPER
#define LBT_RPER 4
#endif
constexpr int kRPer = LBT_RPER;
constexpr int kRBlock = 256 * kRPer;
LBT_DEV void rjob_block(const lbt_rjob* __restrict__ jobs, int njobs, int blk, uint8_t* lds, const lbt_xchg& x,
                        const lbt_update& u) {
  int64_t* nbs = reinterpret_cast<int64_t*>(lds);                   // [256]
  long long* colsum = reinterpret_cast<long long*>(lds + 2048);      // [256]
  int* s_job = reinterpret_cast<int*>(lds + 4096);
  int64_t* s_base = reinterpret_cast<int64_t*>(lds + 4104);
  // every job's block count loaded in parallel (a serial scan of device memory would cost one
  // memory round trip per job), then scanned: <= 64 jobs as an inclusive scan across wave 0's lanes
  // (the owning lane is the one whose [start, end) holds blk), more jobs serially in LDS
  if (njobs <= 64) {
    if (threadIdx.x < 64) {
      const int l = (int)threadIdx.x;
      const int64_t nb = l < njobs ? ((int64_t)jobs[l].K * jobs[l].Cout + kRBlock - 1) / kRBlock : 0;
      int64_t end = nb;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int64_t v = __shfl_up(end, o, 64);
        if (l >= o) end += v;
      }
      const bool own = l < njobs && (int64_t)blk < end && (int64_t)blk >= end - nb;
      const unsigned long long m = __ballot(own);
      if (l == 0) *s_job = m ? __ffsll((long long)m) - 1 : njobs;
      if (own) *s_base = ((int64_t)blk - (end - nb)) * kRBlock;
    }
    __syncthreads();
  } else {
    for (int j = threadIdx.x; j < njobs; j += 256) nbs[j] = ((int64_t)jobs[j].K * jobs[j].Cout + kRBlock - 1) / kRBlock;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t b = blk;
      int jj = njobs;  // past the end: nothing to do
      for (int j = 0; j < njobs; ++j) {
        if (b < nbs[j]) { jj = j; break; }
        b -= nbs[j];
      }
      *s_job = jj;
      *s_base = b * kRBlock;
    }
    __syncthreads();
  }
  if (*s_job >= njobs) return;
  const lbt_rjob j = jobs[*s_job];
  const int64_t total = (int64_t)j.K * j.Cout;
  const int64_t i0 = *s_base + threadIdx.x;  // this thread's outputs: i0 + 256 e, e < kRPer
  const bool corr = j.x_u8off && j.gcolsum;
  // the column sums' shard loads, the slab loads and the optimiser's operands are issued back to back,
  // so all arrive in one memory round trip. Cout <= 256 (colsum's LDS capacity): thread c < Cout sums
  // column c once into LDS; wider jobs: each output's column summed by its own thread (below)
  const bool lds_cols = j.Cout <= 256;
  const int c = (int)threadIdx.x;
  const bool col = corr && lds_cols && c < j.Cout;
  long long v[LBT_NSHARD];
  if (col) {
#pragma unroll
    for (int k = 0; k < LBT_NSHARD; ++k) v[k] = j.gcolsum[(int64_t)k * 2 * j.Cout + c];
  }
  long long s[kRPer];
  float wv[kRPer], am[kRPer];
  const int64_t ob = u.w ? (j.dw - u.g) : 0;
#pragma unroll
  for (int e = 0; e < kRPer; ++e) {
    const int64_t i = i0 + 256 * e;
    s[e] = 0;
    wv[e] = 0.f;
    am[e] = 0.f;
    if (i < total && !x.buf) {
      wv[e] = j.w[i];
      if (u.w) am[e] = u.a[ob + i];
    }
  }
  // the slab's shards (1-2 for the block convs, 32 for the stem's): 8 at a time, every load of a group
  // in flight before its adds (a plain loop waited on each load in turn: 32 round trips for the stem)
  int b = 0;
  for (; b + 8 <= j.nsplit; b += 8) {
    int sv[8][kRPer];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < kRPer; ++e) {
        const int64_t i = i0 + 256 * e;
        sv[q][e] = j.slab[(int64_t)(b + q) * total + (i < total ? i : 0)];
      }
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < kRPer; ++e) s[e] += sv[q][e];
  }
  for (; b < j.nsplit; ++b) {
    int sv[kRPer];
#pragma unroll
    for (int e = 0; e < kRPer; ++e) {
      const int64_t i = i0 + 256 * e;
      sv[e] = j.slab[(int64_t)b * total + (i < total ? i : 0)];
    }
#pragma unroll
    for (int e = 0; e < kRPer; ++e) s[e] += sv[e];
  }
  if (corr && lds_cols) {
    if (col) {
      long long t = 0;
#pragma unroll
      for (int k = 0; k < LBT_NSHARD; ++k) t += v[k];
      colsum[c] = t;
    }
    __syncthreads();
  }
  const float scale = ldexpf(1.0f, -(frac_exp(j.qx) + frac_exp(j.qg)));
#pragma unroll
  for (int e = 0; e < kRPer; ++e) {
    const int64_t i = i0 + 256 * e;
    if (i >= total) break;
    if (corr) {
      long long t;
      if (lds_cols) {
        t = colsum[i % j.Cout];
      } else {
        const int ce = (int)(i % j.Cout);
        t = 0;
        for (int k = 0; k < LBT_NSHARD; ++k) t += j.gcolsum[(int64_t)k * 2 * j.Cout + ce];
      }
      s[e] += 128ll * t;
    }
    if (x.buf) {  // data-parallel exchange: the exact numerator, dequantised after the all-reduce
      x.buf[(j.dw - x.gbase) + i] = s[e];
      continue;
    }
    const float a = (float)s[e] * scale;
    const float b = j.wd2 * wv[e];
    const float gv = a + b;
    if (u.w) {  // lbt_step_reduce_update: the gradient, then MomentumOptimizer on the same element
      LBT_ST_TAIL(j.dw + i, gv);
      sgd_update(wv[e], am[e], gv, u, ob + i);
      continue;
    }
    j.dw[i] = gv;
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_many_kernel(const lbt_rjob* __restrict__ jobs, int njobs) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4112];
  rjob_block(jobs, njobs, blockIdx.x, lds, lbt_xchg{}, lbt_update{});
}

LBT_DEV void pjob_channel(const lbt_pjob& j, int c, const lbt_xchg& x, const lbt_update& u) {
  if (c >= j.C) return;
  int64_t og = 0, ob = 0;
  float wg = 0.f, ag = 0.f, wb = 0.f, ab = 0.f;
  if (u.w) {  // the optimiser's operands, loaded with the sums
    og = (j.dgamma - u.g) + c;
    ob = (j.dbeta - u.g) + c;
    wg = u.w[og]; ag = u.a[og]; wb = u.w[ob]; ab = u.a[ob];
  }
  long long vr[LBT_NSHARD], vg[LBT_NSHARD];  // all shard loads in flight at once
#pragma unroll
  for (int k = 0; k < LBT_NSHARD; ++k) {
    vr[k] = j.sums[(int64_t)k * 4 * j.C + c];
    vg[k] = j.sums[(int64_t)k * 4 * j.C + j.C + c];
  }
  long long sgr = 0, sg = 0;
#pragma unroll
  for (int k = 0; k < LBT_NSHARD; ++k) {
    sgr += vr[k];
    sg += vg[k];
  }
  if (x.buf) {
    x.buf[(j.dgamma - x.gbase) + c] = sgr * x.pjob_scale;
    x.buf[(j.dbeta - x.gbase) + c] = sg * x.pjob_scale;
    return;
  }
  const double g2 = ldexp(1.0, -frac_exp(j.qrg)), r = ldexp(1.0, -frac_exp(j.qr));
  const float a = (float)((double)sgr * (g2 * r));
  if (u.w) {
    const float b = j.wd2 * wg;  // j.gamma[c] == u.w[og]
    const float dg = a + b, db = (float)((double)sg * g2);
    LBT_ST_TAIL(j.dgamma + c, dg);
    LBT_ST_TAIL(j.dbeta + c, db);
    sgd_update(wg, ag, dg, u, og);
    sgd_update(wb, ab, db, u, ob);
    return;
  }
  const float b = j.wd2 * j.gamma[c];
  j.dgamma[c] = a + b;
  j.dbeta[c] = (float)((double)sg * g2);
}

__global__ void param_grads_many_kernel(const lbt_pjob* __restrict__ jobs) {
  pjob_channel(jobs[blockIdx.y], blockIdx.x * blockDim.x + threadIdx.x, lbt_xchg{}, lbt_update{});
}

// One wave per slot: lane k < LBT_NSHARD reads (and zeroes) shard k of the overflow counters.
LBT_DEV void fold_slot_x(const lbt_xchg& x, int i) {
  const int lane = threadIdx.x & 63;
  int a = 0, b = 0;
  if (lane < LBT_NSHARD) {
    int32_t* c = x.counts + ((int64_t)i * LBT_NSHARD + lane) * LBT_CSTRIDE;
    a = c[0];
    b = c[1];
    c[0] = 0;
    c[1] = 0;
  }
  a = wave_sum_i32(a);
  b = wave_sum_i32(b);
  if (lane == 0) {
    x.buf[x.cnt_off + 2 * i] = a;
    x.buf[x.cnt_off + 2 * i + 1] = b;
  }
}

// lbt_step_reduce(_x / _update): [1 head block][update only: ceil(nslots / 4) range-update blocks]
// [np * pblk param-grad blocks][exchange only: ceil(nslots / 4) counter-fold blocks][r_blocks
// wgrad-reduce blocks]. The head block (a serial chain of ~7 us: the records, the Dense_q dW, the
// ordered loss sum) is dispatched first: placed last, it started only after the ~1 000 wgrad-reduce
// blocks had been dispatched (~5 us) and ended the launch.
__global__ __launch_bounds__(256) void step_reduce_kernel(const lbt_rjob* __restrict__ rjobs, int nr, int r_blocks,
                                                          const lbt_pjob* __restrict__ pjobs, int np, int pblk,
                                                          lbt_head head, int has_head, lbt_xchg x, int fold,
                                                          lbt_update u, int ublocks) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kHeadLds];
  int b = blockIdx.x;
  LBT_TS(0);
  if (has_head) {
    if (b == 0) {
      LBT_TROLE(3);
      head_reduce(head, x, lds, u);
      LBT_TS(1);
      return;
    }
    --b;
  }
  if (b < ublocks) {  // update_range (dynamic_fixed_point.py:70-94): one wave per slot
    LBT_TROLE(5);
    const int i = b * 4 + (int)(threadIdx.x >> 6);
    if (i < u.nslots && u.nelem[i] > 0.f) {
      int c1, c2;
      if (wave_shard_totals(u.counts, i, c1, c2)) range_apply(i, c1, c2, u.exps, u.bits, u.target, u.nelem);
    }
    if (b == 0 && threadIdx.x == 0) u.step[0] += 1ull;
    return;
  }
  b -= ublocks;
  if (b < np * pblk) {
    LBT_TROLE(2);
    pjob_channel(pjobs[b / pblk], (b % pblk) * 256 + threadIdx.x, x, u);
    LBT_TS(1);
    return;
  }
  b -= np * pblk;
  if (b < fold) {
    LBT_TROLE(4);
    const int i = b * 4 + (int)(threadIdx.x >> 6);
    if (x.buf && i < x.nslots) fold_slot_x(x, i);
    return;
  }
  b -= fold;
  LBT_TROLE(1);
  rjob_block(rjobs, nr, b, lds, x, u);
  LBT_TS(1);
}

// grid (blocks, njobs): thread -> noise blocks b, b + gx * kThreads, ... (kNoisePer of them; 4 values,
// one Philox call each)
constexpr int kNoisePer = 4;
// (every block also clears its share of the sums arena: 4 x int64 per thread over the gx * gy blocks)
LBT_DEV void noise_fill_block(const lbt_njob* __restrict__ jobs, int64_t* zero, int64_t nzero, int bx, int by, int gx,
                              int per = 1, int gy = 1) {
  const int64_t b = (int64_t)bx * kThreads + threadIdx.x;
  if (per == 1 ? by == 0 : true) {
    const int64_t zb = per == 1 ? b : ((int64_t)by * gx + bx) * kThreads + threadIdx.x;
    const int64_t zs = 4 * (int64_t)gx * kThreads * (per == 1 ? 1 : gy);
    for (int64_t z = 4 * zb; z < nzero; z += zs) {
      if (z + 4 <= nzero) {
#ifdef LBT_PLAIN_PRO
        *reinterpret_cast<longlong2*>(zero + z) = make_longlong2(0, 0);
        *reinterpret_cast<longlong2*>(zero + z + 2) = make_longlong2(0, 0);
#else
        st_out8(zero + z, 0);
        st_out8(zero + z + 1, 0);
        st_out8(zero + z + 2, 0);
        st_out8(zero + z + 3, 0);
#endif
      } else {
        for (int64_t t = z; t < nzero; ++t) zero[t] = 0;
      }
    }
  }
  const lbt_njob j = jobs[by];
  if (4 * b >= j.n) return;
  const uint64_t step = *j.step;
  for (int i = 0; i < per; ++i) {
    const int64_t bb = b + (int64_t)i * gx * kThreads;
    if (4 * bb >= j.n) break;
    const Noise4 n = noise4((uint64_t)bb, j.qid, step, j.seed);
#ifdef LBT_PLAIN_PRO
    *reinterpret_cast<float4*>(j.out + 4 * bb) = make_float4(n.u[0], n.u[1], n.u[2], n.u[3]);
#else
    st_out4(j.out, (uint32_t)(4 * bb), make_float4(n.u[0], n.u[1], n.u[2], n.u[3]));  // tables < 2^29 floats
#endif
  }
}

__global__ __launch_bounds__(kThreads) void noise_fill_kernel(const lbt_njob* __restrict__ jobs, int64_t* zero,
                                                             int64_t nzero) {
  noise_fill_block(jobs, zero, nzero, blockIdx.x, blockIdx.y, gridDim.x);
}

// The step's input images -> int16 codes: 4 consecutive elements per thread (one Philox call),
// quant1 per element exactly as lbt_dfxp_quantize (noise index = element mod inner).
LBT_DEV void quantize_input_block(const lbt_qjob& j, int bx) {
  __shared__ int sh_cnt[2 * kThreads / 64];
  const QState s = qstate(j.q);
  const int64_t e0 = 4 * ((int64_t)bx * kThreads + threadIdx.x);
  int ov1 = 0, ov2 = 0;
  if (e0 < j.n) {  // n % 4 == 0, inner % 4 == 0 (launcher)
    const float4 v = *reinterpret_cast<const float4*>(j.x + e0);
    Noise4 nz = {{0.f, 0.f, 0.f, 0.f}};
    if (j.q.stochastic) nz = qnoise4(j.q, s.step, (uint64_t)((e0 % j.inner) >> 2));
    const int c0 = quant1(s, j.q.stochastic, v.x, nz.u[0], ov1, ov2);
    const int c1 = quant1(s, j.q.stochastic, v.y, nz.u[1], ov1, ov2);
    const int c2 = quant1(s, j.q.stochastic, v.z, nz.u[2], ov1, ov2);
    const int c3 = quant1(s, j.q.stochastic, v.w, nz.u[3], ov1, ov2);
    short4 o;
    o.x = (short)c0; o.y = (short)c1; o.z = (short)c2; o.w = (short)c3;
#ifdef LBT_PLAIN_PRO
    *reinterpret_cast<short4*>((int16_t*)j.out + e0) = o;
#else
    st_out8((int16_t*)j.out + e0, *reinterpret_cast<const long long*>(&o));
#endif
  }
  block_flush_counts(j.q, ov1, ov2, sh_cnt);
}

// lbt_step_prologue: [max_cout x nw weight blocks][input blocks][nq parameter blocks][noise rows x njobs]: the
// weight quantisers (the longest blocks: a Philox call per weight, strided operand-image stores) are
// dispatched first and the short noise-table blocks (kNoisePer Philox calls per thread) fill in behind
// them (traced: with the noise rows first, the ~4 us weight blocks started ~2.7 us late)
struct Prologue {
  const lbt_njob* njobs; int nn, nbx; int64_t* zero; int64_t nzero;
  const lbt_wjob* wjobs; int nw, max_cout;
  const lbt_qjob* qjobs; int nq;
  lbt_qjob input; int nin;
  const int32_t* snap_src; int32_t* snap_dst; int nsnap;
};

__global__ __launch_bounds__(kThreads, 8) void step_prologue_kernel(Prologue a) {
  int b = blockIdx.x;
  LBT_TS(0);
  const int nbw = (a.max_cout + 3) / 4;  // weight blocks per job (4 output channels each)
  const int n2 = nbw * a.nw;
  if (b < n2) {
    LBT_TROLE(2);
    quantize_weights_block4(a.wjobs, b % nbw, b / nbw, nbw);
    LBT_TS(1);
    return;
  }
  b -= n2;
  if (b < a.nin) {
    LBT_TROLE(4);
    quantize_input_block(a.input, b);
    LBT_TS(1);
    return;
  }
  b -= a.nin;
  if (b < a.nq) {
    LBT_TROLE(3);
    quantize_many_block(a.qjobs, b);
    LBT_TS(1);
    return;
  }
  b -= a.nq;
  if (b < (a.nsnap > 0 ? 1 : 0)) {  // the step's exponents, for lbt_step_reduce_update's dequantisations
    for (int i = threadIdx.x; i < a.nsnap; i += kThreads) a.snap_dst[i] = a.snap_src[i];
    return;
  }
  if (a.nsnap > 0) --b;
  LBT_TROLE(1);
  noise_fill_block(a.njobs, a.zero, a.nzero, b % a.nbx, b / a.nbx, a.nbx, kNoisePer, a.nn);
  LBT_TS(1);
}

}  // namespace

LBT_TRACE_SETTER(batched)

extern "C" int lbt_dfxp_noise_fill(const lbt_njob* jobs, int32_t njobs, int64_t max_n, int64_t* zero, int64_t nzero,
                                   void* stream) {
  if (njobs <= 0 || max_n <= 0) return LBT_OK;
  if (nzero > 0 && (reinterpret_cast<uintptr_t>(zero) % 16)) return LBT_EINVAL;
  if (max_n >= ((int64_t)1 << 29)) return LBT_EINVAL;  // the tables' 32-bit store offsets
  const int64_t blocks = (max_n + 4 * kThreads - 1) / (4 * kThreads);
  if (njobs > 65535 || blocks > 0x7fffffff) return LBT_EINVAL;
  hipLaunchKernelGGL(noise_fill_kernel, dim3((unsigned)blocks, njobs), dim3(kThreads), 0, (hipStream_t)stream, jobs,
                     zero, nzero > 0 ? nzero : 0);
  return (int)hipGetLastError();
}

extern "C" int lbt_step_prologue(const lbt_njob* njobs, int32_t nn, int64_t max_n, int64_t* zero, int64_t nzero,
                                 const lbt_wjob* wjobs, int32_t nw, int32_t max_cout, const lbt_qjob* qjobs, int32_t nq,
                                 const lbt_qjob* input, const int32_t* snap_src, int32_t* snap_dst, int32_t snap_n,
                                 void* stream) {
  if (nn < 0 || nw < 0 || nq < 0 || (nn > 0 && max_n <= 0) || (nw > 0 && max_cout <= 0)) return LBT_EINVAL;
  if (snap_n < 0 || (snap_n > 0 && (!snap_src || !snap_dst))) return LBT_EINVAL;
  if (nn > 0 && max_n >= ((int64_t)1 << 29)) return LBT_EINVAL;  // the tables' 32-bit store offsets
  if (nzero > 0 && (reinterpret_cast<uintptr_t>(zero) % 16)) return LBT_EINVAL;
  Prologue a{};
  a.njobs = njobs; a.nn = nn; a.zero = zero; a.nzero = nzero > 0 ? nzero : 0;
  a.nbx = nn > 0 ? (int)((max_n + 4 * kNoisePer * kThreads - 1) / (4 * kNoisePer * kThreads)) : 0;
  a.wjobs = wjobs; a.nw = nw; a.max_cout = nw > 0 ? max_cout : 0;
  a.qjobs = qjobs; a.nq = nq;
  if (input) {
    a.input = *input;
    if (a.input.n % 4 || a.input.inner % 4 || a.input.out_kind != LBT_OUT_I16 ||
        (reinterpret_cast<uintptr_t>(a.input.x) % 16))
      return LBT_EINVAL;
    a.nin = (int)((a.input.n / 4 + kThreads - 1) / kThreads);
  }
  a.snap_src = snap_src; a.snap_dst = snap_dst; a.nsnap = snap_n;
  const int64_t blocks = (int64_t)a.nbx * nn + (int64_t)((a.max_cout + 3) / 4) * nw + nq + a.nin + (snap_n > 0 ? 1 : 0);
  if (blocks <= 0) return LBT_OK;
  if (blocks > 0x7fffffff) return LBT_EINVAL;
  hipLaunchKernelGGL(step_prologue_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

namespace {

// Element-parallel form of quantize_weights_block for wide layers (ResNet-50: 23.5 M weights in
// 54 tensors): block b of the 1-D grid takes 1024 consecutive HWIO elements of the job whose range
// [starts[j], starts[j+1]) holds b; a thread quantises 4 consecutive elements (one float4 load,
// one Philox call for their 4 noise indices: Cout % 4 == 0 keeps them in one noise block) and
// writes them to every image. Same codes and counters as quantize_weights_block; no column sums.
constexpr int kFlatPerBlock = 4 * kThreads;

__global__ __launch_bounds__(kThreads) void quantize_weights_flat_kernel(const lbt_wjob* __restrict__ jobs,
                                                                         const int32_t* __restrict__ starts,
                                                                         int njobs) {
  __shared__ int sh_cnt[2 * kThreads / 64];
  const int b = (int)blockIdx.x;
  int jlo = 0, jhi = njobs;  // starts[jlo] <= b < starts[jhi]
  while (jhi - jlo > 1) {
    const int mid = (jlo + jhi) >> 1;
    if (starts[mid] <= b) jlo = mid; else jhi = mid;
  }
  const lbt_wjob j = jobs[jlo];
  const QState s = qstate(j.q);
  const int64_t n = (int64_t)j.KH * j.KW * j.Cin * j.Cout;
  const int64_t inner = (int64_t)j.KW * j.Cin * j.Cout;
  const int csi = (j.Cin + 15) / 16, cso = (j.Cout + 15) / 16;
  const int64_t idx = ((int64_t)(b - starts[jlo]) * kFlatPerBlock) + 4 * threadIdx.x;
  int ov1 = 0, ov2 = 0;
  if (idx < n) {
    const float4 wv = *reinterpret_cast<const float4*>(j.w + idx);
    const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
    const Noise4 nz = j.q.stochastic ? qnoise4(j.q, s.step, (uint64_t)((idx % inner) >> 2)) : Noise4{{0.f, 0.f, 0.f, 0.f}};
    int c[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) c[e] = quant1(s, j.q.stochastic, w4[e], nz.u[e], ov1, ov2);
    if (j.w_hwio) {
      char4 v;
      v.x = (char)c[0]; v.y = (char)c[1]; v.z = (char)c[2]; v.w = (char)c[3];
      *reinterpret_cast<char4*>(j.w_hwio + idx) = v;
    }
    const int64_t k = idx / j.Cout;
    const int co0 = (int)(idx - k * j.Cout);
    const int tap = (int)(k / j.Cin), ci = (int)(k - (int64_t)tap * j.Cin);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + e;
      if (j.wf) j.wf[((int64_t)co * j.ksf + tap * csi + ci / 16) * 16 + (ci & 15)] = (int8_t)c[e];
      if (j.wd) j.wd[((int64_t)ci * j.ksd + tap * cso + co / 16) * 16 + (co & 15)] = (int8_t)c[e];
    }
  }
  block_flush_counts(j.q, ov1, ov2, sh_cnt);
}

}  // namespace

extern "C" int lbt_rjob_blocks(int64_t n) { return (int)((n + kRBlock - 1) / kRBlock); }

extern "C" int lbt_flat_weight_blocks(int64_t n) { return (int)((n + kFlatPerBlock - 1) / kFlatPerBlock); }

extern "C" int lbt_dfxp_quantize_weights_flat(const lbt_wjob* jobs, const int32_t* starts, int32_t njobs,
                                              int32_t total_blocks, void* stream) {
  if (njobs <= 0 || total_blocks <= 0) return LBT_OK;
  hipLaunchKernelGGL(quantize_weights_flat_kernel, dim3((unsigned)total_blocks), dim3(kThreads), 0,
                     (hipStream_t)stream, jobs, starts, njobs);
  return (int)hipGetLastError();
}

extern "C" int lbt_dfxp_quantize_weights(const lbt_wjob* jobs, int32_t njobs, int32_t max_cout, void* stream) {
  if (njobs <= 0) return LBT_OK;
  if (njobs > 65535 || max_cout <= 0) return LBT_EINVAL;
  hipLaunchKernelGGL(quantize_weights_kernel, dim3(max_cout, njobs), dim3(kThreads), 0, (hipStream_t)stream, jobs);
  return (int)hipGetLastError();
}

extern "C" int lbt_dfxp_quantize_many(const lbt_qjob* jobs, int32_t njobs, void* stream) {
  if (njobs <= 0) return LBT_OK;
  if (njobs > 65535) return LBT_EINVAL;
  hipLaunchKernelGGL(quantize_many_kernel, dim3(1, njobs), dim3(kThreads), 0, (hipStream_t)stream, jobs);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_wgrad_reduce_many(const lbt_rjob* jobs, int32_t njobs, int32_t total_blocks, void* stream) {
  if (njobs <= 0) return LBT_OK;
  if (total_blocks <= 0 || njobs > 256) return LBT_EINVAL;
  hipLaunchKernelGGL(wgrad_reduce_many_kernel, dim3(total_blocks), dim3(256), 0, (hipStream_t)stream, jobs, njobs);
  return (int)hipGetLastError();
}

namespace {
int step_reduce_launch(const lbt_rjob* rjobs, int32_t nr, int32_t r_blocks, const lbt_pjob* pjobs, int32_t np,
                       int32_t max_c, const lbt_head* head, const lbt_xchg& x, const lbt_update& u, void* stream) {
  if (nr < 0 || np < 0 || nr > 256 || r_blocks < 0 || (nr > 0 && r_blocks == 0) || (np > 0 && max_c <= 0))
    return LBT_EINVAL;
  lbt_head h = {};
  if (head) {
    h = *head;
    if (h.N <= 0 || h.C <= 0 || h.C > 256 || h.C % 8 || h.K <= 0 || h.K > 64 || !h.scratch || !h.w || !h.dw || !h.loss)
      return LBT_EINVAL;
  }
  if (x.buf && (!x.gbase || x.nslots < 0 || (x.nslots > 0 && !x.counts) || x.cnt_off < 0 || x.loss_off < 0 ||
                (x.pjob_scale != 0 && x.pjob_scale != 1)))
    return LBT_EINVAL;
  if (u.w && (x.buf || !u.a || !u.g || u.nslots < 0 || !u.exps || !u.counts || !u.bits || !u.target || !u.nelem ||
              !u.step))
    return LBT_EINVAL;
  const int pblk = np > 0 ? (max_c + 255) / 256 : 0;
  const int fold = x.buf ? (x.nslots + 3) / 4 : 0;
  const int ublocks = u.w ? (u.nslots > 0 ? (u.nslots + 3) / 4 : 1) : 0;
  const int64_t blocks = (int64_t)r_blocks + (int64_t)np * pblk + (head ? 1 : 0) + fold + ublocks;
  if (blocks <= 0) return LBT_OK;
  hipLaunchKernelGGL(step_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, rjobs, nr, r_blocks,
                     pjobs, np, pblk, h, head ? 1 : 0, x, fold, u, ublocks);
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int lbt_step_reduce(const lbt_rjob* rjobs, int32_t nr, int32_t r_blocks, const lbt_pjob* pjobs, int32_t np,
                               int32_t max_c, const lbt_head* head, void* stream) {
  return step_reduce_launch(rjobs, nr, r_blocks, pjobs, np, max_c, head, lbt_xchg{}, lbt_update{}, stream);
}

extern "C" int lbt_step_reduce_x(const lbt_rjob* rjobs, int32_t nr, int32_t r_blocks, const lbt_pjob* pjobs, int32_t np,
                                 int32_t max_c, const lbt_head* head, const lbt_xchg* x, void* stream) {
  if (!x || !x->buf) return LBT_EINVAL;
  return step_reduce_launch(rjobs, nr, r_blocks, pjobs, np, max_c, head, *x, lbt_update{}, stream);
}

extern "C" int lbt_step_reduce_update(const lbt_rjob* rjobs, int32_t nr, int32_t r_blocks, const lbt_pjob* pjobs,
                                      int32_t np, int32_t max_c, const lbt_head* head, const lbt_update* u,
                                      void* stream) {
  if (!u || !u->w) return LBT_EINVAL;
  return step_reduce_launch(rjobs, nr, r_blocks, pjobs, np, max_c, head, lbt_xchg{}, *u, stream);
}

namespace {

// lbt_step_finish: blocks are dealt to the segments in order, ceil(n / 256) each (like rjob_block);
// the last block also writes the loss.
__global__ __launch_bounds__(256) void step_finish_kernel(const lbt_fseg* __restrict__ segs, int nseg,
                                                          const int64_t* __restrict__ xbuf, float* __restrict__ w,
                                                          float* __restrict__ a, float* __restrict__ g, float lr,
                                                          float mu, float* loss, int64_t loss_off, int loss_n) {
  __shared__ int64_t nbs[256];
  __shared__ int s_seg;
  __shared__ int64_t s_base;
  for (int j = threadIdx.x; j < nseg; j += 256) nbs[j] = (segs[j].n + 255) / 256;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t b = blockIdx.x;
    int jj = nseg;
    for (int j = 0; j < nseg; ++j) {
      if (b < nbs[j]) { jj = j; break; }
      b -= nbs[j];
    }
    s_seg = jj;
    s_base = b * 256;
  }
  __syncthreads();
  if (loss && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    loss[0] = (float)((double)xbuf[loss_off] * 2.3283064365386963e-10 / (double)loss_n);  // * 2^-32
  if (s_seg >= nseg) return;
  const lbt_fseg sg = segs[s_seg];
  const int64_t k = s_base + threadIdx.x;
  if (k >= sg.n) return;
  const int64_t i = sg.off + k;
  const long long S = xbuf[i];
  float gv;
  if (sg.kind == 0) {  // wgrad_reduce / rjob_block / head_reduce: (float)S * 2^-(ex+eg) + wd2 * w
    const float scale = ldexpf(1.0f, -(frac_exp(sg.qx) + frac_exp(sg.qg)));
    const float p = (float)S * scale;
    const float q = sg.wd2 * w[i];
    gv = p + q;
  } else if (sg.kind == 1) {  // pjob_channel dgamma
    const double g2 = ldexp(1.0, -frac_exp(sg.qg)), r = ldexp(1.0, -frac_exp(sg.qx));
    const float p = (float)((double)S * (g2 * r));
    const float q = sg.wd2 * w[i];
    gv = p + q;
  } else {  // pjob_channel dbeta
    gv = (float)((double)S * ldexp(1.0, -frac_exp(sg.qg)));
  }
  if (g) g[i] = gv;
  const float t = mu * a[i];
  const float an = t + gv;
  a[i] = an;
  const float step = lr * an;
  w[i] = w[i] - step;
}

__global__ void range_update_x_kernel(int32_t* exps, const int64_t* xbuf, int64_t cnt_off, const int32_t* bits,
                                      const float* target, const float* nelem, int nslots, uint64_t* step) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  // update_range (dynamic_fixed_point.py:70-94) on the summed counts; a 32-bit slot has no range op
  // (the bits==32 bypass, :22-23), as in range_apply
  if (i < nslots && nelem[i] > 0.f && bits[i] < 32) {
    const long long c1 = xbuf[cnt_off + 2 * i], c2 = xbuf[cnt_off + 2 * i + 1];
    const float r1 = (float)c1 / nelem[i];
    const float r2 = (float)c2 / nelem[i];
    const float t = target[i];
    const int delta = r1 > t ? 1 : (r2 <= t ? -1 : 0);
    int I = exps[i] + delta;
    const int hi = bits[i] - 1, lo = bits[i] - 1 - kEMax;
    I = I > hi ? hi : (I < lo ? lo : I);
    exps[i] = I;
  }
  if (i == 0) step[0] += 1ull;
}

}  // namespace

extern "C" int lbt_step_finish(const lbt_fseg* segs, int32_t nseg, int32_t total_blocks, const int64_t* xbuf, float* w,
                               float* a, float* g, float lr, float mu, float* loss, int64_t loss_off, int32_t loss_n,
                               void* stream) {
  if (nseg <= 0 || nseg > 256 || total_blocks <= 0 || !xbuf || !w || !a || (loss && loss_n <= 0)) return LBT_EINVAL;
  hipLaunchKernelGGL(step_finish_kernel, dim3((unsigned)total_blocks), dim3(256), 0, (hipStream_t)stream, segs, nseg,
                     xbuf, w, a, g, lr, mu, loss, loss_off, loss_n);
  return (int)hipGetLastError();
}

extern "C" int lbt_dfxp_range_update_x(int32_t* exps, const int64_t* xbuf, int64_t cnt_off, const int32_t* bits,
                                       const float* target, const float* nelem, int32_t nslots, uint64_t* step,
                                       void* stream) {
  if (nslots < 0 || !xbuf || cnt_off < 0) return LBT_EINVAL;
  const int blocks = nslots > 0 ? (nslots + 255) / 256 : 1;
  hipLaunchKernelGGL(range_update_x_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, exps, xbuf, cnt_off, bits,
                     target, nelem, nslots, step);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_param_grads_many(const lbt_pjob* jobs, int32_t njobs, int32_t max_c, void* stream) {
  if (njobs <= 0) return LBT_OK;
  if (njobs > 65535 || max_c <= 0) return LBT_EINVAL;
  hipLaunchKernelGGL(param_grads_many_kernel, dim3((max_c + 255) / 256, njobs), dim3(256), 0, (hipStream_t)stream,
                     jobs);
  return (int)hipGetLastError();
}

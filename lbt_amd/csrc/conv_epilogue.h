// conv_epilogue.h -- the quantising epilogue shared by the int8 MFMA convolutions and the
// fp16-MFMA stem convolution: the Normalization_q input quantiser (dynamic_fixed_point.py:
// 575-590 -> :26-38) fused into the producing GEMM.
//
// Each wave has written its 16 x (16*ntw) fp32 output tile into its own LDS tile; the tile is
// re-read so that each lane owns 4 CONSECUTIVE channels of one row: one Philox call per 4
// outputs (its 4 noise indices share a Philox block), char4 stores, and exact per-channel sums
// (S1 = sum q, S2 = sum q^2) reduced across the lanes sharing a channel quad, then LDS, then
// one shard of the global sums; overflow counters likewise.  Noise index of output (row, col)
// = (row mod Ho*Wo) * ncol + col: the reference's noise over X.shape[1:].
#pragma once
#include "dfxp_device.h"

namespace lbt {

struct QOut {
  int8_t* yq;       // [M][ncol] int8 codes
  lbt_qdesc q;
  int64_t* chsum;   // sharded [LBT_NSHARD][2*ncol] or NULL
  int64_t M;
  int ncol;
  int64_t HWo;
};

// Make this wave's LDS tile writes visible to the wave (the tile is wave-private).
LBT_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Every thread of the block calls it. sh_sum (2*ncol long long) must have been zeroed and the
// zeroing made visible (barrier) before any wave got here; sh_cnt holds 2 ints per wave.
LBT_DEV void quant_epilogue(const QOut& o, float (*tile)[33], bool wave_live, int64_t mtile, int nt0, int ntw,
                            long long* sh_sum, int* sh_cnt) {
  const int lane = threadIdx.x & 63;
  const QState qs = qstate(o.q);
  const bool want_sum = o.chsum != nullptr;
  int ov1 = 0, ov2 = 0;
  const int quads = 4 * ntw;  // channel quads per row of this wave's tile
  int s1[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, s2[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass >= ntw) continue;
    const int id = pass * 64 + lane;
    const int rr = id / quads, cq = id - rr * quads;
    const int64_t row = mtile * 16 + rr;
    if (!wave_live || row >= o.M) continue;
    const int col0 = nt0 * 16 + cq * 4;
    const uint32_t pix = (uint32_t)row % (uint32_t)o.HWo;  // M < 2^31 (checked by the launchers)
    const Noise4 n = o.q.stochastic ? qnoise4(o.q, qs.step, ((uint64_t)pix * o.ncol + col0) >> 2)
                                    : Noise4{{0.f, 0.f, 0.f, 0.f}};
    char4 w;
    int c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c[k] = quant1(qs, o.q.stochastic, tile[rr][cq * 4 + k], n.u[k], ov1, ov2);
      s1[pass][k] = c[k];
      s2[pass][k] = c[k] * c[k];
    }
    w.x = (int8_t)c[0]; w.y = (int8_t)c[1]; w.z = (int8_t)c[2]; w.w = (int8_t)c[3];
    *reinterpret_cast<char4*>(o.yq + row * o.ncol + col0) = w;
  }
  if (want_sum) {
    // lanes with equal (lane % quads) hold the same channel quad: xor-reduce over quads..32
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (pass >= ntw) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int a1 = s1[pass][k], a2 = s2[pass][k];
        for (int off = quads; off < 64; off <<= 1) {
          a1 += __shfl_xor(a1, off, 64);
          a2 += __shfl_xor(a2, off, 64);
        }
        const int cq = (pass * 64 + lane) % quads;
        if (wave_live && lane < quads) {
          const int ch = nt0 * 16 + cq * 4 + k;
          if (a1) atomicAdd((unsigned long long*)&sh_sum[ch], (unsigned long long)(long long)a1);
          if (a2) atomicAdd((unsigned long long*)&sh_sum[o.ncol + ch], (unsigned long long)(long long)a2);
        }
      }
    }
  }
  if (o.q.counts) counts_stage(0, 1, ov1, ov2, sh_cnt);
  if (!(want_sum || o.q.counts)) return;
  __syncthreads();  // one barrier publishes counters and channel sums
  counts_publish(0, 1, o.q, sh_cnt);
  if (want_sum) block_flush_sums(sh_sum, 2 * o.ncol, o.chsum, 2 * o.ncol);
}

}  // namespace lbt

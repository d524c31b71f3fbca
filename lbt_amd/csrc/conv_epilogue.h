// conv_epilogue.h -- the quantising epilogue shared by the int8 MFMA convolutions and the
// fp16-MFMA stem convolution: the Normalization_q input quantiser (dynamic_fixed_point.py:
// 575-590 -> :26-38) fused into the producing GEMM, working directly on the accumulator layout.
//
// Block = 4 waves; the GEMM's NT 16-column tiles are spread over WPM = min(NT, 4) waves (NTW
// tiles each) and a block covers MTB = 4 / WPM 16-row tiles.  In a 16x16 MFMA accumulator lane l
// holds column l&15 of rows 4*(l>>4) + i, i < 4, so each lane quantises 4 * NTW outputs of ONE
// column per tile: noise u[(row mod Ho*Wo) * ncol + col] (the reference's noise over
// X.shape[1:]) comes from the quantiser's per-step table and is PREFETCHED with the GEMM
// operands; the exact per-channel sums (S1 = sum q, S2 = sum q^2) reduce in registers (rows of
// the lane, then xor-16 / xor-32 across the lanes of the column), each wave parks its column
// totals in LDS with plain stores, and ONE barrier later every counter and channel sum of the
// block is published with one atomic per (channel, sum) into the block's shard.
#pragma once
#include "dfxp_device.h"

namespace lbt {

struct QOut {
  int8_t* yq;       // [M][ncol] int8 codes
  lbt_qdesc q;
  int64_t* chsum;   // sharded [LBT_NSHARD][2*ncol] or NULL
  int64_t M;        // < 2^31
  int ncol;
  int64_t HWo;
};

template <int NT>
struct EpiGeom {
  static constexpr int WPM = NT < 4 ? NT : 4;  // waves per 16-row tile
  static constexpr int NTW = NT / WPM;         // 16-column tiles per wave
  static constexpr int MTB = 4 / WPM;          // 16-row tiles per block
};

// LDS a block needs for the epilogue
template <int NT>
struct EpiShared {
  int cnt[2 * 4];                          // counters staged per wave
  int part[4][2][16 * EpiGeom<NT>::NTW];   // per wave: S1 / S2 of its columns
};

// Noise of this lane's outputs (rows mtile*16 + 4*kg + i, columns (nt0 + j)*16 + r), from the
// quantiser's per-step table (a stochastic quantising epilogue requires one: see the header).
template <int NTW>
LBT_DEV void epi_noise(const QOut& o, int64_t mtile, int nt0, int lane, float (&u)[NTW][4]) {
  const int r = lane & 15, kg = lane >> 4;
  const bool tab = o.q.stochastic && o.q.noise;   // else quant1 ignores u: read zeros
  const float* src = tab ? o.q.noise : zf();
  const uint32_t mask = tab ? 0xffffffffu : 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = mtile * 16 + 4 * kg + i;
    const uint32_t pix = (uint32_t)(row < o.M ? row : 0) % (uint32_t)o.HWo;
#pragma unroll
    for (int j = 0; j < NTW; ++j) u[j][i] = src[(pix * (uint32_t)o.ncol + (nt0 + j) * 16 + r) & mask];
  }
}

// Quantise + store + publish. v holds the fp32 outputs (acc * scale) of this lane. Every thread
// of the block calls it (one barrier).
template <int NT>
LBT_DEV void epi_quant(const QOut& o, const QState& qs, int64_t mtile, int nt0, int wave, int lane,
                       const float (&v)[EpiGeom<NT>::NTW][4], const float (&u)[EpiGeom<NT>::NTW][4],
                       EpiShared<NT>& sh) {
  constexpr int NTW = EpiGeom<NT>::NTW, WPM = EpiGeom<NT>::WPM, MTB = EpiGeom<NT>::MTB;
  const int r = lane & 15, kg = lane >> 4;
  int ov1 = 0, ov2 = 0;
  int s1[NTW], s2[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    s1[j] = 0;
    s2[j] = 0;
    const int col = (nt0 + j) * 16 + r;
    int cc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = mtile * 16 + 4 * kg + i;
      cc[i] = 0;
      if (row < o.M) {
        const int c = quant_w<-1>(qs, o.q.stochastic, v[j][i], u[j][i], ov1, ov2);
        cc[i] = c;
        s1[j] += c;
        s2[j] += c * c;
      }
    }
    // the 4 lanes of a column quad swap codes so lane r stores row 4 kg + (r & 3)'s 4 columns as one
    // write-through dword (the next launch reads them) instead of 4 scattered byte stores
    const uint32_t packed = quad_pack_codes(cc, r & 3);
    const int64_t rowp = mtile * 16 + 4 * kg + (r & 3);
    if (rowp < o.M) st_out(o.yq + (uint32_t)rowp * (uint32_t)o.ncol + (col & ~3), (int)packed);  // M * ncol < 2^31
  }
  const bool want_sum = o.chsum != nullptr;
  if (want_sum) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      // lanes r, r+16, r+32, r+48 share a column: row 0 ends with s1's total, row 1 with s2's
      const int t = rows_scatter2(s1[j], s2[j]);
      if (kg < 2) sh.part[wave][kg][j * 16 + r] = t;
    }
  }
  if (o.q.counts) counts_stage_w(0, 1, ov1, ov2, sh.cnt);  // wave totals (quant_w)
  if (!(want_sum || o.q.counts)) return;
  __syncthreads();  // the only barrier: counters and channel sums of the whole block
  counts_publish(0, 1, o.q, sh.cnt);
  if (want_sum) {
    const int t = threadIdx.x;
    if (t < 2 * o.ncol) {
      const int which = t >= o.ncol, col = t - which * o.ncol;
      const int wcol = (col >> 4) / NTW;           // which wave column-group covers col
      const int lc = col - wcol * NTW * 16;        // its column within that wave
      long long tot = 0;
#pragma unroll
      for (int mt = 0; mt < MTB; ++mt) {
        const int64_t row0 = (mtile - wave / WPM + mt) * 16;  // the block's first m-tile from this wave's
        if (row0 < o.M) tot += sh.part[mt * WPM + wcol][which][lc];
      }
      if (tot) LBT_GADD((unsigned long long*)&o.chsum[(int64_t)shard_id() * 2 * o.ncol + t], (unsigned long long)tot);
    }
  }
}

}  // namespace lbt

// ============================================================================ pass-A epilogue
// Pass A of the BatchNorm backward (bn.hip chain_bwd_a_kernel: ReLU mask, Rescale_q grad
// quantiser + dgamma/dbeta sums, Normalization_q grad quantiser + its sums) applied to a dgrad
// GEMM's outputs, so the fp32 gradient never goes to memory. Same arithmetic, element for
// element, as the chain kernel; the lane owns one column (channel) of 4 * NTW outputs.
#include "chain_flags.h"

namespace lbt {

template <int NT, int NB>
struct ChainShared {
  int cnt[2 * 4 * 4];                              // counters: 4 quantisers x 4 waves
  int part[4][NB][4][16 * EpiGeom<NT>::NTW];       // per wave: the 4 channel sums per branch
};

// Operands of this lane's outputs, fetched with the GEMM operands (every load unconditional).
template <int NT, int NB, int CF>
struct ChainPre {
  static constexpr int NTW = EpiGeom<NT>::NTW;
  float add[NTW][4], ym[NTW][4];
  int R[NB][NTW][4], qn[NB][NTW][4];
  float urg[NB][NTW][4], ung[NB][NTW][4];
  float gam[NB][NTW], bet[NTW];
};

template <int NT, int NB, int CF>
LBT_DEV void chain_prefetch(const lbt_chain_bwd_a& c, const float* add_src, int64_t M, int ncol, uint32_t HW,
                            int64_t mtile, int nt0, int lane, ChainPre<NT, NB, CF>& p) {
  constexpr int NTW = EpiGeom<NT>::NTW;
  const int r = lane & 15, kg = lane >> 4;
  const float* as = add_src ? add_src : zf();
  const uint32_t amask = add_src ? 0xffffffffu : 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = mtile * 16 + 4 * kg + i;
    const int64_t rr = row < M ? row : 0;
    const uint32_t pix = (uint32_t)rr % HW;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int col = (nt0 + j) * 16 + r;
      const uint32_t e = (uint32_t)rr * (uint32_t)ncol + col;  // M * ncol < 2^31 (launcher)
      const uint32_t ni = pix * (uint32_t)ncol + col;
      p.add[j][i] = as[e & amask];
      if (CF & kAYMask) p.ym[j][i] = c.y_mask[e];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const lbt_bwd_branch& B = b == 0 ? c.b1 : c.b2;
        p.R[b][j][i] = B.R[e];
        p.qn[b][j][i] = B.qn_codes[e];
        p.urg[b][j][i] = B.qrg.noise[ni];
        p.ung[b][j][i] = B.qng.noise[ni];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int col = (nt0 + j) * 16 + r;
#pragma unroll
    for (int b = 0; b < NB; ++b) p.gam[b][j] = (b == 0 ? c.b1 : c.b2).gb[col];
    p.bet[j] = c.b1.gb[ncol + col];
  }
}

// v: this lane's dgrad outputs (fp32, exactly the unfused kernel's dx values). Every thread of
// the block calls it (one barrier).
template <int NT, int NB, int CF>
LBT_DEV void chain_epi(const lbt_chain_bwd_a& c, bool has_add, int64_t M, int ncol, int64_t mtile, int nt0, int wave,
                       int lane, const float (&v)[EpiGeom<NT>::NTW][4], const ChainPre<NT, NB, CF>& p,
                       ChainShared<NT, NB>& sh) {
  constexpr int NTW = EpiGeom<NT>::NTW, WPM = EpiGeom<NT>::WPM, MTB = EpiGeom<NT>::MTB;
  constexpr int ST = (CF & kAStoch) ? 1 : 0;
  const int r = lane & 15, kg = lane >> 4;
  QState qrg[2], qng[2];
  float r_inv = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& B = b == 0 ? c.b1 : c.b2;
    qrg[b] = qstate(B.qrg);
    qng[b] = qstate(B.qng);
  }
  if (CF & kAMaskR) r_inv = qstate(c.b1.qr).inv_m;
  int ov[2][2][2] = {{{0, 0}, {0, 0}}, {{0, 0}, {0, 0}}};  // wave totals
  int acc[NB][NTW][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[b][j][s] = 0;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int col = (nt0 + j) * 16 + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = mtile * 16 + 4 * kg + i;
      if (row >= M) continue;
      const uint32_t e = (uint32_t)row * (uint32_t)ncol + col;
      float g = has_add ? v[j][i] + p.add[j][i] : v[j][i];
      if (CF & kAYMask) {
        g = p.ym[j][i] > 0.f ? g : 0.f;
      } else if (CF & kAMaskR) {
        const float xr = (float)p.R[0][j][i] * r_inv;
        const float m1 = xr * p.gam[0][j];
        const float yv = m1 + p.bet[j];
        g = yv > 0.f ? g : 0.f;
      }
      if (CF & kAGmask) c.gmask_out[e] = g;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const lbt_bwd_branch& B = b == 0 ? c.b1 : c.b2;
        const int G2 = quant_w<ST>(qrg[b], B.qrg.stochastic, g, p.urg[b][j][i], ov[b][0][0], ov[b][0][1]);
        acc[b][j][0] += G2 * p.R[b][j][i];
        acc[b][j][1] += G2;
        const float gh = (float)G2 * qrg[b].inv_m;
        const float d = gh * p.gam[b][j];
        const int G = quant_w<ST>(qng[b], B.qng.stochastic, d, p.ung[b][j][i], ov[b][1][0], ov[b][1][1]);
        acc[b][j][2] += G;
        acc[b][j][3] += G * p.qn[b][j][i];
        B.gout[e] = (int8_t)G;
      }
    }
  }
  // column totals: lanes r, r+16, r+32, r+48 share a column
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      // row kg ends with sum kg's column total (rows_scatter4)
      sh.part[wave][b][kg][j * 16 + r] = rows_scatter4(acc[b][j][0], acc[b][j][1], acc[b][j][2], acc[b][j][3]);
    }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& B = b == 0 ? c.b1 : c.b2;
    if (B.qrg.counts) counts_stage_w(2 * b, 4, ov[b][0][0], ov[b][0][1], sh.cnt);
    if (B.qng.counts) counts_stage_w(2 * b + 1, 4, ov[b][1][0], ov[b][1][1], sh.cnt);
  }
  __syncthreads();  // the only barrier
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& B = b == 0 ? c.b1 : c.b2;
    counts_publish(2 * b, 4, B.qrg, sh.cnt);
    counts_publish(2 * b + 1, 4, B.qng, sh.cnt);
  }
  // sums layout per shard: [4][C] (G2*R, G2, G, G*q) -- as chain_bwd_a's S
  for (int t = threadIdx.x; t < NB * 4 * ncol; t += 256) {
    const int b = t / (4 * ncol), rem = t - b * 4 * ncol, s = rem / ncol, col = rem - s * ncol;
    const int wcol = (col >> 4) / NTW, lc = col - wcol * NTW * 16;
    long long tot = 0;
#pragma unroll
    for (int mt = 0; mt < MTB; ++mt) tot += sh.part[mt * WPM + wcol][b][s][lc];
    int64_t* dst = (b == 0 ? c.b1 : c.b2).sums;
    if (tot) LBT_GADD((unsigned long long*)&dst[(int64_t)shard_id() * 4 * ncol + rem], (unsigned long long)tot);
  }
}

}  // namespace lbt

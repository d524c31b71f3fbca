// igemm.hip -- LDS-tiled int8 MFMA implicit GEMM for the wide layers (ResNet-50 shapes, SURVEY 8(f)
// rank 1): channel counts that are multiples of 64 on the gathered side and of 16 on the output
// side, any count (conv_mfma.hip's register-resident kernels take <= 128 channels).
//
//   fwd   : y[m = (n,oh,ow)][co] = sum_{tap,ci} x[n, oh*S+kh-P, ow*S+kw-P, ci] * W[tap][ci][co]
//   dgrad : dx[m = (n,ih,iw)][ci] = sum_{tap,co} g[n, (ih+P-kh)/S, (iw+P-kw)/S, co] * W[tap][ci][co]
//                                   (taps whose position is not an output pixel contribute 0)
// B = the packed weight image of lbt_dfxp_quantize_weight ([col][k], k = (tap, 16-channel slice)).
//
// Workgroup tile 128 rows x 128 columns, 4 waves of 64 x 64 (4 x 4 v_mfma_i32_16x16x64_i8 tiles),
// k-blocks of 64 = one tap x 64 channels; operands staged through double-buffered LDS: the next
// k-block's global loads are in flight while the current one is multiplied.
//
// A16: the gathered operand is int16 codes (9..16-bit: the signed 9-bit image of a Conv2d_q input
// or 16-bit gradient codes, config 4). Each code is split a = 256*hi + lo' + 128 with hi, lo' int8,
// so sum a*w = 256 sum hi*w + sum lo'*w + 128 sum w: two int8 MFMA passes, plus one against an
// all-ones A fragment for sum_k w per column; combined exactly in int64 in the epilogue. Positions
// outside the image (a = 0) are (hi, lo') = (0, -128), which the identity keeps exact.
// A8: int8 codes, either signed (fill 0) or offset-by-128 ("u8off", fill -128, + 128 sum_k w).
#include "dfxp_device.h"
#include "lds_tr.h"
#include "pk2.h"

#include <cstdlib>
#include <type_traits>

namespace {

using namespace lbt;

// tuning knobs read once per process (experiments; the defaults are the measured choice)
int getenv_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

constexpr int kT = 256, kBM = 128, kBN = 128, kBK = 64;
constexpr int kRow = kBK + 16;  // LDS row stride in bytes (16-byte pad staggers the banks)

enum { MODE_FWD = 0, MODE_DGRAD = 1 };

struct IgArgs {
  const void* a;        // x codes (fwd) or g codes (dgrad), NHWC
  const int8_t* b;      // packed weight image [ncol][ks * 16]
  int ks;               // 16-byte slices per column
  int cred;             // channels of the gathered operand (multiple of 64)
  int a_u8off;          // A8 only: codes are q - 128
  lbt_conv_desc d;
  lbt_qdesc qa, qb;
  const int32_t* colsum;  // A8 u8off: sum_k W per column (the wcolsum of the fwd image)
  float* y;
  const float* add_src;
  int64_t M;
  int ncol;
  // split-K: blockIdx.z = split, each taking nk / ksplit consecutive k-blocks and STORING its exact
  // int32 partial sums (A8: one component; A16: hi and lo' + 128 sum W) into part[split][comp][M][ncol];
  // igemm_splitk_reduce_kernel adds the splits and runs the epilogue (ksplit == 1: none of this)
  int ksplit;
  int32_t* part;
  // fwd only, ksplit == 1: the epilogue is the consuming Normalization_q's input quantiser --
  // int8 codes yq, overflow counters of qout, exact per-channel sums chsum[NSHARD][2 * ncol]
  // (sum q, sum q^2); noise index = (row % hw) * ncol + col (noise over shape[1:]); y unused
  int8_t* yq;
  lbt_qdesc qout;
  int64_t* chsum;
  int hw;
  // taps of the k loop: dgrad kh = kh0 + SH * th (th < nkh), kw likewise (fwd and unit-stride dgrad:
  // every tap, kh = th). Strided dgrad runs one launch per parity class (cpy, cpx) of the dx pixels, whose rows are
  // (n, yc, xc) -> (n, yc * SH + cpy, xc * SW + cpx) over a ch x cw grid: only the taps with
  // (ih + PT - kh) % SH == 0 reach such a pixel, and for them the source row is yc + oy - th (no
  // zero rows, no division in the loop).
  int nkh, nkw, kh0, kw0, oy, ox, ch, cw, cpy, cpx;
  // dgrad, A16, 256-row kernel only (has_bna): the BN pass A this dx feeds (lbt_dgrad_bna), run in the
  // epilogue instead of storing dx (bna_epilogue)
  int has_bna;  // 1: bna (mask_r), 2: bn3 (g2 + y_bits, bn3.nbn BNs); sample-blocked row tiles (PERM)
  int npb;      // PERM: 16-pixel blocks per sample
  int perm;     // sample-blocked row tiles (the pass-A epilogues, the PERM quantising forward epilogue)
  lbt_dgrad_bna bna;
  lbt_dgrad_bn3 bn3;
  int dbg;  // igemm_big_kernel diagnostics (LBT_IGEMM_BIG_DBG; 1: no operand loads after the prologue)
};

// every tap, rows = every output pixel (fwd, unit-stride dgrad)
void all_taps(IgArgs& p, int mode) {
  const lbt_conv_desc& d = p.d;
  p.nkh = d.KH; p.nkw = d.KW; p.kh0 = 0; p.kw0 = 0;
  p.oy = d.PT; p.ox = d.PL;
  p.ch = mode == MODE_FWD ? d.Ho : d.H;
  p.cw = mode == MODE_FWD ? d.Wo : d.W;
  p.cpy = 0; p.cpx = 0;
}

// The conv-output quantiser in the GEMM epilogue (fwd, A8). Lane (r, q) holds column cw + 16 j + r
// of rows rtile + 16 i + e. Noise: one Philox4x32 call yields the 4 values of 4 consecutive channels
// of one pixel, so the 4 lanes r = 4g .. 4g+3 each draw the block of one of their 4 rows (e = r & 3)
// and pass values round in 4 shuffle steps -- one Philox call per 4 outputs, the same values as
// quantize_rows_kernel's qnoise4 of that block. Rows past M quantise 0 (no overflow, code 0).
template <int MI, int NJ>
LBT_DEV void quant_epilogue(const IgArgs& p, const v4i (&acc)[MI][NJ], const v4i (&accw)[NJ], int u8, float scale,
                            int64_t rtile, int rlim, bool full, int cw, int r, int q) {
  const QState qs = qstate(p.qout);
  const int ncol = p.ncol;
  const int jj = r & 3;  // this lane's slot in its 4-lane group
  int ov1w = 0, ov2w = 0;
  int cs1[NJ], cs2[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) { cs1[j] = 0; cs2[j] = 0; }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    // the pixel (within its image) of row e = jj of this i: this lane draws its noise block
    const int64_t myrow = rtile + i * 16 + jj;
    const uint32_t pix = (uint32_t)((myrow < p.M ? myrow : 0) % (uint32_t)p.hw);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = cw + j * 16 + r;
      if (cw + j * 16 >= ncol) continue;  // uniform
      const uint64_t blk = ((uint64_t)pix * (uint32_t)ncol + (uint32_t)(col & ~3)) >> 2;
      Noise4 mine = {{0.f, 0.f, 0.f, 0.f}};
      if (p.qout.stochastic) mine = qnoise4(p.qout, qs.step, blk);
      float u[4] = {0.f, 0.f, 0.f, 0.f};
      // step k: lane jj sends its block's value for column (jj - k) & 3 of the group and
      // receives, from lane (jj + k) & 3, the value of this lane's column for row (jj + k) & 3
      auto noise_step = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const int sc = (jj - k) & 3;
        const float send = sc == 0 ? mine.u[0] : sc == 1 ? mine.u[1] : sc == 2 ? mine.u[2] : mine.u[3];
        const float got = quad_from<k>(send);
        const int re = (jj + k) & 3;
        u[0] = re == 0 ? got : u[0];
        u[1] = re == 1 ? got : u[1];
        u[2] = re == 2 ? got : u[2];
        u[3] = re == 3 ? got : u[3];
      };
      noise_step(std::integral_constant<int, 0>{});
      noise_step(std::integral_constant<int, 1>{});
      noise_step(std::integral_constant<int, 2>{});
      noise_step(std::integral_constant<int, 3>{});
      const int wsum = accw[j][0];
      int cc[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = full || i * 16 + e < rlim;
        const float v = ok ? (float)(acc[i][j][e] + u8 * wsum) * scale : 0.f;
        const int c = quant_w<-1>(qs, p.qout.stochastic, v, u[e], ov1w, ov2w);
        cc[e] = c;
        cs1[j] += c;
        cs2[j] += c * c;
      }
      // the same 4-lane transpose on the codes: lane jj collects row jj's codes of the group's 4
      // columns and stores them as one dword
      const uint32_t packed = quad_pack_codes(cc, jj);
      if (full || i * 16 + jj < rlim)
        *reinterpret_cast<uint32_t*>(p.yq + (rtile + i * 16 + jj) * ncol + (col & ~3)) = packed;
    }
  }
  // per-column sums: the 4 q-lanes of a column meet by shuffles, then one int64 atomic per column
  // and sum into this workgroup's shard; overflow counters: wave totals, one atomic each
  const int shard = (int)((blockIdx.x + blockIdx.y * 7u) % LBT_NSHARD);
  int64_t* cs = p.chsum + (int64_t)shard * 2 * ncol;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    // row 0 ends with the column's code sum, row 1 with its sum of squares (rows_scatter2)
    const int t = rows_scatter2(cs1[j], cs2[j]);
    const int col = cw + j * 16 + r;
    if (q < 2 && cw + j * 16 < ncol && t) atomicAdd((unsigned long long*)&cs[q * ncol + col], (unsigned long long)(long long)t);
  }
  if ((threadIdx.x & 63) == 0 && p.qout.counts) {
    int32_t* ct = p.qout.counts + ((int64_t)p.qout.slot * LBT_NSHARD + shard) * LBT_CSTRIDE;
    if (ov1w) atomicAdd(ct, ov1w);
    if (ov2w) atomicAdd(ct + 1, ov2w);
  }
}

// BM x BN workgroup tile (64 or 128 each), 2 x 2 waves of (BM/2) x (BN/2): MI x NJ MFMA tiles
template <int MODE, bool A16, bool ADD, int BM, int BN, int D, bool CLS>
__global__ __launch_bounds__(kT) void igemm_kernel(IgArgs p) {
  constexpr int NA = A16 ? 2 : 1;  // A tiles per k-block: (hi, lo') or one
  constexpr int HA = BM / 64, HB = BN / 64;  // 64-row loader passes of A / B
  constexpr int MI = BM / 32, NJ = BN / 32;  // 16x16 tiles per wave
  __shared__ __attribute__((aligned(16))) int8_t sA[2][NA][BM * kRow];
  __shared__ __attribute__((aligned(16))) int8_t sB[2][BN * kRow];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const lbt_conv_desc& d = p.d;
  const int OH = p.ch, OW = p.cw;  // the row grid (dgrad parity class: its ch x cw pixels)
  const int SH = MODE == MODE_FWD ? d.H : d.Ho, SW = MODE == MODE_FWD ? d.W : d.Wo;
  const int cblocks = p.cred / kBK, nk_all = p.nkh * p.nkw * cblocks;
  const int nk = nk_all / p.ksplit, kbase = (int)blockIdx.z * nk;  // this split's k-blocks

  // ---- loader roles: A rows (t >> 2) and (t >> 2) + 64, 16-byte segment (t & 3) of the 64 channels
  // (A16: 32-byte segments = 16 codes); B columns likewise
  const int lr = t >> 2, seg = t & 3;
  int an[HA], ay[HA], ax[HA];
  bool arow[HA];
#pragma unroll
  for (int h = 0; h < HA; ++h) {
    const int64_t m = m0 + lr + 64 * h;
    arow[h] = m < p.M;
    const uint32_t mu = (uint32_t)(arow[h] ? m : 0);
    ax[h] = (int)(mu % (uint32_t)OW);
    const uint32_t tt = mu / (uint32_t)OW;
    ay[h] = (int)(tt % (uint32_t)OH);
    an[h] = (int)(tt / (uint32_t)OH);
  }
  // global -> register stage of one k-block
  // D register stages: the global loads of k-block b land in stage b % D, D k-blocks ahead of use
  v4i ra[D][HA][A16 ? 2 : 1], rb[D][HB];
  bool rv[D][HA];
  auto load_k = [&](int kbl, int st) {
    const int kb = kbase + kbl;
    const int tap = kb / cblocks, cb = kb - tap * cblocks;
    const int th = tap / p.nkw, tw = tap - th * p.nkw;
    const int kh = MODE == MODE_FWD ? th : p.kh0 + d.SH * th, kw = MODE == MODE_FWD ? tw : p.kw0 + d.SW * tw;
    const int kbw = (kh * d.KW + kw) * cblocks + cb;  // the weight image's k-block
#pragma unroll
    for (int h = 0; h < HA; ++h) {
      int sy, sx;
      if (MODE == MODE_FWD) {
        sy = ay[h] * d.SH + kh - d.PT;
        sx = ax[h] * d.SW + kw - d.PL;
      } else {  // ih = yc * SH + cpy: (ih + PT - kh) / SH = yc + oy - th exactly
        sy = ay[h] + p.oy - th;
        sx = ax[h] + p.ox - tw;
      }
      const bool ok = (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW && arow[h];
      rv[st][h] = ok;
      // 32-bit element offsets (launcher: every operand < 2^31 elements)
      const uint32_t pix = ok ? (uint32_t)((an[h] * SH + sy) * SW + sx) : 0u;
      if constexpr (A16) {
        const int16_t* src = reinterpret_cast<const int16_t*>(p.a) + (pix * (uint32_t)p.cred + (uint32_t)(cb * kBK + seg * 16));
        ra[st][h][0] = *reinterpret_cast<const v4i*>(src);
        ra[st][h][1] = *reinterpret_cast<const v4i*>(src + 8);
      } else {
        const int8_t* src = reinterpret_cast<const int8_t*>(p.a) + (pix * (uint32_t)p.cred + (uint32_t)(cb * kBK + seg * 16));
        ra[st][h][0] = *reinterpret_cast<const v4i*>(src);
      }
    }
#pragma unroll
    for (int h = 0; h < HB; ++h) {
      const int col = n0 + lr + 64 * h;
      const int colc = col < p.ncol ? col : 0;
      rb[st][h] = *reinterpret_cast<const v4i*>(p.b + ((uint32_t)(colc * p.ks + kbw * 4 + seg) << 4));
      if (col >= p.ncol) rb[st][h] = v4i{0, 0, 0, 0};
    }
  };
  auto store_k = [&](int buf, int st) {
#pragma unroll
    for (int h = 0; h < HA; ++h) {
      const int row = lr + 64 * h;
      if constexpr (A16) {
        // 16 codes -> 16 hi bytes and 16 lo' bytes (a = 256 hi + lo' + 128); outside: (0, -128)
        int hi[4], lo[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const uint32_t c01 = (uint32_t)ra[st][h][w >> 1][(w & 1) * 2], c23 = (uint32_t)ra[st][h][w >> 1][(w & 1) * 2 + 1];
          // codes (int16) e0 e1 | e2 e3; hi = arithmetic >> 8 (the high byte), lo' = low byte ^ 0x80
          hi[w] = (int)__builtin_amdgcn_perm(c23, c01, 0x07050301u);
          lo[w] = (int)(__builtin_amdgcn_perm(c23, c01, 0x06040200u) ^ 0x80808080u);
          if (!rv[st][h]) { hi[w] = 0; lo[w] = (int)0x80808080u; }
        }
        *reinterpret_cast<v4i*>(&sA[buf][0][row * kRow + seg * 16]) = v4i{hi[0], hi[1], hi[2], hi[3]};
        *reinterpret_cast<v4i*>(&sA[buf][1][row * kRow + seg * 16]) = v4i{lo[0], lo[1], lo[2], lo[3]};
      } else {
        const int fill = p.a_u8off ? (int)0x80808080u : 0;
        v4i v = ra[st][h][0];
        if (!rv[st][h]) v = v4i{fill, fill, fill, fill};
        *reinterpret_cast<v4i*>(&sA[buf][0][row * kRow + seg * 16]) = v;
      }
    }
#pragma unroll
    for (int h = 0; h < HB; ++h) *reinterpret_cast<v4i*>(&sB[buf][(lr + 64 * h) * kRow + seg * 16]) = rb[st][h];
  };

  v4i acc[NA][MI][NJ], accw[NJ];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[a][i][j] = v4i{0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < NJ; ++j) accw[j] = v4i{0, 0, 0, 0};
  const v4i ones = v4i{0x01010101, 0x01010101, 0x01010101, 0x01010101};
  const bool want_w = A16 || p.a_u8off;  // sum_k W per column (the +128 term)

  // prologue: block 0 into LDS[0], blocks 1 .. D in flight (stage b % D). nk % D == 0 (launcher) and
  // every load / store below is unconditional (block indices clamped, a stale store into the buffer
  // nobody reads any more is harmless): straight-line code, so the compiler's wait counts let the
  // younger stages stay in flight instead of draining them (vmcnt(0)) at every branch
  load_k(0, 0);
  store_k(0, 0);
#pragma unroll
  for (int b = 1; b <= D; ++b) load_k(b < nk ? b : nk - 1, b % D);
  __syncthreads();
  const int r = lane & 15, q = lane >> 4;
  for (int kb0 = 0; kb0 < nk; kb0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {  // kb0 % D == 0: stage indices below are compile-time
      const int kb = kb0 + u;
      const int cur = kb & 1;
      v4i bf[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bf[j] = *reinterpret_cast<const v4i*>(&sB[cur][(wn * (BN / 2) + j * 16 + r) * kRow + q * 16]);
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const v4i af = *reinterpret_cast<const v4i*>(&sA[cur][a][(wm * (BM / 2) + i * 16 + r) * kRow + q * 16]);
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[a][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[j], acc[a][i][j], 0, 0, 0);
        }
      if (want_w) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) accw[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, bf[j], accw[j], 0, 0, 0);
      }
      const int st = (u + 1) % D;  // block kb + 1's stage
      store_k(cur ^ 1, st);  // the other buffer: its readers finished before the last barrier
      load_k(kb + 1 + D < nk ? kb + 1 + D : nk - 1, st);
      __syncthreads();
    }
  }

  // ---- epilogue: lane owns column (tile col + r), rows (tile row + 4q + e). Index math kept
  // off the per-element path: one 64-bit base per column tile, 32-bit row offsets, row checks only
  // on the last (ragged) tile; A8 sums fit int32 (launcher: K * 255 * 128 < 2^31), A16 sums are
  // formed exactly in double (|s| < 2^53) and rounded once to fp32 -- the same value as
  // (float)(int64) s.
  const float scale = ldexpf(1.0f, -(frac_exp(p.qa) + frac_exp(p.qb)));
  constexpr bool addv = MODE == MODE_DGRAD && ADD;
  const int ncol = p.ncol;
  const int64_t rtile = m0 + wm * (BM / 2) + q * 4;  // + i * 16 + e
  const bool full = m0 + BM <= p.M;
  const int rlim = full ? (BM / 2) : (int)(p.M - rtile);  // rows (i * 16 + e) < rlim are real
  const int u8 = p.a_u8off ? 128 : 0;
  if (p.ksplit > 1) {  // uniform: store this split's exact partials
    const int64_t plane = p.M * ncol;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int ctile = n0 + wn * (BN / 2) + j * 16;
      if (ctile >= ncol) continue;
      const int wsum = want_w ? accw[j][0] : 0;
      int32_t* pp = p.part + (int64_t)blockIdx.z * (A16 ? 2 : 1) * plane + rtile * ncol + ctile + r;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (!(full || i * 16 + e < rlim)) continue;
          if constexpr (A16) {
            pp[(i * 16 + e) * ncol] = acc[0][i][j][e];
            pp[plane + (i * 16 + e) * ncol] = acc[1][i][j][e] + 128 * wsum;
          } else {
            pp[(i * 16 + e) * ncol] = acc[0][i][j][e] + u8 * wsum;
          }
        }
    }
    return;
  }
  if constexpr (MODE == MODE_FWD && !A16) {
    if (p.yq) {  // uniform: quantising epilogue
      quant_epilogue<MI, NJ>(p, acc[0], accw, want_w ? u8 : 0, scale, rtile, rlim, full, n0 + wn * (BN / 2), r, q);
      return;
    }
  }
  if constexpr (CLS) {  // parity-class rows: each row's dx pixel, 32-bit (launcher: dx < 2^31 elements)
    uint32_t roff[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t m = rtile + i * 16 + e;
        const uint32_t mu = (uint32_t)(m < p.M ? m : 0);
        const uint32_t xc = mu % (uint32_t)p.cw, t2 = mu / (uint32_t)p.cw;
        const uint32_t yc = t2 % (uint32_t)p.ch, n = t2 / (uint32_t)p.ch;
        roff[i][e] = ((n * (uint32_t)d.H + yc * (uint32_t)d.SH + (uint32_t)p.cpy) * (uint32_t)d.W +
                      xc * (uint32_t)d.SW + (uint32_t)p.cpx) * (uint32_t)ncol;
      }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int ctile = n0 + wn * (BN / 2) + j * 16;
      if (ctile >= ncol) continue;
      const uint32_t col = (uint32_t)(ctile + r);
      const int wsum = want_w ? accw[j][0] : 0;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (!(full || i * 16 + e < rlim)) continue;
          float v;
          if constexpr (A16) {
            const double hs = (double)acc[0][i][j][e] * 256.0;
            const double ls = (double)(acc[1][i][j][e] + 128 * wsum);
            v = (float)(hs + ls) * scale;
          } else {
            v = (float)(acc[0][i][j][e] + u8 * wsum) * scale;
          }
          if constexpr (addv) v = v + p.add_src[roff[i][e] + col];
          p.y[roff[i][e] + col] = v;
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int ctile = n0 + wn * (BN / 2) + j * 16;
    if (ctile >= ncol) continue;  // uniform: ncol % 16 == 0
    const int col = ctile + r;
    float* yp = p.y + rtile * ncol + col;
    const float* ap = addv ? p.add_src + rtile * ncol + col : nullptr;
    float av[MI][4];
    if constexpr (addv) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) av[i][e] = (i * 16 + e < rlim) ? ap[(i * 16 + e) * ncol] : 0.f;
    }
    const int wsum = want_w ? accw[j][0] : 0;  // every row of accw holds sum_k W[col][k]
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v;
        if constexpr (A16) {
          const double hs = (double)acc[0][i][j][e] * 256.0;  // exact
          const double ls = (double)(acc[1][i][j][e] + 128 * wsum);  // |.| < 2^31: K * 255 * 128 bound
          v = (float)(hs + ls) * scale;  // hs + ls exact (< 2^53): one rounding, as (float)(int64)
        } else {
          v = (float)(acc[0][i][j][e] + u8 * wsum) * scale;
        }
        if (full || i * 16 + e < rlim) yp[(i * 16 + e) * ncol] = addv ? v + av[i][e] : v;
      }
  }
}

// Sum of the split partials + the epilogue of igemm_kernel, element-wise (4 per thread).
template <bool A16, bool ADD>
__global__ __launch_bounds__(256) void igemm_splitk_reduce_kernel(IgArgs p) {
  const int64_t plane = p.M * p.ncol;
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= plane) return;
  const float scale = ldexpf(1.0f, -(frac_exp(p.qa) + frac_exp(p.qb)));
  int4 s0 = make_int4(0, 0, 0, 0), s1 = make_int4(0, 0, 0, 0);
  for (int z = 0; z < p.ksplit; ++z) {
    const int4 a = *reinterpret_cast<const int4*>(p.part + (int64_t)z * (A16 ? 2 : 1) * plane + i4);
    s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
    if constexpr (A16) {
      const int4 b = *reinterpret_cast<const int4*>(p.part + ((int64_t)z * 2 + 1) * plane + i4);
      s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
    }
  }
  const int h[4] = {s0.x, s0.y, s0.z, s0.w}, l[4] = {s1.x, s1.y, s1.z, s1.w};
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if constexpr (A16)
      v[k] = (float)((double)h[k] * 256.0 + (double)l[k]) * scale;  // exact sum, one rounding
    else
      v[k] = (float)h[k] * scale;
  }
  if constexpr (ADD) {
    const float4 a = *reinterpret_cast<const float4*>(p.add_src + i4);
    v[0] = v[0] + a.x; v[1] = v[1] + a.y; v[2] = v[2] + a.z; v[3] = v[3] + a.w;
  }
  *reinterpret_cast<float4*>(p.y + i4) = make_float4(v[0], v[1], v[2], v[3]);
}

// ---------------------------------------------------------------------------- 256-row tiles
// igemm_big_kernel: the same implicit GEMMs (no split-K, no parity classes) on 256-row x BN-column
// workgroup tiles of 8 waves (wave tile (256 / WM) x 64, WM x WN = 8, WN = BN / 64), with BOTH operands
// staged by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, no ds_write pass) through an S-stage
// LDS ring: k-block kb + S - 1 is in flight while kb is multiplied, ordered by a counted vmcnt and a
// raw s_barrier per k-block (a __syncthreads would drain the DMA ring with vmcnt(0)). The DMA writes
// each wave-instruction's 1 KiB lane-linearly, so the bank-conflict swizzle is applied on the SOURCE
// side: 16-byte segment s of row r lands at segment s ^ f(r) (A8 / B: f = (r >> 2) & 3 over 64-byte
// rows; A16: f = (r >> 1) & 7 over 128-byte rows of raw int16 codes, split into hi / lo' on the
// fragment read), and the fragment reads apply the same XOR. Out-of-image taps and rows past M read a
// 16-byte fill block (0, or 0x80 for offset codes).
constexpr int kBT = 512;
static __device__ __attribute__((aligned(16))) uint32_t kFill80[4] = {0x80808080u, 0x80808080u, 0x80808080u,
                                                                      0x80808080u};

template <int N>
LBT_DEV void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((address_space(3))) void* lds_vptr;

// XCD-contiguous logical id of workgroup b of n: the hardware deals workgroups round-robin over the 8
// XCDs, so logical ids [start_x, start_x + count_x) all run on XCD x, in dispatch order (bijective)
LBT_DEV uint32_t xcd_logical(uint32_t b, uint32_t n) {
  const uint32_t x = b % 8, q = n / 8, r = n % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// A 16-byte store that is ALWAYS issued (one vector-memory op on the counter whatever `ok` is): a raw buffer
// store at byte offset off of base (< 2^31), or at an out-of-range offset -- dropped by the buffer range
// check -- when !ok. The persistent kernels count their epilogue stores into the ring's vmcnt waits.
// PRECONDITION (host side): every byte the caller may store lies below 2^31 - 16; an offset past it is
// dropped like a masked one. launch_fwdq_persist checks M * ncol < 2^31 (int8 yq), launch_dgrada_persist
// 2 * rows * Cin < 2^31 (16-bit G); a new caller must check its own bound the same way.
LBT_DEV void st16_always(void* base, uint32_t off, bool ok, uint4 v) {
  typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  const v4u_ x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, rs, ok ? (int)off : (int)0x80000000u, 0, 0);
}
// The ring wait of a persistent kernel at k-step s: DMA group s has landed when at most the younger ops are
// outstanding -- the S - 2 later groups (CNT each) and the NST stores of each epilogue run in steps
// s - S + 1 .. s - 1 (ne of them; vector-memory ops complete in issue order).
template <int S, int CNT, int NST>
LBT_DEV void ring_wait(int ne) {
  static_assert(S >= 3 && S <= 4, "ring depth");
  if (ne <= 0) vm_wait<(S - 2) * CNT>();
  else if (ne == 1) vm_wait<(S - 2) * CNT + NST>();
  else if (S == 3 || ne == 2) vm_wait<(S - 2) * CNT + 2 * NST>();
  else vm_wait<(S - 2) * CNT + (S == 4 ? 3 : 2) * NST>();
}

// Segment swizzles of the LDS images, conflict-free for ds_read_b128's lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32): a fragment read by lanes (r = lane & 15, q = lane >> 4)
// of rows base + r (base % 16 == 0) hits 16 distinct 4-bank quads in every group.
// 64-byte rows (4 segments; bank quad = (row & 3, segment)): f = {0, 2, 3, 1}[(row >> 2) & 3].
LBT_DEV int swz64(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
// 128-byte rows (8 segments; quad = (row & 1, segment)), segments 2q ^ f and 2q + 1 ^ f: f = (row >> 1) & 5.
LBT_DEV int swz128(int row) { return (row >> 1) & 5; }

// waves per SIMD the register allocation must leave room for (4: two 512-thread workgroups per CU).
// 16-bit codes at BN 64: 142 -> 128 VGPRs (20 bytes of spill), two workgroups per CU: l1_c2 dgrad16
// 170.6 -> 155.6 us, the other shapes unchanged (profiles/r04l_ab probe_*.txt); A8 BN 128 at 3-4 stages
// would spill 200+ bytes. HALO int8 at BN 64: 98 VGPRs, two per CU. The pass-A epilogues (BNA) at BN 64
// fit 128 VGPRs (78 KiB of LDS: two workgroups per CU).
#ifndef LBT_BIG_OCC
#define LBT_BIG_OCC(A16, BN, S, HALO, BNA) \
  (((A16 && BN == 64 && !HALO && S <= 2) || (!A16 && HALO && BN == 64) || BNA == 4) ? 4 \
   : (A16 && BN == 64 && !HALO) ? 2 : 1)
#endif
// BN pass A (bn_wide.hip bn_bwd_a_wide_kernel) on the dgrad accumulators, element for element.
// MA = 1 (lbt_dgrad_bna): dx -> ReLU mask recomputed from R -> the BN's two quantisers. MA = 2, 3
// (lbt_dgrad_bn3): d = dx + g2 masked by y_bits (optionally stored) -> MA - 1 BNs' quantisers. Per BN:
// G2 = Q_rg(d) -> gamma-scaled rescale gradient -> G = Q_ng (stored) + the four channel sums + the
// counters. These launches tile the rows SAMPLE-blocked (igemm_big_kernel PERM): a 256-row x 64-column
// tile is 16 pixels x 16 samples. The dequantised dx tile is staged in LDS ([pixel][sample][column],
// padded: conflict-free writes from the MFMA layout and reads by quads), then pass A runs with
// bn_bwd_a_wide_kernel's thread layout: a thread owns one position (pixel, 4 channels) and walks 8
// samples, so its two Philox calls (or table reads) per BN are made once for 8 samples and a wave's
// loads / stores are 4 pixels x 64 contiguous channels of one sample (coalesced; the MFMA layout
// would touch 16 rows x 16 bytes per instruction). Channel sums: lanes of a quad column by shuffles,
// the 8 waves in LDS (int32: 16 samples x 16 pixels x 2^22), one int64 atomic per (BN, column, sum)
// into shard tile % NSHARD. Rows outside (sample >= N, pixel >= H*W) are skipped.
struct BnaBn {
  lbt_qdesc qrg, qng;
  const int8_t *R, *qn;
  const float* gamma;
  int16_t* gout;
  int64_t* sums;
};
template <int MA, int k>
LBT_DEV BnaBn bna_bn(const IgArgs& p) {
  if constexpr (MA == 1) {
    const lbt_dgrad_bna& b = p.bna;
    return BnaBn{b.qrg, b.qng, b.R, b.qn, b.gb, b.gout, b.sums};
  } else {
    const lbt_bna_bn& b = p.bn3.bn[k];
    return BnaBn{b.qrg, b.qng, b.R, b.qn, b.gamma_q, b.gout, b.sums};
  }
}
#ifndef LBT_EPI_UNROLL
#define LBT_EPI_UNROLL 8  // samples a thread of the staged epilogues has in flight (2: 1.1x slower, 4: spills; profiles/r04u)
#endif
constexpr int kXRow = 68;                // floats per (pixel, sample) row of the staged dx tile
constexpr int kXPix = 16 * kXRow + 4;    // floats per pixel: 16 samples + 4 (bank offset per pixel)
constexpr int kXBytes = 16 * kXPix * 4;  // 69 888 bytes

template <int MI, int NJ, int WM, int BN, int MA>
LBT_DEV void passa_epilogue(const IgArgs& p, const v4i (&acc)[2][MI][NJ], const v4i (&accw)[NJ], float scale,
                            int sb, int pb, int n0, int r, int q, int wm, uint32_t tile, int8_t* lds) {
  static_assert(BN == 64 && WM == 8 && MI == 2, "the pass-A epilogue runs 256 x 64 tiles of 8 waves");
  constexpr int NB = MA == 3 ? 2 : 1;
  const int C = p.ncol;
  const int N = p.d.N;
  const int hw = p.ch * p.cw;
  float* xs = reinterpret_cast<float*>(lds);
  // ---- the dequantised dx tile into LDS: lane (r, q) holds column 16 j + r of samples 4 q + e at pixel
  // MI wm + i
  __syncthreads();  // every wave's last fragment reads of the LDS ring are done
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int wsum = accw[j][0];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double hs = (double)acc[0][i][j][e] * 256.0;
        const double ls = (double)(acc[1][i][j][e] + 128 * wsum);
        xs[(wm * MI + i) * kXPix + (4 * q + e) * kXRow + j * 16 + r] = (float)(hs + ls) * scale;
      }
  }
  __syncthreads();
  // ---- pass A: thread = (quad cq, pixel pl, sample half sh)
  const int t = threadIdx.x;
  const int cq = t & 15, pl = (t >> 4) & 15, sh = t >> 8;
  const int c0 = n0 + 4 * cq;
  const int pix = pb * 16 + pl;
  const bool pv = pix < hw;
  float bet[4] = {0.f, 0.f, 0.f, 0.f};
  float sr = 0.f;
  if constexpr (MA == 1) {
    const float4 b4 = *reinterpret_cast<const float4*>(p.bna.gb + C + c0);
    bet[0] = b4.x; bet[1] = b4.y; bet[2] = b4.z; bet[3] = b4.w;
    sr = qstate(p.bna.qr).inv_m;
  }
  const uint64_t blk = ((uint64_t)(pv ? pix : 0) * (uint32_t)C + (uint32_t)c0) >> 2;
  const int sbase = sb * 16 + sh * 8;
  const int shard = (int)(tile % LBT_NSHARD);
  const int wv = t >> 6;
  int* red = reinterpret_cast<int*>(lds + kXBytes);  // [8 waves][4 sums][64 columns]
  // one pass over the thread's samples per BN (the projection blocks' two BNs one after the other: the
  // same registers)
  auto bn_pass = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const BnaBn bn = bna_bn<MA, k>(p);
    const QState srg = qstate(bn.qrg), sng = qstate(bn.qng);
    const float4 g4 = *reinterpret_cast<const float4*>(bn.gamma + c0);
    const float gam[4] = {g4.x, g4.y, g4.z, g4.w};
    const Noise4 z{{0.f, 0.f, 0.f, 0.f}};
    const Noise4 u1 = bn.qrg.stochastic ? qnoise4(bn.qrg, srg.step, blk) : z;
    const Noise4 u2 = bn.qng.stochastic ? qnoise4(bn.qng, sng.step, blk) : z;
    int sm[4][4];  // [sum][channel]
#pragma unroll
    for (int a = 0; a < 4; ++a) sm[a][0] = sm[a][1] = sm[a][2] = sm[a][3] = 0;
    int ov[4] = {0, 0, 0, 0};
    // PK: both gradient quantisers stochastic (the models' configuration): quant4_w on packed pairs, the
    // counts as wave totals (lane 0 is active whenever a lane of its wave is: the inactive lanes of a sample
    // step are the wave's highest, past the image's last pixel); else quant1 per element, per-lane counts
    auto samples = [&](auto pkc) {
      constexpr bool PK = decltype(pkc)::value;
#pragma unroll LBT_EPI_UNROLL
      for (int u = 0; u < 8; ++u) {
        const int s_ = sbase + u;
        if (!pv || s_ >= N) break;  // samples ascend: the rest of this thread's are outside too
        const int64_t off = ((int64_t)s_ * hw + pix) * C + c0;
        const float4 xv = *reinterpret_cast<const float4*>(xs + pl * kXPix + (sh * 8 + u) * kXRow + 4 * cq);
        float d[4] = {xv.x, xv.y, xv.z, xv.w};
        const char4 rv = *reinterpret_cast<const char4*>(bn.R + off);
        const char4 qv = *reinterpret_cast<const char4*>(bn.qn + off);
        const int R[4] = {rv.x, rv.y, rv.z, rv.w};
        const int Q[4] = {qv.x, qv.y, qv.z, qv.w};
        if constexpr (MA >= 2) {  // bn_wide.hip :123-138
          const float4 g2 = *reinterpret_cast<const float4*>(p.bn3.g2 + off);
          const uint32_t yb = p.bn3.y_bits[off >> 2];
          d[0] = (yb & 1u) ? d[0] + g2.x : 0.f;
          d[1] = (yb & 2u) ? d[1] + g2.y : 0.f;
          d[2] = (yb & 4u) ? d[2] + g2.z : 0.f;
          d[3] = (yb & 8u) ? d[3] + g2.w : 0.f;
          if (k == 0 && p.bn3.gmask_out)
            *reinterpret_cast<float4*>(p.bn3.gmask_out + off) = make_float4(d[0], d[1], d[2], d[3]);
        } else {  // bn.hip chain_bwd_a's mask recomputation, op for op (bn_wide.hip :139-147)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float xr = (float)R[c] * sr;
            const float m1 = xr * gam[c];
            const float yv = m1 + bet[c];
            d[c] = yv > 0.f ? d[c] : 0.f;
          }
        }
        int G[4];
        if constexpr (PK) {  // bn_wide.hip :150-175 on packed pairs
          int G2[4];
          quant4_w<true>(srg, make_float4(d[0], d[1], d[2], d[3]), make_float4(u1.u[0], u1.u[1], u1.u[2], u1.u[3]), G2,
                         ov[0], ov[1]);
          const pf2 im = pk(srg.inv_m, srg.inv_m);
          const pf2 gh0 = pcvt(G2[0], G2[1]) * im, gh1 = pcvt(G2[2], G2[3]) * im;
          const pf2 dd0 = gh0 * pk(gam[0], gam[1]), dd1 = gh1 * pk(gam[2], gam[3]);
          quant4_w<true>(sng, make_float4(dd0.x, dd0.y, dd1.x, dd1.y), make_float4(u2.u[0], u2.u[1], u2.u[2], u2.u[3]),
                         G, ov[2], ov[3]);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            sm[0][c] += G2[c] * R[c];
            sm[1][c] += G2[c];
            sm[2][c] += G[c];
            sm[3][c] += G[c] * Q[c];
          }
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {  // bn_wide.hip :150-175
            const int G2 = quant1(srg, bn.qrg.stochastic, d[c], u1.u[c], ov[0], ov[1]);
            sm[0][c] += G2 * R[c];
            sm[1][c] += G2;
            const float gh = (float)G2 * srg.inv_m;
            const float dd = gh * gam[c];
            G[c] = quant1(sng, bn.qng.stochastic, dd, u2.u[c], ov[2], ov[3]);
            sm[2][c] += G[c];
            sm[3][c] += G[c] * Q[c];
          }
        }
        short4 o;
        o.x = (short)G[0]; o.y = (short)G[1]; o.z = (short)G[2]; o.w = (short)G[3];
        *reinterpret_cast<short4*>(bn.gout + off) = o;
      }
    };
    const bool pkq = bn.qrg.stochastic && bn.qng.stochastic;  // uniform
    if (pkq)
      samples(std::true_type{});
    else
      samples(std::false_type{});
    // channel sums: the 4 pixel lanes of a wave sharing cq (shuffles), the 8 waves in LDS
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        int v = sm[a][c];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if ((t & 63) < 16) red[(wv * 4 + a) * 64 + 4 * cq + c] = v;
      }
    // overflow counts -> wave totals in lane 0 (already wave totals on the packed path)
    int a0 = ov[0], a1 = ov[1], b0 = ov[2], b1 = ov[3];
    if (!pkq) {
      a0 = wave_sum_i32(a0); a1 = wave_sum_i32(a1);
      b0 = wave_sum_i32(b0); b1 = wave_sum_i32(b1);
    }
    if ((t & 63) == 0) {
      if (bn.qrg.counts) {
        int32_t* ct = bn.qrg.counts + ((int64_t)bn.qrg.slot * LBT_NSHARD + shard) * LBT_CSTRIDE;
        if (a0) atomicAdd(ct, a0);
        if (a1) atomicAdd(ct + 1, a1);
      }
      if (bn.qng.counts) {
        int32_t* ct = bn.qng.counts + ((int64_t)bn.qng.slot * LBT_NSHARD + shard) * LBT_CSTRIDE;
        if (b0) atomicAdd(ct, b0);
        if (b1) atomicAdd(ct + 1, b1);
      }
    }
    __syncthreads();
    if (t < 256) {
      const int a = t >> 6, cl = t & 63;
      long long v = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += red[(w * 4 + a) * 64 + cl];
      if (v) atomicAdd((unsigned long long*)&bn.sums[(int64_t)shard * 4 * C + a * C + n0 + cl], (unsigned long long)v);
    }
    if (k + 1 < NB) __syncthreads();  // red is rewritten by the next BN's pass
  };
  bn_pass(std::integral_constant<int, 0>{});
  if constexpr (NB == 2) bn_pass(std::integral_constant<int, 1>{});
}

// The conv-output quantiser (Normalization_q's input, quant_epilogue's arithmetic) on sample-blocked
// tiles (BNA 4): per 64-column half, the dequantised tile is staged in LDS as for passa_epilogue, then a
// thread owns (pixel, 4 channels), draws that position's noise once (table or Philox) and walks 8
// samples -- int8 codes stored as coalesced char4 runs, exact channel sums (sum q, sum q^2) in
// registers, one int64 atomic per (column, sum) per workgroup (quant_epilogue: per column per wave).
template <int MI, int NJ, int WM, int BN>
LBT_DEV void quantq_epilogue(const IgArgs& p, const v4i (&acc)[MI][NJ], const v4i (&accw)[NJ], int u8, float scale,
                             int sb, int pb, int n0, int r, int q, int wm, int wn, uint32_t tile, int8_t* lds) {
  static_assert((BN == 64 && WM == 8 && MI == 2) || (BN == 128 && WM == 4 && MI == 4), "256 x 64 / 128 tiles");
  const int C = p.ncol;
  const int N = p.d.N;
  const int hw = p.ch * p.cw;
  const QState qs = qstate(p.qout);
  const int st = p.qout.stochastic;
  float* xs = reinterpret_cast<float*>(lds);
  int* red = reinterpret_cast<int*>(lds + kXBytes);  // [8 waves][2 sums][64 columns]
  const int t = threadIdx.x;
  const int cq = t & 15, pl = (t >> 4) & 15, sh = t >> 8, wv = t >> 6;
  const int pix = pb * 16 + pl;
  const bool pv = pix < hw;
  const int sbase = sb * 16 + sh * 8;
  const int shard = (int)(tile % LBT_NSHARD);
  int ov1 = 0, ov2 = 0;
  __syncthreads();  // every wave's last fragment reads of the LDS ring are done
#pragma unroll
  for (int h = 0; h < BN / 64; ++h) {
    if (wn == h) {  // this half's waves stage their rows: pixel MI wm + i, samples 4 q + e, column 16 j + r
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int wsum = accw[j][0];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            xs[(wm * MI + i) * kXPix + (4 * q + e) * kXRow + j * 16 + r] = (float)(acc[i][j][e] + u8 * wsum) * scale;
      }
    }
    __syncthreads();
    const int c0 = n0 + h * 64 + 4 * cq;
    const uint64_t blk = ((uint64_t)(pv ? pix : 0) * (uint32_t)C + (uint32_t)c0) >> 2;
    Noise4 u = {{0.f, 0.f, 0.f, 0.f}};
    if (st) u = qnoise4(p.qout, qs.step, blk);
    const float4 u4 = make_float4(u.u[0], u.u[1], u.u[2], u.u[3]);
    int s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
    // this lane's samples sbase .. sbase + nsm - 1 (uniform per wave but for the pixel check): the
    // output pointer and the LDS row advance by one sample per step (no per-sample 64-bit offsets)
    const int nsm = pv ? (N - sbase < 8 ? (N - sbase > 0 ? N - sbase : 0) : 8) : 0;
    int8_t* yp = p.yq + ((int64_t)sbase * hw + pix) * C + c0;
    const int64_t ystep = (int64_t)hw * C;
    const float* xp = xs + pl * kXPix + (sh * 8) * kXRow + 4 * cq;
    auto samples = [&](auto stc) {
      constexpr bool ST = decltype(stc)::value;
#pragma unroll LBT_EPI_UNROLL
      for (int k = 0; k < 8; ++k) {
        if (k >= nsm) break;  // samples ascend
        const float4 xv = *reinterpret_cast<const float4*>(xp + k * kXRow);
        int c[4];
        quant4_w<ST>(qs, xv, u4, c, ov1, ov2);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[e] += c[e];
          s2[e] += c[e] * c[e];
        }
        *reinterpret_cast<char4*>(yp) = make_char4((char)c[0], (char)c[1], (char)c[2], (char)c[3]);
        yp += ystep;
      }
    };
    if (st)
      samples(std::true_type{});
    else
      samples(std::false_type{});
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int a = s1[e], b = s2[e];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      if ((t & 63) < 16) {
        red[(wv * 2 + 0) * 64 + 4 * cq + e] = a;
        red[(wv * 2 + 1) * 64 + 4 * cq + e] = b;
      }
    }
    __syncthreads();  // xs read and red written: the next half may restage
    if (t < 128) {
      const int a = t >> 6, cl = t & 63;
      long long v = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += red[(w * 2 + a) * 64 + cl];
      if (v)
        atomicAdd((unsigned long long*)&p.chsum[(int64_t)shard * 2 * C + a * C + n0 + h * 64 + cl], (unsigned long long)v);
    }
    if (h + 1 < BN / 64) __syncthreads();  // red is rewritten by the next half
  }
  // (wave totals, quant4_w: lane 0 was active whenever a lane of its wave was -- the inactive lanes of a
  // sample step are the ones past the image's last pixel, the wave's highest)
  if ((t & 63) == 0 && p.qout.counts) {
    int32_t* ct = p.qout.counts + ((int64_t)p.qout.slot * LBT_NSHARD + shard) * LBT_CSTRIDE;
    if (ov1) atomicAdd(ct, ov1);
    if (ov2) atomicAdd(ct + 1, ov2);
  }
}

// HALO (3x3, stride 1, pad 1: fwd, and the unit-stride dgrad of such a conv): the k loop runs
// channel-block-major, and per channel block ONE window of A is staged -- the tile's 256 pixels plus
// W + 1 on either side in the same row-major pixel order, 256 + 2W + 2 <= 384 rows -- instead of one
// 256-row A block per tap: the 9 taps read the window shifted by dy * W + dx (invalid taps -- outside
// the image -- read the fill value in registers). A leaves L2 ~1.4x instead of 9x per channel block.
// Window: two buffers, the next block's window DMA'd one instruction per wave per tap step while the
// current block's 9 taps run; B: a 3-stage ring, two taps ahead.
template <int MODE, bool A16, bool ADD, int BN, int S, int BNA = 0, bool HALO = false>
__global__ __launch_bounds__(kBT, LBT_BIG_OCC(A16, BN, S, HALO, BNA)) void igemm_big_kernel(IgArgs p) {
  constexpr int BM = 256, WN = BN / 64, WM = 8 / WN, TR = BM / WM, MI = TR / 16, NJ = 4;
  constexpr int NA = A16 ? 2 : 1;
  constexpr int ROWB = A16 ? 128 : 64;                 // bytes of one A row per k-block
  constexpr int ABYTES = BM * ROWB, BBYTES = BN * 64, STAGE = ABYTES + BBYTES;
  constexpr int NIA = ABYTES / 1024, NIB = BBYTES / 1024;  // 1-KiB DMA wave-instructions per stage
  constexpr int GA = NIA / 8;                          // A instructions per wave (2 or 4)
  constexpr int RPI = A16 ? 8 : 16;                    // A rows per instruction
  static_assert(NIA % 8 == 0 && (NIB % 8 == 0 || NIB == 4) && (!A16 || BN <= 128), "geometry");
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;
  const int r = lane & 15, q = lane >> 4;
  // XCD-aware bijective tile order: the WN column tiles of one row tile share an XCD's L2
  const int ntn = p.ncol / BN;
  const uint32_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const uint32_t tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  // PERM (the pass-A epilogues): row tile rt = (sample block sb, pixel block pb), tile row
  // (16 px + s) = pixel 16 pb + px of sample 16 sb + s; else rows m0 .. m0 + 255 in pixel order
  constexpr bool PERM = BNA >= 1;
  const uint32_t rt = tile / (uint32_t)ntn;
  const int64_t m0 = PERM ? 0 : (int64_t)rt * BM;
  const int sb = PERM ? (int)(rt / (uint32_t)p.npb) : 0, pb = PERM ? (int)(rt % (uint32_t)p.npb) : 0;
  const int n0 = (int)(tile % (uint32_t)ntn) * BN;
  const lbt_conv_desc& d = p.d;
  const int OH = p.ch, OW = p.cw;
  const int SH = MODE == MODE_FWD ? d.H : d.Ho, SW = MODE == MODE_FWD ? d.W : d.Wo;
  const int cblocks = p.cred / kBK, nk = p.nkh * p.nkw * cblocks;
  const int8_t* fill = (!A16 && p.a_u8off) ? reinterpret_cast<const int8_t*>(kFill80)
                                           : reinterpret_cast<const int8_t*>(zi());

  // ---- this lane's DMA rows: A row (i = wave + 8 g) * RPI + lane / (64 / RPI), segment lane % (64 / RPI)
  constexpr int SPR = 64 / RPI;  // lanes (16-byte segments) per row: 4 (A8) or 8 (A16)
  int an[GA], ay[GA], ax[GA], aseg[GA];
  bool arow[GA];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int row = (wave + 8 * g) * RPI + lane / SPR;
    if constexpr (PERM) {
      const int sm = sb * 16 + (row & 15), px = pb * 16 + (row >> 4);
      arow[g] = sm < d.N && px < OH * OW;
      const uint32_t pu = (uint32_t)(arow[g] ? px : 0);
      ax[g] = (int)(pu % (uint32_t)OW);
      ay[g] = (int)(pu / (uint32_t)OW);
      an[g] = arow[g] ? sm : 0;
    } else {
      const int64_t m = m0 + row;
      arow[g] = m < p.M;
      const uint32_t mu = (uint32_t)(arow[g] ? m : 0);
      ax[g] = (int)(mu % (uint32_t)OW);
      const uint32_t tt = mu / (uint32_t)OW;
      ay[g] = (int)(tt % (uint32_t)OH);
      an[g] = (int)(tt / (uint32_t)OH);
    }
    const int ps = lane % SPR;  // the LDS segment this lane fills; its source is segment ps ^ f(row)
    aseg[g] = A16 ? (ps ^ swz128(row)) : (ps ^ swz64(row));
  }
  // B: instruction i covers weight-image columns n0 + 16 i .. + 15 (64 bytes of the k-block each)
  constexpr int GB = NIB >= 8 ? NIB / 8 : 1;
  const bool bact = NIB >= 8 || wave < NIB;
  int bcolx[GB], bseg[GB];
#pragma unroll
  for (int g = 0; g < GB; ++g) {
    const int cl = (wave + 8 * g) * 16 + lane / 4;
    bcolx[g] = n0 + cl;
    bseg[g] = (lane % 4) ^ swz64(cl);
  }
  auto issue = [&](int kb, int st) {
    const int tap = kb / cblocks, cb = kb - tap * cblocks;
    const int th = tap / p.nkw, tw = tap - th * p.nkw;
    const int kh = MODE == MODE_FWD ? th : p.kh0 + d.SH * th, kw = MODE == MODE_FWD ? tw : p.kw0 + d.SW * tw;
    const int kbw = (kh * d.KW + kw) * cblocks + cb;
    int8_t* sb = lds + st * STAGE;
#pragma unroll
    for (int g = 0; g < GA; ++g) {
      int sy, sx;
      if (MODE == MODE_FWD) {
        sy = ay[g] * d.SH + kh - d.PT;
        sx = ax[g] * d.SW + kw - d.PL;
      } else {
        sy = ay[g] + p.oy - th;
        sx = ax[g] + p.ox - tw;
      }
      const bool ok = (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW && arow[g];
      const int8_t* src;
      if (ok) {
        const uint32_t pix = (uint32_t)((an[g] * SH + sy) * SW + sx);
        src = reinterpret_cast<const int8_t*>(p.a) +
              (uint64_t)(pix * (uint32_t)p.cred + (uint32_t)(cb * kBK)) * (A16 ? 2 : 1) + aseg[g] * 16;
      } else {
        src = fill;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_vptr)(sb + (wave + 8 * g) * 1024), 16, 0, 0);
    }
    if (bact) {
#pragma unroll
      for (int g = 0; g < GB; ++g) {
        const int8_t* src = p.b + ((uint32_t)(bcolx[g] * p.ks + kbw * 4 + bseg[g]) << 4);
        __builtin_amdgcn_global_load_lds(src, (lds_vptr)(sb + ABYTES + (wave + 8 * g) * 1024), 16, 0, 0);
      }
    }
  };
  auto wait_landed = [&]() {  // k-block kb's DMA landed: at most S-2 younger groups in flight
    if constexpr (NIB >= 8) {
      vm_wait<(S - 2) * (GA + GB)>();
    } else {
      if (bact) vm_wait<(S - 2) * (GA + 1)>(); else vm_wait<(S - 2) * GA>();
    }
  };

  v4i acc[NA][MI][NJ], accw[NJ];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[a][i][j] = v4i{0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < NJ; ++j) accw[j] = v4i{0, 0, 0, 0};
  // sum_k W per column (the +128 term of offset / split codes): from the caller's column sums when it
  // has them, else summed from the B fragments on the VALU (16-bit codes; offset codes of
  // lbt_conv_fwd_igemm_q) -- 4 v_dot4 per fragment instead of an MFMA against ones (an extra 4 of
  // the 16 (A8) / 32 (A16) MFMAs per k-block of a 64 x 64 wave tile)
  const bool wmfma = A16 || (p.a_u8off && !p.colsum);  // uniform
  int csw[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) csw[j] = 0;

  // fragments of one k-block (A16: the raw int16 code pairs, split into hi / lo' at the MFMA)
  typedef v4i FragA[MI][NA];
  typedef v4i FragB[NJ];
  auto read_frags = [&](int st, FragA& fa, FragB& fb) {
    const int8_t* sb = lds + st * STAGE;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = wn * 64 + j * 16 + r;
      fb[j] = *reinterpret_cast<const v4i*>(sb + ABYTES + col * 64 + ((q ^ swz64(col)) << 4));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * TR + i * 16 + r;
      if constexpr (A16) {
        const int f = swz128(row);
        fa[i][0] = *reinterpret_cast<const v4i*>(sb + row * 128 + (((2 * q) ^ f) << 4));
        fa[i][NA - 1] = *reinterpret_cast<const v4i*>(sb + row * 128 + (((2 * q + 1) ^ f) << 4));
      } else {
        fa[i][0] = *reinterpret_cast<const v4i*>(sb + row * 64 + ((q ^ swz64(row)) << 4));
      }
    }
  };
  auto mma = [&](const FragA& fa, const FragB& fb) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if constexpr (A16) {
        // codes (int16) e0 e1 | e2 e3 per dword: hi = high bytes, lo' = low bytes ^ 0x80 (a = 256 hi + lo' + 128)
        const v4i c0 = fa[i][0], c1 = fa[i][NA - 1];
        const uint32_t w[8] = {(uint32_t)c0[0], (uint32_t)c0[1], (uint32_t)c0[2], (uint32_t)c0[3],
                               (uint32_t)c1[0], (uint32_t)c1[1], (uint32_t)c1[2], (uint32_t)c1[3]};
        v4i hi, lo;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          hi[u] = (int)__builtin_amdgcn_perm(w[2 * u + 1], w[2 * u], 0x07050301u);
          lo[u] = (int)(__builtin_amdgcn_perm(w[2 * u + 1], w[2 * u], 0x06040200u) ^ 0x80808080u);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          acc[0][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(hi, fb[j], acc[0][i][j], 0, 0, 0);
          acc[NA - 1][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(lo, fb[j], acc[NA - 1][i][j], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[0][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i][0], fb[j], acc[0][i][j], 0, 0, 0);
      }
    }
    if (wmfma) {  // sum_k W of the column: the lane's 16 k-bytes on the VALU (dot4 with ones), beside the MFMAs
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) csw[j] = __builtin_amdgcn_sdot4(fb[j][u], 0x01010101, csw[j], false);
    }
  };

  if constexpr (HALO) {
    constexpr int GW = A16 ? 6 : 3;        // window DMA instructions per wave: 8 * GW * RPI = 384 rows
    constexpr int NWR = 8 * GW * RPI, WINB = NWR * ROWB, BST = BN * 64;
    constexpr int GBI = NIB >= 8 ? NIB / 8 : 1;  // B instructions per issuing wave per tap
    int8_t* win = lds;                     // [2][NWR][ROWB]
    int8_t* bring = lds + 2 * WINB;        // [3][BN][64]
    const int Wd = OW, Hd = OH;
    const int nwin = 256 + 2 * Wd + 2;     // window rows that can be read
    const int64_t wbase = m0 - (Wd + 1);
    uint32_t soff[GW];
    bool sv[GW];
#pragma unroll
    for (int g = 0; g < GW; ++g) {
      const int wr = (wave + 8 * g) * RPI + lane / SPR;
      const int64_t px = wbase + wr;
      sv[g] = wr < nwin && px >= 0 && px < p.M;
      const int ps = lane % SPR;
      const int sg = A16 ? (ps ^ swz128(wr)) : (ps ^ swz64(wr));
      soff[g] = sv[g] ? (uint32_t)px * (uint32_t)p.cred * (A16 ? 2u : 1u) + (uint32_t)sg * 16u : 0u;
    }
    auto issue_win = [&](int cb, int buf, int g) {
      const int8_t* src = sv[g] ? reinterpret_cast<const int8_t*>(p.a) + soff[g] + (uint32_t)cb * (A16 ? 128u : 64u)
                                : fill;
      __builtin_amdgcn_global_load_lds(src, (lds_vptr)(win + buf * WINB + (wave + 8 * g) * 1024), 16, 0, 0);
    };
    auto issue_b = [&](int k, int st) {
      const int cb = k / 9, tp = k - cb * 9;
      const int kbw = tp * cblocks + cb;  // (kh * 3 + kw) * cblocks + cb
      if (bact) {
#pragma unroll
        for (int g = 0; g < GB; ++g) {
          const int8_t* src = p.b + ((uint32_t)(bcolx[g] * p.ks + kbw * 4 + bseg[g]) << 4);
          __builtin_amdgcn_global_load_lds(src, (lds_vptr)(bring + st * BST + (wave + 8 * g) * 1024), 16, 0, 0);
        }
      }
    };
    // this lane's fragment rows: pixel (x, y) within its image, and whether the row exists
    int fx[MI], fy[MI];
    bool fok[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + wm * TR + i * 16 + r;
      fok[i] = m < p.M;
      const uint32_t mu = (uint32_t)(fok[i] ? m : 0);
      fx[i] = (int)(mu % (uint32_t)Wd);
      fy[i] = (int)((mu / (uint32_t)Wd) % (uint32_t)Hd);
    }
    const int afill = (!A16 && p.a_u8off) ? (int)0x80808080u : 0;
#pragma unroll
    for (int g = 0; g < GW; ++g) issue_win(0, 0, g);
    issue_b(0, 0);
    issue_b(nk > 1 ? 1 : 0, 1);
    for (int cb = 0; cb < cblocks; ++cb) {
      const bool more = cb + 1 < cblocks;
      const int8_t* wsb = win + (cb & 1) * WINB;
      auto tap_step = [&](auto tc) {
        constexpr int tp = decltype(tc)::value;
        constexpr int th = tp / 3, tw = tp % 3;
        constexpr int dy = MODE == MODE_FWD ? th - 1 : 1 - th, dx = MODE == MODE_FWD ? tw - 1 : 1 - tw;
        // B(k) landed: younger are B(k + 1) and the window pieces of steps k - 2, k - 1
        constexpr int P = (tp >= 2 && tp - 2 < GW ? 1 : 0) + (tp >= 1 && tp - 1 < GW ? 1 : 0);
        if (bact) {
          if (more) vm_wait<GBI + P>(); else vm_wait<GBI>();
        } else {
          if (more) vm_wait<P>(); else vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
        const int k = cb * 9 + tp;
        issue_b(k + 2 < nk ? k + 2 : nk - 1, (tp + 2) % 3);
        if (tp < GW && more) issue_win(cb + 1, (cb + 1) & 1, tp);
        FragA fa;
        FragB fb;
        const int8_t* bsb = bring + (tp % 3) * BST;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int col = wn * 64 + j * 16 + r;
          fb[j] = *reinterpret_cast<const v4i*>(bsb + col * 64 + ((q ^ swz64(col)) << 4));
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int wr = wm * TR + i * 16 + r + (dy + 1) * Wd + dx + 1;
          const bool v = fok[i] && (unsigned)(fx[i] + dx) < (unsigned)Wd && (unsigned)(fy[i] + dy) < (unsigned)Hd;
          if constexpr (A16) {
            const int f = swz128(wr);
            const v4i c0 = *reinterpret_cast<const v4i*>(wsb + wr * 128 + (((2 * q) ^ f) << 4));
            const v4i c1 = *reinterpret_cast<const v4i*>(wsb + wr * 128 + (((2 * q + 1) ^ f) << 4));
            const v4i z = v4i{0, 0, 0, 0};
            fa[i][0] = v ? c0 : z;
            fa[i][NA - 1] = v ? c1 : z;
          } else {
            const v4i c0 = *reinterpret_cast<const v4i*>(wsb + wr * 64 + ((q ^ swz64(wr)) << 4));
            fa[i][0] = v ? c0 : v4i{afill, afill, afill, afill};
          }
        }
        mma(fa, fb);
      };
      tap_step(std::integral_constant<int, 0>{});
      tap_step(std::integral_constant<int, 1>{});
      tap_step(std::integral_constant<int, 2>{});
      tap_step(std::integral_constant<int, 3>{});
      tap_step(std::integral_constant<int, 4>{});
      tap_step(std::integral_constant<int, 5>{});
      tap_step(std::integral_constant<int, 6>{});
      tap_step(std::integral_constant<int, 7>{});
      tap_step(std::integral_constant<int, 8>{});
    }
  } else {
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s < nk ? s : nk - 1, s);
  if constexpr (S >= 3) {
    // Software-pipelined: k-block kb + 1's fragments are read from LDS while kb's MFMAs run. Step kb
    // waits for DMA group kb + 1 (at most S - 3 younger groups in flight) and the barrier, which also
    // retires every wave's reads of the stage the new DMA (group kb + S - 1) overwrites (read in step kb - 2).
    auto wait_next = [&]() {
      if constexpr (NIB >= 8) {
        vm_wait<(S - 3) * (GA + GB)>();
      } else {
        if (bact) vm_wait<(S - 3) * (GA + 1)>(); else vm_wait<(S - 3) * GA>();
      }
    };
    auto step = [&](int kb, const FragA& ca, const FragB& cb, FragA& na, FragB& nb) {
      wait_next();
      __builtin_amdgcn_s_barrier();
      if (!(p.dbg & 1)) {
        const int nx = kb + S - 1;
        issue(nx < nk ? nx : nk - 1, nx % S);
      }
      read_frags((kb + 1) % S, na, nb);  // past the last k-block: an unused read of a stale stage
      mma(ca, cb);
    };
    wait_landed();
    __builtin_amdgcn_s_barrier();
    FragA fa0, fa1;
    FragB fb0, fb1;
    read_frags(0, fa0, fb0);
    for (int kb = 0; kb < nk; kb += 2) {
      step(kb, fa0, fb0, fa1, fb1);
      if (kb + 1 < nk) step(kb + 1, fa1, fb1, fa0, fb0);
    }
  } else {
    for (int kb = 0; kb < nk; ++kb) {
      wait_landed();
      __builtin_amdgcn_s_barrier();
      if (!(p.dbg & 1)) {
        const int nx = kb + S - 1;
        issue(nx < nk ? nx : nk - 1, nx % S);  // refills the stage read in iteration kb - 1
      }
      FragA fa;
      FragB fb;
      read_frags(kb % S, fa, fb);
      mma(fa, fb);
    }
  }
  }
  vm_wait<0>();  // the ring's trailing (clamped) DMAs: nothing may still write LDS when the block ends
  if (wmfma) {  // the column totals: lanes r, r + 16, r + 32, r + 48 hold a quarter of column r's k each
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const auto h = __builtin_amdgcn_permlane32_swap(csw[j], csw[j], false, false);
      const int t1 = (int)h[0] + (int)h[1];
      const auto g = __builtin_amdgcn_permlane16_swap(t1, t1, false, false);
      const int t = (int)g[0] + (int)g[1];
      accw[j] = v4i{t, t, t, t};
    }
  }

  // ---- epilogue (igemm_kernel's): lane owns column (tile col + r), rows (tile row + 4q + e)
  const float scale = ldexpf(1.0f, -(frac_exp(p.qa) + frac_exp(p.qb)));
  constexpr bool addv = MODE == MODE_DGRAD && ADD;
  const int ncol = p.ncol;
  const int64_t rtile = m0 + wm * TR + q * 4;  // + i * 16 + e
  const bool full = m0 + BM <= p.M;
  const int rlim = full ? TR : (int)(p.M - rtile);
  const int cw = n0 + wn * 64;
  // the +128 sum_k W term of offset codes: the weight image's column sums (fwd); 16-bit codes: accw
  if constexpr (!A16) {
    if (p.a_u8off && p.colsum) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int cs = p.colsum[cw + j * 16 + r];
        accw[j] = v4i{cs, cs, cs, cs};
      }
    }
  }
  const int u8 = (!A16 && p.a_u8off) ? 128 : 0;
  if constexpr (BNA == 4) {
    if constexpr (MODE == MODE_FWD && !A16)
      quantq_epilogue<MI, NJ, WM, BN>(p, acc[0], accw, u8, scale, sb, pb, n0, r, q, wm, wn, tile, lds);
    return;
  }
  if constexpr (MODE == MODE_FWD && !A16) {
    if (p.yq) {  // uniform: quantising epilogue
      quant_epilogue<MI, NJ>(p, acc[0], accw, u8, scale, rtile, rlim, full, cw, r, q);
      return;
    }
  }
  if constexpr (BNA >= 1 && BNA <= 3) {
    if constexpr (BN == 64) passa_epilogue<MI, NJ, WM, BN, BNA>(p, acc, accw, scale, sb, pb, n0, r, q, wm, tile, lds);
    return;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = cw + j * 16 + r;
    float* yp = p.y + rtile * ncol + col;
    const float* ap = addv ? p.add_src + rtile * ncol + col : nullptr;
    float av[MI][4];
    if constexpr (addv) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) av[i][e] = (i * 16 + e < rlim) ? ap[(i * 16 + e) * ncol] : 0.f;
    }
    const int wsum = (A16 || p.a_u8off) ? accw[j][0] : 0;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v;
        if constexpr (A16) {
          const double hs = (double)acc[0][i][j][e] * 256.0;
          const double ls = (double)(acc[1][i][j][e] + 128 * wsum);
          v = (float)(hs + ls) * scale;
        } else {
          v = (float)(acc[0][i][j][e] + u8 * wsum) * scale;
        }
        if (full || i * 16 + e < rlim) yp[(i * 16 + e) * ncol] = addv ? v + av[i][e] : v;
      }
  }
}

// ------------------------------------------------------------ persistent quantising forward
// igemm_fwdq_kernel: lbt_conv_fwd_igemm_q on sample-blocked 256-row tiles (16 pixels x 16 samples, as
// quantq_epilogue) with a stochastic qout that reads a noise table (or a nearest-rounding one), for the
// short-K GEMMs where igemm_big_kernel's one-tile workgroups spend their life in latency (ResNet-50
// l1_c3, K = 64: one k-block, then a 64 KiB LDS staging pass; profiles/r05 pmc: waves waiting 44 %).
//  * one workgroup per CU, each owning ONE column tile and a strided set of row tiles; an S-stage
//    LDS-DMA ring runs across tile boundaries, so the next tiles' operands are in flight during a
//    tile's epilogue (every wave issues exactly GA + 2 DMA instructions per k-step -- idle slots write
//    a dummy KiB -- so the counted vmcnt waits are constants);
//  * the epilogue quantises straight from the accumulators: the MFMA runs with the operands swapped
//    (weights as the A operand), and the weight image's columns are loaded into LDS permuted (LDS row
//    16 j + 4 g + e of a 64-column slice <- channel 16 g + 4 j + e), so lane (r, q) ends with 16
//    CONSECUTIVE channels (16 q .. 16 q + 15 of its wave's slice) of one row: one 16-byte store per
//    row, no LDS staging of the tile;
//  * the tile's noise (16 pixels x BN channels of the table) rides the ring with the operands of the
//    tile's last k-block; lanes of one pixel read it as LDS broadcasts;
//  * channel sums (sum q, sum q^2) stay in registers across every tile of the workgroup (its column
//    tile is fixed) and leave once: 16-lane shuffles, the waves in LDS, one int64 atomic per (column,
//    sum); overflow counters are wave totals (quant4_w), one atomic each at the end.
// Rows outside the image or batch hold the fill code, whose dequantised value is exactly 0: code 0, no
// overflow, nothing added to the sums, and their stores are skipped -- quantq_epilogue's results bit for bit.
template <int BN, int S, bool ST>
__global__ __launch_bounds__(kBT, 1) void igemm_fwdq_kernel(IgArgs p, int nrg, int rtiles) {
  constexpr int BM = 256, WN = BN / 64, WM = 8 / WN, TR = BM / WM, MI = TR / 16, NJ = 4;
  constexpr int ABYTES = BM * 64, BBYTES = BN * 64, NBYTES = 16 * BN * 4;
  constexpr int STAGE = ABYTES + BBYTES + NBYTES;
  constexpr int GA = ABYTES / 1024 / 8;  // A instructions per wave per k-block (2)
  constexpr int NIB = BBYTES / 1024, NIN = NBYTES / 1024;  // B / noise instructions per k-block (<= 8)
  constexpr int CNT = GA + 2;
  constexpr int PARTS = kBT / BN;
  static_assert(NIB <= 8 && NIN <= 8 && (BN == 64 || BN == 128), "geometry");
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  int8_t* dummy = lds + S * STAGE;                   // 1 KiB sink of the idle DMA slots
  int* wsl = reinterpret_cast<int*>(dummy + 1024);   // [BN] sum_k W per column (offset codes)
  int* wpart = wsl + BN;                             // [PARTS][BN]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;
  const int r = lane & 15, q = lane >> 4;
  const int ntn = p.ncol / BN;
  const uint32_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const uint32_t L = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int cn = (int)(L % (uint32_t)ntn), rg = (int)(L / (uint32_t)ntn);
  const int n0 = cn * BN;
  const int T = rg < rtiles ? (rtiles - 1 - rg) / nrg + 1 : 0;
  if (T == 0) return;  // uniform over the workgroup, before any barrier
  const lbt_conv_desc& d = p.d;
  const int C = p.ncol, N = d.N, hw = p.hw, OW = p.cw, npb = p.npb;
  const int cblocks = p.cred / kBK, nk = p.nkh * p.nkw * cblocks;
  const int8_t* fill = p.a_u8off ? reinterpret_cast<const int8_t*>(kFill80) : reinterpret_cast<const int8_t*>(zi());
  const int u8 = p.a_u8off ? 128 : 0;

  // ---- sum_k W of this workgroup's columns (offset codes): from the caller's colsum, else from the image
  int ws[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) ws[k] = 0;
  if (u8) {
    {
      const int ch = t % BN, part = t / BN;
      int s = 0;
      if (p.colsum) {
        if (part == 0) s = p.colsum[n0 + ch];
      } else {
        const int8_t* col = p.b + (int64_t)(n0 + ch) * p.ks * 16;
        for (int c = part; c < nk * 4; c += PARTS) {
          const int4 v = *reinterpret_cast<const int4*>(col + c * 16);
          s = __builtin_amdgcn_sdot4(v.x, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(v.y, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(v.z, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(v.w, 0x01010101, s, false);
        }
      }
      wpart[part * BN + ch] = s;
    }
    __syncthreads();
    if (t < BN) {
      int s = 0;
#pragma unroll
      for (int k = 0; k < PARTS; ++k) s += wpart[k * BN + t];
      wsl[t] = s;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) ws[k] = wsl[wn * 64 + 16 * q + k];
  }

  // ---- DMA geometry. A: instruction g of a wave covers tile rows (wave + 8 g) * 16 .. + 15, 4 lanes a row
  int aseg[GA];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int row = (wave + 8 * g) * 16 + lane / 4;
    aseg[g] = (lane % 4) ^ swz64(row);
  }
  // B: LDS row cl (16 rows per instruction) <- weight column n0 + perm(cl)
  const bool bact = wave < NIB;
  int bcol, bseg;
  {
    const int cl = wave * 16 + lane / 4;
    const int pc = (cl & ~63) | (((cl & 15) >> 2) << 4) | (((cl >> 4) & 3) << 2) | (cl & 3);
    bcol = n0 + (bact ? pc : 0);
    bseg = (lane % 4) ^ swz64(cl);
  }
  // noise: instruction w covers pixels (1024 / (4 BN)) w .. of the tile, lane-linear [pixel][BN] floats
  constexpr int NPX = 1024 / (4 * BN), NSEG = BN / 4;  // pixels per instruction, 16-byte segments per pixel
  const bool nact = ST && wave < NIN;
  const int npl = wave * NPX + lane / NSEG, nseg = lane % NSEG;

  // issue side: tile it, k-block ikb, and its rows
  int it = 0, ikb = 0;
  int an[GA], ay[GA], ax[GA];
  bool arow[GA];
  int64_t noff = 0;
  auto set_rows = [&](int k) {
    const uint32_t rt = (uint32_t)(rg + k * nrg);
    const int sb = (int)(rt / (uint32_t)npb), pb = (int)(rt % (uint32_t)npb);
#pragma unroll
    for (int g = 0; g < GA; ++g) {
      const int row = (wave + 8 * g) * 16 + lane / 4;
      const int sm = sb * 16 + (row & 15), px = pb * 16 + (row >> 4);
      arow[g] = sm < N && px < hw;
      const uint32_t pu = (uint32_t)(arow[g] ? px : 0);
      ax[g] = (int)(pu % (uint32_t)OW);
      ay[g] = (int)(pu / (uint32_t)OW);
      an[g] = arow[g] ? sm : 0;
    }
    const int px = pb * 16 + npl;
    noff = (int64_t)(px < hw ? px : 0) * C + n0 + 4 * nseg;
  };
  set_rows(0);
  auto issue = [&](int st) {
    int8_t* sb = lds + st * STAGE;
    if (it < T) {
      const int kb = ikb;
      const int tap = kb / cblocks, cb = kb - tap * cblocks;
      const int kh = tap / p.nkw, kw = tap - kh * p.nkw;
      const int kbw = (kh * d.KW + kw) * cblocks + cb;
#pragma unroll
      for (int g = 0; g < GA; ++g) {
        const int sy = ay[g] * d.SH + kh - d.PT, sx = ax[g] * d.SW + kw - d.PL;
        const bool ok = (unsigned)sy < (unsigned)d.H && (unsigned)sx < (unsigned)d.W && arow[g];
        const int8_t* src = fill;
        if (ok) {
          const uint32_t pix = (uint32_t)((an[g] * d.H + sy) * d.W + sx);
          src = reinterpret_cast<const int8_t*>(p.a) + (uint64_t)(pix * (uint32_t)p.cred + (uint32_t)(cb * kBK)) +
                aseg[g] * 16;
        }
        __builtin_amdgcn_global_load_lds(src, (lds_vptr)(sb + (wave + 8 * g) * 1024), 16, 0, 0);
      }
      {
        const int8_t* src = bact ? p.b + ((uint32_t)(bcol * p.ks + kbw * 4 + bseg) << 4) : fill;
        __builtin_amdgcn_global_load_lds(src, (lds_vptr)(bact ? sb + ABYTES + wave * 1024 : dummy), 16, 0, 0);
      }
      {
        const bool nl = nact && kb == nk - 1;
        const int8_t* src = nl ? reinterpret_cast<const int8_t*>(p.qout.noise + noff) : fill;
        __builtin_amdgcn_global_load_lds(src, (lds_vptr)(nl ? sb + ABYTES + BBYTES + wave * 1024 : dummy), 16, 0, 0);
      }
      if (++ikb == nk) {
        ikb = 0;
        if (++it < T) set_rows(it);
      }
    } else {
#pragma unroll
      for (int g = 0; g < CNT; ++g) __builtin_amdgcn_global_load_lds(fill, (lds_vptr)dummy, 16, 0, 0);
    }
  };

  const QState qs = qstate(p.qout);
  const float scale = ldexpf(1.0f, -(frac_exp(p.qa) + frac_exp(p.qb)));
  v4i acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  int s1[16], s2[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { s1[k] = 0; s2[k] = 0; }
  int ov1 = 0, ov2 = 0;

  auto epilogue = [&](int k, const int8_t* sbase) {
    const uint32_t rt = (uint32_t)(rg + k * nrg);
    const int sb = (int)(rt / (uint32_t)npb), pb = (int)(rt % (uint32_t)npb);
    const int sample = sb * 16 + r;
    const float* nimg = reinterpret_cast<const float*>(sbase + ABYTES + BBYTES);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int pt = wm * MI + i, px = pb * 16 + pt;
      const bool ok = sample < N && px < hw;
      uint32_t w4[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float4 xv = make_float4((float)(acc[i][j][0] + u8 * ws[4 * j + 0]) * scale,
                                      (float)(acc[i][j][1] + u8 * ws[4 * j + 1]) * scale,
                                      (float)(acc[i][j][2] + u8 * ws[4 * j + 2]) * scale,
                                      (float)(acc[i][j][3] + u8 * ws[4 * j + 3]) * scale);
        float4 u4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (ST) u4 = *reinterpret_cast<const float4*>(nimg + pt * BN + wn * 64 + 16 * q + 4 * j);
        int c[4];
        quant4_w<ST>(qs, xv, u4, c, ov1, ov2);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[4 * j + e] += c[e];
          s2[4 * j + e] += c[e] * c[e];
        }
        w4[j] = (uint32_t)(c[0] & 0xff) | ((uint32_t)(c[1] & 0xff) << 8) | ((uint32_t)(c[2] & 0xff) << 16) |
                ((uint32_t)c[3] << 24);
        // the quad's overflow counts are added here (left to itself, the compiler sinks all 4 MI NJ x 8
        // ballot masks to the end of the epilogue and spills them)
        asm volatile("" : "+s"(ov1), "+s"(ov2));
      }
      st16_always(p.yq, (uint32_t)(((int64_t)sample * hw + px) * C + n0 + wn * 64 + 16 * q), ok,
                  make_uint4(w4[0], w4[1], w4[2], w4[3]));
    }
  };

  // ---- the ring: k-step s reads stage s % S; step s issues step s + S - 1 into the stage step s - 1 read
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  const int nsteps = T * nk;
  int ct = 0, ckb = 0;
  uint32_t ehist = 0;  // bit k: an epilogue (MI stores) ran k + 1 steps ago
  for (int s = 0; s < nsteps; ++s) {
    ring_wait<S, CNT, MI>(__popc(ehist & ((1u << (S - 1)) - 1u)));
    __builtin_amdgcn_s_barrier();
    issue((s + S - 1) % S);
    const int8_t* sbase = lds + (s % S) * STAGE;
    ehist <<= 1;
    v4i fa[MI], fb[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = wn * 64 + j * 16 + r;
      fb[j] = *reinterpret_cast<const v4i*>(sbase + ABYTES + col * 64 + ((q ^ swz64(col)) << 4));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * TR + i * 16 + r;
      fa[i] = *reinterpret_cast<const v4i*>(sbase + row * 64 + ((q ^ swz64(row)) << 4));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fb[j], fa[i], acc[i][j], 0, 0, 0);
    if (++ckb == nk) {
      ckb = 0;
      epilogue(ct, sbase);
      ehist |= 1u;
      ++ct;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = v4i{0, 0, 0, 0};
    }
  }
  vm_wait<0>();  // the trailing dummy DMAs: nothing writes LDS past here

  // ---- channel sums: the 16 rows of a lane group by shuffles, the WM waves of a column slice in LDS
#pragma unroll
  for (int k = 0; k < 16; ++k) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      s1[k] += __shfl_xor(s1[k], m, 64);
      s2[k] += __shfl_xor(s2[k], m, 64);
    }
  }
  __syncthreads();  // every wave's last ring reads are done: the ring is reused as the exchange
  int* red = reinterpret_cast<int*>(lds);  // [WM][BN][2]
  if (r == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      red[((wm * BN) + wn * 64 + 16 * q + k) * 2 + 0] = s1[k];
      red[((wm * BN) + wn * 64 + 16 * q + k) * 2 + 1] = s2[k];
    }
  }
  __syncthreads();
  const int shard = (int)(L % LBT_NSHARD);
  if (t < 2 * BN) {
    const int a = t / BN, cl = t % BN;
    long long v = 0;
#pragma unroll
    for (int w = 0; w < WM; ++w) v += red[(w * BN + cl) * 2 + a];
    if (v) atomicAdd((unsigned long long*)&p.chsum[(int64_t)shard * 2 * C + a * C + n0 + cl], (unsigned long long)v);
  }
  if (lane == 0 && p.qout.counts) {
    int32_t* ctr = p.qout.counts + ((int64_t)p.qout.slot * LBT_NSHARD + shard) * LBT_CSTRIDE;
    if (ov1) atomicAdd(ctr, ov1);
    if (ov2) atomicAdd(ctr + 1, ov2);
  }
}

template <int BN, int S, bool ST>
void fwdq_go(const IgArgs& p, int nwg, int nrg, int rtiles, hipStream_t st) {
  constexpr size_t shm = (size_t)S * (256 * 64 + BN * 64 + 16 * BN * 4) + 1024 + (size_t)4 * BN + (size_t)4 * kBT;
  static bool attr_ = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&igemm_fwdq_kernel<BN, S, ST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    return true;
  }();
  (void)attr_;
  hipLaunchKernelGGL((igemm_fwdq_kernel<BN, S, ST>), dim3((unsigned)nwg), dim3(kBT), shm, st, p, nrg, rtiles);
}

// The persistent quantising forward (tuning fwdq_perm >= 2) takes a sample-blocked fwdq GEMM when its
// noise is a table (or rounding is to nearest), its column tiles divide the workgroup count (256: one per
// CU; fwdq_perm > 2: that many, to put many tiles on each in tests), and the int32 lane sums stay exact
// (<= 2047 tiles a workgroup). Ring stages: the tuning's 3 or 4, else LBT_FWDQ_S (default 4).
template <int BN>
bool launch_fwdq_persist(const IgArgs& p, int tstages, hipStream_t st) {
  static const int dstages = getenv_int("LBT_FWDQ_S", 4);
  const int stages = tstages >= 3 ? tstages : dstages;
  const int wgs = p.perm > 2 ? p.perm : 256;
  if (p.perm < 2 || !p.yq) return false;
  // default (2): only the one-k-block GEMMs (1x1, K = 64: ResNet-50 stage 1's conv-3 / shortcut), where it
  // measured faster (l1_c3 188 -> 147 us); the longer-K ones ran slower than the staged two-workgroup form
  // (l1_c2 108 -> 117 us; the ResNet-50 step 34.65 vs 36.34 ms with every fwdq GEMM persistent,
  // profiles/round5/persist_ab.txt). > 2: every sample-blocked fwdq GEMM (tests)
  if (p.perm == 2 && p.nkh * p.nkw * (p.cred / kBK) != 1) return false;
  const bool stoch = p.qout.stochastic != 0;
  if (stoch && !p.qout.noise) return false;
  const int ntn = p.ncol / BN;
  if (p.ncol % BN || wgs % ntn) return false;
  if ((int64_t)p.d.N * p.d.Ho * p.d.Wo * p.ncol >= ((int64_t)1 << 31)) return false;  // st16_always bound
  const int rtiles = (p.d.N + 15) / 16 * p.npb;
  int nrg = wgs / ntn;
  if (nrg > rtiles) nrg = rtiles;
  if ((rtiles + nrg - 1) / nrg > 2047) return false;
  const int nwg = nrg * ntn;
#define LBT_FQ(S_)                                                      \
  do {                                                                  \
    if (stoch) fwdq_go<BN, S_, true>(p, nwg, nrg, rtiles, st);          \
    else fwdq_go<BN, S_, false>(p, nwg, nrg, rtiles, st);               \
  } while (0)
  if (stages <= 3) LBT_FQ(3); else LBT_FQ(4);
#undef LBT_FQ
  return true;
}

// ------------------------------------------------------ persistent 16-bit dgrad + BN pass A (bn1 / bn2)
// igemm_dgrada_kernel: lbt_conv_dgrad_igemm_bna (unit-stride 16-bit dgrad whose dx feeds ReLU_q +
// Rescale_q + Normalization_q backward, mask from R) in igemm_fwdq_kernel's form, when both gradient
// quantisers are stochastic with noise tables (the models' configuration): one workgroup per CU owning a
// 64-column tile (dx channels) and a strided set of sample-blocked row tiles, an S-stage LDS-DMA ring
// across tile boundaries carrying A (256 rows x 64 16-bit codes), B (64 weight columns, loaded PERMUTED
// so a lane's accumulators are 16 consecutive channels of one row) and, with a tile's last k-block, both
// quantisers' noise for its 16 pixels. The epilogue runs pass A straight from the accumulators
// (passa_epilogue's arithmetic, element for element): the lane's R and qn codes are one 16-byte load
// each, its G codes one 32-byte store; the four channel sums stay in registers across the workgroup's
// tiles (its columns are fixed) and leave once. Rows outside the batch / image carry dx = 0 exactly
// (a = 0 codes), so they quantise to 0 and add nothing; their loads read row 0 and their stores are skipped.
template <int S>
__global__ __launch_bounds__(kBT, 1) void igemm_dgrada_kernel(IgArgs p, int nrg, int rtiles) {
  constexpr int BN = 64, BM = 256, WM = 8, TR = BM / WM, MI = TR / 16, NJ = 4;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 64, NBYTES = 2 * 16 * BN * 4;
  constexpr int STAGE = ABYTES + BBYTES + NBYTES;
  constexpr int GA = ABYTES / 1024 / 8;  // 4: A instructions per wave per k-block (8 rows each)
  constexpr int CNT = GA + 2;            // + B (waves 0-3, else dummy) + noise (waves 0-3 qrg, 4-7 qng)
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  int8_t* dummy = lds + S * STAGE;
  int* wsl = reinterpret_cast<int*>(dummy + 1024);            // [64] sum_k W per column
  float* gbl = reinterpret_cast<float*>(wsl + BN);            // [2][64] gamma_q | beta_q of the columns
  int* wpart = reinterpret_cast<int*>(gbl + 2 * BN);          // [8][64]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave;
  const int r = lane & 15, q = lane >> 4;
  const int ntn = p.ncol / BN;
  const uint32_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const uint32_t L = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int cn = (int)(L % (uint32_t)ntn), rg = (int)(L / (uint32_t)ntn);
  const int n0 = cn * BN;
  const int T = rg < rtiles ? (rtiles - 1 - rg) / nrg + 1 : 0;
  if (T == 0) return;
  const lbt_conv_desc& d = p.d;
  const lbt_dgrad_bna& bn = p.bna;
  const int C = p.ncol, N = d.N, hw = p.ch * p.cw, OW = p.cw, npb = p.npb;
  const int SH = d.Ho, SW = d.Wo;  // the gathered image (g) of a unit-stride dgrad
  const int cblocks = p.cred / kBK, nk = p.nkh * p.nkw * cblocks;
  const int8_t* fill = reinterpret_cast<const int8_t*>(zi());

  // ---- per-column constants: sum_k W (16-bit codes: the + 128 sum W term), gamma_q, beta_q
  {
    const int ch = t % BN, part = t / BN;
    int s = 0;
    const int8_t* col = p.b + (int64_t)(n0 + ch) * p.ks * 16;
    for (int c = part; c < nk * 4; c += 8) {
      const int4 v = *reinterpret_cast<const int4*>(col + c * 16);
      s = __builtin_amdgcn_sdot4(v.x, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(v.y, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(v.z, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(v.w, 0x01010101, s, false);
    }
    wpart[part * BN + ch] = s;
    if (t < 2 * BN) gbl[t] = bn.gb[(t / BN) * C + n0 + t % BN];
  }
  __syncthreads();
  if (t < BN) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += wpart[k * BN + t];
    wsl[t] = s;
  }
  __syncthreads();

  // ---- DMA geometry. A (16-bit codes, 128-byte rows): instruction g covers rows (wave + 8 g) * 8 .. + 7
  int aseg[GA];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int row = (wave + 8 * g) * 8 + lane / 8;
    aseg[g] = (lane % 8) ^ swz128(row);
  }
  const bool bact = wave < 4;
  int bcol, bseg;
  {
    const int cl = (wave & 3) * 16 + lane / 4;
    const int pc = (((cl & 15) >> 2) << 4) | (((cl >> 4) & 3) << 2) | (cl & 3);
    bcol = n0 + pc;
    bseg = (lane % 4) ^ swz64(cl);
  }
  // noise: waves 0-3 qrg, 4-7 qng; instruction covers 4 pixels x 64 floats of its quantiser's tile image
  const float* ntab = wave < 4 ? bn.qrg.noise : bn.qng.noise;
  const int npl = (wave & 3) * 4 + lane / 16, nseg = lane % 16;

  int it = 0, ikb = 0;
  int an[GA], ay[GA], ax[GA];
  bool arow[GA];
  int64_t noff = 0;
  auto set_rows = [&](int k) {
    const uint32_t rt = (uint32_t)(rg + k * nrg);
    const int sb = (int)(rt / (uint32_t)npb), pb = (int)(rt % (uint32_t)npb);
#pragma unroll
    for (int g = 0; g < GA; ++g) {
      const int row = (wave + 8 * g) * 8 + lane / 8;
      const int sm = sb * 16 + (row & 15), px = pb * 16 + (row >> 4);
      arow[g] = sm < N && px < hw;
      const uint32_t pu = (uint32_t)(arow[g] ? px : 0);
      ax[g] = (int)(pu % (uint32_t)OW);
      ay[g] = (int)(pu / (uint32_t)OW);
      an[g] = arow[g] ? sm : 0;
    }
    const int px = pb * 16 + npl;
    noff = (int64_t)(px < hw ? px : 0) * C + n0 + 4 * nseg;
  };
  set_rows(0);
  auto issue = [&](int st) {
    int8_t* sb = lds + st * STAGE;
    if (it < T) {
      const int kb = ikb;
      const int tap = kb / cblocks, cb = kb - tap * cblocks;
      const int th = tap / p.nkw, tw = tap - th * p.nkw;
      const int kbw = (th * d.KW + tw) * cblocks + cb;  // unit stride: kh = th, kw = tw
#pragma unroll
      for (int g = 0; g < GA; ++g) {
        const int sy = ay[g] + p.oy - th, sx = ax[g] + p.ox - tw;
        const bool ok = (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW && arow[g];
        const int8_t* src = fill;
        if (ok) {
          const uint32_t pix = (uint32_t)((an[g] * SH + sy) * SW + sx);
          src = reinterpret_cast<const int8_t*>(p.a) + (uint64_t)(pix * (uint32_t)p.cred + (uint32_t)(cb * kBK)) * 2 +
                aseg[g] * 16;
        }
        __builtin_amdgcn_global_load_lds(src, (lds_vptr)(sb + (wave + 8 * g) * 1024), 16, 0, 0);
      }
      {
        const int8_t* src = bact ? p.b + ((uint32_t)(bcol * p.ks + kbw * 4 + bseg) << 4) : fill;
        __builtin_amdgcn_global_load_lds(src, (lds_vptr)(bact ? sb + ABYTES + wave * 1024 : dummy), 16, 0, 0);
      }
      {
        const bool nl = kb == nk - 1;
        const int8_t* src = nl ? reinterpret_cast<const int8_t*>(ntab + noff) : fill;
        __builtin_amdgcn_global_load_lds(src, (lds_vptr)(nl ? sb + ABYTES + BBYTES + wave * 1024 : dummy), 16, 0, 0);
      }
      if (++ikb == nk) {
        ikb = 0;
        if (++it < T) set_rows(it);
      }
    } else {
#pragma unroll
      for (int g = 0; g < CNT; ++g) __builtin_amdgcn_global_load_lds(fill, (lds_vptr)dummy, 16, 0, 0);
    }
  };

  const QState srg = qstate(bn.qrg), sng = qstate(bn.qng);
  const float sr = qstate(bn.qr).inv_m;
  const float scale = ldexpf(1.0f, -(frac_exp(p.qa) + frac_exp(p.qb)));
  v4i acc[2][MI][NJ];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[a][i][j] = v4i{0, 0, 0, 0};
  int sm[4][16];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int k = 0; k < 16; ++k) sm[a][k] = 0;
  int ov0 = 0, ov1 = 0, ov2 = 0, ov3 = 0;

  auto epilogue = [&](int k, const int8_t* sbase) {
    const uint32_t rt = (uint32_t)(rg + k * nrg);
    const int sb = (int)(rt / (uint32_t)npb), pb = (int)(rt % (uint32_t)npb);
    const int sample = sb * 16 + r;
    const float* n1 = reinterpret_cast<const float*>(sbase + ABYTES + BBYTES);
    const float* n2 = n1 + 16 * BN;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int pt = wm * MI + i, px = pb * 16 + pt;
      const bool ok = sample < N && px < hw;
      const int64_t off = ok ? ((int64_t)sample * hw + px) * C + n0 + 16 * q : 0;
      const int4 R16 = *reinterpret_cast<const int4*>(bn.R + off);
      const int4 Q16 = *reinterpret_cast<const int4*>(bn.qn + off);
      const int Rw[4] = {R16.x, R16.y, R16.z, R16.w}, Qw[4] = {Q16.x, Q16.y, Q16.z, Q16.w};
      uint32_t gw[8];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int4 ws4 = *reinterpret_cast<const int4*>(wsl + 16 * q + 4 * j);
        const float4 g4 = *reinterpret_cast<const float4*>(gbl + 16 * q + 4 * j);
        const float4 b4 = *reinterpret_cast<const float4*>(gbl + BN + 16 * q + 4 * j);
        const int wsv[4] = {ws4.x, ws4.y, ws4.z, ws4.w};
        const float gam[4] = {g4.x, g4.y, g4.z, g4.w}, bet[4] = {b4.x, b4.y, b4.z, b4.w};
        int R[4], Q[4];
        float dv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          R[e] = (int)(int8_t)(Rw[j] >> (8 * e));
          Q[e] = (int)(int8_t)(Qw[j] >> (8 * e));
          const double hs = (double)acc[0][i][j][e] * 256.0;
          const double ls = (double)(acc[1][i][j][e] + 128 * wsv[e]);
          const float dx = (float)(hs + ls) * scale;
          const float xr = (float)R[e] * sr;  // the ReLU mask recomputed from R (bn.hip chain_bwd_a)
          const float m1 = xr * gam[e];
          const float yv = m1 + bet[e];
          dv[e] = yv > 0.f ? dx : 0.f;
        }
        const float4 u1 = *reinterpret_cast<const float4*>(n1 + pt * BN + 16 * q + 4 * j);
        const float4 u2 = *reinterpret_cast<const float4*>(n2 + pt * BN + 16 * q + 4 * j);
        int G2[4], G[4];
        quant4_w<true>(srg, make_float4(dv[0], dv[1], dv[2], dv[3]), u1, G2, ov0, ov1);
        const pf2 im = pk(srg.inv_m, srg.inv_m);
        const pf2 gh0 = pcvt(G2[0], G2[1]) * im, gh1 = pcvt(G2[2], G2[3]) * im;
        const pf2 dd0 = gh0 * pk(gam[0], gam[1]), dd1 = gh1 * pk(gam[2], gam[3]);
        quant4_w<true>(sng, make_float4(dd0.x, dd0.y, dd1.x, dd1.y), u2, G, ov2, ov3);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sm[0][4 * j + e] += G2[e] * R[e];
          sm[1][4 * j + e] += G2[e];
          sm[2][4 * j + e] += G[e];
          sm[3][4 * j + e] += G[e] * Q[e];
        }
        gw[2 * j] = (uint32_t)(G[0] & 0xffff) | ((uint32_t)G[1] << 16);
        gw[2 * j + 1] = (uint32_t)(G[2] & 0xffff) | ((uint32_t)G[3] << 16);
        asm volatile("" : "+s"(ov0), "+s"(ov1), "+s"(ov2), "+s"(ov3));  // (see igemm_fwdq_kernel)
      }
      st16_always(bn.gout, (uint32_t)(off * 2), ok, make_uint4(gw[0], gw[1], gw[2], gw[3]));
      st16_always(bn.gout, (uint32_t)(off * 2 + 16), ok, make_uint4(gw[4], gw[5], gw[6], gw[7]));
    }
  };

  // ---- the ring (igemm_fwdq_kernel's), 16-bit A fragments split into hi / lo' at the MFMA
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  const int nsteps = T * nk;
  int ct = 0, ckb = 0;
  uint32_t ehist = 0;  // bit k: an epilogue (2 MI stores) ran k + 1 steps ago
  for (int s = 0; s < nsteps; ++s) {
    ring_wait<S, CNT, 2 * MI>(__popc(ehist & ((1u << (S - 1)) - 1u)));
    __builtin_amdgcn_s_barrier();
    issue((s + S - 1) % S);
    const int8_t* sbase = lds + (s % S) * STAGE;
    ehist <<= 1;
    v4i fb[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = j * 16 + r;
      fb[j] = *reinterpret_cast<const v4i*>(sbase + ABYTES + col * 64 + ((q ^ swz64(col)) << 4));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * TR + i * 16 + r;
      const int f = swz128(row);
      const v4i c0 = *reinterpret_cast<const v4i*>(sbase + row * 128 + (((2 * q) ^ f) << 4));
      const v4i c1 = *reinterpret_cast<const v4i*>(sbase + row * 128 + (((2 * q + 1) ^ f) << 4));
      const uint32_t w[8] = {(uint32_t)c0[0], (uint32_t)c0[1], (uint32_t)c0[2], (uint32_t)c0[3],
                             (uint32_t)c1[0], (uint32_t)c1[1], (uint32_t)c1[2], (uint32_t)c1[3]};
      v4i hi, lo;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        hi[u] = (int)__builtin_amdgcn_perm(w[2 * u + 1], w[2 * u], 0x07050301u);
        lo[u] = (int)(__builtin_amdgcn_perm(w[2 * u + 1], w[2 * u], 0x06040200u) ^ 0x80808080u);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[0][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fb[j], hi, acc[0][i][j], 0, 0, 0);
        acc[1][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fb[j], lo, acc[1][i][j], 0, 0, 0);
      }
    }
    if (++ckb == nk) {
      ckb = 0;
      epilogue(ct, sbase);
      ehist |= 1u;
      ++ct;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[a][i][j] = v4i{0, 0, 0, 0};
    }
  }
  vm_wait<0>();

  // ---- the four channel sums (a lane's int32 partials are exact for <= 255 tiles: 2 T products of
  // <= 2^22), widened: the 16 rows of a lane group by shuffles, the 8 waves in LDS
  __syncthreads();
  long long* red = reinterpret_cast<long long*>(lds);  // [8 waves][4 sums][64 columns]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      long long v = sm[a][k];
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m, 64);
      if (r == 0) red[(wm * 4 + a) * BN + 16 * q + k] = v;
    }
  __syncthreads();
  const int shard = (int)(L % LBT_NSHARD);
  if (t < 4 * BN) {
    const int a = t / BN, cl = t % BN;
    long long v = 0;
#pragma unroll
    for (int w = 0; w < WM; ++w) v += red[(w * 4 + a) * BN + cl];
    if (v) atomicAdd((unsigned long long*)&bn.sums[(int64_t)shard * 4 * C + a * C + n0 + cl], (unsigned long long)v);
  }
  if (lane == 0) {
    if (bn.qrg.counts) {
      int32_t* ct2 = bn.qrg.counts + ((int64_t)bn.qrg.slot * LBT_NSHARD + shard) * LBT_CSTRIDE;
      if (ov0) atomicAdd(ct2, ov0);
      if (ov1) atomicAdd(ct2 + 1, ov1);
    }
    if (bn.qng.counts) {
      int32_t* ct2 = bn.qng.counts + ((int64_t)bn.qng.slot * LBT_NSHARD + shard) * LBT_CSTRIDE;
      if (ov2) atomicAdd(ct2, ov2);
      if (ov3) atomicAdd(ct2 + 1, ov3);
    }
  }
}

template <int S>
void dgrada_go(const IgArgs& p, int nwg, int nrg, int rtiles, hipStream_t st) {
  constexpr size_t shm = (size_t)S * (256 * 128 + 64 * 64 + 2 * 16 * 64 * 4) + 1024 + 64 * 4 + 128 * 4 + 512 * 4;
  static bool attr_ = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&igemm_dgrada_kernel<S>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    return true;
  }();
  (void)attr_;
  hipLaunchKernelGGL((igemm_dgrada_kernel<S>), dim3((unsigned)nwg), dim3(kBT), shm, st, p, nrg, rtiles);
}

// The persistent dgrad + pass A (tuning fwdq_perm > 2, on that many workgroups): both gradient quantisers
// stochastic with noise tables, 64-column tiles dividing the workgroups, <= 255 tiles a workgroup; a
// 3-stage ring (132 KiB).
bool launch_dgrada_persist(const IgArgs& p, hipStream_t st) {
  // opt-in (fwdq_perm > 2, on that many workgroups): bit-exact, but slower than the staged form on every
  // ResNet-50 shape measured (l1_c2 206 -> 247 us, l1_c3 175 -> 199, l3_c2 131 -> 187;
  // profiles/round5/persist_ab.txt)
  const int wgs = p.perm;
  if (p.perm <= 2 || p.has_bna != 1) return false;
  const lbt_dgrad_bna& b = p.bna;
  if (!b.qrg.stochastic || !b.qng.stochastic || !b.qrg.noise || !b.qng.noise) return false;
  const int ntn = p.ncol / 64;
  if (p.ncol % 64 || wgs % ntn || p.cred % kBK) return false;
  // the 16-bit G codes leave through st16_always at byte offset off * 2 of a buffer resource whose
  // num_records is 2^31 - 1: a larger image would wrap or be dropped silently, so it takes the staged form
  if ((int64_t)p.d.N * p.d.H * p.d.W * p.d.Cin * 2 >= ((int64_t)1 << 31)) return false;
  const int rtiles = (p.d.N + 15) / 16 * p.npb;
  int nrg = wgs / ntn;
  if (nrg > rtiles) nrg = rtiles;
  if ((rtiles + nrg - 1) / nrg > 255) return false;  // int32 lane sums exact (see the kernel)
  dgrada_go<3>(p, nrg * ntn, nrg, rtiles, st);
  return true;
}

// one igemm_big_kernel instantiation: dynamic LDS = the S-stage ring, or (HALO) two A windows of 384
// rows + a 3-stage B ring
template <int MODE, bool A16, bool ADD, int BN, int S, int BNA, bool HALO>
void big_go(const IgArgs& p, int64_t tiles, hipStream_t st) {
  constexpr int BM = 256, ROWB = A16 ? 128 : 64;
  constexpr size_t ring = HALO ? (size_t)2 * 384 * ROWB + (size_t)3 * BN * 64 : (size_t)S * (BM * ROWB + BN * 64);
  // the staged dx tile + the channel-sum exchange of the pass-A epilogue
  constexpr size_t shm = (BNA && ring < (size_t)kXBytes + 8192) ? (size_t)kXBytes + 8192 : ring;
  static bool attr_ = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&igemm_big_kernel<MODE, A16, ADD, BN, S, BNA, HALO>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    return true;
  }();
  (void)attr_;
  hipLaunchKernelGGL((igemm_big_kernel<MODE, A16, ADD, BN, S, BNA, HALO>), dim3((unsigned)tiles), dim3(kBT), shm, st,
                     p);
}

template <int MODE, bool A16, int BN, int S, bool HALO = false>
void launch_big_bn(IgArgs p, hipStream_t st) {
  static const int dbg = getenv_int("LBT_IGEMM_BIG_DBG", 0);
  p.dbg = dbg;
  // sample-blocked tiles only for the instantiations that decode them (the kernel's PERM)
  const bool qperm = MODE == MODE_FWD && !A16 && BN <= 128 && S == 2 && !HALO && p.perm && p.yq;
  const bool bna = MODE == MODE_DGRAD && A16 && BN == 64 && !HALO && p.has_bna;
  if (!qperm && !bna) p.perm = 0;
  const int64_t rtiles = p.perm ? (int64_t)((p.d.N + 15) / 16) * p.npb : (p.M + 255) / 256;
  const int64_t tiles = rtiles * (p.ncol / BN);
  if constexpr (MODE == MODE_DGRAD && A16 && BN == 64 && !HALO) {
    if (p.has_bna == 1) return big_go<MODE, A16, false, BN, S, 1, HALO>(p, tiles, st);
    if (p.has_bna == 2 && p.bn3.nbn == 1) return big_go<MODE, A16, false, BN, S, 2, HALO>(p, tiles, st);
    if (p.has_bna == 2) return big_go<MODE, A16, false, BN, S, 3, HALO>(p, tiles, st);
  }
  if constexpr (MODE == MODE_FWD && !A16 && BN <= 128 && S == 2 && !HALO) {
    if (qperm) return big_go<MODE, A16, false, BN, S, 4, HALO>(p, tiles, st);
  }
  if (MODE == MODE_DGRAD && p.add_src) big_go<MODE, A16, MODE == MODE_DGRAD, BN, S, 0, HALO>(p, tiles, st);
  else big_go<MODE, A16, false, BN, S, 0, HALO>(p, tiles, st);
}

// Selection of the 256-row LDS-DMA kernel (lbt_igemm_tuning, include/lbt_dfxp.h): read per call,
// so a test can force the kernel onto any shape and variant. Defaults from the environment at the
// first use (LBT_IGEMM_BIG, LBT_IGEMM_BIG_MIN, LBT_IGEMM_BIG_S, LBT_IGEMM_BIG_BN256) -- the measured
// choice: on, >= 200 tiles, 2 stages, 128-column tiles at most.
lbt_igemm_tuning& big_tuning() {
  static lbt_igemm_tuning t = [] {
    lbt_igemm_tuning v;
    v.big = getenv_int("LBT_IGEMM_BIG", 1);
    v.min_tiles = getenv_int("LBT_IGEMM_BIG_MIN", 200);
    v.stages = getenv_int("LBT_IGEMM_BIG_S", 2);
    v.max_bn = getenv_int("LBT_IGEMM_BIG_BN256", 0) ? 256 : 128;
    v.halo = getenv_int("LBT_IGEMM_HALO", 1);  // bit 0: int8 codes (fwd), bit 1: 16-bit codes (dgrad16)
    v.fwdq_perm = getenv_int("LBT_FWDQ_PERM", 2);
    v.launches = 0;
    return v;
  }();
  return t;
}

// The 256-row LDS-DMA kernel takes a GEMM when it is big enough to give every CU about one tile
// (min_tiles, default 200; big = 0: never) and is not split / classed.
template <int MODE, bool A16>
bool launch_big(const IgArgs& p, hipStream_t st) {
  const lbt_igemm_tuning tu = big_tuning();
  const int64_t tmin = tu.min_tiles;
  if (!tu.big || p.ksplit != 1 || p.ncol % 64 || p.cred % kBK) return false;
  if ((p.M + 255) / 256 * (p.ncol / 64) > 0x7fffffff) return false;
  // column tile: the widest (<= max_bn) that still gives min_tiles tiles (256 only without the
  // quantising epilogue and on request: its 8 x 4 accumulator tiles per wave spill)
  const int64_t mt = p.perm ? (int64_t)((p.d.N + 15) / 16) * p.npb : (p.M + 255) / 256;
  int bn = 0;
  if (!A16 && !p.yq && p.ncol % 256 == 0 && tu.max_bn >= 256 && mt * (p.ncol / 256) >= tmin) bn = 256;
  else if (tu.max_bn >= 128 && p.ncol % 128 == 0 && mt * (p.ncol / 128) >= tmin) bn = 128;
  else if (mt * (p.ncol / 64) >= tmin) bn = 64;
  if (!bn) return false;
  if (p.has_bna) bn = 64;  // the pass-A epilogues: 64-column tiles, 256 VGPRs (one workgroup per CU)
  // LDS ring depth (stages): 2 by default -- the probe on the ResNet-50 shapes measured the
  // occupancy of 2 stages (A8 BN 128: 48 KiB, two workgroups per CU) ahead of the latency hiding of 3-4
  // (72-96 KiB, one; the software-pipelined loop), except 3x3 dgrad16 at 28x28 / 14x14 (3-5 %).
  // A16 runs 3 stages for any request above 2 (4 stages of 128-byte A rows at BN 128 would take 160 KiB).
  const int S = tu.stages;
  // 3x3 / stride 1 / pad 1 with every tap (fwd, unit-stride dgrad) and W <= 63: the A window per
  // channel block (HALO), 64- and 128-column tiles
  const lbt_conv_desc& d = p.d;
  const bool halo = (tu.halo & (A16 ? 2 : 1)) && !p.perm && bn <= 128 && d.KH == 3 && d.KW == 3 && d.SH == 1 && d.SW == 1 && d.PT == 1 &&
                    d.PL == 1 && d.Ho == d.H && d.Wo == d.W && p.nkh == 3 && p.nkw == 3 && p.kh0 == 0 &&
                    p.kw0 == 0 && p.cw == d.W && p.ch == d.H && d.W <= 63 &&
                    // where it measured faster (profiles/r04p): one column tile (the window is not
                    // re-staged per column tile), or a chip the 128-column tiles would under-fill
                    (p.ncol == 64 || mt * (p.ncol / bn) < 256);
  if constexpr (MODE == MODE_DGRAD && A16) {
    if (p.has_bna == 1 && p.perm >= 2 && launch_dgrada_persist(p, st)) {
      ++big_tuning().launches;
      return true;
    }
  }
  if constexpr (MODE == MODE_FWD && !A16) {
    if (p.yq && p.perm >= 2 && bn <= 128 &&
        (bn == 128 ? launch_fwdq_persist<128>(p, S, st) : launch_fwdq_persist<64>(p, S, st))) {
      ++big_tuning().launches;
      return true;
    }
  }
  if (halo) {  // 64-column tiles: int8 codes two workgroups per CU (98 VGPRs, 60 KiB); 16-bit one (2 x 48 KiB windows)
    launch_big_bn<MODE, A16, 64, 2, true>(p, st);
  } else if (bn == 256) {
    if constexpr (!A16) launch_big_bn<MODE, A16, 256, 4>(p, st);
  } else if (bn == 128) {
    if (S <= 2) launch_big_bn<MODE, A16, 128, 2>(p, st);
    else if (S == 3 || A16) launch_big_bn<MODE, A16, 128, 3>(p, st);
    else launch_big_bn<MODE, A16, 128, 4>(p, st);
  } else {
    if (S <= 2) launch_big_bn<MODE, A16, 64, 2>(p, st);
    else if (S == 3) launch_big_bn<MODE, A16, 64, 3>(p, st);
    else launch_big_bn<MODE, A16, 64, 4>(p, st);
  }
  ++big_tuning().launches;
  return true;
}

template <int MODE, bool A16, int BM, int BN, bool CLS = false>
void launch_tile(const IgArgs& p, hipStream_t st) {
  const dim3 grid((unsigned)((p.M + BM - 1) / BM), (unsigned)((p.ncol + BN - 1) / BN), (unsigned)p.ksplit);
  // register stages in flight: a divisor of the split's k-block count (3x3 convs: 9 * Cin/64 -> 3;
  // 1x1: 2), 1 for the VGPR-heavy 128x128 tiles
  const int nk = p.nkh * p.nkw * (p.cred / kBK) / p.ksplit;
  const int D = (BM == 128 && BN == 128) ? 1 : (nk % 3 == 0 && !CLS ? 3 : (nk % 2 == 0 ? 2 : 1));
#define LBT_IG(DD)                                                                      \
  do {                                                                                  \
    if (MODE == MODE_DGRAD && p.add_src)                                                \
      hipLaunchKernelGGL((igemm_kernel<MODE, A16, true, BM, BN, DD, CLS>), grid, dim3(kT), 0, st, p);  \
    else                                                                                \
      hipLaunchKernelGGL((igemm_kernel<MODE, A16, false, BM, BN, DD, CLS>), grid, dim3(kT), 0, st, p); \
  } while (0)
  if constexpr (CLS) {
    if (D == 2) LBT_IG(2); else LBT_IG(1);
  } else {
    if (D == 3) LBT_IG(3); else if (D == 2) LBT_IG(2); else LBT_IG(1);
  }
#undef LBT_IG
  if (p.ksplit > 1) {
    const dim3 g2((unsigned)((p.M * p.ncol / 4 + 255) / 256));
    if (MODE == MODE_DGRAD && p.add_src)
      hipLaunchKernelGGL((igemm_splitk_reduce_kernel<A16, true>), g2, dim3(256), 0, st, p);
    else
      hipLaunchKernelGGL((igemm_splitk_reduce_kernel<A16, false>), g2, dim3(256), 0, st, p);
  }
}

// Split-K factor: when even 64 x 64-row tiles leave the chip with fewer than ~2 workgroups per CU
// and the k loop is long, the smallest divisor of the k-block count that reaches ~512 workgroups
// (each split keeping >= 4 k-blocks). 1 = no split.
int choose_ksplit(int64_t M, int ncol, int nk) {
  const int64_t tiles = ((M + 63) / 64) * ((ncol + 127) / 128);
  if (tiles >= 256 || nk < 8 || getenv_int("LBT_IGEMM_SPLITK", 1) == 0) return 1;
  static const int cand[] = {2, 3, 4, 6, 8, 9, 12, 16};
  int best = 1;
  for (int c : cand) {
    if (nk % c || nk / c < 4) continue;
    best = c;
    if (tiles * c >= 512) break;
  }
  return best;
}

// workspace bytes a split launch needs (0: none)
int64_t splitk_bytes(int64_t M, int ncol, int nk, bool a16) {
  const int ks = choose_ksplit(M, ncol, nk);
  return ks > 1 ? (int64_t)ks * (a16 ? 2 : 1) * M * ncol * 4 : 0;
}

// Tile choice: 64 columns when the GEMM has <= 64 (no MFMAs on padding columns), and 64 rows
// when 128-row tiles would leave the 256 CUs without two workgroups each.
template <int MODE, bool A16, bool CLS = false>
int launch(const IgArgs& p, hipStream_t st) {
  const int64_t mb = (p.M + kBM - 1) / kBM;
  if (mb > 0x7fffffff / 2 || (p.ncol + 63) / 64 > 65535) return LBT_EINVAL;
  const bool bn64 = p.ncol <= 64 || getenv_int("LBT_IGEMM_BN", 128) == 64;
  if constexpr (CLS) {  // parity classes of a strided dgrad: 64-row tiles only (fewer variants)
    if (bn64) launch_tile<MODE, A16, 64, 64, true>(p, st); else launch_tile<MODE, A16, 64, 128, true>(p, st);
    return (int)hipGetLastError();
  }
  if (launch_big<MODE, A16>(p, st)) return (int)hipGetLastError();
  const int64_t nb = (p.ncol + (bn64 ? 63 : 127)) / (bn64 ? 64 : 128);
  // ... and always for 16-bit codes when the tile would be 128 x 128: that variant needs 256 VGPRs
  // (one wave per SIMD), which leaves its fp32 epilogue stores unhidden
  const bool bm64 = mb * nb < getenv_int("LBT_IGEMM_MIN_WG", 512) || (A16 && !bn64) || p.ksplit > 1;
  if (bm64) {
    if (bn64) launch_tile<MODE, A16, 64, 64>(p, st); else launch_tile<MODE, A16, 64, 128>(p, st);
  } else {
    if (bn64) launch_tile<MODE, A16, 128, 64>(p, st); else launch_tile<MODE, A16, 128, 128>(p, st);
  }
  return (int)hipGetLastError();
}

bool desc_ok(const lbt_conv_desc& d) {
  return d.N > 0 && d.H > 0 && d.W > 0 && d.KH > 0 && d.KW > 0 && d.SH > 0 && d.SW > 0 && d.Ho > 0 && d.Wo > 0 &&
         d.Cin > 0 && d.Cout > 0;
}

// dx of a parity class no tap reaches (a 1x1 stride-2 conv's odd pixels): add_src, or 0
__global__ __launch_bounds__(256) void dgrad_fill_class_kernel(IgArgs p) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= p.M * p.ncol) return;
  const int64_t m = i4 / p.ncol;
  const int c = (int)(i4 - m * p.ncol);
  const lbt_conv_desc& d = p.d;
  const int64_t xc = m % p.cw, t2 = m / p.cw, yc = t2 % p.ch, n = t2 / p.ch;
  const int64_t off = ((n * d.H + yc * d.SH + p.cpy) * d.W + xc * d.SW + p.cpx) * p.ncol + c;
  *reinterpret_cast<float4*>(p.y + off) =
      p.add_src ? *reinterpret_cast<const float4*>(p.add_src + off) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Strided dgrad as SH x SW parity-class GEMMs (IgArgs: nkh ...): each class runs only the taps that
// reach it, so no MFMA multiplies the zero rows of the stride's implicit upsampling. Never split.
template <bool A16>
int dgrad_classes(IgArgs p, hipStream_t st) {
  const lbt_conv_desc& d = p.d;
  if ((int64_t)d.N * d.H * d.W * d.Cin >= ((int64_t)1 << 31)) return LBT_EINVAL;  // 32-bit row offsets
  p.ksplit = 1;
  for (int py = 0; py < d.SH; ++py)
    for (int px = 0; px < d.SW; ++px) {
      const int ch = py < d.H ? (d.H - py + d.SH - 1) / d.SH : 0;
      const int cw = px < d.W ? (d.W - px + d.SW - 1) / d.SW : 0;
      if (!ch || !cw) continue;
      const int kh0 = (py + d.PT) % d.SH, kw0 = (px + d.PL) % d.SW;
      p.nkh = kh0 < d.KH ? (d.KH - kh0 + d.SH - 1) / d.SH : 0;
      p.nkw = kw0 < d.KW ? (d.KW - kw0 + d.SW - 1) / d.SW : 0;
      p.kh0 = kh0; p.kw0 = kw0;
      p.oy = (py + d.PT - kh0) / d.SH; p.ox = (px + d.PL - kw0) / d.SW;
      p.cpy = py; p.cpx = px; p.ch = ch; p.cw = cw;
      p.M = (int64_t)d.N * ch * cw;
      int rc;
      if (!p.nkh || !p.nkw) {
        hipLaunchKernelGGL(dgrad_fill_class_kernel, dim3((unsigned)((p.M * p.ncol / 4 + 255) / 256)), dim3(256), 0, st,
                           p);
        rc = (int)hipGetLastError();
      } else {
        rc = launch<MODE_DGRAD, A16, true>(p, st);
      }
      if (rc) return rc;
    }
  return 0;
}

}  // namespace

// a_kind: 0 int8 signed, 1 int8 offset (q - 128; needs colsum = sum_k W per output channel), 2 int16
extern "C" int lbt_conv_fwd_igemm(const void* xq, int32_t a_kind, const int8_t* wf, int32_t ksf,
                                  const int32_t* colsum, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y,
                                  void* stream) {
  if (!desc_ok(d) || d.Cin % kBK || d.Cout % 16 || !y || !wf) return LBT_EINVAL;
  if ((int64_t)d.KH * d.KW * d.Cin * 255 * 128 >= ((int64_t)1 << 31)) return LBT_EINVAL;  // int32 epilogue sums
  if ((int64_t)d.N * d.H * d.W * d.Cin >= ((int64_t)1 << 31) || (int64_t)ksf * 16 * d.Cout >= ((int64_t)1 << 31))
    return LBT_EINVAL;  // 32-bit operand offsets
  if (ksf * 16 < d.KH * d.KW * d.Cin) return LBT_EINVAL;
  IgArgs p{};
  p.a = xq; p.b = wf; p.ks = ksf; p.cred = d.Cin; p.a_u8off = a_kind == 1; p.d = d; p.qa = qx; p.qb = qw;
  p.colsum = colsum; p.y = y; p.add_src = nullptr; p.M = (int64_t)d.N * d.Ho * d.Wo; p.ncol = d.Cout;
  if (p.M * p.ncol >= ((int64_t)1 << 40)) return LBT_EINVAL;
  p.ksplit = 1;
  all_taps(p, MODE_FWD);
  hipStream_t st = (hipStream_t)stream;
  return a_kind == 2 ? launch<MODE_FWD, true>(p, st) : launch<MODE_FWD, false>(p, st);
}

// Forward whose epilogue is the consuming Normalization_q's input quantiser (no fp32 y): int8 codes
// yq + qout's overflow counters + exact channel sums chsum[NSHARD][2 * Cout]. A8 codes only (a_kind
// 0 / 1); never split (short-M GEMMs use lbt_conv_fwd_igemm_ws + lbt_dfxp_quantize).
extern "C" int lbt_conv_fwd_igemm_q(const void* xq, int32_t a_kind, const int8_t* wf, int32_t ksf, lbt_conv_desc d,
                                    lbt_qdesc qx, lbt_qdesc qw, int8_t* yq, lbt_qdesc qout, int64_t* chsum,
                                    void* stream) {
  if (!desc_ok(d) || d.Cin % kBK || d.Cout % 16 || !yq || !wf || !chsum || a_kind == 2) return LBT_EINVAL;
  if (qout.bits < 2 || qout.bits > 8) return LBT_EINVAL;
  if ((int64_t)d.KH * d.KW * d.Cin * 255 * 128 >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if ((int64_t)d.N * d.H * d.W * d.Cin >= ((int64_t)1 << 31) || (int64_t)ksf * 16 * d.Cout >= ((int64_t)1 << 31))
    return LBT_EINVAL;
  if (ksf * 16 < d.KH * d.KW * d.Cin) return LBT_EINVAL;
  IgArgs p{};
  p.a = xq; p.b = wf; p.ks = ksf; p.cred = d.Cin; p.a_u8off = a_kind == 1; p.d = d; p.qa = qx; p.qb = qw;
  p.M = (int64_t)d.N * d.Ho * d.Wo; p.ncol = d.Cout;
  if (p.M * p.ncol >= ((int64_t)1 << 31)) return LBT_EINVAL;
  p.ksplit = 1;
  all_taps(p, MODE_FWD);
  p.yq = yq; p.qout = qout; p.chsum = chsum; p.hw = d.Ho * d.Wo;
  // the 256-row kernels' quantising epilogue on sample-blocked tiles (1: quantq_epilogue, >= 2: the
  // persistent igemm_fwdq_kernel where it applies)
  p.perm = big_tuning().fwdq_perm > 0 ? big_tuning().fwdq_perm : 0;
  p.npb = (d.Ho * d.Wo + 15) / 16;
  return launch<MODE_FWD, false>(p, (hipStream_t)stream);
}

// Workspace of the split-K variants below (0: that GEMM does not split). mode 0 fwd, 1 dgrad.
extern "C" int64_t lbt_igemm_workspace_bytes(lbt_conv_desc d, int32_t mode, int32_t a16) {
  if (!desc_ok(d)) return 0;
  if (mode == 0)
    return splitk_bytes((int64_t)d.N * d.Ho * d.Wo, d.Cout, d.KH * d.KW * (d.Cin / kBK), a16 != 0);
  if (d.SH > 1 || d.SW > 1) return 0;  // strided dgrad: parity classes, never split
  return splitk_bytes((int64_t)d.N * d.H * d.W, d.Cin, d.KH * d.KW * (d.Cout / kBK), a16 != 0);
}

// lbt_igemm_tuning: the 256-row kernel's selection, read by every wide fwd / dgrad call after this
extern "C" int lbt_igemm_get_tuning(lbt_igemm_tuning* out) {
  if (!out) return LBT_EINVAL;
  *out = big_tuning();
  return 0;
}

extern "C" int lbt_igemm_set_tuning(const lbt_igemm_tuning* t) {
  if (!t || t->min_tiles < 1 || t->stages < 2 || t->stages > 4 || (t->max_bn != 64 && t->max_bn != 128 && t->max_bn != 256) ||
      t->fwdq_perm < 0 || t->fwdq_perm > 4096)
    return LBT_EINVAL;
  lbt_igemm_tuning& cur = big_tuning();
  cur.big = t->big; cur.min_tiles = t->min_tiles; cur.stages = t->stages; cur.max_bn = t->max_bn;
  cur.halo = t->halo;
  cur.fwdq_perm = t->fwdq_perm;
  return 0;
}

// lbt_conv_fwd_igemm with a caller-owned workspace (ws_bytes >= lbt_igemm_workspace_bytes): the
// short-M / long-K GEMMs split K over workgroups, exact int32 partials, one reduce launch after.
extern "C" int lbt_conv_fwd_igemm_ws(const void* xq, int32_t a_kind, const int8_t* wf, int32_t ksf,
                                     const int32_t* colsum, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y,
                                     void* ws, int64_t ws_bytes, void* stream) {
  if (!desc_ok(d) || d.Cin % kBK || d.Cout % 16 || !y || !wf) return LBT_EINVAL;
  if ((int64_t)d.KH * d.KW * d.Cin * 255 * 128 >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if ((int64_t)d.N * d.H * d.W * d.Cin >= ((int64_t)1 << 31) || (int64_t)ksf * 16 * d.Cout >= ((int64_t)1 << 31))
    return LBT_EINVAL;
  if (ksf * 16 < d.KH * d.KW * d.Cin) return LBT_EINVAL;
  IgArgs p{};
  p.a = xq; p.b = wf; p.ks = ksf; p.cred = d.Cin; p.a_u8off = a_kind == 1; p.d = d; p.qa = qx; p.qb = qw;
  p.colsum = colsum; p.y = y; p.add_src = nullptr; p.M = (int64_t)d.N * d.Ho * d.Wo; p.ncol = d.Cout;
  if (p.M * p.ncol >= ((int64_t)1 << 31)) return LBT_EINVAL;
  const int64_t need = lbt_igemm_workspace_bytes(d, 0, a_kind == 2);
  p.ksplit = (need > 0 && ws && ws_bytes >= need) ? choose_ksplit(p.M, p.ncol, d.KH * d.KW * (d.Cin / kBK)) : 1;
  p.part = reinterpret_cast<int32_t*>(ws);
  all_taps(p, MODE_FWD);
  hipStream_t st = (hipStream_t)stream;
  return a_kind == 2 ? launch<MODE_FWD, true>(p, st) : launch<MODE_FWD, false>(p, st);
}

// g_i16: gradient codes are int16 (9..16-bit) instead of int8
extern "C" int lbt_conv_dgrad_igemm(const void* gq, int32_t g_i16, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                                    lbt_qdesc qg, lbt_qdesc qw, float* dx, const float* add_src, void* stream) {
  if (!desc_ok(d) || d.Cout % kBK || d.Cin % 16 || !dx || !wd) return LBT_EINVAL;
  if ((int64_t)d.KH * d.KW * d.Cout * 255 * 128 >= ((int64_t)1 << 31)) return LBT_EINVAL;  // int32 epilogue sums
  if ((int64_t)d.N * d.Ho * d.Wo * d.Cout >= ((int64_t)1 << 31) || (int64_t)ksd * 16 * d.Cin >= ((int64_t)1 << 31))
    return LBT_EINVAL;  // 32-bit operand offsets
  if (ksd * 16 < d.KH * d.KW * d.Cout) return LBT_EINVAL;
  IgArgs p{};
  p.a = gq; p.b = wd; p.ks = ksd; p.cred = d.Cout; p.a_u8off = 0; p.d = d; p.qa = qg; p.qb = qw;
  p.colsum = nullptr; p.y = dx; p.add_src = add_src; p.M = (int64_t)d.N * d.H * d.W; p.ncol = d.Cin;
  p.ksplit = 1;
  all_taps(p, MODE_DGRAD);
  hipStream_t st = (hipStream_t)stream;
  if (d.SH > 1 || d.SW > 1) return g_i16 ? dgrad_classes<true>(p, st) : dgrad_classes<false>(p, st);
  return g_i16 ? launch<MODE_DGRAD, true>(p, st) : launch<MODE_DGRAD, false>(p, st);
}

extern "C" int lbt_conv_dgrad_igemm_ws(const void* gq, int32_t g_i16, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                                       lbt_qdesc qg, lbt_qdesc qw, float* dx, const float* add_src, void* ws,
                                       int64_t ws_bytes, void* stream) {
  if (!desc_ok(d) || d.Cout % kBK || d.Cin % 16 || !dx || !wd) return LBT_EINVAL;
  if ((int64_t)d.KH * d.KW * d.Cout * 255 * 128 >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if ((int64_t)d.N * d.Ho * d.Wo * d.Cout >= ((int64_t)1 << 31) || (int64_t)ksd * 16 * d.Cin >= ((int64_t)1 << 31))
    return LBT_EINVAL;
  if (ksd * 16 < d.KH * d.KW * d.Cout) return LBT_EINVAL;
  IgArgs p{};
  p.a = gq; p.b = wd; p.ks = ksd; p.cred = d.Cout; p.a_u8off = 0; p.d = d; p.qa = qg; p.qb = qw;
  p.colsum = nullptr; p.y = dx; p.add_src = add_src; p.M = (int64_t)d.N * d.H * d.W; p.ncol = d.Cin;
  if (p.M * p.ncol >= ((int64_t)1 << 31)) return LBT_EINVAL;
  const int64_t need = lbt_igemm_workspace_bytes(d, 1, g_i16);
  p.ksplit = (need > 0 && ws && ws_bytes >= need) ? choose_ksplit(p.M, p.ncol, d.KH * d.KW * (d.Cout / kBK)) : 1;
  p.part = reinterpret_cast<int32_t*>(ws);
  all_taps(p, MODE_DGRAD);
  hipStream_t st = (hipStream_t)stream;
  if (d.SH > 1 || d.SW > 1) return g_i16 ? dgrad_classes<true>(p, st) : dgrad_classes<false>(p, st);
  return g_i16 ? launch<MODE_DGRAD, true>(p, st) : launch<MODE_DGRAD, false>(p, st);
}

// The dgrad with the mask_r BN pass A it feeds (include/lbt_dfxp.h lbt_dgrad_bna): in the 256-row
// kernel's epilogue when that kernel takes the GEMM, else dgrad into dx + lbt_bn_bwd_a_wide_masked.
// LBT_DGRAD_BNA=0: always the second form (A/B).
extern "C" int lbt_conv_dgrad_igemm_bna(const int16_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                                        lbt_qdesc qg, lbt_qdesc qw, const lbt_dgrad_bna* bna, float* dx, void* ws,
                                        int64_t ws_bytes, void* stream) {
  if (!bna || !dx || !desc_ok(d)) return LBT_EINVAL;
  const lbt_dgrad_bna& b = *bna;
  if (!b.R || !b.gb || !b.qn || !b.gout || !b.sums || b.qr.bits <= 0) return LBT_EINVAL;
  if (b.qrg.bits <= 0 || b.qrg.bits > 16 || b.qng.bits <= 0 || b.qng.bits > 16 || d.Cin % 4) return LBT_EINVAL;
  const int64_t rows = (int64_t)d.N * d.H * d.W, inner = (int64_t)d.H * d.W * d.Cin;
  hipStream_t st = (hipStream_t)stream;
  static const int fuse = getenv_int("LBT_DGRAD_BNA", 1);
  if (fuse && d.SH == 1 && d.SW == 1 && d.Cout % kBK == 0 && d.Cin % 64 == 0 &&
      (int64_t)d.KH * d.KW * d.Cout * 255 * 128 < ((int64_t)1 << 31) &&
      (int64_t)d.N * d.Ho * d.Wo * d.Cout < ((int64_t)1 << 31) && (int64_t)ksd * 16 * d.Cin < ((int64_t)1 << 31) &&
      ksd * 16 >= d.KH * d.KW * d.Cout && rows * d.Cin < ((int64_t)1 << 31) && lbt_igemm_workspace_bytes(d, 1, 1) == 0) {
    IgArgs p{};
    p.a = gq; p.b = wd; p.ks = ksd; p.cred = d.Cout; p.a_u8off = 0; p.d = d; p.qa = qg; p.qb = qw;
    p.colsum = nullptr; p.y = nullptr; p.add_src = nullptr; p.M = rows; p.ncol = d.Cin;
    p.ksplit = 1;
    all_taps(p, MODE_DGRAD);
    p.has_bna = 1;
    p.perm = big_tuning().fwdq_perm >= 2 ? big_tuning().fwdq_perm : 1;  // >= 2: the persistent form where it applies
    p.npb = (d.H * d.W + 15) / 16;
    p.bna = b;
    if (launch_big<MODE_DGRAD, true>(p, st)) return (int)hipGetLastError();
  }
  int rc = lbt_conv_dgrad_igemm_ws(gq, 1, wd, ksd, d, qg, qw, dx, nullptr, ws, ws_bytes, stream);
  if (rc) return rc;
  return lbt_bn_bwd_a_wide_masked(dx, nullptr, nullptr, nullptr, 1, b.qr, b.gb, nullptr, b.qrg, b.R, b.qng, b.qn,
                                  b.gout, nullptr, b.sums, rows, inner, d.Cin, stream);
}

extern "C" int lbt_conv_dgrad_igemm_bn3(const int16_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                                        lbt_qdesc qg, lbt_qdesc qw, const lbt_dgrad_bn3* bn3, float* dx, void* ws,
                                        int64_t ws_bytes, void* stream) {
  if (!bn3 || !dx || !desc_ok(d)) return LBT_EINVAL;
  const lbt_dgrad_bn3& b = *bn3;
  if (!b.g2 || !b.y_bits || b.nbn < 1 || b.nbn > 2 || d.Cin % 4) return LBT_EINVAL;
  for (int k = 0; k < b.nbn; ++k) {
    const lbt_bna_bn& n = b.bn[k];
    if (!n.R || !n.gamma_q || !n.qn || !n.gout || !n.sums) return LBT_EINVAL;
    if (n.qrg.bits <= 0 || n.qrg.bits > 16 || n.qng.bits <= 0 || n.qng.bits > 16) return LBT_EINVAL;
  }
  const int64_t rows = (int64_t)d.N * d.H * d.W, inner = (int64_t)d.H * d.W * d.Cin;
  hipStream_t st = (hipStream_t)stream;
  static const int fuse = getenv_int("LBT_DGRAD_BN3", 1);
  if (fuse && d.SH == 1 && d.SW == 1 && d.Cout % kBK == 0 && d.Cin % 64 == 0 &&
      (int64_t)d.KH * d.KW * d.Cout * 255 * 128 < ((int64_t)1 << 31) &&
      (int64_t)d.N * d.Ho * d.Wo * d.Cout < ((int64_t)1 << 31) && (int64_t)ksd * 16 * d.Cin < ((int64_t)1 << 31) &&
      ksd * 16 >= d.KH * d.KW * d.Cout && rows * d.Cin < ((int64_t)1 << 31) && lbt_igemm_workspace_bytes(d, 1, 1) == 0) {
    IgArgs p{};
    p.a = gq; p.b = wd; p.ks = ksd; p.cred = d.Cout; p.a_u8off = 0; p.d = d; p.qa = qg; p.qb = qw;
    p.colsum = nullptr; p.y = nullptr; p.add_src = nullptr; p.M = rows; p.ncol = d.Cin;
    p.ksplit = 1;
    all_taps(p, MODE_DGRAD);
    p.has_bna = 2;
    p.perm = 1;
    p.npb = (d.H * d.W + 15) / 16;
    p.bn3 = b;
    if (launch_big<MODE_DGRAD, true>(p, st)) return (int)hipGetLastError();
  }
  int rc = lbt_conv_dgrad_igemm_ws(gq, 1, wd, ksd, d, qg, qw, dx, nullptr, ws, ws_bytes, stream);
  for (int k = 0; k < b.nbn && !rc; ++k) {
    const lbt_bna_bn& n = b.bn[k];
    rc = lbt_bn_bwd_a_wide_masked(dx, b.g2, nullptr, b.y_bits, 0, lbt_qdesc{}, n.gamma_q, k == 0 ? b.gmask_out : nullptr,
                                  n.qrg, n.R, n.qng, n.qn, n.gout, nullptr, n.sums, rows, inner, d.Cin, stream);
  }
  return rc;
}

namespace {

// ----------------------------------------------------------------------------- wide wgrad
// dW[tap][ci][co] = sum_p x[p shifted by tap][ci] * g[p][co] for the wide layers. x is offset int8
// (x' = x - 128, post-ReLU 9-bit codes 0..255); g is int8 or int16 (G16: g = 256 gh + gl' + 128).
// Per workgroup: one tap, 64 ci x 64 co, a pixel range; each wave walks 64-pixel chunks, stores
// [pixel][16 B] LDS images and multiplies ds_read_b64_tr_b8 fragments (as conv_mfma.hip's wgrad).
// Exact identity (over every processed lane, invalid ones carrying x' = -128, g = 0):
//   sum x g = 256 sum x' gh + sum x' gl' + 128 sum x' + 128 (256 sum gh + sum gl' + 128 npix)
// (G8: sum x g = sum x' g + 128 sum g); the row / column sums come from MFMAs against ones.
// The 4 waves meet in LDS (int64), then one int64 atomic per output into shard (split % nshard).

constexpr int kWP = 64;

// STORE: the workgroup's partial is STORED into slab[split] (every element of slab[nsplit][K][Cout]
// has exactly one writer -- no zeroing, no atomics); else atomically added into shard split % nshard.
// Grid: 1-D over (split, tap x ci block, co block). xmap = 1 (default): XCD-aware order -- the
// workgroups of one pixel split (every ci / co block, which share that split's X and G chunks) are
// consecutive on ONE XCD, meant to serve the Cout/64-fold X and Cin/64-fold G re-reads of a 64 x 64 tile
// from that XCD's L2 (LBT_WGRAD_XMAP=1; measured 0.3 ms per ResNet-50 step SLOWER); xmap = 0 (default):
// split fastest (the former 3-D grid's order).
template <bool G16, bool STORE>
__global__ __launch_bounds__(kT, 1) void wgrad_wide_kernel(const int8_t* __restrict__ xq, const void* __restrict__ gq,
                                                        lbt_conv_desc d, long long* __restrict__ slab, int64_t P,
                                                        int nsplit, int nshard, int xmap) {
  constexpr int NG = G16 ? 2 : 1;  // G images: (gh, gl') or g
  constexpr int NBS = 4, COW = 16 * NBS;  // output-channel slices per workgroup
  // per wave: X [4 slices][64 px][16 B], G [NG][4 slices][64 px][16 B]; reused as the int64 tile
  __shared__ __attribute__((aligned(16))) int8_t lds[4][(4 + NBS * NG) * kWP * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int cib = d.Cin / 64, cob = d.Cout / 64;
  const uint32_t gy = (uint32_t)(d.KH * d.KW * cib), nblk = gy * (uint32_t)cob;
  uint32_t split, by, ob_;
  if (xmap) {
    const uint32_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
    const uint32_t t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
    split = t / nblk;
    const uint32_t b = t - split * nblk;
    by = b / (uint32_t)cob;
    ob_ = b - by * (uint32_t)cob;
  } else {
    split = blockIdx.x % (uint32_t)nsplit;
    const uint32_t b = blockIdx.x / (uint32_t)nsplit;
    ob_ = b / gy;
    by = b - ob_ * gy;
  }
  const int tap = (int)by / cib, cb = (int)by - tap * cib, ob = (int)ob_;
  const int kh = tap / d.KW, kw = tap - kh * d.KW;
  int8_t* Xi = lds[wave];
  int8_t* Gi = lds[wave] + 4 * kWP * 16;
  const int64_t per = (P + nsplit - 1) / nsplit;
  const int64_t p0 = (int64_t)split * per;
  const int64_t p1 = p0 + per < P ? p0 + per : P;
  const uint32_t HWo = (uint32_t)d.Ho * d.Wo;
  v4i acc[NG][4][NBS], ax[4], ag[NG][NBS];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    ax[a] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < NBS; ++b)
#pragma unroll
      for (int h = 0; h < NG; ++h) acc[h][a][b] = v4i{0, 0, 0, 0};
  }
#pragma unroll
  for (int h = 0; h < NG; ++h)
#pragma unroll
    for (int b = 0; b < NBS; ++b) ag[h][b] = v4i{0, 0, 0, 0};
  const v4i ones = v4i{0x01010101, 0x01010101, 0x01010101, 0x01010101};
  long long nchunks = 0;
  // operand registers of one 64-pixel chunk; the next chunk's loads are issued right after this
  // chunk's registers are in LDS, so they fly during its MFMAs (no extra registers)
  v4i xs[4], gs[G16 ? 2 * NBS : NBS];
  bool xv = false, pv = false;
  auto issue = [&](int64_t c0) {
    const int64_t p = c0 + lane;
    pv = p < p1;
    const uint32_t pu = (uint32_t)(pv ? p : p0);
    const uint32_t n = pu / HWo, rem = pu - n * HWo;
    const int oh = (int)(rem / (uint32_t)d.Wo), ow = (int)(rem - (uint32_t)oh * (uint32_t)d.Wo);
    const int ih = oh * d.SH + kh - d.PT, iw = ow * d.SW + kw - d.PL;
    xv = pv && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
    const int8_t* xp = xq + (xv ? ((((int64_t)n * d.H + ih) * d.W + iw) * d.Cin + cb * 64) : 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) xs[s] = *reinterpret_cast<const v4i*>(xp + s * 16);
    if constexpr (G16) {
      const int16_t* gp = reinterpret_cast<const int16_t*>(gq) + (int64_t)pu * d.Cout + ob * COW;
#pragma unroll
      for (int s = 0; s < 2 * NBS; ++s) gs[s] = *reinterpret_cast<const v4i*>(gp + s * 8);
    } else {
      const int8_t* gp = reinterpret_cast<const int8_t*>(gq) + (int64_t)pu * d.Cout + ob * COW;
#pragma unroll
      for (int s = 0; s < NBS; ++s) gs[s] = *reinterpret_cast<const v4i*>(gp + s * 16);
    }
  };
  const int64_t cfirst = p0 + (int64_t)wave * kWP;
  issue(cfirst < p1 ? cfirst : p0);
  for (int64_t c0 = cfirst; c0 < p1; c0 += 4 * kWP) {
    ++nchunks;
    const int fx = (int)0x80808080u;  // x' = -128: x = 0 (padding, pixels past the range)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (!xv) xs[s] = v4i{fx, fx, fx, fx};
      *reinterpret_cast<v4i*>(Xi + (s * kWP + lane) * 16) = xs[s];
    }
    if constexpr (G16) {
#pragma unroll
      for (int s = 0; s < NBS; ++s) {  // 16 codes -> 16 gh bytes, 16 gl' bytes; past the range g = 0
        int hi[4], lo[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const uint32_t c01 = (uint32_t)gs[2 * s + (w >> 1)][(w & 1) * 2];
          const uint32_t c23 = (uint32_t)gs[2 * s + (w >> 1)][(w & 1) * 2 + 1];
          hi[w] = pv ? (int)__builtin_amdgcn_perm(c23, c01, 0x07050301u) : 0;
          lo[w] = pv ? (int)(__builtin_amdgcn_perm(c23, c01, 0x06040200u) ^ 0x80808080u) : (int)0x80808080u;
        }
        *reinterpret_cast<v4i*>(Gi + (s * kWP + lane) * 16) = v4i{hi[0], hi[1], hi[2], hi[3]};
        *reinterpret_cast<v4i*>(Gi + ((NBS + s) * kWP + lane) * 16) = v4i{lo[0], lo[1], lo[2], lo[3]};
      }
    } else {
#pragma unroll
      for (int s = 0; s < NBS; ++s) {
        if (!pv) gs[s] = v4i{0, 0, 0, 0};
        *reinterpret_cast<v4i*>(Gi + (s * kWP + lane) * 16) = gs[s];
      }
    }
    const int64_t cn = c0 + 4 * kWP;
    issue(cn < p1 ? cn : c0);  // the next chunk (clamped: straight-line, a redundant last load)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    v4i gf[NG][NBS];
#pragma unroll
    for (int h = 0; h < NG; ++h)
#pragma unroll
      for (int b = 0; b < NBS; ++b) {
        gf[h][b] = tr_frag(Gi + (h * NBS + b) * kWP * 16, 16 * q, lane);
        ag[h][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, gf[h][b], ag[h][b], 0, 0, 0);
      }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const v4i xf = tr_frag(Xi + a * kWP * 16, 16 * q, lane);
      ax[a] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xf, ones, ax[a], 0, 0, 0);
#pragma unroll
      for (int h = 0; h < NG; ++h)
#pragma unroll
        for (int b = 0; b < NBS; ++b) acc[h][a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xf, gf[h][b], acc[h][a][b], 0, 0, 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // ---- combine exactly; the 4 waves meet in LDS (int64 [64 ci][64 co]) one after another
  // (plain read-modify-write, each wave owning the tile between two barriers)
  __syncthreads();
  long long* tile = reinterpret_cast<long long*>(&lds[0][0]);
  const long long npix = nchunks * kWP;
  long long vv[4][NBS][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NBS; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (G16) {
          const long long sg = 256ll * ag[0][b][i] + (long long)ag[1][b][i] + 128ll * npix;  // sum_p g[co]
          vv[a][b][i] = 256ll * acc[0][a][b][i] + (long long)acc[1][a][b][i] + 128ll * ax[a][i] + 128ll * sg;
        } else {
          vv[a][b][i] = (long long)acc[0][a][b][i] + 128ll * ag[0][b][i];
        }
      }
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < NBS; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            long long* t = &tile[(a * 16 + q * 4 + i) * COW + b * 16 + r];
            *t = w == 0 ? vv[a][b][i] : *t + vv[a][b][i];
          }
    }
    __syncthreads();
  }
  const int64_t shard = STORE ? (int64_t)split : (int64_t)(split % (uint32_t)nshard);
  long long* dst = slab + (shard * (d.KH * d.KW) + tap) * d.Cin * d.Cout;
  for (int i = threadIdx.x; i < 64 * COW; i += kT) {
    const long long v = tile[i];
    const int ci = cb * 64 + i / COW, co = ob * COW + i % COW;
    if constexpr (STORE)
      dst[(int64_t)ci * d.Cout + co] = v;
    else if (v)
      atomicAdd((unsigned long long*)&dst[(int64_t)ci * d.Cout + co], (unsigned long long)v);
  }
}


// ----------------------------------------------------------------------------- 3x3 wgrad, all taps
// wgrad3_kernel: a stride-1 SAME 3x3 conv's weight gradient with ALL 9 taps in one workgroup tile, so
// X and G leave L2 once per (ci block, co block) instead of once per tap (wgrad_wide_kernel's 9x).
// Workgroup = (pixel split, 64 ci, 64 co) of 8 waves; a chunk is RB = 64 / W whole output rows of one
// image (RB * W <= 64 pixels = the MFMA k), staged once for all waves: the X halo window
// [4 ci slices][(RB + 2) x (W + 2) pixels][16 B] (fill code outside the image) and G's 64 pixels x
// 64 co ([hi | lo'][4 co slices][64 px][16 B]; past the rows / image: g = 0). Wave w owns ci slice
// w & 3 and co slices 2 (w >> 2) + {0, 1} for all 9 taps; its A fragments are transposed reads of
// the window at the tap's offset (pixels past the chunk read a duplicate of its last pixel: their
// g = 0 cancels them exactly, see the identity of wgrad_wide_kernel), its B fragments the G image.
// The next chunk's loads fly during the MFMAs. Every (split, tap, ci, co) has one writer: STORED
// into slab[split][9 * Cin][Cout] (int64), reduced by lbt_conv_wgrad_reduce64 over the splits.
constexpr int kW3Win = 192;  // window pixels per ci slice: (64 / W + 2) * (W + 2) <= 192 (host check)

// ds_read_b64_tr_b8 as inline asm: the compiler's waitcnt pass makes every ds_read_tr intrinsic wait
// for ALL outstanding LDS-DMA (vmcnt(0): it cannot tell the ring's stages apart), which serialises the
// DMA ring. The asm form is invisible to that pass, so its results are fenced by hand: tr_wait()
// (s_waitcnt lgkmcnt(0)) takes the fragments as in/out operands, so no use can move above it.
LBT_DEV v2i tr8_asm(uint32_t addr) {
  v2i r;
  asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
LBT_DEV v4i tr_frag_asm(uint32_t a, uint32_t b) {
  const v2i lo = tr8_asm(a), hi = tr8_asm(b);
  return v4i{lo.x, lo.y, hi.x, hi.y};
}
LBT_DEV void tr_wait(v4i& a) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a)::"memory"); }

LBT_DEV v4i tr_frag2(const int8_t* img, int oa, int ob) {
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  const v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(img + oa));
  const v2i hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(img + ob));
  return v4i{lo.x, lo.y, hi.x, hi.y};
}

// Operands reach LDS by LDS-DMA (global_load_lds_dwordx4, no staging registers) through an S-stage
// ring of raw chunks -- the X window in its final [slice][pixel][16 B] layout, G as raw codes
// [pixel][64 co] -- with one barrier per chunk: step c waits for chunk c + 1's DMA, splits its raw G
// into the hi / lo' planes of plane buffer (c + 1) & 1, issues chunk c + S - 1's DMA into the stage
// chunk c - 1 left, and runs chunk c's MFMAs. NXW = X DMA instructions per wave per chunk (each wave
// issues exactly NXW + 1 per chunk -- idle slots write a dummy KiB -- so the vmcnt waits are constants).
template <bool G16, int NXW, int S>
__global__ __launch_bounds__(512, 2) void wgrad3_kernel(const int8_t* __restrict__ xq, const void* __restrict__ gq,
                                                      lbt_conv_desc d, long long* __restrict__ slab, int nsplit,
                                                      int dbg) {
  constexpr int NP = G16 ? 2 : 1;                    // G planes: (gh, gl') or g
  constexpr int XB = 4 * kW3Win * 16;                // X window image (12 KiB)
  constexpr int GB = 64 * 64 * (G16 ? 2 : 1);        // raw G codes of a chunk (8 / 4 KiB)
  constexpr int STG = XB + GB;
  constexpr int PB = NP * 4 * 64 * 16;               // one plane buffer
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  int8_t* const planes = lds + S * STG;              // [2][PB]
  int8_t* const dummy = planes + 2 * PB;             // 1 KiB sink of the idle DMA slots
  __shared__ int sax[9 * 64];  // sum_p x' per (tap, ci): waves 0-3 -> all
  __shared__ int sag[NP * 64];  // sum_p g (planes) per co: waves with ci slice 0 -> all
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 15, q = lane >> 4;
  const int H = d.H, W = d.W, Cin = d.Cin, Cout = d.Cout;
  const int RB = 64 / W, NPX = RB * W, Wp = W + 2, WIN = (RB + 2) * Wp;
  const int CPI = (H + RB - 1) / RB;
  const int64_t TC = (int64_t)d.N * CPI;
  const int nblk = (Cin / 64) * (Cout / 64);
  // dbg bit 1: XCD-aware order (a pixel split's channel blocks, which read the same X / G chunks, on one
  // XCD's L2)
  const uint32_t bid = (dbg & 2) ? xcd_logical(blockIdx.x, gridDim.x) : blockIdx.x;
  const int blk = (int)(bid % (uint32_t)nblk), split = (int)(bid / (uint32_t)nblk);
  const int cb = blk / (Cout / 64), ob = blk - cb * (Cout / 64);
  const int64_t c0 = TC * split / nsplit, c1 = TC * (split + 1) / nsplit;
  const int nc = (int)(c1 - c0);
  typedef __attribute__((address_space(3))) int8_t lds_i8;
  const uint32_t lbase = (uint32_t)(uintptr_t)(lds_i8*)lds;  // LDS byte address of the ring
  const int ws = wave & 3, wh = wave >> 2;
  const bool do_ax = G16 && wh == 0, do_ag = ws == 0;
  // transposed-read offsets (X: clamped to the chunk). Lane group q supplies k = pixels 8q .. 8q+7 (first
  // read) and 32+8q .. 32+8q+7 (second) -- any k order serves, A and B use the same -- so lanes 0-31 of
  // each ds_read_b64_tr_b8 cover 16 consecutive 16-byte rows (all 64 banks once; pixels 16q + j/2 put
  // lane groups 0 and 1 on the same 32 banks: 2-way conflicts)
  const int pa = 8 * q + (j >> 1), pb = pa + 32;
  const int xa = pa < NPX ? pa : NPX - 1, xb = pb < NPX ? pb : NPX - 1;
  const int oxa = ((xa / W) * Wp + xa % W) * 16 + 8 * (j & 1);
  const int oxb = ((xb / W) * Wp + xb % W) * 16 + 8 * (j & 1);
  const int oga = pa * 16 + 8 * (j & 1), ogb = pb * 16 + 8 * (j & 1);
  const int ngx = (WIN + 63) >> 6;  // 64-pixel groups of the window per slice

  // DMA of chunk k (clamped to the split's last) into stage st. Everything but the chunk's (image,
  // first row) is loop-invariant per lane, and issue() is called with k = 0, 1, 2, ... (clamped), so
  // (n, row0) advance incrementally -- no divisions in the loop.
  int xhy[NXW], xrel[NXW], xdst[NXW];
  bool xreal[NXW];
#pragma unroll
  for (int u = 0; u < NXW; ++u) {
    const int ins = wave + 8 * u;  // (slice, pixel group) = (ins % 4, ins / 4)
    const int sl = ins & 3, gp = ins >> 2;
    const int pix = gp * 64 + lane;
    const int hy = pix / Wp, hx = pix - hy * Wp;
    xreal[u] = gp < ngx;
    // window pixels past WIN and columns outside the image read the fill (hy = -1 marks them)
    xhy[u] = (pix < WIN && hx >= 1 && hx <= W) ? hy : -1000000;
    xrel[u] = (hy - 1) * W + (hx - 1);
    xdst[u] = xreal[u] ? (sl * kW3Win + gp * 64) * 16 : -1;
  }
  const int gitem = wave * 64 + lane;
  const int gpl = G16 ? gitem >> 3 : gitem >> 2, gseg = G16 ? gitem & 7 : gitem & 3;
  const bool greal = G16 || wave < 4;
  const int grow = gpl < NPX ? gpl / W : 1000000;  // output row of the pixel within the chunk
  int in_n = (int)(c0 / CPI), in_row0 = (int)(c0 - (int64_t)in_n * CPI) * RB, in_k = 0;
  auto issue = [&](int k, int st) {
    if (k < nc && k != in_k) {  // advance to chunk k (= in_k + 1)
      in_row0 += RB;
      if (in_row0 >= H) { in_row0 = 0; ++in_n; }
      in_k = k;
    }
    const int n = in_n, row0 = in_row0;
    int8_t* sb = lds + st * STG;
    const int8_t* xim = xq + ((int64_t)n * H * W + (int64_t)row0 * W) * Cin + cb * 64;
#pragma unroll
    for (int u = 0; u < NXW; ++u) {
      const int sl = (wave + 8 * u) & 3;
      const bool in = (unsigned)(row0 - 1 + xhy[u]) < (unsigned)H;
      const int8_t* src = in ? xim + (int64_t)xrel[u] * Cin + sl * 16 : reinterpret_cast<const int8_t*>(kFill80);
      int8_t* dst = xreal[u] ? sb + xdst[u] : dummy;
      __builtin_amdgcn_global_load_lds(src, (lds_vptr)dst, 16, 0, 0);
    }
    {  // G: wave w moves items 64 w .. 64 w + 63 of the chunk's raw codes (G8: waves 4-7 idle)
      const bool in = greal && row0 + grow < H;
      const int8_t* src = in ? reinterpret_cast<const int8_t*>(gq) +
                                   (((int64_t)n * H * W + (int64_t)row0 * W + gpl) * Cout + ob * 64) * (G16 ? 2 : 1) +
                                   gseg * 16
                             : reinterpret_cast<const int8_t*>(zi());
      int8_t* dst = greal ? sb + XB + wave * 1024 : dummy;
      __builtin_amdgcn_global_load_lds(src, (lds_vptr)dst, 16, 0, 0);
    }
  };
  // raw G of the chunk in stage st -> plane buffer pbuf (one 16-byte item per thread)
  auto split_g = [&](int st, int pbuf) {
    const int8_t* raw = lds + st * STG + XB;
    int8_t* pl8 = planes + pbuf * PB;
    if constexpr (G16) {
      const int pl = tid >> 3, seg = tid & 7;
      const v4i gr = *reinterpret_cast<const v4i*>(raw + tid * 16);
      int hi[2], lo[2];
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const uint32_t c01 = (uint32_t)gr[2 * w], c23 = (uint32_t)gr[2 * w + 1];
        hi[w] = (int)__builtin_amdgcn_perm(c23, c01, 0x07050301u);
        lo[w] = (int)(__builtin_amdgcn_perm(c23, c01, 0x06040200u) ^ 0x80808080u);
      }
      const int o = ((seg >> 1) * 64 + pl) * 16 + (seg & 1) * 8;
      *reinterpret_cast<v2i*>(pl8 + o) = v2i{hi[0], hi[1]};
      *reinterpret_cast<v2i*>(pl8 + 4 * 64 * 16 + o) = v2i{lo[0], lo[1]};
    } else if (tid < 256) {
      *reinterpret_cast<v4i*>(pl8 + ((tid & 3) * 64 + (tid >> 2)) * 16) = *reinterpret_cast<const v4i*>(raw + tid * 16);
    }
  };

  v4i acc[9][2][NP], ax[9], ag[2][NP];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    ax[t] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int h = 0; h < NP; ++h) acc[t][c][h] = v4i{0, 0, 0, 0};
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int h = 0; h < NP; ++h) ag[c][h] = v4i{0, 0, 0, 0};
  const v4i ones = v4i{0x01010101, 0x01010101, 0x01010101, 0x01010101};
  constexpr int G1 = NXW + 1;  // DMA instructions per wave per chunk

  // chunk k's MFMAs; the A fragment of tap t + 1 is read while tap t's MFMAs run
  auto mma = [&](int k) {
    const uint32_t xs = lbase + (uint32_t)((k % S) * STG + ws * kW3Win * 16);
    const uint32_t gp = lbase + (uint32_t)(S * STG + (k & 1) * PB);
    v4i bf[2][NP];
#pragma unroll
    for (int cs = 0; cs < 2; ++cs)
#pragma unroll
      for (int h = 0; h < NP; ++h) {
        const uint32_t b = gp + (uint32_t)(((h * 4 + 2 * wh + cs) * 64) * 16);
        bf[cs][h] = tr_frag_asm(b + oga, b + ogb);
      }
    v4i af = tr_frag_asm(xs + oxa, xs + oxb);
#pragma unroll
    for (int cs = 0; cs < 2; ++cs)
#pragma unroll
      for (int h = 0; h < NP; ++h) tr_wait(bf[cs][h]);
    tr_wait(af);
    if (do_ag) {
#pragma unroll
      for (int cs = 0; cs < 2; ++cs)
#pragma unroll
        for (int h = 0; h < NP; ++h) ag[cs][h] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, bf[cs][h], ag[cs][h], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      v4i an = af;
      if (t < 8) {
        const uint32_t toff = (uint32_t)((((t + 1) / 3) * Wp + (t + 1) % 3) * 16);
        an = tr_frag_asm(xs + oxa + toff, xs + oxb + toff);
      }
      if (do_ax) ax[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, ones, ax[t], 0, 0, 0);
#pragma unroll
      for (int cs = 0; cs < 2; ++cs)
#pragma unroll
        for (int h = 0; h < NP; ++h) acc[t][cs][h] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[cs][h], acc[t][cs][h], 0, 0, 0);
      if (t < 8) {
        tr_wait(an);
        af = an;
      }
    }
  };

  if (nc > 0) {
#pragma unroll
    for (int k = 0; k < S - 1; ++k) issue(k, k);
    vm_wait<(S - 2) * G1>();  // chunk 0 landed
    __builtin_amdgcn_s_barrier();
    split_g(0, 0);
    for (int k = 0; k < nc; ++k) {
      vm_wait<(S - 3) * G1>();  // chunk k + 1 landed (this wave's part)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's plane writes of chunk k
      __builtin_amdgcn_s_barrier();  // every wave's DMA of k + 1 and planes of k; chunk k - 1's readers done
      if (!(dbg & 1)) issue(k + S - 1, (k + S - 1) % S);
      mma(k);
      split_g((k + 1) % S, (k + 1) & 1);  // in the MFMAs' shadow; past the last chunk: a harmless stale split
    }
    vm_wait<0>();  // no DMA may still write LDS when the workgroup ends
  }
  // ---- the row / column sums to every wave, then one exact int64 per output
  if (do_ax && j == 0) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) sax[t * 64 + ws * 16 + 4 * q + i] = ax[t][i];
  }
  if (do_ag && q == 0) {
#pragma unroll
    for (int cs = 0; cs < 2; ++cs)
#pragma unroll
      for (int h = 0; h < NP; ++h) sag[h * 64 + (2 * wh + cs) * 16 + j] = ag[cs][h][0];
  }
  __syncthreads();
  const long long npix = (long long)nc * 64;
  long long* dst = slab + (int64_t)split * 9 * Cin * Cout;
#pragma unroll
  for (int cs = 0; cs < 2; ++cs) {
    const int col = (2 * wh + cs) * 16 + j;
    const long long sgc = G16 ? 256ll * sag[col] + (long long)sag[64 + col] + 128ll * npix : (long long)sag[col];
    const int co = ob * 64 + col;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cl = ws * 16 + 4 * q + i;
        long long v;
        if constexpr (G16)
          v = 256ll * acc[t][cs][0][i] + (long long)acc[t][cs][NP - 1][i] + 128ll * sax[t * 64 + cl] + 128ll * sgc;
        else
          v = (long long)acc[t][cs][0][i] + 128ll * sgc;
        dst[((int64_t)t * Cin + cb * 64 + cl) * Cout + co] = v;
      }
  }
}

template <bool G16, int NXW>
void wgrad3_launch(const int8_t* xq, const void* gq, const lbt_conv_desc& d, long long* slab, int nsplit, dim3 grid,
                   int dbg, hipStream_t st) {
  constexpr int S = 4;
  constexpr int PB = (G16 ? 2 : 1) * 4 * 64 * 16;
  constexpr size_t shm = (size_t)S * (4 * kW3Win * 16 + 64 * 64 * (G16 ? 2 : 1)) + 2 * PB + 1024;
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad3_kernel<G16, NXW, S>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    return true;
  }();
  (void)attr;
  // LBT_WGRAD_XCD bit 1: the XCD-aware order for the 3x3 body (dbg bit 1)
  static const int xmap = getenv_int("LBT_WGRAD_XCD", 1) & 2;
  hipLaunchKernelGGL((wgrad3_kernel<G16, NXW, S>), grid, dim3(512), shm, st, xq, gq, d, slab, nsplit, dbg | xmap);
}

bool wgrad3_ok(const lbt_conv_desc& d) {
  if (d.KH != 3 || d.KW != 3 || d.SH != 1 || d.SW != 1 || d.PT != 1 || d.PB != 1 || d.PL != 1 || d.PR != 1 ||
      d.Ho != d.H || d.Wo != d.W || d.W > 64 || d.Cin % 64 || d.Cout % 64)
    return false;
  const int RB = 64 / d.W;
  return (RB + 2) * (d.W + 2) <= kW3Win;
}

// ----------------------------------------------------------------------------- 1x1 wgrad, 16-bit G
// wgrad1_kernel: a 1x1 conv's weight gradient (pad 0, any stride) with 16-bit gradient codes on a
// workgroup tile of (64 WCI) ci x (32 WCO) co, WCI x WCO = 8 waves of 64 ci x 32 co (wgrad_wide_kernel's
// 64 x 64 tile re-read X Cout/64 times and G Cin/64 times: ~616 MB of operand loads per ResNet-50 1x1
// conv against 100-460 MB of data). A chunk = 64 pixels (the MFMA k); every operand image is
// [64 px][16 B] -- an X slice of 16 ci, or a RAW G group of 8 co as (lo, hi) byte pairs -- moved by
// LDS-DMA through an S-stage ring with one barrier per chunk. The raw G image needs no split pass:
// a transposed read gives lane i byte i of each pixel's 16 bytes, i.e. column i = (co i / 2, byte
// i & 1), so the MFMA runs on 16 "columns" of 8 co x (lo, hi); the lo lanes XOR their bytes with
// 0x80 (lo' = lo - 128, signed), and the epilogue joins lane pairs:
//   sum x g = 256 sum x' gh + sum x' gl' + 128 sum x' + 128 (256 sum gh + sum gl' + 128 npix)
// (x' = x - 128; every processed pixel counts, padding ones carry x' = -128, g = 0, which the
// identity cancels). Every (split, ci, co) has one writer: STORED into slab[split][Cin][Cout].
template <int WCI, int S>
__global__ __launch_bounds__(512, 1) void wgrad1_kernel(const int8_t* __restrict__ xq, const int16_t* __restrict__ gq,
                                                      lbt_conv_desc d, long long* __restrict__ slab, int nsplit,
                                                      int xmap) {
  constexpr int WCO = 8 / WCI;
  constexpr int TCI = 64 * WCI, TCO = 32 * WCO;     // workgroup tile
  constexpr int NXS = TCI / 16, NGG = TCO / 8;       // X slices, G groups (1 KiB images each)
  constexpr int NXW = (NXS + 7) / 8, NGW = NGG / 8;  // DMA instructions per wave per chunk
  constexpr int G1 = NXW + NGW;
  constexpr int STG = (NXS + NGG) * 1024;
  static_assert(NGG % 8 == 0, "geometry");
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  int8_t* const dummy = lds + S * STG;  // 1 KiB sink of idle X slots
  __shared__ int sax[TCI];              // sum_p x' per ci
  __shared__ int sag[2 * TCO];          // sum_p of each raw-G column (co, byte)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 15, q = lane >> 4;
  const int wci = wave / WCO, wco = wave - wci * WCO;
  const int Cin = d.Cin, Cout = d.Cout;
  const int64_t P = (int64_t)d.N * d.Ho * d.Wo;
  const int64_t TC = (P + 63) / 64;
  const int cbn = Cin / TCI, obn = Cout / TCO, nblk = cbn * obn;
  // xmap: XCD-aware order (a pixel split's channel tiles, which read the same X / G chunks, on one XCD)
  const uint32_t bid = xmap ? xcd_logical(blockIdx.x, gridDim.x) : blockIdx.x;
  const int blk = (int)(bid % (uint32_t)nblk), split = (int)(bid / (uint32_t)nblk);
  const int cb = blk / obn, ob = blk - cb * obn;
  const int64_t c0 = TC * split / nsplit, c1 = TC * (split + 1) / nsplit;
  const int nc = (int)(c1 - c0);
  typedef __attribute__((address_space(3))) int8_t lds_i8;
  const uint32_t lbase = (uint32_t)(uintptr_t)(lds_i8*)lds;
  const bool do_ax = wco == 0, do_ag = wci == 0;
  // transposed-read offsets: lane group q supplies k = pixels 8q .. 8q+7 (first read), 32 + 8q .. (second)
  const int pa = 8 * q + (j >> 1);
  const int oa = pa * 16 + 8 * (j & 1), ob2 = oa + 32 * 16;
  const uint32_t hwo = (uint32_t)d.Ho * d.Wo;
  const bool unit = d.SH == 1 && d.SW == 1 && d.Ho == d.H && d.Wo == d.W;

  auto issue = [&](int k, int st) {
    const int64_t p = (c0 + k) * 64 + lane;
    const bool pv = p < P;
    const uint32_t pu = (uint32_t)(pv ? p : 0);
    uint32_t xp = pu;
    if (!unit) {
      const uint32_t n = pu / hwo, rem = pu - n * hwo, oh = rem / (uint32_t)d.Wo, ow = rem - oh * (uint32_t)d.Wo;
      xp = (n * (uint32_t)d.H + oh * (uint32_t)d.SH) * (uint32_t)d.W + ow * (uint32_t)d.SW;
    }
    int8_t* sb = lds + st * STG;
    const int8_t* xs = xq + (int64_t)xp * Cin + cb * TCI;
#pragma unroll
    for (int u = 0; u < NXW; ++u) {
      const int sl = wave + 8 * u;
      const bool real = sl < NXS;
      const int8_t* src = (pv && real) ? xs + sl * 16 : reinterpret_cast<const int8_t*>(kFill80);
      int8_t* dst = real ? sb + sl * 1024 : dummy;
      __builtin_amdgcn_global_load_lds(src, (lds_vptr)dst, 16, 0, 0);
    }
    const int8_t* gs = reinterpret_cast<const int8_t*>(gq + (int64_t)pu * Cout + ob * TCO);
#pragma unroll
    for (int u = 0; u < NGW; ++u) {
      const int g = wave + 8 * u;
      const int8_t* src = pv ? gs + g * 16 : reinterpret_cast<const int8_t*>(zi());
      __builtin_amdgcn_global_load_lds(src, (lds_vptr)(sb + (NXS + g) * 1024), 16, 0, 0);
    }
  };

  v4i acc[4][4], ax[4], ag[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    ax[a] = v4i{0, 0, 0, 0};
    ag[a] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = v4i{0, 0, 0, 0};
  }
  const v4i ones = v4i{0x01010101, 0x01010101, 0x01010101, 0x01010101};
  const int lox = (j & 1) ? 0 : (int)0x80808080u;  // lo-byte columns: lo' = lo ^ 0x80

  auto mma = [&](int k) {
    const uint32_t sb = lbase + (uint32_t)((k % S) * STG);
    v4i af[4], bf[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t g = sb + (uint32_t)((NXS + wco * 4 + b) * 1024);
      bf[b] = tr_frag_asm(g + oa, g + ob2);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const uint32_t x = sb + (uint32_t)((wci * 4 + a) * 1024);
      af[a] = tr_frag_asm(x + oa, x + ob2);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      tr_wait(bf[b]);
      bf[b] = bf[b] ^ v4i{lox, lox, lox, lox};
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) tr_wait(af[a]);
    if (do_ag) {
#pragma unroll
      for (int b = 0; b < 4; ++b) ag[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, bf[b], ag[b], 0, 0, 0);
    }
    if (do_ax) {
#pragma unroll
      for (int a = 0; a < 4; ++a) ax[a] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], ones, ax[a], 0, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[b], acc[a][b], 0, 0, 0);
  };

  if (nc > 0) {
#pragma unroll
    for (int k = 0; k < S - 1; ++k) issue(k < nc ? k : nc - 1, k);
    for (int k = 0; k < nc; ++k) {
      vm_wait<(S - 2) * G1>();       // chunk k landed (this wave's part)
      __builtin_amdgcn_s_barrier();  // every wave's part of chunk k; chunk k - 1's readers done
      const int nx = k + S - 1;
      issue(nx < nc ? nx : nc - 1, nx % S);
      mma(k);
    }
    vm_wait<0>();  // no DMA may still write LDS when the workgroup ends
  }
  // ---- sums to every wave; lo lanes (even columns) join their hi partner and store
  if (do_ax && j == 0) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) sax[(wci * 4 + a) * 16 + 4 * q + i] = ax[a][i];
  }
  if (do_ag && q == 0) {
#pragma unroll
    for (int b = 0; b < 4; ++b) sag[(wco * 4 + b) * 16 + j] = ag[b][0];
  }
  __syncthreads();
  const long long npix = (long long)nc * 64;
  long long* dst = slab + (int64_t)split * Cin * Cout;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int colg = (wco * 4 + b) * 16 + (j & ~1);  // this pair's lo column in the tile
    const long long sgc = 256ll * sag[colg + 1] + (long long)sag[colg] + 128ll * npix;  // sum_p g[co]
    const int co = ob * TCO + (wco * 4 + b) * 8 + (j >> 1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hi = __shfl_xor(acc[a][b][i], 1, 64);
        const int cl = (wci * 4 + a) * 16 + 4 * q + i;
        const long long v = 256ll * hi + (long long)acc[a][b][i] + 128ll * sax[cl] + 128ll * sgc;
        if (!(j & 1)) dst[(int64_t)(cb * TCI + cl) * Cout + co] = v;
      }
  }
}

// the 1x1 body's tile: 0 = not taken, else WCI (waves along ci; 8 / WCI along co)
int wgrad1_wci(const lbt_conv_desc& d) {
  if (d.KH != 1 || d.KW != 1 || d.PT || d.PL || d.PB < 0 || d.PR < 0 || (d.Ho - 1) * d.SH >= d.H ||
      (d.Wo - 1) * d.SW >= d.W)
    return 0;
  if (d.Cin % 128 == 0 && d.Cout % 128 == 0) return 2;
  if (d.Cin % 64 == 0 && d.Cout % 256 == 0) return 1;
  if (d.Cin % 256 == 0 && d.Cout % 64 == 0) return 4;
  return 0;
}

template <int WCI>
void wgrad1_launch(const int8_t* xq, const int16_t* gq, const lbt_conv_desc& d, long long* slab, int nsplit,
                   hipStream_t st) {
  constexpr int S = 3, WCO = 8 / WCI;
  constexpr size_t shm = (size_t)S * (4 * WCI + 4 * WCO) * 1024 + 1024;
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad1_kernel<WCI, S>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    return true;
  }();
  (void)attr;
  const int64_t nblk = (int64_t)(d.Cin / (64 * WCI)) * (d.Cout / (32 * WCO));
  // LBT_WGRAD_XCD (default 1): bit 0 the XCD-aware order for this 1x1 body -- its pixel split's channel
  // tiles share one XCD's L2 for their X / G chunks (ResNet-50 weight gradients 5.33 -> 5.19 ms per step;
  // bit 1, the same for the 3x3 body, measured no change: profiles/round5/wgrad_xcd_ab.txt)
  static const int xmap = getenv_int("LBT_WGRAD_XCD", 1) & 1;
  hipLaunchKernelGGL((wgrad1_kernel<WCI, S>), dim3((unsigned)(nblk * nsplit)), dim3(512), shm, st, xq, gq, d, slab,
                     nsplit, xmap);
}

}  // namespace

// wide wgrad: x offset int8 codes (q - 128), g int8 (g_i16 = 0) or int16 codes; adds into a
// ZEROED int64 slab [nshard][KH*KW*Cin][Cout] (reduce with lbt_conv_wgrad_reduce64 over nshard).
extern "C" int lbt_conv_wgrad_igemm(const int8_t* xq, const void* gq, int32_t g_i16, lbt_conv_desc d, int64_t* slab,
                                    int32_t nsplit, int32_t nshard, void* stream) {
  if (!desc_ok(d) || d.Cin % 64 || d.Cout % 64 || nsplit <= 0 || nshard <= 0 || nshard > nsplit) return LBT_EINVAL;
  const int64_t P = (int64_t)d.N * d.Ho * d.Wo;
  if (P >= ((int64_t)1 << 31)) return LBT_EINVAL;
  const int64_t nwg = (int64_t)d.KH * d.KW * (d.Cin / 64) * (d.Cout / 64) * nsplit;
  if (nwg > 0x7fffffff) return LBT_EINVAL;
  const dim3 grid((unsigned)nwg);
  static const int xmap = getenv_int("LBT_WGRAD_XMAP", 0);
  hipStream_t st = (hipStream_t)stream;
  if (g_i16)
    hipLaunchKernelGGL((wgrad_wide_kernel<true, false>), grid, dim3(kT), 0, st, xq, gq, d, (long long*)slab, P, nsplit,
                       nshard, xmap);
  else
    hipLaunchKernelGGL((wgrad_wide_kernel<false, false>), grid, dim3(kT), 0, st, xq, gq, d, (long long*)slab, P, nsplit,
                       nshard, xmap);
  return (int)hipGetLastError();
}

// ... storing: slab [nsplit][KH*KW*Cin][Cout] is fully WRITTEN (one partial per pixel split; no
// zeroing, no atomics); reduce with lbt_conv_wgrad_reduce64 over nsplit.
extern "C" int lbt_conv_wgrad_igemm_store(const int8_t* xq, const void* gq, int32_t g_i16, lbt_conv_desc d,
                                          int64_t* slab, int32_t nsplit, void* stream) {
  if (!desc_ok(d) || d.Cin % 64 || d.Cout % 64 || nsplit <= 0) return LBT_EINVAL;
  const int64_t P = (int64_t)d.N * d.Ho * d.Wo;
  if (P >= ((int64_t)1 << 31)) return LBT_EINVAL;
  if ((P + nsplit - 1) / nsplit > 4 * 131072) return LBT_EINVAL;  // int32 MFMA sums of a wave stay exact
  hipStream_t st = (hipStream_t)stream;
  static const int w3 = getenv_int("LBT_WGRAD3", 1);
  if (w3 && wgrad3_ok(d)) {  // 3x3 / stride 1: all taps per workgroup; splits over whole-row chunks
    const int RB = 64 / d.W;
    const int64_t chunks = (int64_t)d.N * ((d.H + RB - 1) / RB);
    const int64_t nblk = (int64_t)(d.Cin / 64) * (d.Cout / 64);
    // <= 1024 chunks a split: every int32 MFMA sum stays below 2^31 (64 products of |x' g| <= 2^14 a chunk)
    if (nsplit > chunks || (chunks + nsplit - 1) / nsplit > 1024 || nblk * nsplit > 0x7fffffff) return LBT_EINVAL;
    const dim3 grid((unsigned)(nblk * nsplit));
    static const int dbg = getenv_int("LBT_WGRAD3_DBG", 0);  // diagnostics: 1 = no DMA after the prologue
    const int win = (RB + 2) * (d.W + 2);
    const bool two = 4 * ((win + 63) / 64) > 8;  // X DMA instructions per wave per chunk: 1 or 2
    long long* sl = (long long*)slab;
    if (g_i16) {
      if (two) wgrad3_launch<true, 2>(xq, gq, d, sl, nsplit, grid, dbg, st);
      else wgrad3_launch<true, 1>(xq, gq, d, sl, nsplit, grid, dbg, st);
    } else {
      if (two) wgrad3_launch<false, 2>(xq, gq, d, sl, nsplit, grid, dbg, st);
      else wgrad3_launch<false, 1>(xq, gq, d, sl, nsplit, grid, dbg, st);
    }
    return (int)hipGetLastError();
  }
  static const int w1 = getenv_int("LBT_WGRAD1", 1);
  if (w1 && g_i16 && wgrad1_wci(d)) {  // 1x1, 16-bit G: (64 WCI) ci x (32 WCO) co workgroup tiles
    const int wci = wgrad1_wci(d);
    const int64_t chunks = (P + 63) / 64;
    const int64_t nblk = (int64_t)(d.Cin / (64 * wci)) * (d.Cout / (256 / wci));
    // <= 2047 chunks a split: every int32 MFMA sum stays below 2^31 (|x' g| <= 2^14 a pixel; 2048
    // chunks of saturated codes, x' = -128 and both G bytes -128, would reach 2^31 exactly)
    if (nsplit > chunks || (chunks + nsplit - 1) / nsplit > 2047 || nblk * nsplit > 0x7fffffff) return LBT_EINVAL;
    const int16_t* g16 = reinterpret_cast<const int16_t*>(gq);
    long long* sl = (long long*)slab;
    if (wci == 2) wgrad1_launch<2>(xq, g16, d, sl, nsplit, st);
    else if (wci == 1) wgrad1_launch<1>(xq, g16, d, sl, nsplit, st);
    else wgrad1_launch<4>(xq, g16, d, sl, nsplit, st);
    return (int)hipGetLastError();
  }
  const int64_t nwg = (int64_t)d.KH * d.KW * (d.Cin / 64) * (d.Cout / 64) * nsplit;
  if (nwg > 0x7fffffff) return LBT_EINVAL;
  const dim3 grid((unsigned)nwg);
  static const int xmap = getenv_int("LBT_WGRAD_XMAP", 0);
  if (g_i16)
    hipLaunchKernelGGL((wgrad_wide_kernel<true, true>), grid, dim3(kT), 0, st, xq, gq, d, (long long*)slab, P, nsplit,
                       nsplit, xmap);
  else
    hipLaunchKernelGGL((wgrad_wide_kernel<false, true>), grid, dim3(kT), 0, st, xq, gq, d, (long long*)slab, P, nsplit,
                       nsplit, xmap);
  return (int)hipGetLastError();
}

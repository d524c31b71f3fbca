// conv_mfma.hip -- int8 implicit-GEMM convolution on gfx950 v_mfma_i32_16x16x64_i8.
//
//  lbt_conv_fwd_i8       Conv2d_q.forward  y = conv(Xq, Wq)          (dynamic_fixed_point.py:287-291)
//  lbt_conv_dgrad_i8     Conv2d_q.backward dX = conv^T(gradq, Wq)    (dynamic_fixed_point.py:305)
//  lbt_conv_wgrad_i8     Conv2d_q.backward dW = sum_p Xq (x) gradq   (dynamic_fixed_point.py:302)
//  lbt_conv_wgrad_reduce     + 2*wd*W, dequant, split reduction
//
// Operand maps (probed on MI355X with exact integer data): for 16x16x64_i8 lane l supplies
// A[row l&15][k = 16*(l>>4) .. +15] and B[k = 16*(l>>4) .. +15][col l&15] as 16 int8 each;
// C/D: col = l&15, row = 4*(l>>4) + reg.
//
// fwd / dgrad: GEMM rows = output pixels (fwd) or input pixels (dgrad), cols = output channels,
// k = (tap, 16-channel slice).  Every A fragment is one 16-byte NHWC channel slice of one
// pixel, gathered straight from global memory by its lane (the 9x tap re-reads of a 3x3 conv
// hit L1/L2; the whole activation is a few MB).  B (packed weights, <= 37 KB) is L2-resident.
// Out-of-bounds taps read the encoding of 0: -128 for the unsigned-9-bit offset encoding
// (q - 128), 0 otherwise; the offset is undone in the epilogue with 128 * sum_k W[k][co].
//
// wgrad: GEMM rows = (tap, ci), cols = co, k = pixels.  Each wave stages 64 pixels of G and of
// the tap-shifted X into LDS transposed ([channel][pixel]) and issues 16x16x64 MFMAs; each
// workgroup owns a pixel range and one tap and writes an int32 partial (exact, no atomics).
#include "conv_epilogue.h"
#include "chain_flags.h"
#include "lds_tr.h"
#include "stem_bwd.h"

using namespace lbt;


namespace {

constexpr int kThreads = 256;

enum { MODE_FWD = 0, MODE_DGRAD = 1 };

struct GemmArgs {
  const int8_t* a;      // gathered operand (xq for fwd, gq for dgrad), NHWC
  const int8_t* b;      // packed weights [ncol][ks*16]
  int ks;               // 16-byte k-slices per column (multiple of 4)
  int nslices;          // real k-slices = taps * CS
  int a_fill;           // fill word for out-of-bounds taps
  const int32_t* colsum;
  lbt_conv_desc d;
  lbt_qdesc qa, qb;     // scale sources
  float* y;             // fp32 output
  const float* add_src; // fp32 addend (dgrad)
  int8_t* yq;           // quantised output (fwd epilogue quantiser)
  lbt_qdesc qout;
  int64_t* ychsum;
  int64_t M;            // GEMM rows
  int ncol;             // GEMM cols
  lbt_chain_bwd_a chain;  // dgrad epilogue = pass A of this chain (CF != 0)
};

// 16 signed 4-bit codes (element e = nibble e: low nibble of byte e/2 first) -> 16 int8 lanes of an
// MFMA operand: lo / hi nibbles interleaved with v_perm_b32, then sign-extended bytewise without
// carries: (b & 7) | ((b & 8) * 0x1F) sets bits 3-7 exactly when bit 3 (the sign) is set.
LBT_DEV v4i unpack_i4x16(v2i pk) {
  v4i o;
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    const uint32_t x = (uint32_t)(w == 0 ? pk.x : pk.y);
    const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x0F0F0F0Fu;
    const uint32_t a = __builtin_amdgcn_perm(hi, lo, 0x05010400u);  // e0 e1 e2 e3
    const uint32_t b = __builtin_amdgcn_perm(hi, lo, 0x07030602u);  // e4 e5 e6 e7
    o[2 * w] = (int)((a & 0x07070707u) | ((a & 0x08080808u) * 0x1Fu));
    o[2 * w + 1] = (int)((b & 0x07070707u) | ((b & 0x08080808u) * 0x1Fu));
  }
  return o;
}

// W4: the B operand (weights) is stored as packed signed 4-bit codes, 8 bytes per 16-element
// k-slice (no int4 MFMA on gfx950 -- unpacked to int8 in registers).
// One workgroup's tile (bid = its index in the GEMM's grid); the body of conv_gemm_kernel and of
// the dgrad half of dgrad_wgrad_kernel.
// DUAL (dgrad with pass A only): p2 is a second dgrad GEMM into the same output pixels (a projection
// block's 1x1/2 shortcut beside its 3x3/2 first conv); its fp32 result float(acc2) * scale2 is the
// pass-A addend, exactly the value the shortcut's own dgrad launch would have stored and this one
// re-loaded as add_src.
template <int MODE, int CS, int NT, int CF, int NB, bool W4, bool DUAL = false>
__device__ __forceinline__ void conv_gemm_body(const GemmArgs& p, uint32_t bid, const GemmArgs* p2 = nullptr) {
  using G = EpiGeom<NT>;
  constexpr int NTW = G::NTW, WPM = G::WPM, MTB = G::MTB;
  __shared__ EpiShared<NT> sh;
  __shared__ ChainShared<NT, (CF ? NB : 1)> csh;
  ChainPre<NT, NB, CF> cp;
  LBT_TS(0);
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int mt_local = wave / WPM;
  const int nt0 = (wave % WPM) * NTW;
  const int64_t mtile = (int64_t)bid * MTB + mt_local;
  const int r = lane & 15, kg = lane >> 4;
  const lbt_conv_desc& d = p.d;
  const bool want_q = p.yq != nullptr;

  // this lane's GEMM row -> pixel (n, y, x) of the "row" space (M < 2^31: 32-bit math)
  const int OH = MODE == MODE_FWD ? d.Ho : d.H, OW = MODE == MODE_FWD ? d.Wo : d.W;
  const int64_t m = mtile * 16 + r;
  const bool row_ok = m < p.M;
  int n = 0, py = 0, px = 0;
  if (row_ok) {
    const uint32_t mu = (uint32_t)m;
    px = (int)(mu % (uint32_t)OW);
    const uint32_t t = mu / (uint32_t)OW;
    py = (int)(t % (uint32_t)OH);
    n = (int)(t / (uint32_t)OH);
  }
  const int cred = CS * 16;  // channels of the gathered operand
  const int SH = MODE == MODE_FWD ? d.H : d.Ho, SW = MODE == MODE_FWD ? d.W : d.Wo;

  // A fragment of k-step kk (slice s = 4*kk + kg) for this lane's row: its address, and the
  // value it takes instead when the slice is padding (0) or the tap is outside the image (fill)
  auto addr_aq = [&](const GemmArgs& q, int kk, bool& use, int& alt) -> const v4i* {
    const lbt_conv_desc& d = q.d;
    const int s = kk * 4 + kg;
    use = false;
    alt = 0;
    if (s >= q.nslices) return reinterpret_cast<const v4i*>(q.a);
    alt = MODE == MODE_DGRAD ? 0 : q.a_fill;
    const int tap = s / CS, cs = s - tap * CS;
    const int kh = tap / d.KW, kw = tap - kh * d.KW;
    int sy, sx;
    bool ok;
    if (MODE == MODE_FWD) {
      sy = py * d.SH + kh - d.PT;
      sx = px * d.SW + kw - d.PL;
      ok = (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
    } else {
      const int ny = py + d.PT - kh, nx = px + d.PL - kw;
      sy = ny / d.SH;
      sx = nx / d.SW;
      ok = ny >= 0 && nx >= 0 && sy * d.SH == ny && sx * d.SW == nx && sy < SH && sx < SW;
    }
    use = ok && row_ok;
    if (!use) return reinterpret_cast<const v4i*>(q.a);
    return reinterpret_cast<const v4i*>(q.a + (((int64_t)n * SH + sy) * SW + sx) * cred + cs * 16);
  };
  auto addr_a = [&](int kk, bool& use, int& alt) -> const v4i* { return addr_aq(p, kk, use, alt); };
  auto load_bq = [&](const GemmArgs& q, int kk, int j) -> v4i {
    const int col = (nt0 + j) * 16 + r;
    if constexpr (W4)
      return unpack_i4x16(*reinterpret_cast<const v2i*>(q.b + ((int64_t)col * q.ks + kk * 4 + kg) * 8));
    else
      return *reinterpret_cast<const v4i*>(q.b + ((int64_t)col * q.ks + kk * 4 + kg) * 16);
  };
  auto load_b = [&](int kk, int j) -> v4i { return load_bq(p, kk, j); };

  v4i acc[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) acc[j] = v4i{0, 0, 0, 0};
  // epilogue operands, fetched together with the GEMM operands: noise (fwd) / addend (dgrad)
  float ea[NTW][4];
  int corr[NTW];
  const QOut qo{p.yq, p.qout, p.ychsum, p.M, p.ncol, (int64_t)OH * OW};
  const QState qs = qstate(p.qout);

  const int nks = p.ks >> 2;
  // every operand of a 3x3 conv's k loop fits in registers: issue ALL loads (no branches around
  // them), then the MFMAs -- one memory round trip per wave instead of one per k-step
  constexpr int kMaxKS = (9 * CS + 3) / 4;
  const bool preload = nks <= kMaxKS;
  v4i af[kMaxKS], bf[kMaxKS][NTW];
  if (preload) {
    bool use[kMaxKS];
    int alt[kMaxKS];
    const v4i* pa[kMaxKS];
#pragma unroll
    for (int kk = 0; kk < kMaxKS; ++kk) {
      pa[kk] = addr_a(kk < nks ? kk : 0, use[kk], alt[kk]);
      if (kk >= nks) { use[kk] = false; alt[kk] = 0; }  // zero A: its MFMA adds nothing
    }
#pragma unroll
    for (int kk = 0; kk < kMaxKS; ++kk) {
      af[kk] = *pa[kk];
#pragma unroll
      for (int j = 0; j < NTW; ++j) bf[kk][j] = load_b(kk < nks ? kk : 0, j);
    }
    const int* cs_src = (MODE == MODE_FWD && p.colsum) ? p.colsum : zi();
    const uint32_t cmask = (MODE == MODE_FWD && p.colsum) ? 0xffffffffu : 0u;
#pragma unroll
    for (int j = 0; j < NTW; ++j) corr[j] = 128 * cs_src[((nt0 + j) * 16 + r) & cmask];
    if constexpr (CF != 0) {
      chain_prefetch<NT, NB, CF>(p.chain, p.add_src, p.M, p.ncol, (uint32_t)(OH * OW), mtile, nt0, lane, cp);
    } else if constexpr (MODE == MODE_FWD) {
      epi_noise<NTW>(qo, mtile, nt0, lane, ea);
    } else {
      const float* as = p.add_src ? p.add_src : zf();
      const uint32_t amask = p.add_src ? 0xffffffffu : 0u;
#pragma unroll
      for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t row = mtile * 16 + kg * 4 + i;
          ea[j][i] = as[(uint32_t)((row < p.M ? row : 0) * p.ncol + (nt0 + j) * 16 + r) & amask];
        }
    }
#pragma unroll
    for (int kk = 0; kk < kMaxKS; ++kk)
      if (!use[kk]) af[kk] = v4i{alt[kk], alt[kk], alt[kk], alt[kk]};
#pragma unroll
    for (int kk = 0; kk < kMaxKS; ++kk)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[kk], bf[kk][j], acc[j], 0, 0, 0);
  } else {
    for (int kk = 0; kk < nks; ++kk) {
      bool use;
      int alt;
      const v4i* pa = addr_a(kk, use, alt);
      v4i a = *pa;
      if (!use) a = v4i{alt, alt, alt, alt};
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, load_b(kk, j), acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j) corr[j] = (MODE == MODE_FWD && p.colsum) ? 128 * p.colsum[(nt0 + j) * 16 + r] : 0;
    if constexpr (CF != 0) {
      chain_prefetch<NT, NB, CF>(p.chain, p.add_src, p.M, p.ncol, (uint32_t)(OH * OW), mtile, nt0, lane, cp);
    } else if constexpr (MODE == MODE_FWD) {
      epi_noise<NTW>(qo, mtile, nt0, lane, ea);
    } else {
#pragma unroll
      for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t row = mtile * 16 + kg * 4 + i;
          ea[j][i] = (p.add_src && row < p.M) ? p.add_src[row * p.ncol + (nt0 + j) * 16 + r] : 0.f;
        }
    }
  }
  if constexpr (DUAL) {
    static_assert(MODE == MODE_DGRAD && CF != 0, "dual GEMM: dgrad + pass A only");
    const GemmArgs& q = *p2;
    v4i acc2[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc2[j] = v4i{0, 0, 0, 0};
    const int nks2 = q.ks >> 2;
    for (int kk = 0; kk < nks2; ++kk) {
      bool use;
      int alt;
      const v4i* pa = addr_aq(q, kk, use, alt);
      v4i a = *pa;
      if (!use) a = v4i{alt, alt, alt, alt};
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc2[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, load_bq(q, kk, j), acc2[j], 0, 0, 0);
    }
    const float scale2 = ldexpf(1.0f, -(frac_exp(q.qa) + frac_exp(q.qb)));
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) cp.add[j][i] = (float)acc2[j][i] * scale2;
  }
  LBT_TS(1);

  // ---------------- epilogue: lane owns column (nt0+j)*16 + r of rows mtile*16 + 4*kg + i
  const float scale = ldexpf(1.0f, -(frac_exp(p.qa) + frac_exp(p.qb)));
  float v[NTW][4];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) v[j][i] = (float)(acc[j][i] + corr[j]) * scale;
  if constexpr (CF != 0) {
    LBT_TS(2);
    chain_epi<NT, NB, CF>(p.chain, DUAL || p.add_src != nullptr, p.M, p.ncol, mtile, nt0, wave, lane, v, cp, csh);
    LBT_TS(3);
    return;
  }
  if (!want_q) {
    const bool addv = MODE == MODE_DGRAD && p.add_src;
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = mtile * 16 + kg * 4 + i;
        if (row < p.M) p.y[row * p.ncol + (nt0 + j) * 16 + r] = addv ? v[j][i] + ea[j][i] : v[j][i];
      }
    return;
  }
  if constexpr (MODE == MODE_FWD) {
    LBT_TS(2);
    epi_quant<NT>(qo, qs, mtile, nt0, wave, lane, v, ea, sh);
    LBT_TS(3);
  }
}

template <int MODE, int CS, int NT, int CF = 0, int NB = 1, bool W4 = false>
__global__ __launch_bounds__(kThreads, (CS == 1 && MODE == MODE_DGRAD && NB == 1) ? 8 : 1) void conv_gemm_kernel(
    GemmArgs p) {
  conv_gemm_body<MODE, CS, NT, CF, NB, W4>(p, blockIdx.x);
}

// dgrad + pass A of a projection block's input gradient: its 3x3/2 conv's dgrad (p) plus the 1x1/2
// shortcut's (p2) in one launch (was: the shortcut's dgrad to an fp32 buffer, then p with it as
// add_src)
template <int CS, int NT, int CF, int NB, bool W4>
__global__ __launch_bounds__(kThreads) void conv_dgrad2_kernel(GemmArgs p, GemmArgs p2) {
  conv_gemm_body<MODE_DGRAD, CS, NT, CF, NB, W4, true>(p, blockIdx.x, &p2);
}

// Two independent GEMMs of one geometry class (same CS / NT / M) in one grid: workgroups [0, nb0)
// run p0's tiles, the rest p1's (a projection block's 3x3/2 conv and its 1x1/2 shortcut, which
// read the same input codes: one launch instead of two).
template <int MODE, int CS, int NT, bool W4>
__global__ __launch_bounds__(kThreads) void conv_gemm2_kernel(GemmArgs p0, GemmArgs p1, uint32_t nb0) {
  if (blockIdx.x < nb0)
    conv_gemm_body<MODE, CS, NT, 0, 1, W4>(p0, blockIdx.x);
  else
    conv_gemm_body<MODE, CS, NT, 0, 1, W4>(p1, blockIdx.x - nb0);
}

// ----------------------------------------------------------------------------- wgrad
// dW[tap][ci][co] = sum_p X[p shifted by tap][ci] * G[p][co]: GEMM rows = ci, cols = co, k = pixels.
// grid (nsplit, taps, Cout/16): workgroup = one tap, one 16-channel co slice, a pixel range; each
// wave walks 64-pixel chunks. A lane loads one pixel's 16-byte channel slices (X: CSI of them,
// G: one) and stores them as rows of [pixel][16 B] LDS images (one ds_write_b128 each); the MFMA
// fragments -- 16 consecutive pixels of one channel -- come back with the gfx950 transposing read
// ds_read_b64_tr_b8 (probed: in a 16-lane group, lane i receives byte i of the 8 rows formed by
// lane pairs 2r, 2r+1). Each workgroup adds its exact int32 partial [CI][16] into shard
// (split % nshard) of a zeroed slab[nshard][tap][ci][co] for the batched reduce.
constexpr int kWP = 64;  // pixels per wave chunk


struct WgradArgs {
  const int8_t* xq;
  const int8_t* gq;
  lbt_conv_desc d;
  int x_fill;
  int32_t* slab;
  int64_t P;
  int nsplit, nshard;
};

// LDS of one wgrad workgroup: per wave an X image [CSI][64 px][16 B] and a G image [64 px][16 B],
// then the per-wave partials [4][CI][16]
template <int CSI, int NW = 4>
struct WgradShared {
  int8_t lds[NW][(CSI + 1) * kWP * 16];
  int red[NW][CSI * 16 * 16];
};

// NW waves per workgroup (4 in the wgrad / dgrad_wgrad kernels, 8 in conv_bwd_kernel)
template <int CSI, int NW = 4>
__device__ __forceinline__ void conv_wgrad_body(const WgradArgs& wa, uint32_t bid, WgradShared<CSI, NW>& sm) {
  const int8_t* __restrict__ xq = wa.xq;
  const int8_t* __restrict__ gq = wa.gq;
  const lbt_conv_desc& d = wa.d;
  const int x_fill = wa.x_fill, nsplit = wa.nsplit, nshard = wa.nshard;
  int32_t* __restrict__ slab = wa.slab;
  const int64_t P = wa.P;
  constexpr int CI = CSI * 16;
  auto& lds = sm.lds;
  auto& red = sm.red;
  LBT_TS(0);
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int r = lane & 15, kg = lane >> 4;
  // XCD-aware unit order: workgroups are dealt round-robin over the 8 XCDs, so unit u of the
  // split-major order (split, tap, co-slice) goes to linear block (u % chunk) * 8 + u / chunk:
  // all taps / co-slices of one pixel split -- which re-read the same G and X bytes -- share one
  // XCD's L2 (speed only; any order gives the same integer sums).
  const int ntap = d.KH * d.KW, ncos = d.Cout >> 4, total = nsplit * ntap * ncos;
  const int chunk = (total + 7) >> 3;
  const int u = (int)(bid & 7) * chunk + (int)(bid >> 3);
  if (u >= total) return;
  const int split = u / (ntap * ncos), urem = u - split * (ntap * ncos);
  const int tap = urem / ncos, cso = urem - tap * ncos;
  const int kh = tap / d.KW, kw = tap - kh * d.KW;
  int8_t* Xi = lds[wave];
  int8_t* Gi = lds[wave] + CSI * kWP * 16;
  const int64_t per = (P + nsplit - 1) / nsplit;
  const int64_t p0 = (int64_t)split * per;
  const int64_t p1 = p0 + per < P ? p0 + per : P;
  const uint32_t HWo = (uint32_t)d.Ho * d.Wo;

  v4i acc[CSI];
#pragma unroll
  for (int a = 0; a < CSI; ++a) acc[a] = v4i{0, 0, 0, 0};

  // chunks are interleaved across the NW waves of the block, two in flight per wave: chunk k + 2's
  // loads are issued while chunk k is computed. Every load is unconditional (a chunk past the end has
  // no valid pixel: clamped addresses, zero gradient), so the compiler's vmcnt waits count exactly the
  // loads issued since instead of waiting for all of them (each chunk then paid a memory round trip:
  // the strided jobs' 32 chunks per wave took ~23 us of the batched launch, profiles/round6/budget)
  struct Chunk {
    v4i xs[CSI], g;
    bool xv, pv;
  };
  // whole-row chunks (the ResNet shapes: 64-pixel chunks of whole output rows of one image, aligned
  // splits): the lane's row / column within a chunk are chunk-invariant and the chunk's image and first
  // row wave-uniform -- no per-lane divisions per chunk
  const bool rows64 = 64 % d.Wo == 0 && HWo % 64 == 0 && per % 64 == 0 && p0 % 64 == 0;
  const int lrow = rows64 ? lane / d.Wo : 0, lcol = rows64 ? lane - lrow * d.Wo : 0;
  auto fetch = [&](int64_t c0, Chunk& b) {
    const int64_t p = c0 + lane;
    const bool pv = p < p1;
    const uint32_t pu = (uint32_t)(pv ? p : p0);  // P < 2^31 (launcher)
    uint32_t n;
    int oh, ow;
    if (rows64) {  // wave-uniform branch
      const uint32_t cu = (uint32_t)(c0 < p1 ? c0 : p0);
      n = cu / HWo;
      oh = (int)((cu - n * HWo) / (uint32_t)d.Wo) + lrow;
      ow = lcol;
    } else {
      n = pu / HWo;
      const uint32_t rem = pu - n * HWo;
      oh = (int)(rem / (uint32_t)d.Wo);
      ow = (int)(rem - (uint32_t)oh * (uint32_t)d.Wo);
    }
    const int ih = oh * d.SH + kh - d.PT, iw = ow * d.SW + kw - d.PL;
    const bool xv = pv && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
    // all loads first (clamped addresses, no branches), fills selected afterwards
    const int8_t* xp = xq + (xv ? ((((int64_t)n * d.H + ih) * d.W + iw) * CI) : 0);
#pragma unroll
    for (int cs = 0; cs < CSI; ++cs) b.xs[cs] = *reinterpret_cast<const v4i*>(xp + cs * 16);
    b.g = *reinterpret_cast<const v4i*>(gq + (int64_t)pu * d.Cout + cso * 16);
    b.xv = xv;
    b.pv = pv;
  };
  auto consume = [&](Chunk& b, int64_t cnext) {
    const int xf = b.pv ? x_fill : 0;
#pragma unroll
    for (int cs = 0; cs < CSI; ++cs)
      *reinterpret_cast<v4i*>(Xi + (cs * kWP + lane) * 16) = b.xv ? b.xs[cs] : v4i{xf, xf, xf, xf};
    *reinterpret_cast<v4i*>(Gi + lane * 16) = b.pv ? b.g : v4i{0, 0, 0, 0};
    // the images are read by other lanes of the same wave only: a wave's LDS instructions execute in
    // issue order, so only the compiler must keep the reads after the writes
    asm volatile("" ::: "memory");
    fetch(cnext, b);
    const v4i bfrag = tr_frag(Gi, 16 * kg, lane);
#pragma unroll
    for (int a = 0; a < CSI; ++a) {
      const v4i afrag = tr_frag(Xi + a * kWP * 16, 16 * kg, lane);
      acc[a] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag, bfrag, acc[a], 0, 0, 0);
    }
    asm volatile("" ::: "memory");  // the next chunk's stores after these reads (in-order LDS)
  };
  const int64_t cw = p0 + (int64_t)wave * kWP, cstep = (int64_t)NW * kWP;
  const int64_t nch = p1 > cw ? (p1 - cw + cstep - 1) / cstep : 0;  // this wave's chunks
  if (nch > 0) {
    Chunk b0, b1;
    fetch(cw, b0);
    fetch(cw + cstep, b1);
    for (int64_t k = 0; k < nch; k += 2) {
      consume(b0, cw + (k + 2) * cstep);
      consume(b1, cw + (k + 3) * cstep);
    }
  }
  LBT_TS(1);
  // acc[a] element i: row = a*16 + 4*kg + i (ci), col = r (co within the slice)
#pragma unroll
  for (int a = 0; a < CSI; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][(a * 16 + kg * 4 + i) * 16 + r] = acc[a][i];
  __syncthreads();
  LBT_TS(2);
  int32_t* dst = slab + ((int64_t)(split % nshard) * (d.KH * d.KW) + tap) * CI * d.Cout + cso * 16;
  for (int i = threadIdx.x; i < CI * 16; i += NW * 64) {
    const int ci = i >> 4, co = i & 15;
    int v = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][i];
    if (v) LBT_GADD(&dst[(int64_t)ci * d.Cout + co], v);  // integer atomics: exact, order-independent
  }
  LBT_TS(3);
}

template <int CSI>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(WgradArgs wa) {
  __shared__ __attribute__((aligned(16))) WgradShared<CSI> sm;
  conv_wgrad_body<CSI>(wa, blockIdx.x, sm);
}

// Horizontal fusion of one conv's two backward GEMMs, which read the same gradient codes and
// are independent of each other: workgroups [0, nwg) are the wgrad's (the longer ones, dispatched
// first), the rest the dgrad (+ chain pass A) tiles. One launch instead of two; nwg is a multiple
// of 8, so both halves keep their XCD-aware block order.
template <int CS, int NT, int CF, int NB, bool W4>
__global__ __launch_bounds__(kThreads, (CS == 1 && NB == 1) ? 8 : 1) void dgrad_wgrad_kernel(GemmArgs p, WgradArgs wa,
                                                                                          uint32_t nwg) {
  if (blockIdx.x < nwg) {
    __shared__ __attribute__((aligned(16))) WgradShared<NT> sm;
    conv_wgrad_body<NT>(wa, blockIdx.x, sm);
  } else
    conv_gemm_body<MODE_DGRAD, CS, NT, CF, NB, W4>(p, blockIdx.x - nwg);
}

// 256 threads = 32 outputs x 8 split groups; coalesced 128-B slab rows; exact int64 sums.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const int32_t* __restrict__ slab, int nsplit, int K,
                                                           int Cout, int x_u8off, const int64_t* __restrict__ gcolsum,
                                                           lbt_qdesc qx, lbt_qdesc qg, const float* __restrict__ w,
                                                           float wd2, float* __restrict__ dw,
                                                           long long* __restrict__ num) {
  __shared__ long long red[8][32];
  const int lo = threadIdx.x & 31, sg = threadIdx.x >> 5;
  const int64_t total = (int64_t)K * Cout;
  const int64_t i = (int64_t)blockIdx.x * 32 + lo;
  long long s = 0;
  if (i < total) {
#pragma unroll 4
    for (int b = sg; b < nsplit; b += 8) s += slab[(int64_t)b * total + i];
  }
  red[sg][lo] = s;
  __syncthreads();
  if (sg != 0 || i >= total) return;
  for (int k = 1; k < 8; ++k) s += red[k][lo];
  if (x_u8off && gcolsum) {
    const int co = (int)(i % Cout);
    long long cs = 0;
    for (int k = 0; k < LBT_NSHARD; ++k) cs += gcolsum[(int64_t)k * 2 * Cout + co];
    s += 128ll * cs;
  }
  if (num) {  // the exact exchange: the numerator, dequantised after the all-reduce
    num[i] = s;
    return;
  }
  const float scale = ldexpf(1.0f, -(frac_exp(qx) + frac_exp(qg)));
  const float a = (float)s * scale;
  const float b = wd2 * w[i];
  dw[i] = a + b;
}

template <int MODE, int NT, bool W4>
int launch_gemm_nt(const GemmArgs& p, int cs, hipStream_t st) {
  constexpr int MTB = EpiGeom<NT>::MTB;
  const int64_t mtiles = (p.M + 15) / 16;
  const int64_t blocks = (mtiles + MTB - 1) / MTB;
  if (blocks > 0x7fffffff) return LBT_EINVAL;
  switch (cs) {
    case 1: hipLaunchKernelGGL((conv_gemm_kernel<MODE, 1, NT, 0, 1, W4>), dim3((unsigned)blocks), dim3(kThreads), 0, st, p); break;
    case 2: hipLaunchKernelGGL((conv_gemm_kernel<MODE, 2, NT, 0, 1, W4>), dim3((unsigned)blocks), dim3(kThreads), 0, st, p); break;
    case 4: hipLaunchKernelGGL((conv_gemm_kernel<MODE, 4, NT, 0, 1, W4>), dim3((unsigned)blocks), dim3(kThreads), 0, st, p); break;
    case 8: hipLaunchKernelGGL((conv_gemm_kernel<MODE, 8, NT, 0, 1, W4>), dim3((unsigned)blocks), dim3(kThreads), 0, st, p); break;
    default: return LBT_EINVAL;
  }
  return (int)hipGetLastError();
}

template <int MODE, bool W4 = false>
int launch_gemm(const GemmArgs& p, int cs, hipStream_t st) {
  if (p.M * p.ncol >= (int64_t)1 << 31) return LBT_EINVAL;  // 32-bit row / element arithmetic
  switch (p.ncol / 16) {
    case 1: return launch_gemm_nt<MODE, 1, W4>(p, cs, st);
    case 2: return launch_gemm_nt<MODE, 2, W4>(p, cs, st);
    case 4: return launch_gemm_nt<MODE, 4, W4>(p, cs, st);
    case 8: return launch_gemm_nt<MODE, 8, W4>(p, cs, st);
    default: return LBT_EINVAL;
  }
}

bool desc_ok(const lbt_conv_desc& d) {
  return d.N > 0 && d.H > 0 && d.W > 0 && d.KH > 0 && d.KW > 0 && d.SH > 0 && d.SW > 0 && d.Ho > 0 &&
         d.Wo > 0 && d.Cin > 0 && d.Cout > 0;
}

}  // namespace

LBT_TRACE_SETTER(conv)

namespace {
int fwd_setup(const int8_t* xq, int32_t x_u8off, const int8_t* wf, int32_t ksf, const int32_t* wcolsum,
              lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y, int8_t* yq, lbt_qdesc qout, int64_t* ychsum,
              GemmArgs& p) {
  if (!desc_ok(d) || d.Cin % 16 || d.Cout % 16 || d.Cout > 128) return LBT_EINVAL;
  const int cs = d.Cin / 16;
  p.a = xq; p.b = wf; p.ks = ksf; p.nslices = d.KH * d.KW * cs;
  if (ksf % 4 || ksf < p.nslices) return LBT_EINVAL;
  p.a_fill = x_u8off ? (int)0x80808080u : 0;
  p.colsum = x_u8off ? wcolsum : nullptr;
  if (x_u8off && !wcolsum) return LBT_EINVAL;
  if (yq && qout.stochastic && !qout.noise) return LBT_EINVAL;  // quantising epilogue reads the noise table
  p.d = d; p.qa = qx; p.qb = qw; p.y = y; p.add_src = nullptr; p.yq = yq; p.qout = qout; p.ychsum = ychsum;
  p.M = (int64_t)d.N * d.Ho * d.Wo; p.ncol = d.Cout;
  return 0;
}

template <bool W4>
int conv_fwd(const int8_t* xq, int32_t x_u8off, const int8_t* wf, int32_t ksf, const int32_t* wcolsum,
             lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y, int8_t* yq, lbt_qdesc qout, int64_t* ychsum,
             void* stream) {
  GemmArgs p;
  const int e = fwd_setup(xq, x_u8off, wf, ksf, wcolsum, d, qx, qw, y, yq, qout, ychsum, p);
  if (e) return e;
  return launch_gemm<MODE_FWD, W4>(p, d.Cin / 16, (hipStream_t)stream);
}

template <int CS, int NT, bool W4>
int launch_fwd_pair(const GemmArgs& p0, const GemmArgs& p1, hipStream_t st) {
  constexpr int MTB = EpiGeom<NT>::MTB;
  const int64_t blocks = ((p0.M + 15) / 16 + MTB - 1) / MTB;
  if (2 * blocks > 0x7fffffff) return LBT_EINVAL;
  hipLaunchKernelGGL((conv_gemm2_kernel<MODE_FWD, CS, NT, W4>), dim3((unsigned)(2 * blocks)), dim3(kThreads), 0, st,
                     p0, p1, (uint32_t)blocks);
  return (int)hipGetLastError();
}

int conv_fwd_pair(const lbt_conv_fwd_job* j0, const lbt_conv_fwd_job* j1, void* stream) {
  if (!j0 || !j1 || j0->w4 != j1->w4) return LBT_EINVAL;
  GemmArgs p[2];
  const lbt_conv_fwd_job* j[2] = {j0, j1};
  for (int i = 0; i < 2; ++i) {
    if (j[i]->w4 && j[i]->qw.bits > 4) return LBT_EINVAL;
    const int e = fwd_setup(j[i]->xq, j[i]->x_u8off, j[i]->wf, j[i]->ksf, j[i]->wcolsum, j[i]->d, j[i]->qx, j[i]->qw,
                            j[i]->y, j[i]->yq, j[i]->qout, j[i]->ychsum, p[i]);
    if (e) return e;
  }
  if (p[0].M != p[1].M || p[0].ncol != p[1].ncol || j0->d.Cin != j1->d.Cin) return LBT_EINVAL;
  if (p[0].M * p[0].ncol >= (int64_t)1 << 31) return LBT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int key = ((j0->d.Cin / 16) << 8) | ((p[0].ncol / 16) << 1) | (j0->w4 ? 1 : 0);
#define LBT_FP(CS_, NT_)                                                                   \
  if (key == ((CS_ << 8) | (NT_ << 1))) return launch_fwd_pair<CS_, NT_, false>(p[0], p[1], st); \
  if (key == ((CS_ << 8) | (NT_ << 1) | 1)) return launch_fwd_pair<CS_, NT_, true>(p[0], p[1], st);
  // ResNet-20 / CIFAR projection blocks: 16 -> 32 and 32 -> 64 channels
  LBT_FP(1, 2)
  LBT_FP(2, 4)
#undef LBT_FP
  return LBT_EINVAL;
}

template <bool W4>
int conv_dgrad(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg, lbt_qdesc qw,
               float* dx, const float* add_src, void* stream) {
  if (!desc_ok(d) || d.Cin % 16 || d.Cout % 16 || d.Cin > 128) return LBT_EINVAL;
  const int cs = d.Cout / 16;
  GemmArgs p;
  p.a = gq; p.b = wd; p.ks = ksd; p.nslices = d.KH * d.KW * cs;
  if (ksd % 4 || ksd < p.nslices) return LBT_EINVAL;
  p.a_fill = 0; p.colsum = nullptr;
  p.d = d; p.qa = qg; p.qb = qw; p.y = dx; p.add_src = add_src; p.yq = nullptr; p.qout = lbt_qdesc{};
  p.ychsum = nullptr;
  p.M = (int64_t)d.N * d.H * d.W; p.ncol = d.Cin;
  return launch_gemm<MODE_DGRAD, W4>(p, cs, (hipStream_t)stream);
}
}  // namespace

extern "C" int lbt_conv_fwd_i8(const int8_t* xq, int32_t x_u8off, const int8_t* wf, int32_t ksf,
                               const int32_t* wcolsum, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y,
                               int8_t* yq, lbt_qdesc qout, int64_t* ychsum, void* stream) {
  return conv_fwd<false>(xq, x_u8off, wf, ksf, wcolsum, d, qx, qw, y, yq, qout, ychsum, stream);
}
extern "C" int lbt_conv_fwd_i8w4(const int8_t* xq, int32_t x_u8off, const uint8_t* wf4, int32_t ksf,
                                 const int32_t* wcolsum, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y,
                                 int8_t* yq, lbt_qdesc qout, int64_t* ychsum, void* stream) {
  if (qw.bits > 4) return LBT_EINVAL;
  return conv_fwd<true>(xq, x_u8off, (const int8_t*)wf4, ksf, wcolsum, d, qx, qw, y, yq, qout, ychsum, stream);
}
extern "C" int lbt_conv_fwd_pair_i8(const lbt_conv_fwd_job* j0, const lbt_conv_fwd_job* j1, void* stream) {
  return conv_fwd_pair(j0, j1, stream);
}
extern "C" int lbt_conv_dgrad_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                                 lbt_qdesc qw, float* dx, const float* add_src, void* stream) {
  return conv_dgrad<false>(gq, wd, ksd, d, qg, qw, dx, add_src, stream);
}
extern "C" int lbt_conv_dgrad_i8w4(const int8_t* gq, const uint8_t* wd4, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                                   lbt_qdesc qw, float* dx, const float* add_src, void* stream) {
  if (qw.bits > 4) return LBT_EINVAL;
  return conv_dgrad<true>(gq, (const int8_t*)wd4, ksd, d, qg, qw, dx, add_src, stream);
}

namespace {

// The wgrad launch of one conv: its argument block and grid (a multiple of 8 workgroups).
int wgrad_setup(const int8_t* xq, int32_t x_u8off, const int8_t* gq, const lbt_conv_desc& d, int32_t* slab,
                int32_t nsplit, int32_t nshard, WgradArgs& wa, uint32_t& blocks) {
  if (!desc_ok(d) || d.Cin % 16 || d.Cout % 16 || nsplit <= 0 || nshard <= 0 || nshard > nsplit) return LBT_EINVAL;
  if (d.Cin / 16 != 1 && d.Cin / 16 != 2 && d.Cin / 16 != 4 && d.Cin / 16 != 8) return LBT_EINVAL;
  const int64_t P = (int64_t)d.N * d.Ho * d.Wo;
  if (P >= ((int64_t)1 << 31)) return LBT_EINVAL;
  // int32 shard totals: the pixels of one shard times |x*g| <= 255*128 stay below 2^31
  if ((P + nsplit - 1) / nsplit * ((nsplit + nshard - 1) / nshard) > 65536) return LBT_EINVAL;
  const int64_t units = (int64_t)nsplit * d.KH * d.KW * (d.Cout / 16);
  if (units >= ((int64_t)1 << 30)) return LBT_EINVAL;
  wa = WgradArgs{xq, gq, d, x_u8off ? (int)0x80808080u : 0, slab, P, nsplit, nshard};
  blocks = (uint32_t)((units + 7) / 8 * 8);
  return 0;
}

// dgrad + pass A, optionally with the same conv's wgrad in the same launch (wa != nullptr)
template <int CS, int NT, int CF, int NB, bool W4>
int launch_dgrad_chain(const GemmArgs& p, const WgradArgs* wa, uint32_t wblocks, hipStream_t st) {
  constexpr int MTB = EpiGeom<NT>::MTB;
  const int64_t blocks = ((p.M + 15) / 16 + MTB - 1) / MTB;
  if (wa) {
    if (wa->d.Cin != NT * 16 || blocks + wblocks > 0x7fffffff) return LBT_EINVAL;
    hipLaunchKernelGGL((dgrad_wgrad_kernel<CS, NT, CF, NB, W4>), dim3((unsigned)(blocks + wblocks)), dim3(kThreads), 0,
                       st, p, *wa, wblocks);
  } else {
    hipLaunchKernelGGL((conv_gemm_kernel<MODE_DGRAD, CS, NT, CF, NB, W4>), dim3((unsigned)blocks), dim3(kThreads), 0,
                       st, p);
  }
  return (int)hipGetLastError();
}

constexpr int kAFused = kAFB | kAStoch;


template <bool W4>
int dgrad_chain(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg, lbt_qdesc qw,
                const float* add_src, const lbt_chain_bwd_a* a, const WgradArgs* wa, uint32_t wblocks, void* stream) {
  if (!desc_ok(d) || d.Cin % 16 || d.Cout % 16 || d.Cin > 128 || !a) return LBT_EINVAL;
  if (a->C != d.Cin || a->rows != d.N || a->inner != (int64_t)d.H * d.W * d.Cin) return LBT_EINVAL;
  const int f = bwd_a_flags(*a);
  if ((f & kAFused) != kAFused) return LBT_EINVAL;
  const lbt_bwd_branch* br[2] = {&a->b1, &a->b2};
  for (int b = 0; b < (a->has_b2 ? 2 : 1); ++b)
    if (!br[b]->qrg.noise || !br[b]->qng.noise || !br[b]->gb) return LBT_EINVAL;
  const int cs = d.Cout / 16;
  GemmArgs p;
  p.a = gq; p.b = wd; p.ks = ksd; p.nslices = d.KH * d.KW * cs;
  if (ksd % 4 || ksd < p.nslices) return LBT_EINVAL;
  p.a_fill = 0; p.colsum = nullptr;
  p.d = d; p.qa = qg; p.qb = qw; p.y = nullptr; p.add_src = add_src; p.yq = nullptr; p.qout = lbt_qdesc{};
  p.ychsum = nullptr;
  p.M = (int64_t)d.N * d.H * d.W; p.ncol = d.Cin;
  p.chain = *a;
  if (p.M * p.ncol >= ((int64_t)1 << 31)) return LBT_EINVAL;  // 32-bit element offsets
  hipStream_t st = (hipStream_t)stream;
  const int nt = d.Cin / 16;
  const int key = (cs << 8) | (nt << 4) | (a->has_b2 ? 1 : 0);
#define LBT_DC(CS_, NT_, CF_, NB_)                                                                  \
  if (key == ((CS_ << 8) | (NT_ << 4) | (NB_ == 2)) && f == (CF_))                                  \
    return launch_dgrad_chain<CS_, NT_, CF_, NB_, W4>(p, wa, wblocks, st);
#define LBT_DC_SHAPES(CF_, NB_) \
  LBT_DC(1, 1, CF_, NB_) LBT_DC(2, 2, CF_, NB_) LBT_DC(4, 4, CF_, NB_) LBT_DC(2, 1, CF_, NB_) LBT_DC(4, 2, CF_, NB_)
  LBT_DC_SHAPES(kAFused | kAMaskR, 1)             // block, first BN (mask from R1)
  LBT_DC_SHAPES(kAFused | kAYMask | kAGmask, 1)   // block end, identity shortcut
  LBT_DC_SHAPES(kAFused | kAYMask, 2)             // block end, projection shortcut
  LBT_DC_SHAPES(kAFused | kAYMask, 1)             // stem
#undef LBT_DC_SHAPES
#undef LBT_DC
  return LBT_EINVAL;
}

template <int CS, int NT, int CF, int NB, bool W4>
int launch_dgrad2(const GemmArgs& p, const GemmArgs& p2, hipStream_t st) {
  constexpr int MTB = EpiGeom<NT>::MTB;
  const int64_t blocks = ((p.M + 15) / 16 + MTB - 1) / MTB;
  hipLaunchKernelGGL((conv_dgrad2_kernel<CS, NT, CF, NB, W4>), dim3((unsigned)blocks), dim3(kThreads), 0, st, p, p2);
  return (int)hipGetLastError();
}

// dgrad (gq, wd, d) + dgrad (gq2, wd2, d2) + pass A, one launch (see conv_dgrad2_kernel)
template <bool W4>
int dgrad2_chain(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg, lbt_qdesc qw,
                 const int8_t* gq2, const int8_t* wd2, int32_t ksd2, lbt_conv_desc d2, lbt_qdesc qg2, lbt_qdesc qw2,
                 const lbt_chain_bwd_a* a, void* stream) {
  if (!desc_ok(d) || !desc_ok(d2) || d.Cin % 16 || d.Cout % 16 || d.Cin > 128 || !a) return LBT_EINVAL;
  // same input-gradient pixels and channels, same gathered-gradient geometry
  if (d2.N != d.N || d2.H != d.H || d2.W != d.W || d2.Cin != d.Cin || d2.Cout != d.Cout || d2.Ho != d.Ho ||
      d2.Wo != d.Wo)
    return LBT_EINVAL;
  if (a->C != d.Cin || a->rows != d.N || a->inner != (int64_t)d.H * d.W * d.Cin) return LBT_EINVAL;
  const int f = bwd_a_flags(*a);
  if ((f & kAFused) != kAFused) return LBT_EINVAL;
  const lbt_bwd_branch* br[2] = {&a->b1, &a->b2};
  for (int b = 0; b < (a->has_b2 ? 2 : 1); ++b)
    if (!br[b]->qrg.noise || !br[b]->qng.noise || !br[b]->gb) return LBT_EINVAL;
  const int cs = d.Cout / 16;
  GemmArgs p, p2;
  p.a = gq; p.b = wd; p.ks = ksd; p.nslices = d.KH * d.KW * cs;
  p2.a = gq2; p2.b = wd2; p2.ks = ksd2; p2.nslices = d2.KH * d2.KW * cs;
  if (ksd % 4 || ksd < p.nslices || ksd2 % 4 || ksd2 < p2.nslices) return LBT_EINVAL;
  p.a_fill = p2.a_fill = 0; p.colsum = p2.colsum = nullptr;
  p.d = d; p.qa = qg; p.qb = qw; p.y = nullptr; p.add_src = nullptr; p.yq = nullptr; p.qout = lbt_qdesc{};
  p.ychsum = nullptr;
  p.M = (int64_t)d.N * d.H * d.W; p.ncol = d.Cin;
  p.chain = *a;
  p2.d = d2; p2.qa = qg2; p2.qb = qw2; p2.y = nullptr; p2.add_src = nullptr; p2.yq = nullptr; p2.qout = lbt_qdesc{};
  p2.ychsum = nullptr; p2.M = p.M; p2.ncol = p.ncol; p2.chain = lbt_chain_bwd_a{};
  if (p.M * p.ncol >= ((int64_t)1 << 31)) return LBT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int nt = d.Cin / 16;
  const int key = (cs << 8) | (nt << 4) | (a->has_b2 ? 1 : 0);
#define LBT_D2(CS_, NT_, CF_, NB_)                                                                \
  if (key == ((CS_ << 8) | (NT_ << 4) | (NB_ == 2)) && f == (CF_))                                  \
    return launch_dgrad2<CS_, NT_, CF_, NB_, W4>(p, p2, st);
  // projection blocks (Cout = 2 Cin) whose input gradient feeds an identity block's end chain or
  // the stem's
  LBT_D2(2, 1, kAFused | kAYMask | kAGmask, 1) LBT_D2(4, 2, kAFused | kAYMask | kAGmask, 1)
  LBT_D2(2, 1, kAFused | kAYMask, 1) LBT_D2(4, 2, kAFused | kAYMask, 1)
#undef LBT_D2
  return LBT_EINVAL;
}

template <bool W4>
int dgrad_chain_wgrad(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg, lbt_qdesc qw,
                      const float* add_src, const lbt_chain_bwd_a* a, const int8_t* xq, int32_t x_u8off,
                      int32_t* slab, int32_t nsplit, int32_t nshard, void* stream) {
  WgradArgs wa;
  uint32_t wblocks = 0;
  const int e = wgrad_setup(xq, x_u8off, gq, d, slab, nsplit, nshard, wa, wblocks);
  if (e) return e;
  return dgrad_chain<W4>(gq, wd, ksd, d, qg, qw, add_src, a, &wa, wblocks, stream);
}

}  // namespace

extern "C" int lbt_conv_dgrad2_chain_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                                        lbt_qdesc qw, const int8_t* gq2, const int8_t* wd2, int32_t ksd2,
                                        lbt_conv_desc d2, lbt_qdesc qg2, lbt_qdesc qw2, int32_t w4,
                                        const lbt_chain_bwd_a* a, void* stream) {
  if (w4) {
    if (qw.bits > 4 || qw2.bits > 4) return LBT_EINVAL;
    return dgrad2_chain<true>(gq, wd, ksd, d, qg, qw, gq2, wd2, ksd2, d2, qg2, qw2, a, stream);
  }
  return dgrad2_chain<false>(gq, wd, ksd, d, qg, qw, gq2, wd2, ksd2, d2, qg2, qw2, a, stream);
}
extern "C" int lbt_conv_dgrad_chain_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                                       lbt_qdesc qw, const float* add_src, const lbt_chain_bwd_a* a, void* stream) {
  return dgrad_chain<false>(gq, wd, ksd, d, qg, qw, add_src, a, nullptr, 0, stream);
}
extern "C" int lbt_conv_dgrad_chain_i8w4(const int8_t* gq, const uint8_t* wd4, int32_t ksd, lbt_conv_desc d,
                                         lbt_qdesc qg, lbt_qdesc qw, const float* add_src, const lbt_chain_bwd_a* a,
                                         void* stream) {
  if (qw.bits > 4) return LBT_EINVAL;
  return dgrad_chain<true>(gq, (const int8_t*)wd4, ksd, d, qg, qw, add_src, a, nullptr, 0, stream);
}
extern "C" int lbt_conv_dgrad_chain_wgrad_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                                             lbt_qdesc qg, lbt_qdesc qw, const float* add_src,
                                             const lbt_chain_bwd_a* a, const int8_t* xq, int32_t x_u8off,
                                             int32_t* slab, int32_t nsplit, int32_t nshard, void* stream) {
  return dgrad_chain_wgrad<false>(gq, wd, ksd, d, qg, qw, add_src, a, xq, x_u8off, slab, nsplit, nshard, stream);
}
extern "C" int lbt_conv_dgrad_chain_wgrad_i8w4(const int8_t* gq, const uint8_t* wd4, int32_t ksd, lbt_conv_desc d,
                                               lbt_qdesc qg, lbt_qdesc qw, const float* add_src,
                                               const lbt_chain_bwd_a* a, const int8_t* xq, int32_t x_u8off,
                                               int32_t* slab, int32_t nsplit, int32_t nshard, void* stream) {
  if (qw.bits > 4) return LBT_EINVAL;
  return dgrad_chain_wgrad<true>(gq, (const int8_t*)wd4, ksd, d, qg, qw, add_src, a, xq, x_u8off, slab, nsplit,
                                 nshard, stream);
}

extern "C" int lbt_conv_wgrad_i8(const int8_t* xq, int32_t x_u8off, const int8_t* gq, lbt_conv_desc d,
                                    int32_t* slab, int32_t nsplit, int32_t nshard, void* stream) {
  WgradArgs wa;
  uint32_t blocks = 0;
  const int e = wgrad_setup(xq, x_u8off, gq, d, slab, nsplit, nshard, wa, blocks);
  if (e) return e;
  hipStream_t st = (hipStream_t)stream;
  switch (d.Cin / 16) {
    case 1: hipLaunchKernelGGL(conv_wgrad_kernel<1>, dim3(blocks), dim3(kThreads), 0, st, wa); break;
    case 2: hipLaunchKernelGGL(conv_wgrad_kernel<2>, dim3(blocks), dim3(kThreads), 0, st, wa); break;
    case 4: hipLaunchKernelGGL(conv_wgrad_kernel<4>, dim3(blocks), dim3(kThreads), 0, st, wa); break;
    case 8: hipLaunchKernelGGL(conv_wgrad_kernel<8>, dim3(blocks), dim3(kThreads), 0, st, wa); break;
    default: return LBT_EINVAL;
  }
  return (int)hipGetLastError();
}

// ---- many convs' weight gradients in ONE launch (lbt_conv_wgrad_many_i8): the jobs travel in the
// kernel arguments; job j owns blocks [start[j], start[j+1]) (multiples of 8: each job keeps its
// XCD-aware unit order). 3x3 / stride-1 / SAME jobs whose image rows tile 64-pixel chunks run
// wgrad_s1_body, the others conv_wgrad_body (one unit = pixel split x tap x co slice).
//
// wgrad_s1_body: workgroup = (pixel split, ci slice, co slice) of kFW waves. A wave takes 64
// consecutive output pixels at a time (whole image rows: 64 % W == 0, H % (64 / W) == 0), stages the
// X slices of those rows plus a one-pixel halo ([64/W + 2][W + 2][16 B], the fill code outside the
// image) and the 64 G slices in its own LDS region, and runs all 9 taps' MFMAs from there with
// per-lane transposed reads: X and G leave L2 once per (ci, co) slice pair instead of once per tap,
// and the next chunk's loads are in flight during the MFMAs. The waves' partials are summed in
// LDS and added into the job's slab (shard = split % nshard) with one integer atomic per output.
namespace {
constexpr int kMaxWJobs = 24;
#ifndef LBT_WGM_OCC
#define LBT_WGM_OCC 4  // waves per SIMD the batched launch's registers are budgeted for
#endif
#ifndef LBT_WGM_BUFS
#define LBT_WGM_BUFS 2
#endif
#ifndef LBT_WGX
#define LBT_WGX 0
#endif
constexpr int kWgmBufs = LBT_WGM_BUFS;  // chunks of loads in flight per wave (register buffers)
constexpr int kFW = 8;        // waves per workgroup of the batched launch
constexpr int kHaloMax = 3;   // halo slices per lane: (64/W + 2) * (W + 2) <= 192 (W | 64, 2 <= W <= 32)
struct WgradMany {
  WgradArgs j[kMaxWJobs];
  uint32_t start[kMaxWJobs + 1];
  int32_t fast[kMaxWJobs];
  int n;
};
union WgradManyShared {
  WgradShared<1, kFW> s1;
  WgradShared<2, kFW> s2;
  int8_t stage[kFW][5 * 1024];               // wgrad_s1_body: per wave X halo | G (at +4096)
  // wgrad_s1_body: partials [tap][kg][r][4] of wave pair (w, w + kFW/2), summed in place (the LDS of
  // three workgroups per CU: the batched launch fits one round)
  int red[kFW / 2][9 * 256];
};

bool wgrad_s1_ok(const lbt_conv_desc& d, int nsplit) {
  if (d.KH != 3 || d.KW != 3 || d.SH != 1 || d.SW != 1 || d.PT != 1 || d.PB != 1 || d.PL != 1 || d.PR != 1 ||
      d.Ho != d.H || d.Wo != d.W || d.W > 64 || 64 % d.W || d.H % (64 / d.W) ||
      (64 / d.W + 2) * (d.W + 2) > 64 * kHaloMax)
    return false;
  const int64_t chunks = (int64_t)d.N * d.H * d.W / 64;
  return nsplit > 0 && chunks % nsplit == 0;
}

LBT_DEV v4i tr_frag_at(const int8_t* img, int oa, int ob) {
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  const v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(img + oa));
  const v2i hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(img + ob));
  return v4i{lo.x, lo.y, hi.x, hi.y};
}

__device__ __forceinline__ void wgrad_s1_body(const WgradArgs& wa, uint32_t bid, WgradManyShared& sm) {
  const lbt_conv_desc& d = wa.d;
  const int H = d.H, W = d.W, Cin = d.Cin, Cout = d.Cout;
  const int ncs = Cin >> 4, ncos = Cout >> 4, nsplit = wa.nsplit;
  const int total = nsplit * ncs * ncos;
  const int xchunk = (total + 7) >> 3;
  const int u = (int)(bid & 7) * xchunk + (int)(bid >> 3);  // XCD-aware: a split's slices share an L2
  if (u >= total) return;
  const int split = u / (ncs * ncos), urem = u - split * (ncs * ncos);
  const int cis = urem / ncos, cos = urem - cis * ncos;
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int j = lane & 15, kg = lane >> 4;
  const int RB = 64 / W, Wp = W + 2, nhalo = (RB + 2) * Wp;
  const int64_t cps = (int64_t)d.N * H * W / 64 / nsplit;  // chunks per split (exact: host check)
  const int64_t c0 = (int64_t)split * cps;
  const int nmine = cps > wave ? (int)((cps - wave + kFW - 1) / kFW) : 0;
  const int HW = H * W;
  const int fill = wa.x_fill;
  int8_t* st = sm.stage[wave];
  int8_t* gs = st + 4096;
  // per-lane transposed-read offsets (chunk-invariant): pixels pa = 16kg + j/2 and pa + 8
  const int pa = 16 * kg + (j >> 1), pb = pa + 8;
  const int oxa = ((pa / W) * Wp + pa % W) * 16 + 8 * (j & 1);
  const int oxb = ((pb / W) * Wp + pb % W) * 16 + 8 * (j & 1);
  const int oga = pa * 16 + 8 * (j & 1), ogb = pb * 16 + 8 * (j & 1);
  // chunk-invariant geometry of this lane's halo slices t = lane + 64 i of the [RB + 2][W + 2] window:
  // the offset from the chunk's first pixel, whether it is a real column inside the window, whether it
  // lies in the window's top / bottom row (outside the image at the first / last row block). The
  // per-chunk part is then wave-uniform (scalar): the per-lane divisions by W + 2 of every chunk were
  // most of the loop's VALU instructions
  int hoff[kHaloMax];
  uint32_t hin = 0, htop = 0, hbot = 0;
#pragma unroll
  for (int i = 0; i < kHaloMax; ++i) {
    const int t = lane + 64 * i;
    const int hy = t / Wp, hx = t - hy * Wp;
    hoff[i] = ((hy - 1) * W + hx - 1) * Cin;
    hin |= (uint32_t)(t < nhalo && hx >= 1 && hx <= W) << i;
    htop |= (uint32_t)(hy == 0) << i;
    hbot |= (uint32_t)(hy == RB + 1) << i;
  }

  // two register buffers: chunk s + 2's loads are issued while chunk s is computed (s + 1's are
  // already in flight), so a wave waits on a load issued two chunks earlier
  struct Buf {
    v4i x[kHaloMax], g;
    uint32_t valid;
  };
  auto load = [&](Buf& b, int64_t c) {
    const int64_t p0 = c * 64;  // wave-uniform: the chunk's first pixel, RB whole rows of image n
    const int n = (int)(p0 / HW), row0 = (int)(p0 - (int64_t)n * HW) / W;
    const int8_t* xim = wa.xq + (p0 * Cin + cis * 16);  // = pixel (n, row0, 0)
    b.valid = hin & ~(row0 == 0 ? htop : 0u) & ~(row0 + RB == H ? hbot : 0u);
#pragma unroll
    for (int i = 0; i < kHaloMax; ++i)
      b.x[i] = *reinterpret_cast<const v4i*>(xim + ((b.valid >> i) & 1 ? hoff[i] : 0));
    b.g = *reinterpret_cast<const v4i*>(wa.gq + (p0 + lane) * Cout + cos * 16);
  };
  v4i acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = v4i{0, 0, 0, 0};
  // this wave's chunk s, clamped to its last one: the refills past the end reload it and every load
  // is UNCONDITIONAL, so the compiler's vmcnt waits count exactly the loads issued since (a load
  // under a branch made it wait for vmcnt(0) -- every chunk then paid a whole memory round trip:
  // 8 chunks ~ 12 us per stage-1 job, tools/trace_phases.py, profiles/round6/budget)
  auto cidx = [&](int s) { return c0 + wave + (int64_t)(s < nmine ? s : nmine - 1) * kFW; };
  // chunk s of this wave: stage b into LDS, refill b with chunk s + kWgmBufs, MFMAs of all 9 taps
  // (a step past the end, s >= nmine, adds a zero gradient fragment)
  // LBT_WGX (scratch timing builds only, wrong results): 1 no refill loads, 2 no LDS staging stores,
  // 4 no transposed LDS reads (register operands), 8 no MFMAs (integer adds)
  auto step = [&](Buf& b, int s) {
    if constexpr (!(LBT_WGX & 2)) {
#pragma unroll
      for (int i = 0; i < kHaloMax; ++i) {
        const int t = lane + 64 * i;
        const v4i v = (b.valid >> i) & 1 ? b.x[i] : v4i{fill, fill, fill, fill};
        if (t < nhalo) *reinterpret_cast<v4i*>(st + t * 16) = v;
      }
      *reinterpret_cast<v4i*>(gs + lane * 16) = s < nmine ? b.g : v4i{0, 0, 0, 0};
    }
    // the images are read by other lanes of the same wave only: a wave's LDS instructions execute in
    // issue order, so only the compiler must keep the reads after the writes (no fence: a workgroup
    // release fence would also wait for the refills in flight)
    asm volatile("" ::: "memory");
    if constexpr (!(LBT_WGX & 1)) load(b, cidx(s + kWgmBufs));
    const v4i bfrag = (LBT_WGX & 4) ? b.g : tr_frag_at(gs, oga, ogb);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int toff = ((t / 3) * Wp + t % 3) * 16;
      const v4i afrag = (LBT_WGX & 4) ? b.x[t % kHaloMax] : tr_frag_at(st, oxa + toff, oxb + toff);
      if constexpr (LBT_WGX & 8)
        acc[t] = acc[t] + afrag + bfrag;
      else
        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag, bfrag, acc[t], 0, 0, 0);
    }
    asm volatile("" ::: "memory");  // the next chunk's stores after these reads (in-order LDS)
  };
  LBT_TS(0);
  if (nmine > 0) {  // kWgmBufs register buffers: chunk s + kWgmBufs's loads issued during chunk s
    Buf bf[kWgmBufs];
#pragma unroll
    for (int k = 0; k < kWgmBufs; ++k) load(bf[k], cidx(k));
    for (int s = 0; s < nmine; s += kWgmBufs) {
#pragma unroll
      for (int k = 0; k < kWgmBufs; ++k) step(bf[k], s + k);
    }
  }
  LBT_TS(1);
  __syncthreads();  // the partials overwrite the staging regions
  // acc[t] element i: ci = 4kg + i, co = j (16x16 C/D map); waves w and w + kFW/2 share slot w
  constexpr int kHalf = kFW / 2;
  if (wave < kHalf) {
#pragma unroll
    for (int t = 0; t < 9; ++t) *reinterpret_cast<v4i*>(&sm.red[wave][(t * 64 + lane) * 4]) = acc[t];
  }
  __syncthreads();
  if (wave >= kHalf) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      v4i* q = reinterpret_cast<v4i*>(&sm.red[wave - kHalf][(t * 64 + lane) * 4]);
      *q = *q + acc[t];
    }
  }
  __syncthreads();
  LBT_TS(2);
  int32_t* dst = wa.slab + (int64_t)(split % wa.nshard) * 9 * Cin * Cout + (int64_t)cis * 16 * Cout + cos * 16;
  for (int i = threadIdx.x; i < 9 * 256; i += kFW * 64) {
    int v = 0;
#pragma unroll
    for (int w = 0; w < kHalf; ++w) v += sm.red[w][i];
    const int t = i >> 8, l = (i >> 2) & 63, ii = i & 3;
    const int ci = 4 * (l >> 4) + ii, co = l & 15;
    if (v) LBT_GADD(&dst[((int64_t)t * Cin + ci) * Cout + co], v);  // integer atomics: exact, order-independent
  }
  LBT_TS(3);
}

// block b of a batched launch: find its job, run that job's body
LBT_DEV void wgrad_many_block(const WgradMany& m, uint32_t b, WgradManyShared& sm) {
  int j = 0;
#pragma unroll 1
  while (j + 1 < m.n && b >= m.start[j + 1]) ++j;
  const WgradArgs& wa = m.j[j];
  const uint32_t rb = b - m.start[j];
#ifdef LBT_TRACE
  if (threadIdx.x == 0 && lbt_trace_buf) lbt_trace_buf[(size_t)blockIdx.x * 8 + 6] = (unsigned long long)(j + 1);
#endif
  if (m.fast[j]) {
    wgrad_s1_body(wa, rb, sm);
    return;
  }
  switch (wa.d.Cin >> 4) {
    case 1: conv_wgrad_body<1, kFW>(wa, rb, sm.s1); break;
    default: conv_wgrad_body<2, kFW>(wa, rb, sm.s2); break;
  }
}

__global__ __launch_bounds__(kFW * 64, LBT_WGM_OCC) void conv_wgrad_many_kernel(const WgradMany m) {
  __shared__ __attribute__((aligned(16))) WgradManyShared sm;
  wgrad_many_block(m, blockIdx.x, sm);
}

// The batched weight gradients with the stem's whole backward (stem_bwd.h, two 256-pixel row blocks
// per 512-thread workgroup) as extra blocks of the same launch: the stem backward reads only the first
// block's dgrad output, like the batched jobs, so it shares the batched launch's rounds of workgroups
// instead of running as a launch of its own after it (lbt_conv_wgrad_many_stem_i8; 25.2 + 13.0 us as
// two launches -> 34.2 us as one).
union WgradManyStemShared {
  WgradManyShared w;
  StemBwdShared<2> s;
};
static_assert(kFW * 64 == 2 * 256, "two stem row blocks per workgroup of the batched launch");
// (stem_first, the default: the stem's workgroups are the launch's FIRST blocks; else its last)
__global__ __launch_bounds__(kFW * 64, LBT_WGM_OCC) void conv_wgrad_many_stem_kernel(const WgradMany m,
                                                                                    const StemBwdArgs st,
                                                                                    uint32_t pairs, int stem_first) {
  __shared__ __attribute__((aligned(16))) WgradManyStemShared sm;
  const uint32_t b = blockIdx.x, nw = m.start[m.n];
  if (stem_first ? b < pairs : b >= nw) {
    stem_bwd_body<2>(st, stem_first ? b : b - nw, sm.s);
    return;
  }
  wgrad_many_block(m, stem_first ? b - pairs : b, sm.w);
}
static_assert(sizeof(WgradMany) + sizeof(StemBwdArgs) + 8 <= 4096, "kernel arguments");
static_assert(sizeof(WgradMany) <= 4096, "kernel arguments");

// WgradArgs + block count of one job of the batched launch
int wgrad_many_setup(const lbt_wgrad_job& w, WgradArgs& wa, uint32_t& blocks, int32_t& fast) {
  if (!w.slab || !w.xq || !w.gq) return LBT_EINVAL;
  const int e = wgrad_setup(w.xq, w.x_u8off, w.gq, w.d, w.slab, w.nsplit, w.nshard, wa, blocks);
  if (e) return e;
  fast = wgrad_s1_ok(w.d, w.nsplit) ? 1 : 0;
  if (fast) {
    const int64_t units = (int64_t)w.nsplit * (w.d.Cin / 16) * (w.d.Cout / 16);
    blocks = (uint32_t)((units + 7) / 8 * 8);
  } else if (w.d.Cin != 16 && w.d.Cin != 32) {
    return LBT_EINVAL;  // conv_wgrad_body<CSI, kFW> instances: CSI 1, 2
  }
  return 0;
}
}  // namespace

extern "C" int lbt_conv_wgrad_many_i8(const lbt_wgrad_job* jobs, int32_t njobs, void* stream) {
  if (njobs < 0 || (njobs > 0 && !jobs)) return LBT_EINVAL;
  for (int i = 0; i < njobs; ++i) {  // every job checked before anything is queued
    WgradArgs wa;
    uint32_t blocks = 0;
    int32_t fast = 0;
    const int e = wgrad_many_setup(jobs[i], wa, blocks, fast);
    if (e) return e;
  }
  for (int base = 0; base < njobs; base += kMaxWJobs) {
    WgradMany m{};
    const int n = njobs - base < kMaxWJobs ? njobs - base : kMaxWJobs;
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) {
      uint32_t blocks = 0;
      wgrad_many_setup(jobs[base + i], m.j[i], blocks, m.fast[i]);
      m.start[i] = (uint32_t)total;
      total += blocks;
    }
    if (total >= 0x7fffffffull) return LBT_EINVAL;
    m.start[n] = (uint32_t)total;
    m.n = n;
    hipLaunchKernelGGL(conv_wgrad_many_kernel, dim3((unsigned)total), dim3(kFW * 64), 0, (hipStream_t)stream, m);
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  return 0;
}

extern "C" int lbt_conv_stem_bwd(const lbt_chain_bwd_b* b, const int16_t* x, lbt_conv_desc d, int32_t* slab,
                                 int32_t nshard, void* stream);

// lbt_conv_wgrad_many_i8(jobs) then lbt_conv_stem_bwd(b, x, d, slab, nshard) with the stem's row
// blocks riding in the batched launch (two per workgroup): as its FIRST workgroups by default (measured
// 0.9 us faster), as its last with LBT_STEM_FIRST=0; the same results (integer atomics). A batch too large for one launch, or an odd number of stem row blocks, runs as the two calls.
extern "C" int lbt_conv_wgrad_many_stem_i8(const lbt_wgrad_job* jobs, int32_t njobs, const lbt_chain_bwd_b* b,
                                           const int16_t* x, lbt_conv_desc d, int32_t* slab, int32_t nshard,
                                           void* stream) {
  if (njobs < 0 || (njobs > 0 && !jobs) || !b || !x || !slab || nshard <= 0) return LBT_EINVAL;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (M <= 0 || !stem_bwd_shape_ok(b, d)) return M <= 0 ? lbt_conv_wgrad_many_i8(jobs, njobs, stream) : LBT_EINVAL;
  const int64_t rblocks = M / kSbPixels, pairs = rblocks / 2;
  // int32 shard totals stay exact: <= 31 row blocks per shard (stem.hip lbt_conv_stem_wgrad)
  if (njobs > kMaxWJobs || rblocks % 2 || (pairs + nshard - 1) / nshard * 2 > 31) {
    const int e = lbt_conv_wgrad_many_i8(jobs, njobs, stream);
    return e ? e : lbt_conv_stem_bwd(b, x, d, slab, nshard, stream);
  }
  WgradMany m{};
  uint64_t total = 0;
  for (int i = 0; i < njobs; ++i) {  // every job checked before anything is queued
    uint32_t blocks = 0;
    const int e = wgrad_many_setup(jobs[i], m.j[i], blocks, m.fast[i]);
    if (e) return e;
    m.start[i] = (uint32_t)total;
    total += blocks;
  }
  m.start[njobs] = (uint32_t)total;
  m.n = njobs;
  if (total + pairs >= 0x7fffffffull) return LBT_EINVAL;
  StemBwdArgs st;
  st.b = *b; st.x = x; st.d = d; st.K = d.KH * d.KW * d.Cin; st.slab = slab; st.nshard = nshard;
  // stem blocks first (A/B on one box, isolated launch: 34.2 / 34.3 us vs 35.0 / 35.2 us placed last);
  // LBT_STEM_FIRST=0 places them last
  static const int stem_first = !(getenv("LBT_STEM_FIRST") != nullptr && getenv("LBT_STEM_FIRST")[0] == '0');
  hipLaunchKernelGGL(conv_wgrad_many_stem_kernel, dim3((unsigned)(total + pairs)), dim3(kFW * 64), 0,
                     (hipStream_t)stream, m, st, (uint32_t)pairs, stem_first);
  return (int)hipGetLastError();
}

extern "C" int lbt_conv_wgrad_reduce(const int32_t* slab, int32_t nsplit, int32_t K, int32_t Cout, int32_t x_u8off,
                                     const int64_t* gcolsum, lbt_qdesc qx, lbt_qdesc qg, const float* w, float wd2,
                                     float* dw, void* stream) {
  const int64_t total = (int64_t)K * Cout;
  const int64_t blocks = (total + 31) / 32;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, slab, nsplit, K,
                     Cout, x_u8off, gcolsum, qx, qg, w, wd2, dw, nullptr);
  return (int)hipGetLastError();
}
extern "C" int lbt_conv_wgrad_reduce_x(const int32_t* slab, int32_t nsplit, int32_t K, int32_t Cout, int32_t x_u8off,
                                       const int64_t* gcolsum, int64_t* num, void* stream) {
  if (!num || nsplit <= 0 || K <= 0 || Cout <= 0) return LBT_EINVAL;
  const int64_t blocks = ((int64_t)K * Cout + 31) / 32;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, slab, nsplit, K,
                     Cout, x_u8off, gcolsum, lbt_qdesc{}, lbt_qdesc{}, nullptr, 0.f, nullptr, (long long*)num);
  return (int)hipGetLastError();
}

// Diagnostics: resident workgroups per CU of a few conv GEMM variants (hipOccupancy API), written
// to out[0..n): fwd<CS1,NT1>, dgrad+A<CS1,NT1,26>, dgrad<CS4,NT2>, dgrad+A<CS2,NT2,26>, wgrad<1>.
extern "C" int lbt_diag_occupancy(int32_t* out, int32_t n) {
  const void* k[5] = {reinterpret_cast<const void*>(&conv_gemm_kernel<MODE_FWD, 1, 1, 0, 1, false>),
                      reinterpret_cast<const void*>(&conv_gemm_kernel<MODE_DGRAD, 1, 1, 26, 1, false>),
                      reinterpret_cast<const void*>(&conv_gemm_kernel<MODE_DGRAD, 4, 2, 0, 1, false>),
                      reinterpret_cast<const void*>(&conv_gemm_kernel<MODE_DGRAD, 2, 2, 26, 1, false>),
                      reinterpret_cast<const void*>(&conv_wgrad_kernel<1>)};
  for (int i = 0; i < n && i < 5; ++i) {
    int b = -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k[i], kThreads, 0) != hipSuccess) b = -1;
    out[i] = b;
  }
  return 0;
}

// ============================================================================ fused conv backward
// lbt_conv_bwd_fused_i8: one stride-1 3x3 conv's backward with both neighbouring BN passes in ONE
// launch. A dgrad workgroup owns tile_rows(CS) image rows of one sample:
//   phase 1  pass B of the BN after the conv (bn.hip chain_bwd_b_kernel's arithmetic) over the rows
//            plus a one-pixel halo -> int8 gq codes in LDS; owned pixels also store gq (the weight
//            gradient's operand), count overflows and add the gq channel sums
//   phase 2  dgrad on v_mfma_i32_16x16x64_i8 with every A fragment a 16-byte ds_read of the LDS
//            gq image (the 9 taps never go back to memory) -> fp32 tile in LDS
//   phase 3  pass A of the BN before the conv (chain_bwd_a_kernel's arithmetic) over the tile, one
//            channel quad per thread with vector loads / stores
// Workgroups [0, nwg) run a weight-gradient job instead (conv_wgrad_body): the deferred wgrad of the
// conv of the previous launch.
namespace {

// Phase stamps of conv_bwd_kernel (scratch -DLBT_TRACE builds); -DLBT_P1STUDY moves them into its load
// phase: slots 1-3 = statistics loads issued / all loads issued / statistics finished, 4 / 5 = the ends of
// the load phase and of phase 1 (tools/trace_phases.py)
#ifdef LBT_P1STUDY
#define LBT_TSS(i) LBT_TS(i)
#define LBT_TSB(i) do { if ((i) == 1) LBT_TS(4); else if ((i) == 2) LBT_TS(5); } while (0)
#else
#define LBT_TSS(i) do { } while (0)
#define LBT_TSB(i) LBT_TS(i)
#endif
constexpr int kBNW = 8;    // waves per workgroup
constexpr int kBThreads = kBNW * 64;
// image rows per workgroup: 8 for the 16-channel stage (1024 4-row tiles would take two rounds of
// two 512-thread workgroups per CU), 4 otherwise (W * C == 512: a 4-row tile is 8 MFMA tiles)
__host__ __device__ constexpr int tile_rows(int CS) { return CS == 1 ? 8 : 4; }
// phase-1 (halo) channel-quad groups per thread
__host__ __device__ constexpr int halo_iters(int CS, int TH) {
  return ((TH + 2) * (512 / (CS * 16) + 2) * CS * 4 + kBThreads - 1) / kBThreads;
}
__host__ __device__ constexpr int halo_iters(int CS) { return halo_iters(CS, tile_rows(CS)); }
// Batch-adaptive tile rows of the fused conv kernels: the 16-channel stage takes 4-row tiles when its
// 8-row tiles leave the launch with fewer workgroups than CUs (N * H / 8 < 256: per-GPU batches below
// 64 -- the strong-scaling shards of configs[2]): twice the workgroups, each with two thirds of the halo
// rows of phase 1, half the phase-3 groups and MFMA pairs per wave. LBT_TILE_ROWS1=8|4 forces one.
// The 32- / 64-channel stages take 2-row tiles when 4-row tiles leave CUs without a workgroup
// (N * H / 4 < 256: per-GPU batches below 64 for the 64-channel stage, below 32 for the 32-channel
// one): B = 16 0.301 -> 0.291 ms per step, bit-identical. Not at one tile per CU: the 64-channel stage
// at B = 128 (256 tiles) measured 0.414 -> 0.433 ms with 2-row tiles (two co-resident workgroups per CU,
// each staging the whole 37 KB weight image and a halo of 2 rows per 2; profiles/round6/tile_rows23_ab.txt).
// LBT_TILE_ROWS23=4|2 forces one.
inline int tile_rows_for(int CS, int64_t N, int H) {
  if (CS != 1) {
    static const int force23 = [] {
      const char* e = getenv("LBT_TILE_ROWS23");
      return e ? atoi(e) : 0;
    }();
    if (force23 == 4 || H % 4) return 4;
    return (force23 == 2 || N * H / 4 < 256) ? 2 : 4;
  }
  static const int force = [] {
    const char* e = getenv("LBT_TILE_ROWS1");
    return e ? atoi(e) : 0;
  }();
  if (force == 2 || force == 4 || force == 8) return H % force ? 8 : force;  // (16-row tiles at B=128: 0.447 vs 0.429 ms)
  if (N * H / 8 >= 256 || H % 4) return 8;
  return (N * H / 4 < 256 && H % 2 == 0) ? 2 : 4;  // (2-row tiles: B = 16, as the wide stages below)
}

// The conv's weight image shared through LDS by the fused conv kernels: [C columns][KS k-slices] of 16
// bytes (W4: 8-byte packed slices), loaded once per workgroup with coalesced 16-byte loads (in the
// launch's first load wave), written to LDS at the end of phase 1 (no extra wait: the loads have long
// landed) and read per fragment in phase 2. Each wave used to load its n-tile's fragments itself: 2
// (C = 64), 4 (32) or 8 (16) waves per n-tile, i.e. 72 KB of weight loads per stage-3 workgroup where the
// image is 36 KB -- through one CU's load path, in the load phase that dominates these launches. LDS
// column stride padded by 16 bytes: the 16 lanes r of a fragment read conflict-free.
template <int C, int KS, bool W4>
struct WImg {
  static constexpr int kBpf = W4 ? 8 : 16;       // bytes per (column, k-slice) fragment
  static constexpr int kColB = KS * kBpf;         // bytes per column in the global image
  static constexpr int kStride = kColB + 16;      // ... in LDS
  static constexpr int kBytes = C * kStride;
  static constexpr int kChunks = C * kColB / 16;  // 16-byte chunks of the global image
  static constexpr int kIt = (kChunks + kBThreads - 1) / kBThreads;
  static_assert(kColB % 16 == 0, "16-byte chunks within a column");
  LBT_DEV static void load(const int8_t* src, v4i (&v)[kIt]) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int i = (int)threadIdx.x + it * kBThreads;
      v[it] = *reinterpret_cast<const v4i*>(src + (int64_t)(i < kChunks ? i : 0) * 16);
    }
  }
  LBT_DEV static void store(int8_t* lds, const v4i (&v)[kIt]) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int i = (int)threadIdx.x + it * kBThreads;
      if (i < kChunks) {
        const int g = i * 16, col = g / kColB;
        *reinterpret_cast<v4i*>(lds + col * kStride + (g - col * kColB)) = v[it];
      }
    }
  }
  LBT_DEV static v4i frag(const int8_t* lds, int col, int slice) {
    if constexpr (W4)
      return unpack_i4x16(*reinterpret_cast<const v2i*>(lds + col * kStride + slice * 8));
    else
      return *reinterpret_cast<const v4i*>(lds + col * kStride + slice * 16);
  }
};

struct ConvBwdArgs {
  lbt_chain_bwd_b b;
  const int8_t* wd;
  int ks, nslices, w4;
  lbt_qdesc qw;
  int H, W;
  const float* add_src;
  lbt_chain_bwd_a a;
};

template <int C, int TH, int WB>
struct BwdShared {
  int8_t w[WB];                                  // the dgrad weight image (WImg)
  int8_t gq[(TH + 2) * (512 / C + 2) * C];   // halo image [(TH+2)][(W+2)][C], W*C == 512
  float tile[TH * (512 / C) * (C + 4)];       // dgrad outputs [TH*W][C+4] (padded rows)
  float pb[2 * C];                               // pass-B constants mg, mgx per channel
  int part[kBNW][(2 * 4 + 2) * C];               // per wave: pass-A sums per branch, gq sums
  int cnt[kBNW * 2 * 5];                         // counters: 5 quantisers x waves
};

LBT_DEV int ld4i8(const int8_t* p, int64_t i) { return *reinterpret_cast<const int*>(p + i); }
LBT_DEV void unpack4(int w, int v[4]) {
  v[0] = (int8_t)(w & 0xff); v[1] = (int8_t)((w >> 8) & 0xff);
  v[2] = (int8_t)((w >> 16) & 0xff); v[3] = (int8_t)(w >> 24);
}
LBT_DEV int pack4(const int c[4]) {
  return (int)((uint32_t)(c[0] & 0xff) | ((uint32_t)(c[1] & 0xff) << 8) | ((uint32_t)(c[2] & 0xff) << 16) |
               ((uint32_t)c[3] << 24));
}
LBT_DEV float4 ld4f(const float* p, int64_t i) { return *reinterpret_cast<const float4*>(p + i); }

// Wave total of the lanes holding the same channel quad (lanes l, l + C4, l + 2*C4, ...): DPP
// rotations inside each 16-lane row, then the rows paired by a lane shuffle (xor 16) and the halves
// by v_permlane32_swap (its two results are the lane's own half and the other half, both ways:
// their sum is the pair total in every lane). The total lands in every lane.
// (The row pairing is v_permlane16_swap: its two results hold the lane's own row and the paired
// row, both ways -- a VALU exchange where __shfl_xor(v, 16) was an LDS ds_bpermute round trip.)
LBT_DEV int row_pair_sum(int v) {
  const auto h = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return (int)h[0] + (int)h[1];
}
LBT_DEV int half_pair_sum(int v) {
  const auto h = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (int)h[0] + (int)h[1];
}
// 64-bit sum over the four 16-lane rows of a wave (permlane16 then permlane32 swaps on both halves)
LBT_DEV long long rows_total64(long long v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)((unsigned long long)v >> 32);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  v = (long long)(((unsigned long long)b[0] << 32) | a[0]) + (long long)(((unsigned long long)b[1] << 32) | a[1]);
  const uint32_t lo2 = (uint32_t)v, hi2 = (uint32_t)((unsigned long long)v >> 32);
  const auto c = __builtin_amdgcn_permlane32_swap(lo2, lo2, false, false);
  const auto d = __builtin_amdgcn_permlane32_swap(hi2, hi2, false, false);
  return (long long)(((unsigned long long)d[0] << 32) | c[0]) + (long long)(((unsigned long long)d[1] << 32) | c[1]);
}
// the whole wave's total in every lane, on DPP / permlane swaps only (no LDS)
LBT_DEV int wave_total(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  return half_pair_sum(row_pair_sum(v));
}

// Stochastic quantiser (quant_w<1>'s arithmetic) with PER-LANE overflow counts, on the VALU only:
// the asymmetric predicate x >= T or x < -T (T a power of two) is max(x, -x*(1-2^-24)) >= T -- for
// x < 0 the product rounds to >= T exactly when -x > T (the float after T, T(1+2^-23), gives
// T(1+2^-24-2^-47), which rounds down to T; -x = T gives T(1-2^-24), representable and < T). A NaN
// threshold (lanes that must not count: halo pixels, which the owning workgroup counts) compares
// false. Two compares + two carry-adds per element and no lane masks live in SGPRs (the __ballot
// form kept one 64-bit mask per predicate live across the unrolled elements and spilled them into
// VGPR lanes); ov_wave turns the lane counts into wave totals once per kernel.
LBT_DEV int quant_sl(const QState& s, float x, float u, float T1, float T2, int& c1, int& c2) {
  const float xm = x * s.m;
  const float a = fmaxf(xm, -xm * 0x1.fffffep-1f);
  c1 += a >= T1;
  c2 += a >= T2;
  float v = xm + u;
  v = fminf(fmaxf(v, -s.L), s.Lm1);
  return (int)floorf(v);
}
// Keep the counts of a phase computed inside it: otherwise the compiler sinks the compares to
// the counts' use at the kernel end and keeps every element's operand live across the phases.
LBT_DEV void pin_counts(int& c1, int& c2) { asm volatile("" : "+v"(c1), "+v"(c2)); }
LBT_DEV float ov_thr(bool cnt, float T) { return cnt ? T : __builtin_nanf(""); }
// lane counts (each < 2^16) -> the wave totals, in every lane
LBT_DEV void ov_wave(int& c1, int& c2) {
  const int t = wave_total(c1 | (c2 << 16));
  c1 = t & 0xffff;
  c2 = t >> 16;
}
// Four quantisers' packed lane counts (c1 | c2 << 16 each, as ov_wave) -> their wave totals,
// staged at counts_stage_w's slots i0 .. i0 + 3 (slots >= nq skipped): one rows_scatter4 leaves
// quantiser r's four-row sums in row r, the DPP steps finish the row (10 VALU exchanges where four
// ov_wave calls spend 24).
LBT_DEV int ov_pack(int c1, int c2) { return c1 | (c2 << 16); }
LBT_DEV void ov_stage4(int i0, int nq, int v0, int v1, int v2, int v3, int* sh) {
  int t = rows_scatter4(v0, v1, v2, v3);
  t += __builtin_amdgcn_update_dpp(0, t, 0x128, 0xf, 0xf, false);  // row_ror:8
  t += __builtin_amdgcn_update_dpp(0, t, 0x124, 0xf, 0xf, false);  // row_ror:4
  t += __builtin_amdgcn_update_dpp(0, t, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  t += __builtin_amdgcn_update_dpp(0, t, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  const int lane = (int)(threadIdx.x & 63), i = i0 + (lane >> 4);
  if ((lane & 15) == 0 && i < nq) {
    int* p = sh + (int)(threadIdx.x >> 6) * 2 * nq + 2 * i;
    p[0] = t & 0xffff;
    p[1] = t >> 16;
  }
}

// ---- channel pairs on packed fp32 (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32: two lanes' worth of
// IEEE fp32 per instruction, each half rounded exactly as the scalar op). The element chains of the
// fused conv kernels are VALU-bound (SQ: VALU busy ~70 % of the kernel), so every multiply / add /
// fma of a channel quad runs as two packed ops; compares, clamps, floors and conversions stay scalar.
typedef float f2 __attribute__((ext_vector_type(2)));
LBT_DEV f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
LBT_DEV f2 mk2(float a, float b) { return f2{a, b}; }
LBT_DEV f2 cvt2(int a, int b) { return f2{(float)a, (float)b}; }
// div_by (the compiler's correctly rounded x / y given y's reciprocal refinement) on a pair
LBT_DEV f2 div_by2(f2 x, f2 y, f2 rc) {
  const f2 q = x * rc;
  const f2 r = fma2(-y, q, x);
  const f2 q1 = fma2(r, rc, q);
  const f2 r1 = fma2(-y, q1, x);
  return __builtin_elementwise_copysign(fma2(r1, rc, q1), x);
}
// div_by2 for numerators that are never -0 -- the copysign only restores div_fixup's -0 / y = -0;
// every other quotient already carries x's sign. True of the BN differences it is used on: x1 - mu
// with x1 = q * 2^-e (an integer code: +0 when q == 0) and t1 - t2 with t1 = G * 2^-e - mg (mg from
// an integer sum: never -0), since a - b is -0 only when a is -0 and b is +0.
LBT_DEV f2 div_by2_nz(f2 x, f2 y, f2 rc) {
  const f2 q = x * rc;
  const f2 r = fma2(-y, q, x);
  const f2 q1 = fma2(r, rc, q);
  const f2 r1 = fma2(-y, q1, x);
  return fma2(r1, rc, q1);
}
// overflow counts of a pair (quant_sl's predicate; NaN thresholds count nothing)
LBT_DEV void ov_count2(f2 xm, float T1, float T2, int& c1, int& c2) {
  const f2 n = xm * mk2(-0x1.fffffep-1f, -0x1.fffffep-1f);
  const float a0 = fmaxf(xm.x, n.x), a1 = fmaxf(xm.y, n.y);
  c1 += (a0 >= T1) + (a1 >= T1);
  c2 += (a0 >= T2) + (a1 >= T2);
}
// the same for xm >= 0 (inputs after a ReLU): x < -T cannot hold
LBT_DEV void ov_count2_pos(f2 xm, float T1, float T2, int& c1, int& c2) {
  c1 += (xm.x >= T1) + (xm.y >= T1);
  c2 += (xm.x >= T2) + (xm.y >= T2);
}
// floor(clip(xm + u, -L, L-1)) of a pair, as floats (the codes, exact); med3 is the clip for
// non-NaN operands
LBT_DEV f2 qfloor2(const QState& s, f2 xm, f2 u) {
  const f2 v = xm + u;
  return mk2(floorf(__builtin_amdgcn_fmed3f(v.x, -s.L, s.Lm1)), floorf(__builtin_amdgcn_fmed3f(v.y, -s.L, s.Lm1)));
}
LBT_DEV int pack4f(f2 a, f2 b) {
  const int c[4] = {(int)a.x, (int)a.y, (int)b.x, (int)b.y};
  return pack4(c);
}

template <int CS, int CF, int NB, bool W4, int WCS, int TH = tile_rows(CS)>
__global__ __launch_bounds__(kBThreads, (CS == 4 && TH >= 4) ? 2 : 4) void conv_bwd_kernel(ConvBwdArgs p, WgradArgs wa, uint32_t nwg) {
  constexpr int C = CS * 16, C4 = C / 4, NT = CS;
  constexpr int kMaxKS = (9 * CS + 3) / 4;
  constexpr int WC = WCS ? WCS : 1;
  // J: phase-3 groups per thread (NQ channel quads per tile: TH x 512 bytes / 4); NPR: (m, n) MFMA
  // pairs per tile (2 TH: one per wave at TH = 4). Two-row tiles (TH = 2, the under-filled 32- /
  // 64-channel launches) leave waves 4-7 without a pair and threads >= 256 without a phase-3 group.
  constexpr int kBIt = halo_iters(CS, TH), NQ = TH * 128, J = (NQ + kBThreads - 1) / kBThreads, NPR = 2 * TH;
  static_assert(TH % 4 == 0 || TH == 2, "whole groups of 4 rows, or 2-row tiles");
  using WI = WImg<C, 4 * kMaxKS, W4>;
  union Smem {
    BwdShared<C, TH, WI::kBytes> b;
    WgradShared<WC, kBNW> w;
  };
  __shared__ __attribute__((aligned(16))) Smem sm;
  if (WCS != 0 && blockIdx.x < nwg) {
    conv_wgrad_body<WC, kBNW>(wa, blockIdx.x, sm.w);
    return;
  }
  BwdShared<C, TH, WI::kBytes>& sh = sm.b;
  LBT_TS(0);
  const lbt_chain_bwd_b& B = p.b;
  const lbt_chain_bwd_a& A = p.a;
  const uint32_t bid = blockIdx.x - nwg;
  constexpr int W = 512 / C, Wp = W + 2;  // W * C == 512 (host check)
  const int H = p.H;
  const int tpi = H / TH;
  const int n = (int)(bid / (uint32_t)tpi), row0 = (int)(bid - (uint32_t)n * tpi) * TH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int cq = (tid % C4) * 4;  // this thread's channel quad (512 % C4 == 0: fixed over its groups)
  const int64_t img = (int64_t)n * H * W * C;

  // ---------------- the pass-B statistics' shard sums first (they gate the first barrier): 16 groups
  // of 32 lanes, lane = shard, group g owning channels g*CPG .. g*CPG+CPG-1 (SG, SGQ)
  // Waves w < C / 16 each own 16 channels: lane l reads channel w*16 + (l & 15) of shards
  // 8*(l >> 4) .. +7, so every load instruction covers 4 shards x 16 consecutive channels (128-byte
  // rows); rows_total64 adds the wave's four lane rows.
  static_assert(LBT_NSHARD == 32 && kBThreads == 512 && C % 16 == 0 && C / 16 <= kBNW, "statistics layout");
  constexpr int kSW = C / 16;  // statistics waves
  long long sv[8][2];
  if (wave < kSW) {  // uniform per wave
    const int64_t* ps = B.sums + (int64_t)(8 * (lane >> 4)) * 4 * C + wave * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sv[i][0] = ps[(int64_t)i * 4 * C + 2 * C];
      sv[i][1] = ps[(int64_t)i * 4 * C + 3 * C];
    }
  }
  LBT_TSS(1);  // the statistics loads issued
  // then every load that does not depend on the sums
  // phase-1 operands: G / q codes and the output quantiser's noise over the halo rows
  const int ngrp = (TH + 2) * Wp * C4;
  int Gv[kBIt], Qv[kBIt];
  float4 Uv[kBIt];
#pragma unroll
  for (int it = 0; it < kBIt; ++it) {
    const int g = tid + it * kBThreads;
    const int pix = g / C4, hy = pix / Wp, hx = pix - hy * Wp;
    const int y = row0 - 1 + hy, x = hx - 1;
    const bool in = g < ngrp && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    const uint32_t off = in ? (uint32_t)((y * W + x) * C + cq) : 0u;
    Gv[it] = ld4i8(B.G, img + off);
    Qv[it] = ld4i8(B.qn_codes, img + off);
    Uv[it] = ld4f(B.qo.noise, off);
  }
  // the phase-2 B operands (the dgrad weight image, ks == 4 * kMaxKS: host check), for LDS (WImg)
  v4i wimg[WI::kIt];
  WI::load(p.wd, wimg);
  float mu[4], sg[4], gam[2][4], bet[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    mu[k] = B.ms[cq + k];
    sg[k] = B.ms[C + cq + k];
#pragma unroll
    for (int b = 0; b < NB; ++b) gam[b][k] = (b == 0 ? A.b1 : A.b2).gb[cq + k];
    bet[k] = A.b1.gb[C + cq + k];
  }
  const QState sgq = qstate(B.qng), sn = qstate(B.qn), so = qstate(B.qo);
  QState qrg[2], qng[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    qrg[b] = qstate((b == 0 ? A.b1 : A.b2).qrg);
    qng[b] = qstate((b == 0 ? A.b1 : A.b2).qng);
  }
  const float r_inv = (CF & kAMaskR) ? qstate(A.b1.qr).inv_m : 0.f;
  const float scale = ldexpf(1.0f, -(frac_exp(B.qo) + frac_exp(p.qw)));
  LBT_TSS(2);  // every other load issued, the descriptors read

  // ---------------- pass-B statistics: the shard sums (loaded first, above) added per lane, then over
  // the statistics wave's four lane rows; lanes < 16 finish their channel in double exactly as
  // chain_bwd_b_kernel
  if (wave < kSW) {
    long long SGi = 0, SGQi = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      SGi += sv[i][0];
      SGQi += sv[i][1];
    }
    SGi = rows_total64(SGi);
    SGQi = rows_total64(SGQi);
    const int c = wave * 16 + (lane & 15);
    if (lane < 16) {
    const double s = (double)sn.inv_m, gsc = (double)sgq.inv_m, nn = (double)B.n;
    const double SG = (double)SGi, SGQ = (double)SGQi;
    const float m = B.ms[c], sig = B.ms[C + c];
    sh.pb[c] = (float)(gsc * SG / nn);
    sh.pb[C + c] = (float)(gsc * (s * SGQ - (double)m * SG) / (nn * (double)sig));
    }
  }
  LBT_TSS(3);  // the statistics finished
  __syncthreads();
  LBT_TSB(1);
  float rmg[4], rmgx[4];
  Recip rsg[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rmg[k] = sh.pb[cq + k];
    rmgx[k] = sh.pb[C + cq + k];
    rsg[k] = recip(sg[k]);
  }
  f2 mu2[2], sg2[2], rsc2[2], rmg2[2], rmgx2[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    mu2[h] = mk2(mu[2 * h], mu[2 * h + 1]);
    sg2[h] = mk2(rsg[2 * h].y, rsg[2 * h + 1].y);
    rsc2[h] = mk2(rsg[2 * h].rc, rsg[2 * h + 1].rc);
    rmg2[h] = mk2(rmg[2 * h], rmg[2 * h + 1]);
    rmgx2[h] = mk2(rmgx[2 * h], rmgx[2 * h + 1]);
  }

  // ---------------- phase 1: pass B over the rows + halo -> LDS gq image
  int ovq1 = 0, ovq2 = 0;
  int s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
#pragma unroll
  for (int it = 0; it < kBIt; ++it) {
    if (it * kBThreads >= ngrp) break;  // uniform
    const int g = tid + it * kBThreads;
    const int pix = g / C4, hy = pix / Wp, hx = pix - hy * Wp;
    const int y = row0 - 1 + hy, x = hx - 1;
    const bool valid = g < ngrp;
    const bool in = valid && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    const bool own = in && hy >= 1 && hy <= TH;
    const float T1 = ov_thr(own, so.L), T2 = ov_thr(own, so.Lh);
    int G[4], q[4], c[4];
    unpack4(Gv[it], G);
    unpack4(Qv[it], q);
    const f2 u[2] = {mk2(Uv[it].x, Uv[it].y), mk2(Uv[it].z, Uv[it].w)};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f2 x1 = cvt2(q[2 * h], q[2 * h + 1]) * sn.inv_m;
      const f2 x2 = x1 - mu2[h];
      const f2 xh = div_by2_nz(x2, sg2[h], rsc2[h]);
      const f2 gh = cvt2(G[2 * h], G[2 * h + 1]) * sgq.inv_m;
      const f2 t1 = gh - rmg2[h];
      const f2 t2 = xh * rmgx2[h];
      const f2 dx = div_by2_nz(t1 - t2, sg2[h], rsc2[h]);
      const f2 xm = dx * so.m;
      ov_count2(xm, T1, T2, ovq1, ovq2);
      const f2 fl = qfloor2(so, xm, u[h]);
      c[2 * h] = in ? (int)fl.x : 0;  // outside the image: the conv's zero padding
      c[2 * h + 1] = in ? (int)fl.y : 0;
    }
    if (valid) *reinterpret_cast<int*>(sh.gq + pix * C + cq) = pack4(c);
    if (own) {
      st_out(B.gq + img + (uint32_t)((y * W + x) * C + cq), pack4(c));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s1[k] += c[k];
        s2[k] += c[k] * c[k];
      }
    }
  }
  pin_counts(ovq1, ovq2);
  WI::store(sh.w, wimg);
  __syncthreads();
  LBT_TSB(2);

  // phase-3 operands (addend, mask source, R / qn codes and both quantisers' noise per branch),
  // issued now: they land while the MFMAs run, and phase 1's registers are free
  float4 av[J], ymv[J], urg[NB][J], ung[NB][J];
  int Rv[NB][J], qnv[NB][J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int q3 = tid + j * kBThreads;
    const int pix = (q3 < NQ ? q3 : 0) / C4;  // (2-row tiles: the idle threads load the tile's first quad)
    const uint32_t off = (uint32_t)(row0 * W * C + pix * C + cq);  // tile rows are consecutive pixels
    av[j] = p.add_src ? ld4f(p.add_src, img + off) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (CF & kAYMask) ymv[j] = ld4f(A.y_mask, img + off);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const lbt_bwd_branch& Bb = b == 0 ? A.b1 : A.b2;
      Rv[b][j] = ld4i8(Bb.R, img + off);
      qnv[b][j] = ld4i8(Bb.qn_codes, img + off);
      urg[b][j] = ld4f(Bb.qrg.noise, off);
      ung[b][j] = ld4f(Bb.qng.noise, off);
    }
  }

  // ---------------- phase 2: dgrad from the LDS image, (m-tile, n-tile) pair wave + 8 pi
#pragma unroll
  for (int pi = 0; pi < (NPR + 7) / 8; ++pi) {
    const int pr = wave + 8 * pi;
    if (NPR % 8 && pr >= NPR) break;  // uniform per wave
    const int mt = pr / NT, nt = pr - mt * NT;
    const int m = mt * 16 + r;
    const int ly = m / W, px = m - ly * W;
    const int8_t* base = sh.gq + ((ly + 2) * Wp + px + 2) * C;
    v4i acc = v4i{0, 0, 0, 0};
    const int col = nt * 16 + r;
#pragma unroll
    for (int kk = 0; kk < kMaxKS; ++kk) {
      const int s = kk * 4 + kg;  // the k-slice this lane group supplies: (tap, 16-channel slice)
      const int tap = s / CS, cs = s - tap * CS;
      const int kh = tap / 3, kw = tap - kh * 3;
      v4i a = *reinterpret_cast<const v4i*>(base - (kh * Wp + kw) * C + cs * 16);
      if (s >= 9 * CS) a = v4i{0, 0, 0, 0};  // zero padding of the k dimension
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, WI::frag(sh.w, col, s), acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) sh.tile[(mt * 16 + 4 * kg + i) * (C + 4) + nt * 16 + r] = (float)acc[i] * scale;
  }
  __syncthreads();
  LBT_TSB(3);

  // ---------------- phase 3: pass A over the tile
  int ov[2][2][2] = {{{0, 0}, {0, 0}}, {{0, 0}, {0, 0}}};
  int acc3[NB][4][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc3[b][s][k] = 0;
  const bool has_add = p.add_src != nullptr;
  f2 gam2a[NB][2], bet2a[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int b = 0; b < NB; ++b) gam2a[b][h] = mk2(gam[b][2 * h], gam[b][2 * h + 1]);
    bet2a[h] = mk2(bet[2 * h], bet[2 * h + 1]);
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (NQ % kBThreads && tid + j * kBThreads >= NQ) break;  // uniform per wave
    const int pix = (tid + j * kBThreads) / C4;
    const uint32_t off = (uint32_t)(row0 * W * C + pix * C + cq);
    const float4 t = *reinterpret_cast<const float4*>(sh.tile + pix * (C + 4) + cq);
    f2 g[2] = {mk2(t.x, t.y), mk2(t.z, t.w)};
    if (has_add) {
      g[0] = g[0] + mk2(av[j].x, av[j].y);
      g[1] = g[1] + mk2(av[j].z, av[j].w);
    }
    int R1[4];
    unpack4(Rv[0][j], R1);
    if (CF & kAYMask) {
      const float ym[4] = {ymv[j].x, ymv[j].y, ymv[j].z, ymv[j].w};
#pragma unroll
      for (int h = 0; h < 2; ++h)
        g[h] = mk2(ym[2 * h] > 0.f ? g[h].x : 0.f, ym[2 * h + 1] > 0.f ? g[h].y : 0.f);
    } else if (CF & kAMaskR) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 xr = cvt2(R1[2 * h], R1[2 * h + 1]) * r_inv;
        const f2 m1 = xr * gam2a[0][h];
        const f2 yv = m1 + bet2a[h];
        g[h] = mk2(yv.x > 0.f ? g[h].x : 0.f, yv.y > 0.f ? g[h].y : 0.f);
      }
    }
    if (CF & kAGmask) st_out4(A.gmask_out, (uint32_t)(img + off), make_float4(g[0].x, g[0].y, g[1].x, g[1].y));
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const lbt_bwd_branch& Bb = b == 0 ? A.b1 : A.b2;
      int R[4], qn[4], Gc[4];
      unpack4(Rv[b][j], R);
      unpack4(qnv[b][j], qn);
      const f2 ur[2] = {mk2(urg[b][j].x, urg[b][j].y), mk2(urg[b][j].z, urg[b][j].w)};
      const f2 un[2] = {mk2(ung[b][j].x, ung[b][j].y), mk2(ung[b][j].z, ung[b][j].w)};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 xm = g[h] * qrg[b].m;
        ov_count2(xm, qrg[b].L, qrg[b].Lh, ov[b][0][0], ov[b][0][1]);
        const f2 f1 = qfloor2(qrg[b], xm, ur[h]);  // G2 codes
        const f2 gh = f1 * qrg[b].inv_m;
        const f2 d = gh * gam2a[b][h];
        const f2 dm = d * qng[b].m;
        ov_count2(dm, qng[b].L, qng[b].Lh, ov[b][1][0], ov[b][1][1]);
        const f2 f2c = qfloor2(qng[b], dm, un[h]);  // Gc codes
        const int G2[2] = {(int)f1.x, (int)f1.y};
        Gc[2 * h] = (int)f2c.x;
        Gc[2 * h + 1] = (int)f2c.y;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int k = 2 * h + i;
          acc3[b][0][k] += G2[i] * R[k];
          acc3[b][1][k] += G2[i];
          acc3[b][2][k] += Gc[k];
          acc3[b][3][k] += Gc[k] * qn[k];
        }
      }
      st_out(Bb.gout + img + off, pack4(Gc));
    }
  }

  // ---------------- channel sums: wave butterfly -> this wave's LDS slots (plain stores, no LDS
  // atomics); counters; one barrier; the waves' slots summed and flushed
  {
    // lanes l, l + C4, ... hold the same channels (C4 <= 16 divides 64); after chan_scatter4 the
    // lanes (lane & 15) < C4 of row lane >> 4 hold channel cq + (lane >> 4)
    const bool own = (lane & 15) < C4;
    int* part = sh.part[wave] + cq + (lane >> 4);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int t = chan_scatter4(acc3[b][s], C4);
        if (own) part[(b * 4 + s) * C] = t;
      }
    const int t1 = chan_scatter4(s1, C4), t2 = chan_scatter4(s2, C4);
    if (own) {
      part[8 * C] = t1;
      part[9 * C] = t2;
    }
  }
  // slots [qo | qrg, qng of branch 1 | qrg, qng of branch 2] (counts_publish sums the kBNW waves)
  ov_stage4(0, 5, ov_pack(ovq1, ovq2), ov_pack(ov[0][0][0], ov[0][0][1]), ov_pack(ov[0][1][0], ov[0][1][1]),
            NB == 2 ? ov_pack(ov[1][0][0], ov[1][0][1]) : 0, sh.cnt);
  if constexpr (NB == 2) {
    ov_wave(ov[1][1][0], ov[1][1][1]);
    counts_stage_w(4, 5, ov[1][1][0], ov[1][1][1], sh.cnt);
  }
  __syncthreads();
  LBT_TSB(4);
  counts_publish_nw<kBNW>(0, 5, B.qo, sh.cnt);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& Bb = b == 0 ? A.b1 : A.b2;
    counts_publish_nw<kBNW>(1 + 2 * b, 5, Bb.qrg, sh.cnt);
    counts_publish_nw<kBNW>(2 + 2 * b, 5, Bb.qng, sh.cnt);
  }
  // slot i of [NB*4C pass-A sums | 2C gq sums]: one thread each, the waves' partials in int64
  const int shard = shard_id();
  for (int i = tid; i < (NB * 4 + 2) * C; i += kBThreads) {
    const int slot = i < NB * 4 * C ? i : 8 * C + (i - NB * 4 * C);
    long long t = 0;
#pragma unroll
    for (int w = 0; w < kBNW; ++w) t += sh.part[w][slot];
    if (!t) continue;
    int64_t* dst;
    if (i < NB * 4 * C) {
      const int b = i / (4 * C);
      dst = (b == 0 ? A.b1 : A.b2).sums + (int64_t)shard * 4 * C + (i - b * 4 * C);
    } else {
      if (!B.gcolsum) continue;
      dst = B.gcolsum + (int64_t)shard * 2 * C + (i - NB * 4 * C);
    }
    LBT_GADD((unsigned long long*)dst, (unsigned long long)t);
  }
  LBT_TSB(5);
}

bool noise_ok(const lbt_qdesc& q) { return q.bits > 0 && q.stochastic && q.noise; }

}  // namespace

extern "C" int lbt_conv_bwd_fused_i8(const lbt_conv_bwd* q, void* stream) {
  if (!q) return LBT_EINVAL;
  const lbt_conv_desc& d = q->d;
  const int C = d.Cin;
  if (!desc_ok(d) || d.KH != 3 || d.KW != 3 || d.SH != 1 || d.SW != 1 || d.PT != 1 || d.PB != 1 || d.PL != 1 ||
      d.PR != 1 || d.Ho != d.H || d.Wo != d.W || d.Cout != C || (C != 16 && C != 32 && C != 64) ||
      d.H % tile_rows(C / 16) || d.W * C != 512 || (int64_t)d.N * d.H * 512 >= ((int64_t)1 << 29))
    return LBT_EINVAL;  // (st_out4's 32-bit byte offsets)
  const int CS = C / 16;
  const int64_t inner = (int64_t)d.H * d.W * C;
  const lbt_chain_bwd_b& b = q->b;
  if (!b.G || !b.qn_codes || !b.ms || !b.sums || !b.gq || b.dx || !noise_ok(b.qo) || b.C != C || b.rows != d.N ||
      b.inner != inner)
    return LBT_EINVAL;
  const lbt_chain_bwd_a& a = q->a;
  if (a.C != C || a.rows != d.N || a.inner != inner) return LBT_EINVAL;
  const int f = bwd_a_flags(a);
  if ((f & kAFused) != kAFused) return LBT_EINVAL;
  for (int br = 0; br < (a.has_b2 ? 2 : 1); ++br) {
    const lbt_bwd_branch& Bb = br ? a.b2 : a.b1;
    if (!noise_ok(Bb.qrg) || !noise_ok(Bb.qng) || !Bb.gb) return LBT_EINVAL;
  }
  if (q->ksd != 4 * ((9 * CS + 3) / 4) || !q->wd) return LBT_EINVAL;
  if (q->w4 && q->qw.bits > 4) return LBT_EINVAL;
  WgradArgs wa{};
  uint32_t wblocks = 0;
  int wcs = 0;
  if (q->w.slab) {
    const int e = wgrad_setup(q->w.xq, q->w.x_u8off, q->w.gq, q->w.d, q->w.slab, q->w.nsplit, q->w.nshard, wa, wblocks);
    if (e) return e;
    wcs = q->w.d.Cin / 16;
  }
  ConvBwdArgs p;
  p.b = b; p.wd = q->wd; p.ks = q->ksd; p.nslices = 9 * CS; p.w4 = q->w4; p.qw = q->qw;
  p.H = d.H; p.W = d.W; p.add_src = q->add_src; p.a = a;
  const int th = tile_rows_for(CS, d.N, d.H);
  const int64_t tiles = (int64_t)d.N * (d.H / th);
  if (tiles + wblocks > 0x7fffffff) return LBT_EINVAL;
  const dim3 grid((unsigned)(tiles + wblocks));
  hipStream_t st = (hipStream_t)stream;
  const int nb = a.has_b2 ? 2 : 1;
  // the combinations the fused ResNet plan runs (c2: mask from R1, deferred wgrad of the next
  // block's c1 or none; c1: its consumer's chain, deferred wgrad of the same block's c2)
#define LBT_BW_TH(CS_, CF_, NB_, WCS_, TH_)                                                                 \
  if (q->w4)                                                                                                \
    hipLaunchKernelGGL((conv_bwd_kernel<CS_, CF_, NB_, true, WCS_, TH_>), grid, dim3(kBThreads), 0, st, p, wa, wblocks); \
  else                                                                                                      \
    hipLaunchKernelGGL((conv_bwd_kernel<CS_, CF_, NB_, false, WCS_, TH_>), grid, dim3(kBThreads), 0, st, p, wa, wblocks);
#define LBT_BW(CS_, CF_, NB_, WCS_)                                                                  \
  if (CS == CS_ && f == (CF_) && nb == NB_ && wcs == WCS_) {                                       \
    if (CS_ == 1 && th == 4) {                                                                     \
      LBT_BW_TH(CS_, CF_, NB_, WCS_, (CS_ == 1 ? 4 : tile_rows(CS_)))                              \
    } else if (th == 2) {                                                                          \
      LBT_BW_TH(CS_, CF_, NB_, WCS_, 2)                                                            \
    } else {                                                                                       \
      LBT_BW_TH(CS_, CF_, NB_, WCS_, tile_rows(CS_))                                               \
    }                                                                                              \
    return (int)hipGetLastError();                                                                 \
  }
  // (WCS = 0 everywhere: the plan's LBT_SIDE_WGRAD mode runs each wgrad as a parallel branch)
#define LBT_BW_CS(CS_)                                          \
  LBT_BW(CS_, kAFused | kAMaskR, 1, 0)                          \
  LBT_BW(CS_, kAFused | kAMaskR, 1, CS_)                        \
  LBT_BW(CS_, kAFused | kAYMask | kAGmask, 1, 0)                \
  LBT_BW(CS_, kAFused | kAYMask | kAGmask, 1, CS_)              \
  LBT_BW(CS_, kAFused | kAYMask, 2, 0)                          \
  LBT_BW(CS_, kAFused | kAYMask, 2, CS_)
  LBT_BW_CS(1)
  LBT_BW_CS(2)
  LBT_BW_CS(4)
  LBT_BW(1, kAFused | kAYMask, 1, 0)
  LBT_BW(1, kAFused | kAYMask, 1, 1)
  // a stage's last c2 carrying the wgrad of the next stage's c2 (across the projection block)
  LBT_BW(1, kAFused | kAMaskR, 1, 2)
  LBT_BW(2, kAFused | kAMaskR, 1, 4)
#undef LBT_BW_CS
#undef LBT_BW
#undef LBT_BW_TH
  return LBT_EINVAL;
}

// ============================================================================ fused transition backward
// lbt_conv_bwd2_fused_i8: a projection block's first-conv / shortcut backward (the stage transition)
// in ONE launch -- what lbt_bn_chain_bwd_b_pair + lbt_conv_dgrad2_chain_i8 computed in two:
//   phase 1  pass B of BOTH BNs after the strided convs (conv-1's bn1 and the shortcut BN, at the
//            low resolution Hq x Wq x Cq, Cq = 2C) over the low-res rows the workgroup's dx rows read
//            (plus the one-row halo above that the 3x3/2 conv's SAME padding (top 0, bottom 1)
//            reaches) -> int8 gradient-code images in LDS; owned rows store gq (the weight
//            gradients' operands), count overflows and add the gq channel sums
//   phase 2  dx = dgrad(3x3/2, gq1) + dgrad(1x1/2, gqs) from LDS: each lane's dx pixel takes the
//            taps of its parity (the stride's zero rows read as 0), the two GEMMs in their own
//            accumulators, summed in fp32 in the order the dual dgrad launch used
//   phase 3  pass A of the BN that consumes dx (conv_bwd_kernel's phase 3)
namespace {

struct ConvBwd2Args {
  lbt_chain_bwd_b b1, bs;
  const int8_t* wd1;
  const int8_t* wds;
  lbt_qdesc qw1, qws;
  int H;  // dx rows
  lbt_chain_bwd_a a;
};

template <int C, int TH>
struct Bwd2Shared {
  int8_t g1[(TH / 2 + 1) * 512];   // conv-1's gradient codes, low-res rows q0-1 .. q0+TH/2-1 ([row][Wq][Cq])
  int8_t gs[(TH / 2) * 512];       // the shortcut's, rows q0 .. q0+TH/2-1
  float tile[TH * (512 / C) * (C + 4)];
  float cst[2][5][2 * C];          // per BN (conv-1's, shortcut's): mu, sigma, sigma's rcp refinement, mg, mgx
  int part[kBNW][(2 * 4 + 8) * C]; // per wave: pass-A sums (<= 2 branches x 4C), gq sums (2 x 2Cq)
  int cnt[kBNW * 2 * 6];           // counters: qo1, qos, qrg / qng per branch
};

template <int CS, int CF, int NB, bool W4>
__global__ __launch_bounds__(kBThreads, CS == 1 ? 4 : 2) void conv_bwd2_kernel(ConvBwd2Args p) {
  constexpr int C = CS * 16, C4 = C / 4, Cq = 2 * C, Cq4 = Cq / 4, CSq = 2 * CS, NT = CS;
  constexpr int W = 512 / C, Wq = W / 2;  // W * C == Wq * Cq == 512 (host check)
  constexpr int TH = tile_rows(CS), J = TH / 4;
  constexpr int kK1 = (9 * CSq + 3) / 4;  // k-steps of the 3x3/2 dgrad
  constexpr int NG1 = (TH / 2 + 1) * Wq * Cq4, NGS = (TH / 2) * Wq * Cq4;
  constexpr int kIt = (NG1 + NGS + kBThreads - 1) / kBThreads;
  static_assert(NG1 % 64 == 0 && CSq <= 4 && LBT_NSHARD == 32 && 2 * Cq / 16 <= kBNW, "layout");
  __shared__ __attribute__((aligned(16))) Bwd2Shared<C, TH> sh;
  LBT_TS(0);
  const lbt_chain_bwd_a& A = p.a;
  const uint32_t bid = blockIdx.x;
  const int H = p.H, Hq = H / 2;
  const int tpi = H / TH;
  const int n = (int)(bid / (uint32_t)tpi), r0 = (int)(bid - (uint32_t)n * tpi) * TH, q0 = r0 / 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int cq = (tid % C4) * 4;     // dx channel quad (phase 3)
  const int cqq = (tid % Cq4) * 4;   // low-res channel quad (phase 1)
  const int64_t img = (int64_t)n * H * W * C, imgq = (int64_t)n * Hq * Wq * Cq;

  // ---------------- both BNs' pass-B statistics shard sums first (they gate the first barrier):
  // wave w < 2 * CSq owns 16 channels of BN w / CSq; lane l reads shards 8 (l >> 4) .. + 7
  constexpr int kSW = 2 * CSq;
  long long sv[8][2];
  if (wave < kSW) {
    const lbt_chain_bwd_b& Bb = wave < CSq ? p.b1 : p.bs;
    const int c = (wave % CSq) * 16 + (lane & 15);
    const int64_t* ps = Bb.sums + (int64_t)(8 * (lane >> 4)) * 4 * Cq + c;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sv[i][0] = ps[(int64_t)i * 4 * Cq + 2 * Cq];
      sv[i][1] = ps[(int64_t)i * 4 * Cq + 3 * Cq];
    }
  }
  // phase-1 operands: G / q codes and the output quantiser's noise of the low-res groups (region 1:
  // conv-1's BN over rows q0-1 .. q0+TH/2-1; region 2: the shortcut BN over rows q0 .. q0+TH/2-1)
  int Gv[kIt], Qv[kIt];
  float4 Uv[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int g = tid + it * kBThreads;
    const bool r1 = g < NG1;  // wave-uniform (NG1 % 64 == 0)
    const int gg = r1 ? g : g - NG1;
    const int pix = gg / Cq4, hy = pix / Wq, x = pix - hy * Wq;
    const int y = r1 ? q0 - 1 + hy : q0 + hy;
    const bool in = (r1 || gg < NGS) && (unsigned)y < (unsigned)Hq;
    const uint32_t off = in ? (uint32_t)((y * Wq + x) * Cq + cqq) : 0u;
    const lbt_chain_bwd_b& Bb = r1 ? p.b1 : p.bs;
    Gv[it] = ld4i8(Bb.G, imgq + off);
    Qv[it] = ld4i8(Bb.qn_codes, imgq + off);
    Uv[it] = ld4f(Bb.qo.noise, off);
  }
  // phase-2 B operands of this wave's n-tile (NT | 8): the 3x3/2 dgrad image and the 1x1/2 one
  v4i bf1[kK1], bfs;
  {
    const int col = (wave % NT) * 16 + r;
#pragma unroll
    for (int kk = 0; kk < kK1; ++kk) {
      if constexpr (W4)
        bf1[kk] = unpack_i4x16(*reinterpret_cast<const v2i*>(p.wd1 + ((int64_t)col * (4 * kK1) + kk * 4 + kg) * 8));
      else
        bf1[kk] = *reinterpret_cast<const v4i*>(p.wd1 + ((int64_t)col * (4 * kK1) + kk * 4 + kg) * 16);
    }
    if constexpr (W4)
      bfs = unpack_i4x16(*reinterpret_cast<const v2i*>(p.wds + ((int64_t)col * 4 + kg) * 8));
    else
      bfs = *reinterpret_cast<const v4i*>(p.wds + ((int64_t)col * 4 + kg) * 16);
  }
  float gam[NB][4], bet[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int b = 0; b < NB; ++b) gam[b][k] = (b == 0 ? A.b1 : A.b2).gb[cq + k];
    bet[k] = A.b1.gb[C + cq + k];
  }
  const QState so1 = qstate(p.b1.qo), sos = qstate(p.bs.qo);
  QState qrg[2], qng[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    qrg[b] = qstate((b == 0 ? A.b1 : A.b2).qrg);
    qng[b] = qstate((b == 0 ? A.b1 : A.b2).qng);
  }
  const float r_inv = (CF & kAMaskR) ? qstate(A.b1.qr).inv_m : 0.f;
  const float scale1 = ldexpf(1.0f, -(frac_exp(p.b1.qo) + frac_exp(p.qw1)));
  const float scale2 = ldexpf(1.0f, -(frac_exp(p.bs.qo) + frac_exp(p.qws)));

  // ---------------- pass-B constants of both BNs (chain_bwd_b_kernel's double arithmetic)
  if (wave < kSW) {
    long long SGi = 0, SGQi = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      SGi += sv[i][0];
      SGQi += sv[i][1];
    }
    SGi = rows_total64(SGi);
    SGQi = rows_total64(SGQi);
    const int bn = wave < CSq ? 0 : 1, c = (wave % CSq) * 16 + (lane & 15);
    if (lane < 16) {
      const lbt_chain_bwd_b& Bb = bn == 0 ? p.b1 : p.bs;
      const double s = (double)qstate(Bb.qn).inv_m, gsc = (double)qstate(Bb.qng).inv_m, nn = (double)Bb.n;
      const double SG = (double)SGi, SGQ = (double)SGQi;
      const float m = Bb.ms[c], sig = Bb.ms[Cq + c];
      const Recip rc = recip(sig);
      sh.cst[bn][0][c] = m;
      sh.cst[bn][1][c] = sig;
      sh.cst[bn][2][c] = rc.rc;
      sh.cst[bn][3][c] = (float)(gsc * SG / nn);
      sh.cst[bn][4][c] = (float)(gsc * (s * SGQ - (double)m * SG) / (nn * (double)sig));
    }
  }
  const QState sn1 = qstate(p.b1.qn), sns = qstate(p.bs.qn), sg1 = qstate(p.b1.qng), sgs = qstate(p.bs.qng);
  __syncthreads();
  LBT_TS(1);

  // ---------------- phase 1: both pass-B chains -> LDS gradient-code images
  int ov1a = 0, ov2a = 0, ov1b = 0, ov2b = 0;
  int s1a[4] = {0, 0, 0, 0}, s2a[4] = {0, 0, 0, 0}, s1b[4] = {0, 0, 0, 0}, s2b[4] = {0, 0, 0, 0};
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    if (it * kBThreads >= NG1 + NGS) break;  // uniform
    const int g = tid + it * kBThreads;
    const bool r1 = g < NG1;  // wave-uniform
    const int gg = r1 ? g : g - NG1;
    const bool valid = r1 || gg < NGS;
    const int pix = gg / Cq4, hy = pix / Wq, x = pix - hy * Wq;
    const int y = r1 ? q0 - 1 + hy : q0 + hy;
    const bool in = valid && (unsigned)y < (unsigned)Hq;
    const bool own = in && (!r1 || hy >= 1);
    const int bn = r1 ? 0 : 1;
    const QState& so = r1 ? so1 : sos;
    const QState& sn = r1 ? sn1 : sns;
    const QState& sgq = r1 ? sg1 : sgs;
    const float4 mu4 = *reinterpret_cast<const float4*>(&sh.cst[bn][0][cqq]);
    const float4 sg4 = *reinterpret_cast<const float4*>(&sh.cst[bn][1][cqq]);
    const float4 rc4 = *reinterpret_cast<const float4*>(&sh.cst[bn][2][cqq]);
    const float4 mg4 = *reinterpret_cast<const float4*>(&sh.cst[bn][3][cqq]);
    const float4 mx4 = *reinterpret_cast<const float4*>(&sh.cst[bn][4][cqq]);
    const f2 mu2[2] = {mk2(mu4.x, mu4.y), mk2(mu4.z, mu4.w)}, sg2[2] = {mk2(sg4.x, sg4.y), mk2(sg4.z, sg4.w)};
    const f2 rc2[2] = {mk2(rc4.x, rc4.y), mk2(rc4.z, rc4.w)}, mg2[2] = {mk2(mg4.x, mg4.y), mk2(mg4.z, mg4.w)};
    const f2 mx2[2] = {mk2(mx4.x, mx4.y), mk2(mx4.z, mx4.w)};
    const float T1 = ov_thr(own, so.L), T2 = ov_thr(own, so.Lh);
    int G[4], q[4], c[4];
    unpack4(Gv[it], G);
    unpack4(Qv[it], q);
    const f2 u[2] = {mk2(Uv[it].x, Uv[it].y), mk2(Uv[it].z, Uv[it].w)};
    int o1 = 0, o2 = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f2 x1 = cvt2(q[2 * h], q[2 * h + 1]) * sn.inv_m;
      const f2 x2 = x1 - mu2[h];
      const f2 xh = div_by2_nz(x2, sg2[h], rc2[h]);
      const f2 gh = cvt2(G[2 * h], G[2 * h + 1]) * sgq.inv_m;
      const f2 t1 = gh - mg2[h];
      const f2 t2 = xh * mx2[h];
      const f2 dx = div_by2_nz(t1 - t2, sg2[h], rc2[h]);
      const f2 xm = dx * so.m;
      ov_count2(xm, T1, T2, o1, o2);
      const f2 fl = qfloor2(so, xm, u[h]);
      c[2 * h] = in ? (int)fl.x : 0;  // outside the image: the conv's zero padding
      c[2 * h + 1] = in ? (int)fl.y : 0;
    }
    const int w = pack4(c);
    if (r1) {
      ov1a += o1;
      ov2a += o2;
      *reinterpret_cast<int*>(sh.g1 + pix * Cq + cqq) = w;
      if (own) {
        st_out(p.b1.gq + imgq + (uint32_t)((y * Wq + x) * Cq + cqq), w);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s1a[k] += c[k];
          s2a[k] += c[k] * c[k];
        }
      }
    } else {
      ov1b += o1;
      ov2b += o2;
      if (valid) *reinterpret_cast<int*>(sh.gs + pix * Cq + cqq) = w;
      if (own) {
        st_out(p.bs.gq + imgq + (uint32_t)((y * Wq + x) * Cq + cqq), w);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s1b[k] += c[k];
          s2b[k] += c[k] * c[k];
        }
      }
    }
  }
  pin_counts(ov1a, ov2a);
  pin_counts(ov1b, ov2b);
  __syncthreads();
  LBT_TS(2);

  // phase-3 operands, issued now (they land while the MFMAs run)
  float4 ymv[J], urg[NB][J], ung[NB][J];
  int Rv[NB][J], qnv[NB][J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int pix = (tid + j * kBThreads) / C4;
    const uint32_t off = (uint32_t)(r0 * W * C + pix * C + cq);
    if (CF & kAYMask) ymv[j] = ld4f(A.y_mask, img + off);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const lbt_bwd_branch& Bb = b == 0 ? A.b1 : A.b2;
      Rv[b][j] = ld4i8(Bb.R, img + off);
      qnv[b][j] = ld4i8(Bb.qn_codes, img + off);
      urg[b][j] = ld4f(Bb.qrg.noise, off);
      ung[b][j] = ld4f(Bb.qng.noise, off);
    }
  }

  // ---------------- phase 2: dx = dgrad(3x3/2) + dgrad(1x1/2) from the LDS images
#pragma unroll
  for (int pi = 0; pi < TH / 4; ++pi) {
    const int pr = wave + 8 * pi;
    const int mt = pr / NT, nt = pr - mt * NT;
    const int m = mt * 16 + r;
    const int ly = m / W, px = m - ly * W;
    v4i acc = v4i{0, 0, 0, 0}, acc2 = v4i{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < kK1; ++kk) {
      const int s = kk * 4 + kg;  // (tap, 16-channel slice of Cq)
      const int tap = s / CSq, cs = s - tap * CSq;
      const int kh = tap / 3, kw = tap - kh * 3;
      // dx row r0 + ly reads gq row (r0 + ly - kh) / 2 = local row (ly - kh) / 2 + 1 when even
      const bool ok = s < 9 * CSq && ((ly - kh) & 1) == 0 && ((px - kw) & 1) == 0 && px >= kw;
      const int lr = ((ly - kh) >> 1) + 1, ox = (px - kw) >> 1;
      v4i a = *reinterpret_cast<const v4i*>(sh.g1 + (ok ? (lr * Wq + ox) * Cq + cs * 16 : 0));
      if (!ok) a = v4i{0, 0, 0, 0};
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bf1[kk], acc, 0, 0, 0);
    }
    {
      const bool ok = kg < CSq && (ly & 1) == 0 && (px & 1) == 0;
      v4i a = *reinterpret_cast<const v4i*>(sh.gs + (ok ? ((ly >> 1) * Wq + (px >> 1)) * Cq + kg * 16 : 0));
      if (!ok) a = v4i{0, 0, 0, 0};
      acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bfs, acc2, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = (float)acc[i] * scale1, add = (float)acc2[i] * scale2;
      sh.tile[(mt * 16 + 4 * kg + i) * (C + 4) + nt * 16 + r] = v + add;
    }
  }
  __syncthreads();
  LBT_TS(3);

  // ---------------- phase 3: pass A over the tile (conv_bwd_kernel's phase 3)
  int ov[2][2][2] = {{{0, 0}, {0, 0}}, {{0, 0}, {0, 0}}};
  int acc3[NB][4][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc3[b][s][k] = 0;
  f2 gam2a[NB][2], bet2a[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int b = 0; b < NB; ++b) gam2a[b][h] = mk2(gam[b][2 * h], gam[b][2 * h + 1]);
    bet2a[h] = mk2(bet[2 * h], bet[2 * h + 1]);
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int pix = (tid + j * kBThreads) / C4;
    const uint32_t off = (uint32_t)(r0 * W * C + pix * C + cq);
    const float4 t = *reinterpret_cast<const float4*>(sh.tile + pix * (C + 4) + cq);
    f2 g[2] = {mk2(t.x, t.y), mk2(t.z, t.w)};
    int R1[4];
    unpack4(Rv[0][j], R1);
    if (CF & kAYMask) {
      const float ym[4] = {ymv[j].x, ymv[j].y, ymv[j].z, ymv[j].w};
#pragma unroll
      for (int h = 0; h < 2; ++h)
        g[h] = mk2(ym[2 * h] > 0.f ? g[h].x : 0.f, ym[2 * h + 1] > 0.f ? g[h].y : 0.f);
    } else if (CF & kAMaskR) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 xr = cvt2(R1[2 * h], R1[2 * h + 1]) * r_inv;
        const f2 m1 = xr * gam2a[0][h];
        const f2 yv = m1 + bet2a[h];
        g[h] = mk2(yv.x > 0.f ? g[h].x : 0.f, yv.y > 0.f ? g[h].y : 0.f);
      }
    }
    if (CF & kAGmask) st_out4(A.gmask_out, (uint32_t)(img + off), make_float4(g[0].x, g[0].y, g[1].x, g[1].y));
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const lbt_bwd_branch& Bb = b == 0 ? A.b1 : A.b2;
      int R[4], qn[4], Gc[4];
      unpack4(Rv[b][j], R);
      unpack4(qnv[b][j], qn);
      const f2 ur[2] = {mk2(urg[b][j].x, urg[b][j].y), mk2(urg[b][j].z, urg[b][j].w)};
      const f2 un[2] = {mk2(ung[b][j].x, ung[b][j].y), mk2(ung[b][j].z, ung[b][j].w)};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 xm = g[h] * qrg[b].m;
        ov_count2(xm, qrg[b].L, qrg[b].Lh, ov[b][0][0], ov[b][0][1]);
        const f2 f1 = qfloor2(qrg[b], xm, ur[h]);  // G2 codes
        const f2 gh = f1 * qrg[b].inv_m;
        const f2 d = gh * gam2a[b][h];
        const f2 dm = d * qng[b].m;
        ov_count2(dm, qng[b].L, qng[b].Lh, ov[b][1][0], ov[b][1][1]);
        const f2 f2c = qfloor2(qng[b], dm, un[h]);  // Gc codes
        const int G2[2] = {(int)f1.x, (int)f1.y};
        Gc[2 * h] = (int)f2c.x;
        Gc[2 * h + 1] = (int)f2c.y;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int k = 2 * h + i;
          acc3[b][0][k] += G2[i] * R[k];
          acc3[b][1][k] += G2[i];
          acc3[b][2][k] += Gc[k];
          acc3[b][3][k] += Gc[k] * qn[k];
        }
      }
      st_out(Bb.gout + img + off, pack4(Gc));
    }
  }

  // ---------------- channel sums and counters (conv_bwd_kernel's publish, plus a second gq sum set)
  {
    const bool own = (lane & 15) < C4;
    int* part = sh.part[wave] + cq + (lane >> 4);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int t = chan_scatter4(acc3[b][s], C4);
        if (own) part[(b * 4 + s) * C] = t;
      }
    const bool ownq = (lane & 15) < Cq4;
    int* pq = sh.part[wave] + NB * 4 * C + cqq + (lane >> 4);
    const int t1 = chan_scatter4(s1a, Cq4), t2 = chan_scatter4(s2a, Cq4);
    const int t3 = chan_scatter4(s1b, Cq4), t4 = chan_scatter4(s2b, Cq4);
    if (ownq) {
      pq[0] = t1;
      pq[Cq] = t2;
      pq[2 * Cq] = t3;
      pq[3 * Cq] = t4;
    }
  }
  constexpr int NQ = 2 + 2 * NB;  // [qo1 | qos | qrg, qng of branch 1 | of branch 2]
  ov_stage4(0, NQ, ov_pack(ov1a, ov2a), ov_pack(ov1b, ov2b), ov_pack(ov[0][0][0], ov[0][0][1]),
            ov_pack(ov[0][1][0], ov[0][1][1]), sh.cnt);
  if constexpr (NB == 2) {
    ov_wave(ov[1][0][0], ov[1][0][1]);
    counts_stage_w(4, NQ, ov[1][0][0], ov[1][0][1], sh.cnt);
    ov_wave(ov[1][1][0], ov[1][1][1]);
    counts_stage_w(5, NQ, ov[1][1][0], ov[1][1][1], sh.cnt);
  }
  __syncthreads();
  LBT_TS(4);
  counts_publish_nw<kBNW>(0, NQ, p.b1.qo, sh.cnt);
  counts_publish_nw<kBNW>(1, NQ, p.bs.qo, sh.cnt);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& Bb = b == 0 ? A.b1 : A.b2;
    counts_publish_nw<kBNW>(2 + 2 * b, NQ, Bb.qrg, sh.cnt);
    counts_publish_nw<kBNW>(3 + 2 * b, NQ, Bb.qng, sh.cnt);
  }
  // slot i of [NB*4C pass-A sums | 2Cq conv-1 gq sums | 2Cq shortcut gq sums]
  const int shard = shard_id();
  for (int i = tid; i < NB * 4 * C + 4 * Cq; i += kBThreads) {
    long long t = 0;
#pragma unroll
    for (int w = 0; w < kBNW; ++w) t += sh.part[w][i];
    if (!t) continue;
    int64_t* dst;
    if (i < NB * 4 * C) {
      const int b = i / (4 * C);
      dst = (b == 0 ? A.b1 : A.b2).sums + (int64_t)shard * 4 * C + (i - b * 4 * C);
    } else {
      const int k = i - NB * 4 * C;
      const lbt_chain_bwd_b& Bb = k < 2 * Cq ? p.b1 : p.bs;
      if (!Bb.gcolsum) continue;
      dst = Bb.gcolsum + (int64_t)shard * 2 * Cq + (k < 2 * Cq ? k : k - 2 * Cq);
    }
    LBT_GADD((unsigned long long*)dst, (unsigned long long)t);
  }
  LBT_TS(5);
}

}  // namespace

extern "C" int lbt_conv_bwd2_fused_i8(const lbt_conv_bwd2* q, void* stream) {
  if (!q) return LBT_EINVAL;
  const lbt_conv_desc &d1 = q->d1, &ds = q->ds;
  const int C = d1.Cin, Cq = d1.Cout;
  // the projection block's 3x3/2 SAME conv (pads: top / left 0, bottom / right 1) and 1x1/2 shortcut
  if (!desc_ok(d1) || !desc_ok(ds) || d1.KH != 3 || d1.KW != 3 || d1.SH != 2 || d1.SW != 2 || d1.PT != 0 ||
      d1.PL != 0 || ds.KH != 1 || ds.KW != 1 || ds.SH != 2 || ds.SW != 2 || ds.PT != 0 || ds.PL != 0 ||
      (C != 16 && C != 32) || Cq != 2 * C || d1.W * C != 512 || d1.H % 2 || d1.W % 2 || d1.Ho * 2 != d1.H ||
      d1.Wo * 2 != d1.W || d1.H % tile_rows(C / 16) || ds.N != d1.N || ds.H != d1.H || ds.W != d1.W || ds.Cin != C ||
      ds.Cout != Cq || ds.Ho != d1.Ho || ds.Wo != d1.Wo || (int64_t)d1.N * d1.H * 512 >= ((int64_t)1 << 29))
    return LBT_EINVAL;
  const int CS = C / 16;
  const int64_t inq = (int64_t)d1.Ho * d1.Wo * Cq;
  const lbt_chain_bwd_b* bb[2] = {&q->b1, &q->bs};
  for (int i = 0; i < 2; ++i) {
    const lbt_chain_bwd_b& b = *bb[i];
    if (!b.G || !b.qn_codes || !b.ms || !b.sums || !b.gq || b.dx || !noise_ok(b.qo) || b.C != Cq || b.rows != d1.N ||
        b.inner != inq)
      return LBT_EINVAL;
  }
  const lbt_chain_bwd_a& a = q->a;
  if (a.C != C || a.rows != d1.N || a.inner != (int64_t)d1.H * d1.W * C) return LBT_EINVAL;
  const int f = bwd_a_flags(a);
  if ((f & kAFused) != kAFused) return LBT_EINVAL;
  for (int br = 0; br < (a.has_b2 ? 2 : 1); ++br) {
    const lbt_bwd_branch& Bb = br ? a.b2 : a.b1;
    if (!noise_ok(Bb.qrg) || !noise_ok(Bb.qng) || !Bb.gb) return LBT_EINVAL;
  }
  if (q->ksd1 != 4 * ((9 * 2 * CS + 3) / 4) || q->ksds != 4 || !q->wd1 || !q->wds) return LBT_EINVAL;
  if (q->w4 && (q->qw1.bits > 4 || q->qws.bits > 4)) return LBT_EINVAL;
  ConvBwd2Args p;
  p.b1 = q->b1; p.bs = q->bs; p.wd1 = q->wd1; p.wds = q->wds; p.qw1 = q->qw1; p.qws = q->qws; p.H = d1.H; p.a = a;
  const int64_t tiles = (int64_t)d1.N * (d1.H / tile_rows(CS));
  if (tiles > 0x7fffffff || (int64_t)d1.N * d1.H * d1.W * C >= ((int64_t)1 << 31)) return LBT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int nb = a.has_b2 ? 2 : 1;
#define LBT_B2(CS_, CF_, NB_)                                                                              \
  if (CS == CS_ && f == (CF_) && nb == NB_) {                                                              \
    if (q->w4)                                                                                             \
      hipLaunchKernelGGL((conv_bwd2_kernel<CS_, CF_, NB_, true>), dim3((unsigned)tiles), dim3(kBThreads), 0, st, p); \
    else                                                                                                   \
      hipLaunchKernelGGL((conv_bwd2_kernel<CS_, CF_, NB_, false>), dim3((unsigned)tiles), dim3(kBThreads), 0, st, p); \
    return (int)hipGetLastError();                                                                         \
  }
  // the consumer is an identity block's end chain (mask from y, masked gradient stored) or the
  // stem's (y mask only)
  LBT_B2(1, kAFused | kAYMask | kAGmask, 1)
  LBT_B2(2, kAFused | kAYMask | kAGmask, 1)
  LBT_B2(1, kAFused | kAYMask, 1)
  LBT_B2(2, kAFused | kAYMask, 1)
#undef LBT_B2
  return LBT_EINVAL;
}

// ============================================================================ fused conv forward
// lbt_conv_fwd_fused_i8: the BN element chain that produces a stride-1 3x3 conv's input (bn.hip
// chain_fwd_kernel's arithmetic) runs as the conv's operand staging. A workgroup owns TH image
// rows: phase 1 evaluates the chain over the rows plus a one-pixel halo into an LDS image of the
// conv's input codes (owned pixels also store R codes / y / X codes and count overflows), phase 2
// runs the MFMAs from LDS into an fp32 LDS tile, phase 3 quantises the tile for the next BN (one
// channel quad per thread) and adds its channel sums.
namespace {

struct ConvFwdArgs {
  lbt_chain_fwd c;
  const int8_t* wf;
  const int32_t* wcolsum;
  lbt_qdesc qw;
  int H;
  int8_t* yq;
  lbt_qdesc qout;
  int64_t* ychsum;
};

template <int C, int TH, int WB>
struct FwdShared {
  int8_t w[WB];                               // the forward weight image (WImg)
  int8_t x[(TH + 2) * (512 / C + 2) * C];   // the conv's input codes, halo image (q - 128)
  float tile[TH * (512 / C) * (C + 4)];      // conv outputs [TH*W][C+4]
  float cst[2][2][C];                          // per branch: mu, sigma
  int part[kBNW][2 * C];                       // per wave: S1, S2 of the output codes
  int cnt[kBNW * 2 * 4];                       // counters: R (2 branches), X, output
};

template <int CS, int NB, int F, bool W4, int TH = tile_rows(CS)>
__global__ __launch_bounds__(kBThreads, (CS == 4 && TH >= 4) ? 2 : 4) void conv_fwd_fused_kernel(ConvFwdArgs p) {
  constexpr int C = CS * 16, C4 = C / 4, NT = CS, W = 512 / C, Wp = W + 2;
  constexpr int kMaxKS = (9 * CS + 3) / 4;
  // (as conv_bwd_kernel: NQ channel quads and NPR MFMA pairs per tile; 2-row tiles idle half of each)
  constexpr int kBIt = halo_iters(CS, TH), NQ = TH * 128, J = (NQ + kBThreads - 1) / kBThreads, NPR = 2 * TH;
  static_assert(TH % 4 == 0 || TH == 2, "whole groups of 4 rows, or 2-row tiles");
  using WI = WImg<C, 4 * kMaxKS, W4>;
  __shared__ __attribute__((aligned(16))) FwdShared<C, TH, WI::kBytes> sh;
  LBT_TS(0);
  const lbt_chain_fwd& a = p.c;
  const int H = p.H;
  const uint32_t bid = blockIdx.x;
  const int tpi = H / TH;
  const int n = (int)(bid / (uint32_t)tpi), row0 = (int)(bid - (uint32_t)n * tpi) * TH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int cq = (tid % C4) * 4;
  const int64_t img = (int64_t)n * H * W * C;
  constexpr bool RES = (F & kFRes) != 0, YST = (F & kFY) != 0;

  // ---------------- the moments' shard sums first (they gate the first barrier), then the loads that
  // do not depend on the moments
  // waves w < NB*C/16 each own 16 (branch, channel) pairs: lane l reads pair w*16 + (l & 15) of
  // shards 8*(l >> 4) .. +7 (each load instruction: 4 shards x 16 consecutive channels)
  static_assert(LBT_NSHARD == 32 && kBThreads == 512 && (NB * C) % 16 == 0 && NB * C / 16 <= kBNW,
                "moments layout");
  constexpr int kSW = NB * C / 16;  // statistics waves
  long long sv[8][2];
  if (wave < kSW) {  // uniform per wave
    const int bc = wave * 16 + (lane & 15), b = bc / C, c = bc - b * C;
    const int64_t* cs = (b == 0 ? a.b1 : a.b2).nrm.chsum + (int64_t)(8 * (lane >> 4)) * 2 * C + c;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sv[i][0] = cs[(int64_t)i * 2 * C];
      sv[i][1] = cs[(int64_t)i * 2 * C + C];
    }
  }
  const int ngrp = (TH + 2) * Wp * C4;
  int qv[NB][kBIt];
  float4 rv[kBIt], nrv[NB][kBIt], nov[kBIt];
#pragma unroll
  for (int it = 0; it < kBIt; ++it) {
    const int g = tid + it * kBThreads;
    const int pix = g / C4, hy = pix / Wp, hx = pix - hy * Wp;
    const int y = row0 - 1 + hy, x = hx - 1;
    const bool in = g < ngrp && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    const uint32_t off = in ? (uint32_t)((y * W + x) * C + cq) : 0u;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const lbt_chain_branch& Bb = b == 0 ? a.b1 : a.b2;
      qv[b][it] = ld4i8(Bb.nrm.q, img + off);
      nrv[b][it] = ld4f(Bb.qr.noise, off);
    }
    if constexpr (RES) rv[it] = ld4f(a.res, img + off);
    nov[it] = ld4f(a.qo1.noise, off);
  }
  // the B operands (the forward weight image, for LDS: WImg): loaded in this first load wave, stored
  // to LDS at the end of phase 1
  v4i wimg[WI::kIt];
  WI::load(p.wf, wimg);
  const int bcol = (wave % NT) * 16 + r;
  const int corr = 128 * p.wcolsum[bcol];  // the unsigned-9-bit offset encoding undone: + 128 * sum_k W[k][col]
  float gam[NB][4], bet[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      gam[b][k] = (b == 0 ? a.b1 : a.b2).gb[cq + k];
      bet[b][k] = (b == 0 ? a.b1 : a.b2).gb[C + cq + k];
    }
  QState qr[2];
  float sn[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    qr[b] = qstate((b == 0 ? a.b1 : a.b2).qr);
    sn[b] = qscale((b == 0 ? a.b1 : a.b2).nrm.qn);
  }
  const QState so1 = qstate(a.qo1), sq = qstate(p.qout);
  const float scale = ldexpf(1.0f, -(frac_exp(a.qo1) + frac_exp(p.qw)));

  // ---------------- Normalization_q moments (bn.hip bn_moments) from the shard sums loaded above: each
  // statistics wave adds its 8 shards per lane, then its four lane rows; lanes < 16 finish a pair.
  // (Was: threads c < C loading all 2 x 32 shards each -- 64 dependent-issue loads in one wave on
  // the launch's critical path.)
  if (wave < kSW) {
    long long S1 = 0, S2 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      S1 += sv[i][0];
      S2 += sv[i][1];
    }
    S1 = rows_total64(S1);
    S2 = rows_total64(S2);
    const int bc = wave * 16 + (lane & 15), b = bc / C, c = bc - b * C;
    if (lane < 16) {
    const lbt_bn_norm& nb = b == 0 ? a.b1.nrm : a.b2.nrm;
    const double s = ldexp(1.0, -frac_exp(nb.qn));
    const double mean_d = (double)S1 * s / (double)nb.n;
    const double var_d = (double)S2 * (s * s) / (double)nb.n - mean_d * mean_d;
    const float m = (float)mean_d, vv = (float)var_d;
    const float sigma = sqrtf(vv + nb.eps);
    sh.cst[b][0][c] = m;
    sh.cst[b][1][c] = sigma;
    if (bid == 0) {  // one writer: ms for the backward, the running averages (:601-612)
      if (nb.ms) { nb.ms[c] = m; nb.ms[C + c] = sigma; }
      if (nb.run_mean) {
        nb.run_mean[c] = nb.momentum * nb.run_mean[c] + nb.one_minus_momentum * m;
        nb.run_var[c] = nb.momentum * nb.run_var[c] + nb.one_minus_momentum * vv;
      }
    }
    }
  }
  __syncthreads();
  LBT_TS(1);
  float pm[NB][4];
  Recip ps[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pm[b][k] = sh.cst[b][0][cq + k];
      ps[b][k] = recip(sh.cst[b][1][cq + k]);
    }
  f2 pm2[NB][2], psy2[NB][2], psr2[NB][2], gam2[NB][2], bet2[NB][2];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      pm2[b][h] = mk2(pm[b][2 * h], pm[b][2 * h + 1]);
      psy2[b][h] = mk2(ps[b][2 * h].y, ps[b][2 * h + 1].y);
      psr2[b][h] = mk2(ps[b][2 * h].rc, ps[b][2 * h + 1].rc);
      gam2[b][h] = mk2(gam[b][2 * h], gam[b][2 * h + 1]);
      bet2[b][h] = mk2(bet[b][2 * h], bet[b][2 * h + 1]);
    }

  // ---------------- phase 1: the chain over the rows + halo -> LDS input codes
  int ovr[2][2] = {{0, 0}, {0, 0}}, ovx1 = 0, ovx2 = 0;
#pragma unroll
  for (int it = 0; it < kBIt; ++it) {
    if (it * kBThreads >= ngrp) break;  // uniform
    const int g = tid + it * kBThreads;
    const int pix = g / C4, hy = pix / Wp, hx = pix - hy * Wp;
    const int y = row0 - 1 + hy, x = hx - 1;
    const bool valid = g < ngrp;
    const bool in = valid && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    const bool own = in && hy >= 1 && hy <= TH;
    const uint32_t e = (uint32_t)((y * W + x) * C + cq);
    f2 v[2];  // the channel quad as two packed pairs
    float T1[2], T2[2];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      T1[b] = ov_thr(own, qr[b].L);
      T2[b] = ov_thr(own, qr[b].Lh);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const lbt_chain_branch& Bb = b == 0 ? a.b1 : a.b2;
      int q[4];
      unpack4(qv[b][it], q);
      const f2 u[2] = {mk2(nrv[b][it].x, nrv[b][it].y), mk2(nrv[b][it].z, nrv[b][it].w)};
      f2 fl[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 x1 = cvt2(q[2 * h], q[2 * h + 1]) * sn[b];
        const f2 x2 = x1 - pm2[b][h];
        const f2 t = div_by2_nz(x2, psy2[b][h], psr2[b][h]);
        const f2 xm = t * qr[b].m;
        ov_count2(xm, T1[b], T2[b], ovr[b][0], ovr[b][1]);
        fl[h] = qfloor2(qr[b], xm, u[h]);  // the R codes
        const f2 xr = fl[h] * qr[b].inv_m;
        const f2 m1 = xr * gam2[b][h];
        const f2 tt = m1 + bet2[b][h];
        v[h] = b ? v[h] + tt : tt;
      }
      if (own) st_out(Bb.rout + img + e, pack4f(fl[0], fl[1]));
    }
    if constexpr (RES) {
      v[0] = v[0] + mk2(rv[it].x, rv[it].y);
      v[1] = v[1] + mk2(rv[it].z, rv[it].w);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) v[h] = mk2(v[h].x > 0.f ? v[h].x : 0.f, v[h].y > 0.f ? v[h].y : 0.f);
    if (YST && own) st_out4(a.y, (uint32_t)(img + e), make_float4(v[0].x, v[0].y, v[1].x, v[1].y));
    const f2 uo[2] = {mk2(nov[it].x, nov[it].y), mk2(nov[it].z, nov[it].w)};
    const float X1 = ov_thr(own, so1.L), X2 = ov_thr(own, so1.Lh);
    int co[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // v >= 0 after the ReLU (NaN -> 0): the lower clip and x < -L cannot hold, the codes are >= 0
      const f2 xm = v[h] * so1.m;
      ov_count2_pos(xm, X1, X2, ovx1, ovx2);
      const f2 w = xm + uo[h];
      co[2 * h] = floor_i(fminf(w.x, so1.Lm1));
      co[2 * h + 1] = floor_i(fminf(w.y, so1.Lm1));
    }
    // LBT_OUT_U8OFF: code - 128 (= code ^ 0x80 for codes in [0, 255]); outside the image: the code of 0
    const int cw = in ? (pack4(co) ^ (int)0x80808080) : (int)0x80808080;
    if (valid) *reinterpret_cast<int*>(sh.x + pix * C + cq) = cw;
    if (own) st_out((int8_t*)a.o1 + img + e, cw);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) pin_counts(ovr[b][0], ovr[b][1]);
  pin_counts(ovx1, ovx2);
  WI::store(sh.w, wimg);
  __syncthreads();
  LBT_TS(2);
  // phase-3 noise (the output quantiser), issued under the MFMAs
  float4 u3[J];  // J channel quads per thread: NQ <= J * kBThreads (the idle threads load the first quad)
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int q3 = tid + j * kBThreads;
    u3[j] = ld4f(p.qout.noise, (uint32_t)(row0 * W * C + ((q3 < NQ ? q3 : 0) / C4) * C + cq));
  }

  // ---------------- phase 2: the conv from the LDS image (pair = wave + 8 pi)
#pragma unroll
  for (int pi = 0; pi < (NPR + 7) / 8; ++pi) {
    const int pr = wave + 8 * pi;
    if (NPR % 8 && pr >= NPR) break;  // uniform per wave
    const int mt = pr / NT, nt = pr - mt * NT;
    const int m = mt * 16 + r;
    const int ly = m / W, px = m - ly * W;
    const int8_t* base = sh.x + (ly * Wp + px) * C;
    v4i acc = v4i{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < kMaxKS; ++kk) {
      const int s = kk * 4 + kg;
      const int tap = s / CS, cs = s - tap * CS;
      const int kh = tap / 3, kw = tap - kh * 3;
      v4i av = *reinterpret_cast<const v4i*>(base + (kh * Wp + kw) * C + cs * 16);
      if (s >= 9 * CS) av = v4i{0, 0, 0, 0};  // k padding (its weights are zero too)
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, WI::frag(sh.w, nt * 16 + r, s), acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      sh.tile[(mt * 16 + 4 * kg + i) * (C + 4) + nt * 16 + r] = (float)(acc[i] + corr) * scale;
  }
  __syncthreads();
  LBT_TS(3);

  // ---------------- phase 3: the next BN's input quantiser + its channel sums
  int ovq1 = 0, ovq2 = 0;
  int s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (NQ % kBThreads && tid + j * kBThreads >= NQ) break;  // uniform per wave
    const int pix3 = (tid + j * kBThreads) / C4;
    const float4 t = *reinterpret_cast<const float4*>(sh.tile + pix3 * (C + 4) + cq);
    const f2 tv[2] = {mk2(t.x, t.y), mk2(t.z, t.w)};
    const f2 u[2] = {mk2(u3[j].x, u3[j].y), mk2(u3[j].z, u3[j].w)};
    f2 fl[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f2 xm = tv[h] * sq.m;
      ov_count2(xm, sq.L, sq.Lh, ovq1, ovq2);
      fl[h] = qfloor2(sq, xm, u[h]);
    }
    const int c[4] = {(int)fl[0].x, (int)fl[0].y, (int)fl[1].x, (int)fl[1].y};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s1[k] += c[k];
      s2[k] += c[k] * c[k];
    }
    st_out(p.yq + img + (uint32_t)(row0 * W * C + pix3 * C + cq), pack4(c));
  }
  {
    const int t1 = chan_scatter4(s1, C4), t2 = chan_scatter4(s2, C4);  // row lane >> 4: channel cq + row
    if ((lane & 15) < C4) {
      sh.part[wave][cq + (lane >> 4)] = t1;
      sh.part[wave][C + cq + (lane >> 4)] = t2;
    }
  }
  // slots [qr of branch 1 | qr of branch 2 | qo1 | qout]
  ov_stage4(0, 4, ov_pack(ovr[0][0], ovr[0][1]), NB == 2 ? ov_pack(ovr[NB - 1][0], ovr[NB - 1][1]) : 0,
            ov_pack(ovx1, ovx2), ov_pack(ovq1, ovq2), sh.cnt);
  __syncthreads();
  LBT_TS(4);
#pragma unroll
  for (int b = 0; b < NB; ++b) counts_publish_nw<kBNW>(b, 4, (b == 0 ? a.b1 : a.b2).qr, sh.cnt);
  counts_publish_nw<kBNW>(2, 4, a.qo1, sh.cnt);
  counts_publish_nw<kBNW>(3, 4, p.qout, sh.cnt);
  if (p.ychsum && tid < 2 * C) {
    long long t = 0;
#pragma unroll
    for (int w = 0; w < kBNW; ++w) t += sh.part[w][tid];
    if (t) LBT_GADD((unsigned long long*)&p.ychsum[(int64_t)shard_id() * 2 * C + tid], (unsigned long long)t);
  }
  LBT_TS(5);
}

// ---- lbt_conv_fwd2_fused_i8: a stage transition's forward in ONE launch -- the last identity block's
// end chain (bn2 + residual + ReLU, its R codes and fp32 y, and BOTH of the projection block's input
// quantisers: the 3x3/2 conv's and the 1x1/2 shortcut's) evaluated into LDS code images, the two
// strided convs from LDS, and both BNs' input quantisers + channel sums over the two conv tiles.
// Bit-identical to lbt_bn_chain_fwd + lbt_conv_fwd_pair_i8. A workgroup owns TH2 output rows, i.e.
// input rows 2 oy0 .. 2 oy0 + 2 TH2 - 1 (+ the row below: the 3x3/2 SAME padding is bottom / right).
constexpr int kTH2 = 4;  // output rows per workgroup (2 x 4 m-tiles: one (m, n) pair per wave)

struct ConvFwd2Args {
  lbt_chain_fwd c;
  const int8_t* wf1;
  const int8_t* wfs;
  const int32_t* wcolsum1;
  const int32_t* wcolsums;
  lbt_qdesc qw1, qws;
  int H;  // input rows
  int8_t* yq1;
  int8_t* yqs;
  lbt_qdesc qout1, qouts;
  int64_t* ychsum1;
  int64_t* ychsums;
};

template <int C>
struct Fwd2Shared {
  int8_t xa[(2 * kTH2 + 1) * 512];          // the 3x3/2 conv's input codes (q - 128), rows 2oy0 .. 2oy0+2TH2
  int8_t xs[kTH2 * 256];                     // the shortcut's, even rows / columns only ([TH2][W/2][C])
  float tile[2][kTH2 * (256 / C) * (2 * C + 4)];  // the two conv outputs [pixel][Cq + 4]
  float cst[2][C];                           // bn2: mu, sigma
  int part[kBNW][2 * 2 * 2 * C];             // per wave: S1, S2 of both output code sets (2Cq each)
  int cnt[kBNW * 2 * 5];                     // counters: qr, qo1, qo2, qout1, qouts
};

template <int CS, bool W4>
__global__ __launch_bounds__(kBThreads, CS == 1 ? 4 : 2) void conv_fwd2_kernel(ConvFwd2Args p) {
  constexpr int C = CS * 16, C4 = C / 4, W = 512 / C, Cq = 2 * C, Cq4 = Cq / 4, Wq = W / 2, NTq = Cq / 16;
  constexpr int kK1 = (9 * CS + 3) / 4;
  constexpr int NG = (2 * kTH2 + 1) * W * C4;  // chain groups (rows 2oy0 .. 2oy0 + 2TH2)
  constexpr int kIt = (NG + kBThreads - 1) / kBThreads;
  static_assert(kTH2 * Wq * Cq == 2 * 1024 && C / 16 <= kBNW, "layout");
  __shared__ __attribute__((aligned(16))) Fwd2Shared<C> sh;
  LBT_TS(0);
  const lbt_chain_fwd& a = p.c;
  const int H = p.H, Hq = H / 2;
  const uint32_t bid = blockIdx.x;
  const int tpi = Hq / kTH2;
  const int n = (int)(bid / (uint32_t)tpi), oy0 = (int)(bid - (uint32_t)n * tpi) * kTH2, y0 = 2 * oy0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int cq = (tid % C4) * 4, cqq = (tid % Cq4) * 4;
  const int64_t img = (int64_t)n * H * W * C, imgq = (int64_t)n * Hq * Wq * Cq;

  // ---------------- bn2's moment shard sums first (waves w < C / 16), then every other load
  constexpr int kSW = C / 16;
  long long sv[8][2];
  if (wave < kSW) {
    const int c = wave * 16 + (lane & 15);
    const int64_t* cs = a.b1.nrm.chsum + (int64_t)(8 * (lane >> 4)) * 2 * C + c;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sv[i][0] = cs[(int64_t)i * 2 * C];
      sv[i][1] = cs[(int64_t)i * 2 * C + C];
    }
  }
  int qv[kIt];
  float4 rv[kIt], nrv[kIt], no1[kIt], no2[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int g = tid + it * kBThreads;
    const int pix = g / C4, hy = pix / W, x = pix - hy * W;
    const int y = y0 + hy;
    const bool in = g < NG && y < H;
    const uint32_t off = in ? (uint32_t)((y * W + x) * C + cq) : 0u;
    qv[it] = ld4i8(a.b1.nrm.q, img + off);
    nrv[it] = ld4f(a.b1.qr.noise, off);
    rv[it] = ld4f(a.res, img + off);
    no1[it] = ld4f(a.qo1.noise, off);
    no2[it] = ld4f(a.qo2.noise, off);
  }
  // the two convs' B operands (forward weight images) of this wave's n-tile; one (m, n) pair per wave
  const int mt = wave / NTq, nt = wave - mt * NTq;
  const int bcol = nt * 16 + r;
  v4i bf1[kK1], bfs;
#pragma unroll
  for (int kk = 0; kk < kK1; ++kk) {
    if constexpr (W4)
      bf1[kk] = unpack_i4x16(*reinterpret_cast<const v2i*>(p.wf1 + ((int64_t)bcol * (4 * kK1) + kk * 4 + kg) * 8));
    else
      bf1[kk] = *reinterpret_cast<const v4i*>(p.wf1 + ((int64_t)bcol * (4 * kK1) + kk * 4 + kg) * 16);
  }
  if constexpr (W4)
    bfs = unpack_i4x16(*reinterpret_cast<const v2i*>(p.wfs + ((int64_t)bcol * 4 + kg) * 8));
  else
    bfs = *reinterpret_cast<const v4i*>(p.wfs + ((int64_t)bcol * 4 + kg) * 16);
  const int corr1 = 128 * p.wcolsum1[bcol], corr2 = 128 * p.wcolsums[bcol];
  float gam[4], bet[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    gam[k] = a.b1.gb[cq + k];
    bet[k] = a.b1.gb[C + cq + k];
  }
  const QState qr = qstate(a.b1.qr), so1 = qstate(a.qo1), so2 = qstate(a.qo2);
  const QState sq1 = qstate(p.qout1), sqs = qstate(p.qouts);
  const float sn = qscale(a.b1.nrm.qn);
  const float scale1 = ldexpf(1.0f, -(frac_exp(a.qo1) + frac_exp(p.qw1)));
  const float scale2 = ldexpf(1.0f, -(frac_exp(a.qo2) + frac_exp(p.qws)));

  // ---------------- Normalization_q moments (conv_fwd_fused_kernel's arithmetic)
  if (wave < kSW) {
    long long S1 = 0, S2 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      S1 += sv[i][0];
      S2 += sv[i][1];
    }
    S1 = rows_total64(S1);
    S2 = rows_total64(S2);
    const int c = wave * 16 + (lane & 15);
    if (lane < 16) {
      const lbt_bn_norm& nb = a.b1.nrm;
      const double s = ldexp(1.0, -frac_exp(nb.qn));
      const double mean_d = (double)S1 * s / (double)nb.n;
      const double var_d = (double)S2 * (s * s) / (double)nb.n - mean_d * mean_d;
      const float m = (float)mean_d, vv = (float)var_d;
      const float sigma = sqrtf(vv + nb.eps);
      sh.cst[0][c] = m;
      sh.cst[1][c] = sigma;
      if (bid == 0) {  // one writer: ms for the backward, the running averages (:601-612)
        if (nb.ms) { nb.ms[c] = m; nb.ms[C + c] = sigma; }
        if (nb.run_mean) {
          nb.run_mean[c] = nb.momentum * nb.run_mean[c] + nb.one_minus_momentum * m;
          nb.run_var[c] = nb.momentum * nb.run_var[c] + nb.one_minus_momentum * vv;
        }
      }
    }
  }
  __syncthreads();
  LBT_TS(1);
  f2 pm2[2], psy2[2], psr2[2], gam2[2], bet2[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const Recip r0 = recip(sh.cst[1][cq + 2 * h]), r1 = recip(sh.cst[1][cq + 2 * h + 1]);
    pm2[h] = mk2(sh.cst[0][cq + 2 * h], sh.cst[0][cq + 2 * h + 1]);
    psy2[h] = mk2(r0.y, r1.y);
    psr2[h] = mk2(r0.rc, r1.rc);
    gam2[h] = mk2(gam[2 * h], gam[2 * h + 1]);
    bet2[h] = mk2(bet[2 * h], bet[2 * h + 1]);
  }

  // ---------------- phase 1: the chain over the input rows -> the two LDS code images
  int ovr1 = 0, ovr2 = 0, ovx1 = 0, ovx2 = 0, ovs1 = 0, ovs2 = 0;
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    if (it * kBThreads >= NG) break;  // uniform
    const int g = tid + it * kBThreads;
    const int pix = g / C4, hy = pix / W, x = pix - hy * W;
    const int y = y0 + hy;
    const bool valid = g < NG;
    const bool in = valid && y < H;
    const bool own = in && hy < 2 * kTH2;
    const uint32_t e = (uint32_t)((y * W + x) * C + cq);
    int q[4];
    unpack4(qv[it], q);
    const f2 u[2] = {mk2(nrv[it].x, nrv[it].y), mk2(nrv[it].z, nrv[it].w)};
    const float T1 = ov_thr(own, qr.L), T2 = ov_thr(own, qr.Lh);
    f2 fl[2], v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f2 x1 = cvt2(q[2 * h], q[2 * h + 1]) * sn;
      const f2 x2 = x1 - pm2[h];
      const f2 t = div_by2_nz(x2, psy2[h], psr2[h]);
      const f2 xm = t * qr.m;
      ov_count2(xm, T1, T2, ovr1, ovr2);
      fl[h] = qfloor2(qr, xm, u[h]);  // the R codes
      const f2 xr = fl[h] * qr.inv_m;
      const f2 m1 = xr * gam2[h];
      v[h] = m1 + bet2[h];
    }
    if (own) st_out(a.b1.rout + img + e, pack4f(fl[0], fl[1]));
    v[0] = v[0] + mk2(rv[it].x, rv[it].y);
    v[1] = v[1] + mk2(rv[it].z, rv[it].w);
#pragma unroll
    for (int h = 0; h < 2; ++h) v[h] = mk2(v[h].x > 0.f ? v[h].x : 0.f, v[h].y > 0.f ? v[h].y : 0.f);
    if (own) st_out4(a.y, (uint32_t)(img + e), make_float4(v[0].x, v[0].y, v[1].x, v[1].y));
    const f2 u1[2] = {mk2(no1[it].x, no1[it].y), mk2(no1[it].z, no1[it].w)};
    const f2 u2[2] = {mk2(no2[it].x, no2[it].y), mk2(no2[it].z, no2[it].w)};
    const float X1 = ov_thr(own, so1.L), X2 = ov_thr(own, so1.Lh);
    const float Z1 = ov_thr(own, so2.L), Z2 = ov_thr(own, so2.Lh);
    int c1[4], c2[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // v >= 0 after the ReLU: only the upper clip can act, the codes are >= 0
      const f2 xm = v[h] * so1.m;
      ov_count2_pos(xm, X1, X2, ovx1, ovx2);
      const f2 w1 = xm + u1[h];
      c1[2 * h] = floor_i(fminf(w1.x, so1.Lm1));
      c1[2 * h + 1] = floor_i(fminf(w1.y, so1.Lm1));
      const f2 zm = v[h] * so2.m;
      ov_count2_pos(zm, Z1, Z2, ovs1, ovs2);
      const f2 w2 = zm + u2[h];
      c2[2 * h] = floor_i(fminf(w2.x, so2.Lm1));
      c2[2 * h + 1] = floor_i(fminf(w2.y, so2.Lm1));
    }
    // LBT_OUT_U8OFF (code ^ 0x80); below the image: the code of 0
    const int cw1 = in ? (pack4(c1) ^ (int)0x80808080) : (int)0x80808080;
    const int cw2 = in ? (pack4(c2) ^ (int)0x80808080) : (int)0x80808080;
    if (valid) *reinterpret_cast<int*>(sh.xa + pix * C + cq) = cw1;
    if (own && !(hy & 1) && !(x & 1)) *reinterpret_cast<int*>(sh.xs + ((hy >> 1) * Wq + (x >> 1)) * C + cq) = cw2;
    if (own) {
      st_out((int8_t*)a.o1 + img + e, cw1);
      st_out((int8_t*)a.o2 + img + e, cw2);
    }
  }
  pin_counts(ovr1, ovr2);
  pin_counts(ovx1, ovx2);
  pin_counts(ovs1, ovs2);
  __syncthreads();
  LBT_TS(2);
  // phase-3 noise of both output quantisers (one quad of each tile per thread: TH2*Wq*Cq/4 == 512)
  const uint32_t off3 = (uint32_t)(oy0 * Wq * Cq + (tid / Cq4) * Cq + cqq);
  const float4 un1 = ld4f(p.qout1.noise, off3), uns = ld4f(p.qouts.noise, off3);

  // ---------------- phase 2: both strided convs from LDS (output pixel (ly, px) reads input
  // (2 ly + kh, 2 px + kw); column W is the SAME padding: the code of 0)
  {
    const int m = mt * 16 + r;
    const int ly = m / Wq, px = m - ly * Wq;
    v4i acc = v4i{0, 0, 0, 0}, acc2 = v4i{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < kK1; ++kk) {
      const int s = kk * 4 + kg;
      const int tap = s / CS, cs = s - tap * CS;
      const int kh = tap / 3, kw = tap - kh * 3;
      const int ix = 2 * px + kw;
      const bool okx = ix < W;
      v4i av = *reinterpret_cast<const v4i*>(sh.xa + (((2 * ly + kh) * W + (okx ? ix : 0)) * C + cs * 16));
      if (!okx) av = v4i{(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
      if (s >= 9 * CS) av = v4i{0, 0, 0, 0};  // k padding (its weights are zero too)
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bf1[kk], acc, 0, 0, 0);
    }
    {
      v4i av = *reinterpret_cast<const v4i*>(sh.xs + ((ly * Wq + px) * C + (kg < CS ? kg : 0) * 16));
      if (kg >= CS) av = v4i{0, 0, 0, 0};
      acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bfs, acc2, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (mt * 16 + 4 * kg + i) * (Cq + 4) + nt * 16 + r;
      sh.tile[0][row] = (float)(acc[i] + corr1) * scale1;
      sh.tile[1][row] = (float)(acc2[i] + corr2) * scale2;
    }
  }
  __syncthreads();
  LBT_TS(3);

  // ---------------- phase 3: both BNs' input quantisers + channel sums
  int ovq[2][2] = {{0, 0}, {0, 0}};
  int s1[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, s2[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  {
    const int pix3 = tid / Cq4;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const QState& sq = b ? sqs : sq1;
      const float4 un = b ? uns : un1;
      const float4 t = *reinterpret_cast<const float4*>(sh.tile[b] + pix3 * (Cq + 4) + cqq);
      const f2 tv[2] = {mk2(t.x, t.y), mk2(t.z, t.w)};
      const f2 u[2] = {mk2(un.x, un.y), mk2(un.z, un.w)};
      f2 fl[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 xm = tv[h] * sq.m;
        ov_count2(xm, sq.L, sq.Lh, ovq[b][0], ovq[b][1]);
        fl[h] = qfloor2(sq, xm, u[h]);
      }
      const int c[4] = {(int)fl[0].x, (int)fl[0].y, (int)fl[1].x, (int)fl[1].y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s1[b][k] += c[k];
        s2[b][k] += c[k] * c[k];
      }
      st_out((b ? p.yqs : p.yq1) + imgq + off3, pack4(c));
    }
  }
  {
    const bool ownq = (lane & 15) < Cq4;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int t1 = chan_scatter4(s1[b], Cq4), t2 = chan_scatter4(s2[b], Cq4);
      if (ownq) {
        sh.part[wave][b * 2 * Cq + cqq + (lane >> 4)] = t1;
        sh.part[wave][b * 2 * Cq + Cq + cqq + (lane >> 4)] = t2;
      }
    }
  }
  // slots [qr | qo1 | qo2 | qout1 | qouts]
  ov_stage4(0, 5, ov_pack(ovr1, ovr2), ov_pack(ovx1, ovx2), ov_pack(ovs1, ovs2), ov_pack(ovq[0][0], ovq[0][1]),
            sh.cnt);
  ov_wave(ovq[1][0], ovq[1][1]);
  counts_stage_w(4, 5, ovq[1][0], ovq[1][1], sh.cnt);
  __syncthreads();
  LBT_TS(4);
  counts_publish_nw<kBNW>(0, 5, a.b1.qr, sh.cnt);
  counts_publish_nw<kBNW>(1, 5, a.qo1, sh.cnt);
  counts_publish_nw<kBNW>(2, 5, a.qo2, sh.cnt);
  counts_publish_nw<kBNW>(3, 5, p.qout1, sh.cnt);
  counts_publish_nw<kBNW>(4, 5, p.qouts, sh.cnt);
  if (tid < 4 * Cq) {
    long long t = 0;
#pragma unroll
    for (int w = 0; w < kBNW; ++w) t += sh.part[w][tid];
    int64_t* dst = tid < 2 * Cq ? p.ychsum1 : p.ychsums;
    if (t && dst) LBT_GADD((unsigned long long*)&dst[(int64_t)shard_id() * 2 * Cq + (tid % (2 * Cq))], (unsigned long long)t);
  }
  LBT_TS(5);
}

}  // namespace

extern "C" int lbt_conv_fwd_fused_i8(const lbt_conv_fwd* q, void* stream) {
  if (!q) return LBT_EINVAL;
  const lbt_conv_desc& d = q->d;
  const int C = d.Cin;
  if (!desc_ok(d) || d.KH != 3 || d.KW != 3 || d.SH != 1 || d.SW != 1 || d.PT != 1 || d.PB != 1 || d.PL != 1 ||
      d.PR != 1 || d.Ho != d.H || d.Wo != d.W || d.Cout != C || (C != 16 && C != 32 && C != 64) ||
      d.H % tile_rows(C / 16) || d.W * C != 512 || (int64_t)d.N * d.H * 512 >= ((int64_t)1 << 29))
    return LBT_EINVAL;  // (st_out4's 32-bit byte offsets)
  const int CS = C / 16;
  const lbt_chain_fwd& a = q->c;
  const int64_t inner = (int64_t)d.H * d.W * C;
  if (a.C != C || a.rows != d.N || a.inner != inner || a.o2 || !a.o1 || a.o1_kind != LBT_OUT_U8OFF) return LBT_EINVAL;
  const int f = fwd_flags(a);
  constexpr int kNeed = kFQ | kFRout | kFRelu | kFO1 | kFStoch | kFU8;
  if ((f & kRt) || (f & kNeed) != kNeed || (f & (kFO2 | kFNoR))) return LBT_EINVAL;
  if (!noise_ok(a.qo1)) return LBT_EINVAL;
  for (int br = 0; br < (a.has_b2 ? 2 : 1); ++br) {
    const lbt_chain_branch& Bb = br ? a.b2 : a.b1;
    if (!noise_ok(Bb.qr) || !Bb.gb || !Bb.nrm.chsum || Bb.nrm.frozen) return LBT_EINVAL;
  }
  if (!q->yq || !noise_ok(q->qout) || !q->wcolsum || !q->wf) return LBT_EINVAL;
  if (q->ksf != 4 * ((9 * CS + 3) / 4)) return LBT_EINVAL;
  if (q->w4 && q->qw.bits > 4) return LBT_EINVAL;
  ConvFwdArgs p;
  p.c = a; p.wf = q->wf; p.wcolsum = q->wcolsum; p.qw = q->qw; p.H = d.H;
  p.yq = q->yq; p.qout = q->qout; p.ychsum = q->ychsum;
  const int th = tile_rows_for(CS, d.N, d.H);
  const int64_t tiles = (int64_t)d.N * (d.H / th);
  if (tiles > 0x7fffffff) return LBT_EINVAL;
  const dim3 grid((unsigned)tiles);
  hipStream_t st = (hipStream_t)stream;
  const int nb = a.has_b2 ? 2 : 1;
  const int fl = f & ~kFU8 & ~kFStoch;  // variant key: Y / residual present
#define LBT_FW_TH(CS_, NB_, FL_, TH_)                                                                        \
  if (q->w4)                                                                                                 \
    hipLaunchKernelGGL((conv_fwd_fused_kernel<CS_, NB_, FL_, true, TH_>), grid, dim3(kBThreads), 0, st, p);    \
  else                                                                                                       \
    hipLaunchKernelGGL((conv_fwd_fused_kernel<CS_, NB_, FL_, false, TH_>), grid, dim3(kBThreads), 0, st, p);
#define LBT_FW(CS_, NB_, FL_)                                                                            \
  if (CS == CS_ && nb == NB_ && fl == ((FL_) & ~kFU8 & ~kFStoch)) {                                      \
    if (CS_ == 1 && th == 4) {                                                                           \
      LBT_FW_TH(CS_, NB_, FL_, (CS_ == 1 ? 4 : tile_rows(CS_)))                                          \
    } else if (th == 2) {                                                                                \
      LBT_FW_TH(CS_, NB_, FL_, 2)                                                                        \
    } else {                                                                                             \
      LBT_FW_TH(CS_, NB_, FL_, tile_rows(CS_))                                                           \
    }                                                                                                    \
    return (int)hipGetLastError();                                                                       \
  }
  // c2 (bn1 chain), c1 after an identity / projection block, block 0's c1 (the stem's chain)
#define LBT_FW_CS(CS_)                                  \
  LBT_FW(CS_, 1, kNeed)                                 \
  LBT_FW(CS_, 1, kNeed | kFRes | kFY)                   \
  LBT_FW(CS_, 2, kNeed | kFY)
  LBT_FW(1, 1, kNeed)
  LBT_FW(1, 1, kNeed | kFRes | kFY)
  LBT_FW(1, 1, kNeed | kFY)
  LBT_FW_CS(2)
  LBT_FW_CS(4)
#undef LBT_FW_CS
#undef LBT_FW
#undef LBT_FW_TH
  return LBT_EINVAL;
}

extern "C" int lbt_conv_fwd2_fused_i8(const lbt_conv_fwd2* q, void* stream) {
  if (!q) return LBT_EINVAL;
  const lbt_conv_desc &d1 = q->d1, &ds = q->ds;
  const int C = d1.Cin, Cq = d1.Cout;
  if (!desc_ok(d1) || !desc_ok(ds) || d1.KH != 3 || d1.KW != 3 || d1.SH != 2 || d1.SW != 2 || d1.PT != 0 ||
      d1.PL != 0 || ds.KH != 1 || ds.KW != 1 || ds.SH != 2 || ds.SW != 2 || ds.PT != 0 || ds.PL != 0 ||
      (C != 16 && C != 32) || Cq != 2 * C || d1.W * C != 512 || d1.H % 2 || d1.W % 2 || d1.Ho * 2 != d1.H ||
      d1.Wo * 2 != d1.W || d1.Ho % kTH2 || ds.N != d1.N || ds.H != d1.H || ds.W != d1.W || ds.Cin != C ||
      ds.Cout != Cq || ds.Ho != d1.Ho || ds.Wo != d1.Wo || (int64_t)d1.N * d1.H * 512 >= ((int64_t)1 << 29))
    return LBT_EINVAL;
  const int CS = C / 16;
  const lbt_chain_fwd& a = q->c;
  if (a.C != C || a.rows != d1.N || a.inner != (int64_t)d1.H * d1.W * C || a.has_b2 || !a.o1 || !a.o2 ||
      a.o1_kind != LBT_OUT_U8OFF || a.o2_kind != LBT_OUT_U8OFF || !a.res || !a.y)
    return LBT_EINVAL;
  const int f = fwd_flags(a);
  constexpr int kNeed = kFQ | kFRout | kFRelu | kFO1 | kFO2 | kFStoch | kFU8 | kFRes | kFY;
  if (f != kNeed) return LBT_EINVAL;
  if (!noise_ok(a.qo1) || !noise_ok(a.qo2) || !noise_ok(a.b1.qr) || !a.b1.gb || !a.b1.nrm.chsum || a.b1.nrm.frozen)
    return LBT_EINVAL;
  if (!q->yq1 || !q->yqs || !noise_ok(q->qout1) || !noise_ok(q->qouts) || !q->wcolsum1 || !q->wcolsums || !q->wf1 ||
      !q->wfs)
    return LBT_EINVAL;
  if (q->ksf1 != 4 * ((9 * CS + 3) / 4) || q->ksfs != 4) return LBT_EINVAL;
  if (q->w4 && (q->qw1.bits > 4 || q->qws.bits > 4)) return LBT_EINVAL;
  ConvFwd2Args p;
  p.c = a; p.wf1 = q->wf1; p.wfs = q->wfs; p.wcolsum1 = q->wcolsum1; p.wcolsums = q->wcolsums;
  p.qw1 = q->qw1; p.qws = q->qws; p.H = d1.H; p.yq1 = q->yq1; p.yqs = q->yqs; p.qout1 = q->qout1;
  p.qouts = q->qouts; p.ychsum1 = q->ychsum1; p.ychsums = q->ychsums;
  const int64_t tiles = (int64_t)d1.N * (d1.Ho / kTH2);
  if (tiles > 0x7fffffff || (int64_t)d1.N * d1.H * d1.W * C >= ((int64_t)1 << 31)) return LBT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
#define LBT_F2(CS_)                                                                                           \
  if (CS == CS_) {                                                                                            \
    if (q->w4)                                                                                                \
      hipLaunchKernelGGL((conv_fwd2_kernel<CS_, true>), dim3((unsigned)tiles), dim3(kBThreads), 0, st, p);    \
    else                                                                                                      \
      hipLaunchKernelGGL((conv_fwd2_kernel<CS_, false>), dim3((unsigned)tiles), dim3(kBThreads), 0, st, p);   \
    return (int)hipGetLastError();                                                                            \
  }
  LBT_F2(1)
  LBT_F2(2)
#undef LBT_F2
  return LBT_EINVAL;
}

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
template <int MODE, int CS, int NT, int CF, int NB, bool W4>
__device__ __forceinline__ void conv_gemm_body(const GemmArgs& p, uint32_t bid) {
  using G = EpiGeom<NT>;
  constexpr int NTW = G::NTW, WPM = G::WPM, MTB = G::MTB;
  __shared__ EpiShared<NT> sh;
  __shared__ ChainShared<NT, (CF ? NB : 1)> csh;
  ChainPre<NT, NB, CF> cp;
  LBT_TS(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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
  auto addr_a = [&](int kk, bool& use, int& alt) -> const v4i* {
    const int s = kk * 4 + kg;
    use = false;
    alt = 0;
    if (s >= p.nslices) return reinterpret_cast<const v4i*>(p.a);
    alt = MODE == MODE_DGRAD ? 0 : p.a_fill;
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
    if (!use) return reinterpret_cast<const v4i*>(p.a);
    return reinterpret_cast<const v4i*>(p.a + (((int64_t)n * SH + sy) * SW + sx) * cred + cs * 16);
  };
  auto load_b = [&](int kk, int j) -> v4i {
    const int col = (nt0 + j) * 16 + r;
    if constexpr (W4)
      return unpack_i4x16(*reinterpret_cast<const v2i*>(p.b + ((int64_t)col * p.ks + kk * 4 + kg) * 8));
    else
      return *reinterpret_cast<const v4i*>(p.b + ((int64_t)col * p.ks + kk * 4 + kg) * 16);
  };

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
    chain_epi<NT, NB, CF>(p.chain, p.add_src != nullptr, p.M, p.ncol, mtile, nt0, wave, lane, v, cp, csh);
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

template <int CSI>
__device__ __forceinline__ void conv_wgrad_body(const WgradArgs& wa, uint32_t bid) {
  const int8_t* __restrict__ xq = wa.xq;
  const int8_t* __restrict__ gq = wa.gq;
  const lbt_conv_desc& d = wa.d;
  const int x_fill = wa.x_fill, nsplit = wa.nsplit, nshard = wa.nshard;
  int32_t* __restrict__ slab = wa.slab;
  const int64_t P = wa.P;
  constexpr int CI = CSI * 16;
  // per wave: X image [CSI][64 px][16 B] and G image [64 px][16 B]
  __shared__ __attribute__((aligned(16))) int8_t lds[4][(CSI + 1) * kWP * 16];
  __shared__ int red[4][CI * 16];
  LBT_TS(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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

  // chunks are interleaved across the 4 waves of the block
  for (int64_t c0 = p0 + (int64_t)wave * kWP; c0 < p1; c0 += 4 * kWP) {
    const int64_t p = c0 + lane;
    const bool pv = p < p1;
    const uint32_t pu = (uint32_t)(pv ? p : p0);  // P < 2^31 (launcher)
    const uint32_t n = pu / HWo, rem = pu - n * HWo;
    const int oh = (int)(rem / (uint32_t)d.Wo), ow = (int)(rem - (uint32_t)oh * (uint32_t)d.Wo);
    const int ih = oh * d.SH + kh - d.PT, iw = ow * d.SW + kw - d.PL;
    const bool xv = pv && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
    // all loads first (clamped addresses, no branches), fills selected afterwards
    const int8_t* xp = xq + (xv ? ((((int64_t)n * d.H + ih) * d.W + iw) * CI) : 0);
    v4i xs[CSI];
#pragma unroll
    for (int cs = 0; cs < CSI; ++cs) xs[cs] = *reinterpret_cast<const v4i*>(xp + cs * 16);
    v4i g = *reinterpret_cast<const v4i*>(gq + (int64_t)pu * d.Cout + cso * 16);
    const int xf = pv ? x_fill : 0;
#pragma unroll
    for (int cs = 0; cs < CSI; ++cs) {
      if (!xv) xs[cs] = v4i{xf, xf, xf, xf};
      *reinterpret_cast<v4i*>(Xi + (cs * kWP + lane) * 16) = xs[cs];
    }
    if (!pv) g = v4i{0, 0, 0, 0};
    *reinterpret_cast<v4i*>(Gi + lane * 16) = g;
    // the images are read by other lanes of the same wave only
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const v4i bfrag = tr_frag(Gi, 16 * kg, lane);
#pragma unroll
    for (int a = 0; a < CSI; ++a) {
      const v4i afrag = tr_frag(Xi + a * kWP * 16, 16 * kg, lane);
      acc[a] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag, bfrag, acc[a], 0, 0, 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
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
  for (int i = threadIdx.x; i < CI * 16; i += kThreads) {
    const int ci = i >> 4, co = i & 15;
    const int v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    if (v) LBT_GADD(&dst[(int64_t)ci * d.Cout + co], v);  // integer atomics: exact, order-independent
  }
  LBT_TS(3);
}

template <int CSI>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(WgradArgs wa) {
  conv_wgrad_body<CSI>(wa, blockIdx.x);
}

// Horizontal fusion of one conv's two backward GEMMs, which read the same gradient codes and
// are independent of each other: workgroups [0, nwg) are the wgrad's (the longer ones, dispatched
// first), the rest the dgrad (+ chain pass A) tiles. One launch instead of two; nwg is a multiple
// of 8, so both halves keep their XCD-aware block order.
template <int CS, int NT, int CF, int NB, bool W4>
__global__ __launch_bounds__(kThreads, (CS == 1 && NB == 1) ? 8 : 1) void dgrad_wgrad_kernel(GemmArgs p, WgradArgs wa,
                                                                                          uint32_t nwg) {
  if (blockIdx.x < nwg)
    conv_wgrad_body<NT>(wa, blockIdx.x);
  else
    conv_gemm_body<MODE_DGRAD, CS, NT, CF, NB, W4>(p, blockIdx.x - nwg);
}

// 256 threads = 32 outputs x 8 split groups; coalesced 128-B slab rows; exact int64 sums.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const int32_t* __restrict__ slab, int nsplit, int K,
                                                           int Cout, int x_u8off, const int64_t* __restrict__ gcolsum,
                                                           lbt_qdesc qx, lbt_qdesc qg, const float* __restrict__ w,
                                                           float wd2, float* __restrict__ dw) {
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
template <bool W4>
int conv_fwd(const int8_t* xq, int32_t x_u8off, const int8_t* wf, int32_t ksf, const int32_t* wcolsum,
             lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y, int8_t* yq, lbt_qdesc qout, int64_t* ychsum,
             void* stream) {
  if (!desc_ok(d) || d.Cin % 16 || d.Cout % 16 || d.Cout > 128) return LBT_EINVAL;
  const int cs = d.Cin / 16;
  GemmArgs p;
  p.a = xq; p.b = wf; p.ks = ksf; p.nslices = d.KH * d.KW * cs;
  if (ksf % 4 || ksf < p.nslices) return LBT_EINVAL;
  p.a_fill = x_u8off ? (int)0x80808080u : 0;
  p.colsum = x_u8off ? wcolsum : nullptr;
  if (x_u8off && !wcolsum) return LBT_EINVAL;
  if (yq && qout.stochastic && !qout.noise) return LBT_EINVAL;  // quantising epilogue reads the noise table
  p.d = d; p.qa = qx; p.qb = qw; p.y = y; p.add_src = nullptr; p.yq = yq; p.qout = qout; p.ychsum = ychsum;
  p.M = (int64_t)d.N * d.Ho * d.Wo; p.ncol = d.Cout;
  return launch_gemm<MODE_FWD, W4>(p, cs, (hipStream_t)stream);
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

extern "C" int lbt_conv_wgrad_reduce(const int32_t* slab, int32_t nsplit, int32_t K, int32_t Cout, int32_t x_u8off,
                                     const int64_t* gcolsum, lbt_qdesc qx, lbt_qdesc qg, const float* w, float wd2,
                                     float* dw, void* stream) {
  const int64_t total = (int64_t)K * Cout;
  const int64_t blocks = (total + 31) / 32;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, slab, nsplit, K,
                     Cout, x_u8off, gcolsum, qx, qg, w, wd2, dw);
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

// stem_wide.hip -- the ImageNet ResNet's conv1 (7x7 / 2, 3 -> 64 channels; SURVEY 8(f) rank 1,
// dynamic_fixed_point.py:287-305) on v_mfma_f32_16x16x32_f16, forward and weight gradient.
//
// Like stem.hip, the operand is the image quantised to SIGNED 9-bit codes, which int8 MFMA cannot
// take; fp16 holds them (|x| <= 256) and every 8-bit weight / gradient code exactly, and the fp32
// accumulator stays exact while every partial sum is an integer of magnitude <= 2^24:
//   fwd   : K (= 147 here) products of |x*w| <= 2^8 * 2^7 per output -- the launcher checks
//           K * 2^(xbits-1) * 2^(wbits-1) <= 2^24, so the whole K loop accumulates in fp32;
//   wgrad : k-dim = pixels. A 16-bit gradient code is split g = 256*hi + lo with hi = g >> 8 in
//           [-128, 127] and lo = g & 255 in [0, 255], both exact in fp16; one MFMA step sums 32
//           pixels, and every kFlush = 4 steps (128 pixels, |sum| <= 128 * 256 * 255 < 2^24) the
//           fp32 tiles are moved into int32 accumulators. A workgroup covers <= kMaxWgPixels
//           pixels, so those stay below 2^31; it stores 256*hi + lo as int64 into its own slice of
//           slab[split][k][co] (plain stores: every slab element has exactly one writer), and
//           lbt_conv_wgrad_reduce64 finishes dW exactly as for the generic kernels.
// The results are the integer GEMM's, bit for bit (same as conv_generic.hip and the oracle).
//
// fp16 16x16x32 operand map (gfx950): lane l holds A[row l&15][k = 8*(l>>4) + j] and
// B[k = 8*(l>>4) + j][col l&15], j = 0..7; C/D: col = l&15, row = 4*(l>>4) + reg.
#include "dfxp_device.h"

#include <cstdlib>

using namespace lbt;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

namespace {

constexpr int kThreads = 256;
constexpr int kMaxK = 480;           // patch elements (LDS budget; exactness is checked separately)
constexpr int kFwdRows = 128;        // output pixels per forward workgroup (4 waves x 2 m-tiles)
constexpr int kWgChunk = 64;         // wgrad pixels staged per LDS pass (2 MFMA k-steps)
constexpr int kFlush = 4;            // wgrad MFMA k-steps between fp32 -> int32 flushes
constexpr int kMaxWgPixels = 16384;  // wgrad pixels per workgroup (int32 accumulator bound)

// patch element k = (kh, kw, ci) in HWIO order -> (dy, dx, ci) relative to (oy*SH - PT, ox*SW - PL)
LBT_DEV int patch_code(const lbt_conv_desc& d, int k) {
  const int tap = k / d.Cin, ci = k - tap * d.Cin;
  const int kh = tap / d.KW, kw = tap - kh * d.KW;
  return (kh << 20) | (kw << 10) | ci;
}

// ------------------------------------------------------------------ forward
// grid (ceil(M / 128), ceil(Cout / 64)); wave = 2 m-tiles x NCT column tiles of its 64-column
// group. The W slice lives in LDS as fp16, transposed ([col][k]), so a B fragment is one 16-byte
// read; the patch-element decode table too. A fragments are gathered from the int16 image.
template <int NCT>
__global__ __launch_bounds__(kThreads) void stem_wide_fwd_kernel(const int16_t* __restrict__ x,
                                                                 const int8_t* __restrict__ w, lbt_conv_desc d, int K,
                                                                 int KP, lbt_qdesc qx, lbt_qdesc qw,
                                                                 float* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  _Float16* sW = reinterpret_cast<_Float16*>(smem);        // [NCT*16][KP]
  int* sK = reinterpret_cast<int*>(smem + (size_t)NCT * 16 * KP * 2);  // [KP]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int c0 = blockIdx.y * 64;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  for (int i = threadIdx.x; i < NCT * 16 * KP; i += kThreads) {
    const int col = i / KP, k = i - col * KP;
    const int c = c0 + col;
    const int v = (k < K && c < d.Cout) ? (int)w[(int64_t)k * d.Cout + c] : 0;
    sW[i] = (_Float16)(float)v;
  }
  for (int k = threadIdx.x; k < KP; k += kThreads) sK[k] = k < K ? patch_code(d, k) : -1;
  __syncthreads();

  // this lane's two A rows (output pixels)
  int base[2], iy0[2], ix0[2];
  bool rv[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int64_t m = (int64_t)blockIdx.x * kFwdRows + wave * 32 + mt * 16 + r;
    rv[mt] = m < M;
    const uint32_t mu = (uint32_t)(rv[mt] ? m : 0);
    const int ox = (int)(mu % (uint32_t)d.Wo);
    const uint32_t t = mu / (uint32_t)d.Wo;
    const int oy = (int)(t % (uint32_t)d.Ho), n = (int)(t / (uint32_t)d.Ho);
    iy0[mt] = oy * d.SH - d.PT;
    ix0[mt] = ox * d.SW - d.PL;
    base[mt] = n * d.H;
  }
  f4v acc[2][NCT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[mt][ct] = f4v{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < KP; k0 += 32) {
    int code[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) code[j] = sK[k0 + 8 * kg + j];
    h8 a[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      int off[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = code[j];
        const int iy = iy0[mt] + (c >> 20), ix = ix0[mt] + ((c >> 10) & 1023);
        const bool ok = c >= 0 && rv[mt] && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        off[j] = ok ? ((base[mt] + iy) * d.W + ix) * d.Cin + (c & 1023) : -1;
      }
      int16_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = x[off[j] < 0 ? 0 : off[j]];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[mt][j] = (_Float16)(float)(off[j] < 0 ? 0 : (int)v[j]);
    }
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const h8 b = *reinterpret_cast<const h8*>(sW + (ct * 16 + r) * KP + k0 + 8 * kg);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) acc[mt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt], b, acc[mt][ct], 0, 0, 0);
    }
  }
  const float scale = ldexpf(1.0f, -(frac_exp(qx) + frac_exp(qw)));
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int c = c0 + ct * 16 + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = (int64_t)blockIdx.x * kFwdRows + wave * 32 + mt * 16 + kg * 4 + i;
        if (row < M && c < d.Cout) y[row * d.Cout + c] = acc[mt][ct][i] * scale;  // exact integer * 2^-e
      }
    }
}

// Row-tile forward (the default where it applies: Cin <= 4, KW <= 8, Wo <= 256). A workgroup owns TR
// whole output rows of one image (TR * Wo <= 256 pixels: 8 waves x 2 m-tiles) and loops over such
// tiles. The image rows under a tile are staged ONCE into LDS as fp16 [R][Wimg][4] (zero padding
// and a zero 4th channel written in), so a patch row of 8 taps x 4 channels is 32 consecutive
// halves: one MFMA k-step per kernel row, and a lane's 8 k-elements (2 taps x 4 channels) are one
// 16-byte LDS read at a per-lane offset fixed for the tile -- no per-element gather or decode. The
// weights (zeros at tap 7 / channel 3) are staged once per workgroup, [col][ky*32 + kx*4 + ci].
// Operands are swapped (A = weights, B = pixels) so a lane's accumulator is 4 consecutive output
// channels of one pixel: one 16-byte store each. The next tile's image codes are loaded into registers
// while this tile computes. ResNet-50 conv1 at B=256: 748 us (gather kernel) -> 254 us, one eager launch.
constexpr int kTileThreads = 512;
constexpr int kTileWaves = kTileThreads / 64;
constexpr int kTilePixels = kTileWaves * 2 * 16;  // 2 m-tiles per wave
constexpr int kTilePre = 5;                        // image pixels per thread (R * Wimg <= 2560)
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

template <int NCT>
__global__ __launch_bounds__(kTileThreads) void stem_wide_fwd_tiles_kernel(const int16_t* __restrict__ x,
                                                                           const int8_t* __restrict__ w,
                                                                           lbt_conv_desc d, int TR, int R, int Wimg,
                                                                           int KS, int ntiles, lbt_qdesc qx,
                                                                           lbt_qdesc qw, float* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  _Float16* sW = reinterpret_cast<_Float16*>(smem);  // [NCT*16][KS], KS = KH*32 + 8
  _Float16* sX = sW + NCT * 16 * KS;                 // [R][Wimg][4]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int c0 = blockIdx.y * 64;
  const int KH = d.KH, KW = d.KW, Cin = d.Cin, Cout = d.Cout, Wo = d.Wo;
  for (int i = threadIdx.x; i < NCT * 16 * KS; i += kTileThreads) {
    const int col = i / KS, k = i - col * KS;
    const int ky = k >> 5, kx = (k >> 2) & 7, ci = k & 3, c = c0 + col;
    const int v = (ky < KH && kx < KW && ci < Cin && c < Cout) ? (int)w[((ky * KW + kx) * Cin + ci) * Cout + c] : 0;
    sW[i] = (_Float16)(float)v;
  }
  const int tpi = (d.Ho + TR - 1) / TR;
  const int npx = TR * Wo, nmt = (npx + 15) >> 4;
  const int nimg = R * Wimg;
  const float scale = ldexpf(1.0f, -(frac_exp(qx) + frac_exp(qw)));
  // the tile's image pixels e = t + 512 j (j < kTilePre; host: R * Wimg <= 512 kTilePre) travel through
  // registers: the next tile's loads are issued before this tile's MFMAs and stores
  int raw[kTilePre][2];
  auto load_img = [&](int tile) {
    const int n = tile / tpi, iy0 = (tile - n * tpi) * TR * d.SH - d.PT;
#pragma unroll
    for (int j = 0; j < kTilePre; ++j) {
      const int e = threadIdx.x + j * kTileThreads;
      const int row = e / Wimg, col = e - row * Wimg;
      const int iy = iy0 + row, ix = col - d.PL;
      const bool ok = e < nimg && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
      const int16_t* p = x + (ok ? ((n * d.H + iy) * d.W + ix) * Cin : 0);  // host: N*H*W*Cin < 2^31
      int v[4];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) v[ci] = (ok && ci < Cin) ? (int)p[ci] : 0;
      raw[j][0] = (v[0] & 0xffff) | (v[1] << 16);  // two int16 codes per register
      raw[j][1] = (v[2] & 0xffff) | (v[3] << 16);
    }
  };
  if (blockIdx.x < ntiles) load_img(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tpi, oy0 = (tile - n * tpi) * TR;
    __syncthreads();  // the previous tile's image reads are done (first pass: nothing to wait for)
#pragma unroll
    for (int j = 0; j < kTilePre; ++j) {
      const int e = threadIdx.x + j * kTileThreads;
      if (e < nimg)
        *reinterpret_cast<h4*>(sX + e * 4) =
            h4{(_Float16)(float)(int16_t)raw[j][0], (_Float16)(float)(raw[j][0] >> 16),
               (_Float16)(float)(int16_t)raw[j][1], (_Float16)(float)(raw[j][1] >> 16)};
    }
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load_img(tile + gridDim.x);
    // this lane's pixel in each of its m-tiles (m-tile wave + 8*mt of the tile)
    int xo[2];
    int64_t orow[2];
    bool pv[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int q = (wave + kTileWaves * mt) * 16 + r;
      const int tr = q / Wo, ox = q - tr * Wo;
      pv[mt] = q < npx && oy0 + tr < d.Ho;
      xo[mt] = pv[mt] ? ((tr * d.SH) * Wimg + ox * d.SW) * 4 + kg * 8 : 0;
      orow[mt] = ((int64_t)n * d.Ho + oy0 + tr) * Wo + ox;
    }
    const bool m1 = wave + kTileWaves < nmt;  // uniform: this wave's second m-tile exists
    if (wave < nmt) {
      f4v acc[2][NCT];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[mt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
      for (int ky = 0; ky < KH; ++ky) {
        h8 a[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) a[ct] = *reinterpret_cast<const h8*>(sW + (ct * 16 + r) * KS + ky * 32 + kg * 8);
        const int yo = ky * Wimg * 4;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          if (mt == 1 && !m1) break;
          // two 8-byte reads: the pixel pair is 8-byte aligned only
          const h4 lo = *reinterpret_cast<const h4*>(sX + xo[mt] + yo);
          const h4 hi = *reinterpret_cast<const h4*>(sX + xo[mt] + yo + 4);
          const h8 b = h8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct)
            acc[mt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ct], b, acc[mt][ct], 0, 0, 0);
        }
      }
      // D[row = channel 4kg + i][col = pixel r]: 4 consecutive channels per lane
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        if (mt == 1 && !m1) break;
        if (!pv[mt]) continue;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          const int c = c0 + ct * 16 + 4 * kg;
          if (c < Cout) {  // Cout % 16 == 0: all four channels
            const f4v o = acc[mt][ct] * scale;  // exact integer * 2^-e
            // streamed out (the output is ~800 MB at B=256, read once by the next kernel): 266 -> 254 us
            __builtin_nontemporal_store(o, reinterpret_cast<f4v*>(y + orow[mt] * Cout + c));
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
// grid (nsplit, ceil(K / 64), ceil(Cout / 64)): workgroup = one pixel range, 4 k-tiles (one per
// wave: 16 patch elements), 64 output channels. Per 64-pixel pass the gradient rows are staged
// in LDS transposed and split ([hi|lo][col][pixel] fp16), with the pass's pixel decode; each wave
// gathers its patch rows (A) from the int16 image.
template <bool G16, int NCT>
__global__ __launch_bounds__(kThreads) void stem_wide_wgrad_kernel(const int16_t* __restrict__ x,
                                                                   const void* __restrict__ g_, lbt_conv_desc d,
                                                                   int K, int64_t per, int64_t* __restrict__ slab) {
  constexpr int NH = G16 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) _Float16 sG[NH][NCT * 16][kWgChunk + 8];
  __shared__ int sOff[kWgChunk], sYX[kWgChunk];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int c0 = blockIdx.z * 64;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = p0 + per < M ? p0 + per : M;
  // this lane's A row: patch element k of this wave's k-tile
  const int k = (blockIdx.y * 4 + wave) * 16 + r;
  const int code = k < K ? patch_code(d, k) : -1;
  const int dy = code >> 20, dx = (code >> 10) & 1023, ci = code & 1023;
  const int koff = code >= 0 ? (dy * d.W + dx) * d.Cin + ci : 0;  // the patch element's offset from its pixel's

  f4v facc[NH][NCT];
  int iacc[NH][NCT][4];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      facc[h][ct] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) iacc[h][ct][i] = 0;
    }
  int steps = 0;
  for (int64_t q0 = p0; q0 < p1; q0 += kWgChunk) {
    __syncthreads();  // the previous pass's LDS reads are done
    // stage: pixel decode (64 threads) and the gradient rows, transposed + split
    if (threadIdx.x < kWgChunk) {
      const int64_t p = q0 + threadIdx.x;
      const bool pv = p < p1;
      const uint32_t pu = (uint32_t)(pv ? p : p0);
      const int ox = (int)(pu % (uint32_t)d.Wo);
      const uint32_t t = pu / (uint32_t)d.Wo;
      const int oy = (int)(t % (uint32_t)d.Ho), n = (int)(t / (uint32_t)d.Ho);
      const int y0 = oy * d.SH - d.PT, x0 = ox * d.SW - d.PL;
      // window origin offset (may be negative: only in-range taps are ever added to it); a pixel
      // past the range gets a row far out of [0, H) so every tap of it fails the bounds test
      sOff[threadIdx.x] = ((n * d.H + y0) * d.W + x0) * d.Cin;
      sYX[threadIdx.x] = pv ? ((y0 << 16) | (x0 & 0xFFFF)) : (int)(0x8000u << 16);
    }
    // gradient rows: 8 consecutive channels of one pixel per 16- (8-) byte load, written transposed
    for (int i = threadIdx.x; i < kWgChunk * NCT * 2; i += kThreads) {
      const int px = i / (NCT * 2), col = (i - px * (NCT * 2)) * 8;
      const int64_t p = q0 + px;
      const int c = c0 + col;
      int v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (p < p1 && c < d.Cout) {  // Cout % 16 == 0: the 8 channels are all in range
        if constexpr (G16) {
          const int4 w4 = *reinterpret_cast<const int4*>(reinterpret_cast<const int16_t*>(g_) + p * d.Cout + c);
          const int w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[2 * j] = (int)(int16_t)(w[j] & 0xFFFF); v[2 * j + 1] = w[j] >> 16; }
        } else {
          const int2 w = *reinterpret_cast<const int2*>(reinterpret_cast<const int8_t*>(g_) + p * d.Cout + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[j] = (int)(int8_t)(w.x >> (8 * j)); v[4 + j] = (int)(int8_t)(w.y >> (8 * j)); }
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (G16) {
          sG[0][col + j][px] = (_Float16)(float)(v[j] >> 8);        // hi, arithmetic shift: [-128, 127]
          sG[NH - 1][col + j][px] = (_Float16)(float)(v[j] & 255);  // lo: [0, 255]
        } else {
          sG[0][col + j][px] = (_Float16)(float)v[j];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kWgChunk / 32; ++s) {
      h8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int px = s * 32 + 8 * kg + j;
        const int yx = sYX[px];
        const int iy = (yx >> 16) + dy, ix = (int)(int16_t)(yx & 0xFFFF) + dx;
        const bool ok = code >= 0 && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        const int off = ok ? sOff[px] + koff : 0;
        const int v = x[off];
        a[j] = (_Float16)(float)(ok ? v : 0);
      }
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          const h8 b = *reinterpret_cast<const h8*>(&sG[h][ct * 16 + r][s * 32 + 8 * kg]);
          facc[h][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, facc[h][ct], 0, 0, 0);
        }
      if (++steps == kFlush) {
        steps = 0;
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) {
#pragma unroll
            for (int i = 0; i < 4; ++i) iacc[h][ct][i] += (int)facc[h][ct][i];
            facc[h][ct] = f4v{0.f, 0.f, 0.f, 0.f};
          }
      }
    }
  }
  // D[row = k][col]: row = k-tile*16 + 4*kg + i, col = ct*16 + r
  int64_t* out = slab + (int64_t)blockIdx.x * K * d.Cout;
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int c = c0 + ct * 16 + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = (blockIdx.y * 4 + wave) * 16 + 4 * kg + i;
      int64_t v = (int64_t)(iacc[0][ct][i] + (int)facc[0][ct][i]);
      if constexpr (G16) v = 256 * v + (int64_t)(iacc[1][ct][i] + (int)facc[1][ct][i]);
      if (kk < K && c < d.Cout) out[(int64_t)kk * d.Cout + c] = v;
    }
  }
}

// Weight gradient on output-row chunks (round 4): a chunk is kRwPx (128 since round 5, was 64: twice the
// MFMA work per chunk behind the same load latency) consecutive output pixels of ONE output row (n, oy,
// kRwPx xc ..); its input window (KH rows x ((kRwPx-1) SW + KW) columns x Cin) is staged in LDS as fp16
// once and every patch element -- all K, one 16-row k-tile per wave, up to kRwMaxKT waves -- reads its A
// fragment from it (stem_wide_wgrad_kernel gathers every patch element of every pixel from global
// memory, 64 addresses per load instruction, and re-reads the gradient rows once per 64-row k-block of
// grid.y). Always kRwMaxKT waves: they all stage the window (the k-tiles past K multiply zeros). The next chunk's window and gradient rows are loaded into registers while the current chunk's
// MFMAs run. Same exact arithmetic: fp16 operands, fp32 partial sums flushed to int32 every kFlush
// steps, 256 hi + lo into int64 per split.
constexpr int kRwMaxKT = 10;   // k-tiles (K <= 160)
constexpr int kRwMaxKH = 7;    // window rows
#ifndef LBT_RW_UNROLL
#define LBT_RW_UNROLL 1
#endif
constexpr int kRwPx = 128;     // output pixels per chunk (4 MFMA k-steps)
constexpr int kRwMaxWC = 264;  // window columns (kRwPx - 1) SW + KW
constexpr int kRwMaxCin = 4;
constexpr int kRwWin = kRwMaxKH * kRwMaxWC * kRwMaxCin;
constexpr int kRwWpt = 8;  // window elements a thread stages (host: KH * WC * Cin <= kRwWpt * 64 * kRwMaxKT)

template <bool G16, int NCT>
__global__ __launch_bounds__(64 * kRwMaxKT, NCT <= 2 ? 5 : 3) void stem_wgrad_rows_kernel(const int16_t* __restrict__ x,
                                                                        const void* __restrict__ g_, lbt_conv_desc d,
                                                                        int K, int64_t cper, int64_t nchunks, int xc,
                                                                        int64_t* __restrict__ slab) {
  constexpr int NH = G16 ? 2 : 1;
  constexpr int GV = NCT * 2;  // 16-byte (G16) / 8-byte gradient pieces per pixel (8 channels each)
  __shared__ __attribute__((aligned(16))) _Float16 sG[NH][NCT * 16][kRwPx + 8];
  __shared__ _Float16 sW[kRwWin];
  const int nthr = blockDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const int k = wave * 16 + r;
  const int code = k < K ? patch_code(d, k) : -1;
  const int dy = code >> 20, dx = (code >> 10) & 1023, ci = code & 1023;
  const int WC = ((d.Wo < kRwPx ? d.Wo : kRwPx) - 1) * d.SW + d.KW, wsz = d.KH * WC * d.Cin;
  const int aoff = code >= 0 ? (dy * WC + dx) * d.Cin + ci : 0;  // + px * SW * Cin
  const int astep = d.SW * d.Cin;
  f4v facc[NH][NCT];
  int iacc[NH][NCT][4];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      facc[h][ct] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) iacc[h][ct][i] = 0;
    }
  const int cg0 = blockIdx.y * NCT * 16;  // this workgroup's output channels cg0 .. cg0 + 16 NCT - 1
  const int64_t cb = (int64_t)blockIdx.x * cper;
  const int64_t ce = cb + cper < nchunks ? cb + cper : nchunks;
  // one chunk's operands in registers: window elements threadIdx.x + j * nthr, gradient piece threadIdx.x
  int wv[(kRwWpt + 1) / 2];  // two int16 window codes per register
  constexpr int kGp = (kRwPx * GV + 64 * kRwMaxKT - 1) / (64 * kRwMaxKT);  // gradient pieces a thread stages
  int gw[kGp][4];
  auto load = [&](int64_t c) {
    const int xcc = (int)(c % xc);
    const int64_t t = c / xc;
    const int oy = (int)(t % d.Ho), n = (int)(t / d.Ho);
    const int iy0 = oy * d.SH - d.PT, ix0 = xcc * kRwPx * d.SW - d.PL;
#pragma unroll
    for (int j = 0; j < kRwWpt; ++j) {
      const int e = threadIdx.x + j * nthr;
      int v = 0;
      if (e < wsz) {
        const int cc = e % d.Cin, t2 = e / d.Cin, col = t2 % WC, row = t2 / WC;
        const int iy = iy0 + row, ix = ix0 + col;
        if ((unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W)
          v = x[((int64_t)(n * d.H + iy) * d.W + ix) * d.Cin + cc];
      }
      if (j & 1) wv[j >> 1] |= v << 16;
      else wv[j >> 1] = v & 0xFFFF;
    }
#pragma unroll
    for (int q = 0; q < kGp; ++q) {
      gw[q][0] = gw[q][1] = gw[q][2] = gw[q][3] = 0;
      const int idx = threadIdx.x + q * nthr;
      if (idx < kRwPx * GV) {
        const int px = idx / GV, col = cg0 + (idx % GV) * 8;
        const int ox = xcc * kRwPx + px;
        if (ox < d.Wo && col < d.Cout) {
          const int64_t p = ((int64_t)n * d.Ho + oy) * d.Wo + ox;
          if constexpr (G16) {
            const int4 w4 = *reinterpret_cast<const int4*>(reinterpret_cast<const int16_t*>(g_) + p * d.Cout + col);
            gw[q][0] = w4.x; gw[q][1] = w4.y; gw[q][2] = w4.z; gw[q][3] = w4.w;
          } else {
            const int2 w2 = *reinterpret_cast<const int2*>(reinterpret_cast<const int8_t*>(g_) + p * d.Cout + col);
            gw[q][0] = w2.x; gw[q][1] = w2.y;
          }
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < kRwWpt; ++j) {
      const int e = threadIdx.x + j * nthr;
      if (e < wsz) sW[e] = (_Float16)(float)((j & 1) ? (wv[j >> 1] >> 16) : (int)(int16_t)wv[j >> 1]);
    }
#pragma unroll
    for (int q = 0; q < kGp; ++q) {
      const int idx = threadIdx.x + q * nthr;
      if (idx >= kRwPx * GV) break;
      const int px = idx / GV, col = (idx % GV) * 8;
      int v[8];
      if constexpr (G16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[2 * j] = (int)(int16_t)(gw[q][j] & 0xFFFF); v[2 * j + 1] = gw[q][j] >> 16; }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = (int)(int8_t)(gw[q][0] >> (8 * j));
          v[4 + j] = (int)(int8_t)(gw[q][1] >> (8 * j));
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (G16) {
          sG[0][col + j][px] = (_Float16)(float)(v[j] >> 8);        // hi, arithmetic shift: [-128, 127]
          sG[NH - 1][col + j][px] = (_Float16)(float)(v[j] & 255);  // lo: [0, 255]
        } else {
          sG[0][col + j][px] = (_Float16)(float)v[j];
        }
      }
    }
  };
  static_assert(kRwPx / 32 == kFlush, "one fp32 -> int32 flush per chunk");
  // a window narrower than kRwPx pixels (Wo < kRwPx): the A reads of the pixels past Wo land past wsz
  // (their gradients are zero) -- zeros there, never NaN patterns of stale LDS (0 * NaN)
  for (int e = wsz + threadIdx.x; e < kRwWin; e += nthr) sW[e] = (_Float16)0.f;
  if (cb < ce) load(cb);
  for (int64_t c = cb; c < ce; ++c) {
    __syncthreads();  // the previous chunk's LDS reads are done
    store();
    __syncthreads();
    if (c + 1 < ce) load(c + 1);  // in flight during this chunk's MFMAs
#pragma unroll LBT_RW_UNROLL
    for (int s = 0; s < kRwPx / 32; ++s) {
      h8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int px = s * 32 + 8 * kg + j;
        a[j] = code >= 0 ? sW[aoff + px * astep] : (_Float16)0.f;
      }
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          const h8 b = *reinterpret_cast<const h8*>(&sG[h][ct * 16 + r][s * 32 + 8 * kg]);
          facc[h][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, facc[h][ct], 0, 0, 0);
        }
    }
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
#pragma unroll
        for (int i = 0; i < 4; ++i) iacc[h][ct][i] += (int)facc[h][ct][i];
        facc[h][ct] = f4v{0.f, 0.f, 0.f, 0.f};
      }
  }
  int64_t* out = slab + (int64_t)blockIdx.x * K * d.Cout;
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int c = cg0 + ct * 16 + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = wave * 16 + 4 * kg + i;
      int64_t v = (int64_t)(iacc[0][ct][i] + (int)facc[0][ct][i]);
      if constexpr (G16) v = 256 * v + (int64_t)(iacc[1][ct][i] + (int)facc[1][ct][i]);
      if (kk < K && c < d.Cout) out[(int64_t)kk * d.Cout + c] = v;
    }
  }
}

}  // namespace

extern "C" int lbt_conv_stem_wide_fwd(const int16_t* x, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qx,
                                      lbt_qdesc qw, float* y, void* stream) {
  const int K = d.KH * d.KW * d.Cin;
  // |x| <= 2^11: every image code exact in fp16
  if (K <= 0 || K > kMaxK || d.Cout <= 0 || d.Cout % 16 || qx.bits > 12 || qw.bits > 8) return LBT_EINVAL;
  // exact fp32 accumulation: K * max|x| * max|w| <= 2^24
  if ((double)K * ldexp(1.0, qx.bits - 1) * ldexp(1.0, qw.bits - 1) > 16777216.0) return LBT_EINVAL;
  if (d.KH >= 1024 || d.KW >= 1024 || d.Cin >= 1024 || d.PT >= 1024 || d.PL >= 1024) return LBT_EINVAL;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (M <= 0) return LBT_OK;
  if ((int64_t)d.N * d.H * d.W * d.Cin >= ((int64_t)1 << 31) || M * d.Cout >= ((int64_t)1 << 40)) return LBT_EINVAL;
  const int nct = d.Cout >= 64 ? 4 : d.Cout / 16;
  hipStream_t st = (hipStream_t)stream;
  // row tiles (default; LBT_STEM_WIDE_TILES=0 keeps the gather kernel below)
  const char* tenv = getenv("LBT_STEM_WIDE_TILES");
  const int tiles_env = tenv ? atoi(tenv) : 1;
  if (tiles_env && d.Cin <= 4 && d.KW <= 8 && d.KH <= 15 && d.Wo <= kTilePixels && d.SH <= 16 && d.SW <= 16 &&
      !(reinterpret_cast<uintptr_t>(y) & 15)) {
    const int TR = d.Ho < kTilePixels / d.Wo ? d.Ho : kTilePixels / d.Wo;
    const int R = (TR - 1) * d.SH + d.KH, Wimg = (d.Wo - 1) * d.SW + 8, KS = d.KH * 32 + 8;
    const size_t shm = (size_t)nct * 16 * KS * 2 + (size_t)R * Wimg * 8;
    const int64_t ntiles = (int64_t)d.N * ((d.Ho + TR - 1) / TR);
    if (shm <= 65536 && R * Wimg <= kTilePre * kTileThreads && ntiles < 0x7fffffff) {
      // one round of resident workgroups (102 VGPRs: 2 per CU x 256 CUs), every one the same number
      // of tiles (ResNet-50 conv1, B=256: 512 -> 254 us, 768 -> 282, 1024 -> 257, 14336 -> ~590)
      static const int64_t wgs = [] {
        const char* e = getenv("LBT_STEM_WIDE_WGS");
        return (int64_t)(e && atoi(e) > 0 ? atoi(e) : 512);
      }();
      const int64_t per = (ntiles + wgs - 1) / wgs;
      dim3 grid((unsigned)((ntiles + per - 1) / per), (unsigned)((d.Cout + 63) / 64));
      switch (nct) {
#define LBT_STEM_TILES(n_)                                                                                       \
  case n_:                                                                                                     \
    hipLaunchKernelGGL(stem_wide_fwd_tiles_kernel<n_>, grid, dim3(kTileThreads), shm, st, x, w_hwio, d, TR, R, \
                       Wimg, KS, (int)ntiles, qx, qw, y);                                                      \
    break;
        LBT_STEM_TILES(1)
        LBT_STEM_TILES(2)
        LBT_STEM_TILES(3)
        default: LBT_STEM_TILES(4)
#undef LBT_STEM_TILES
      }
      return (int)hipGetLastError();
    }
  }
  const int KP = (K + 31) / 32 * 32;
  const size_t shm = (size_t)nct * 16 * KP * 2 + (size_t)KP * 4;
  dim3 grid((unsigned)((M + kFwdRows - 1) / kFwdRows), (unsigned)((d.Cout + 63) / 64));
  switch (nct) {
    case 1: hipLaunchKernelGGL(stem_wide_fwd_kernel<1>, grid, dim3(kThreads), shm, st, x, w_hwio, d, K, KP, qx, qw, y); break;
    case 2: hipLaunchKernelGGL(stem_wide_fwd_kernel<2>, grid, dim3(kThreads), shm, st, x, w_hwio, d, K, KP, qx, qw, y); break;
    case 3: hipLaunchKernelGGL(stem_wide_fwd_kernel<3>, grid, dim3(kThreads), shm, st, x, w_hwio, d, K, KP, qx, qw, y); break;
    default: hipLaunchKernelGGL(stem_wide_fwd_kernel<4>, grid, dim3(kThreads), shm, st, x, w_hwio, d, K, KP, qx, qw, y); break;
  }
  return (int)hipGetLastError();
}

// slab: int64 [nsplit][K][Cout], fully written (no zeroing needed); nsplit from lbt_stem_wide_nsplit.
extern "C" int lbt_stem_wide_nsplit(lbt_conv_desc d) {
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  // ~2048 pixels per workgroup (>= 2 waves of workgroups on 256 CUs for conv1 at B=32), within
  // the int32 accumulator bound
  int64_t ns = (M + 2047) / 2048;
  if (ns < 1) ns = 1;
  while ((M + ns - 1) / ns > kMaxWgPixels) ++ns;
  return (int)ns;
}

extern "C" int lbt_conv_stem_wide_wgrad(const int16_t* x, int32_t x_bits, const void* g, int32_t g16, lbt_conv_desc d,
                                        int64_t* slab, int32_t nsplit, void* stream) {
  const int K = d.KH * d.KW * d.Cin;
  if (K <= 0 || K > kMaxK || d.Cout <= 0 || d.Cout % 16 || nsplit <= 0) return LBT_EINVAL;
  // fp32 flush bound (128 pixels x max|x| x 255 <= 2^24) and the int32 accumulator bound
  if (x_bits < 1 || x_bits > 9) return LBT_EINVAL;
  if (d.KH >= 1024 || d.KW >= 1024 || d.Cin >= 1024 || d.PT >= 1024 || d.PL >= 1024) return LBT_EINVAL;
  if (d.H >= 32768 || d.W >= 32768 || (int64_t)d.Ho * d.SH >= 32768 || (int64_t)d.Wo * d.SW >= 32768) return LBT_EINVAL;
  const int64_t M = (int64_t)d.N * d.Ho * d.Wo;
  if (M <= 0) return LBT_OK;
  if ((int64_t)d.N * d.H * d.W * d.Cin >= ((int64_t)1 << 31)) return LBT_EINVAL;
  const int64_t per = (M + nsplit - 1) / nsplit;
  if (per > kMaxWgPixels) return LBT_EINVAL;
  const int nct = d.Cout >= 64 ? 4 : d.Cout / 16;
  hipStream_t st = (hipStream_t)stream;
  // the row-chunk kernel where its LDS window fits (LBT_STEM_ROWS=0 at call time: never)
  {
    const char* e = getenv("LBT_STEM_ROWS");
    const int xc = (d.Wo + kRwPx - 1) / kRwPx;
    const int64_t nchunks = (int64_t)d.N * d.Ho * xc;
    const int64_t cper = (nchunks + nsplit - 1) / nsplit;
    if ((!e || atoi(e) != 0) && K <= 16 * kRwMaxKT && d.Cin <= kRwMaxCin && d.KH <= kRwMaxKH &&
        (kRwPx - 1) * d.SW + d.KW <= kRwMaxWC && d.Cout <= 64 && cper * kRwPx <= kMaxWgPixels &&
        d.KH * (((d.Wo < kRwPx ? d.Wo : kRwPx) - 1) * d.SW + d.KW) * d.Cin <= kRwWpt * 64 * kRwMaxKT) {
      // one group of up to 64 channels; LBT_STEM_CG=32 at call time: 32-channel groups on grid.y (half the
      // accumulators, two 10-wave workgroups per CU, but the window staged twice and 12 spilled registers:
      // 1296 vs 762 us at B=256, profiles/r05/stem_probe.txt)
      const char* cgv = getenv("LBT_STEM_CG");
      const int ncg = (d.Cout % 32 == 0 && cgv && atoi(cgv) == 32) ? d.Cout / 32 : 1;
      const int rn = ncg > 1 ? 2 : nct;
#define LBT_STEM_R(G, N)                                                                                  \
  hipLaunchKernelGGL((stem_wgrad_rows_kernel<G, N>), dim3((unsigned)nsplit, (unsigned)ncg), dim3(64 * kRwMaxKT), 0, st, \
                     x, g, d, K, cper, nchunks, xc, slab)
      if (g16) {
        switch (rn) {
          case 1: LBT_STEM_R(true, 1); break;
          case 2: LBT_STEM_R(true, 2); break;
          case 3: LBT_STEM_R(true, 3); break;
          default: LBT_STEM_R(true, 4); break;
        }
      } else {
        switch (rn) {
          case 1: LBT_STEM_R(false, 1); break;
          case 2: LBT_STEM_R(false, 2); break;
          case 3: LBT_STEM_R(false, 3); break;
          default: LBT_STEM_R(false, 4); break;
        }
      }
#undef LBT_STEM_R
      return (int)hipGetLastError();
    }
  }
  dim3 grid((unsigned)nsplit, (unsigned)((K + 63) / 64), (unsigned)((d.Cout + 63) / 64));
#define LBT_STEM_W(G, N) \
  hipLaunchKernelGGL((stem_wide_wgrad_kernel<G, N>), grid, dim3(kThreads), 0, st, x, g, d, K, per, slab)
  if (g16) {
    switch (nct) {
      case 1: LBT_STEM_W(true, 1); break;
      case 2: LBT_STEM_W(true, 2); break;
      case 3: LBT_STEM_W(true, 3); break;
      default: LBT_STEM_W(true, 4); break;
    }
  } else {
    switch (nct) {
      case 1: LBT_STEM_W(false, 1); break;
      case 2: LBT_STEM_W(false, 2); break;
      case 3: LBT_STEM_W(false, 3); break;
      default: LBT_STEM_W(false, 4); break;
    }
  }
#undef LBT_STEM_W
  return (int)hipGetLastError();
}

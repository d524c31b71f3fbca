/*
 * lbt_dfxp.h -- C-ABI of the MI355X (gfx950) dynamic-fixed-point (DFXP) training hot path.
 *
 * Every entry point is stream-ordered (the last argument is a hipStream_t passed as void*),
 * takes caller-owned DEVICE pointers, allocates nothing and never synchronises, so a caller
 * may capture any sequence of calls into a HIP graph. Return value: 0 on success, otherwise
 * a hipError_t code or one of the LBT_E* argument errors below.
 *
 * The reference (freudh/lbt) is TensorFlow-1 Python; it has no native FFI. Each entry point
 * replaces the TF op sequence named in its comment (file:line in the reference tree), i.e.
 * it is what a ctypes / cffi binding of the reference's quantiser and layers would bind
 * (see INTEGRATION.md).
 *
 * Conventions
 *   - Activations / gradients: NHWC, fp32 or integer codes. Weights: HWIO fp32 master copy.
 *   - A DFXP tensor is (integer codes q, shared exponent e): value = q * 2^-e with
 *     e = bits - I - 1, I = "integer_bits" held per quantiser slot in device memory.
 *   - Quantiser slots live in three device arrays owned by the caller:
 *       exps[slot]      int32  integer bits I (dynamic_fixed_point.py:27,34 "integer_bits")
 *       counts[(slot*LBT_NSHARD + shard)*LBT_CSTRIDE + {0,1}]  int32
 *                              #(x*m >= L or x*m < -L), #(x*m >= L/2 or x*m < -L/2)
 *                              (the numerators of overflow_rate, dynamic_fixed_point.py:48-67)
 *       step[0]         uint64 training-step counter (noise counter)
 *   - Stochastic-rounding noise: Philox4x32-10, counter (i>>2, qid, step_lo, step_hi),
 *     key (seed_lo, seed_hi), u = (r[i&3] >> 8) * 2^-24, i = element index modulo
 *     prod(shape[1:]) -- the reference's tf.random_uniform(X.shape[1:]) broadcast over dim 0
 *     (dynamic_fixed_point.py:36).
 */
#ifndef LBT_DFXP_H
#define LBT_DFXP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBT_OK 0
#define LBT_EINVAL 1001  /* unsupported shape / argument combination */

/* Reduction outputs (overflow counters, per-channel integer sums) are SHARDED: a kernel adds
 * its per-workgroup partial into shard (workgroup id % LBT_NSHARD) so that thousands of
 * workgroups never serialise on one address; consumers sum the shards.                  */
#define LBT_NSHARD 32
/* int32 stride between the overflow-counter shards of one slot: one 128-byte line per shard,
 * so concurrent workgroups' counter atomics never share a cache line.                    */
#define LBT_CSTRIDE 32

/* Output encodings of a quantiser. */
enum {
  LBT_OUT_I8 = 0,     /* signed codes, bits <= 8                                     */
  LBT_OUT_U8OFF = 1,  /* unsigned 9-bit codes q in [0,255] stored as int8 (q - 128)  */
  LBT_OUT_I16 = 2,    /* signed codes, bits <= 16                                    */
  LBT_OUT_F32 = 3     /* dequantised fake-quant value q * 2^-e (the reference's STE output) */
};

/* One quantiser: where its exponent / counters live and how it rounds. */
typedef struct lbt_qdesc {
  const int32_t* exps;   /* device [slots]                                   */
  int32_t* counts;       /* device [slots][LBT_NSHARD][LBT_CSTRIDE]; NULL = no stats */
  const uint64_t* step;  /* device [1]                                       */
  uint64_t seed;         /* noise key                                        */
  uint32_t qid;          /* noise stream id (crc32 of the range variable)    */
  int32_t slot;
  int32_t bits;          /* total bits incl. sign, 2..16                     */
  int32_t stochastic;    /* 1: floor(x*m + u)  0: round-half-even(x*m)       */
  const float* noise;    /* NULL: Philox inline. Else this step's noise table u[i] for
                            i < ceil(inner/4)*4, filled by lbt_dfxp_noise_fill (the noise
                            depends only on (seed, qid, step, i mod inner)).  */
} lbt_qdesc;

/* Convolution geometry, TF padding already resolved into (top,bottom,left,right). */
typedef struct lbt_conv_desc {
  int32_t N, H, W, Cin, Cout, KH, KW, SH, SW, PT, PB, PL, PR, Ho, Wo;
} lbt_conv_desc;

/* ---------------------------------------------------------------- quantiser ---------- */

/* weight_quantization + the overflow statistics of update_range
 * (dynamic_fixed_point.py:4-45 / :48-67).  x is [rows, inner] fp32 (inner = prod(shape[1:])).
 * out is written in `out_kind` encoding, same element order as x.  If chsum != NULL the
 * per-channel integer sums S1[c] = sum q, S2[c] = sum q^2 over all elements with channel
 * c = index % C are ADDED to the sharded int64 buffer chsum[LBT_NSHARD][2C] (S1 at [0,C),
 * S2 at [C,2C) of a shard).  All "chsum"/"sums" buffers below use that sharded layout.   */
int lbt_dfxp_quantize(const float* x, void* out, int out_kind, int64_t rows, int64_t inner,
                      lbt_qdesc q, int64_t* chsum, int32_t C, void* stream);

/* update_range for every slot (dynamic_fixed_point.py:70-94):
 *   c = sum over shards; r1 = c1/n[s], r2 = c2/n[s] (fp32), delta = r1 > t ? +1 : (r2 <= t ? -1 : 0)
 *   I <- clamp(I + delta, bits-31, bits-1); counts zeroed; step[0] += 1.
 * Slots with nelem <= 0 (not fed this step) are left untouched.                          */
int lbt_dfxp_range_update(int32_t* exps, int32_t* counts, const int32_t* bits, const float* target,
                          const float* nelem, int32_t nslots, uint64_t* step, void* stream);

/* Data-parallel form of the range update (the counters must be summed over ranks first).
 * counts_fold sums each slot's shards, zeroes them and writes the totals EXACTLY as fp32
 * (so they can ride in the gradient all-reduce buffer):
 *   folded[4s+0] = c1 >> 12, folded[4s+1] = c1 & 4095, folded[4s+2] = c2 >> 12, [4s+3] = c2 & 4095
 * (any rank count < 2^12 keeps every partial sum of the all-reduce below 2^24).
 * range_update_folded applies the rule above to c = 4096*hi + lo of the (reduced) buffer.  */
int lbt_dfxp_counts_fold(int32_t* counts, int32_t nslots, float* folded, void* stream);
int lbt_dfxp_range_update_folded(int32_t* exps, const float* folded, const int32_t* bits, const float* target,
                                 const float* nelem, int32_t nslots, uint64_t* step, void* stream);

/* Per-step noise tables. Job j writes u[i] = Philox(i>>2, qid, step, seed)[i&3] >> 8 * 2^-24 for
 * i < ceil(n/4)*4 into out (16-byte aligned), reading *step on the device; one launch fills every
 * table (grid.y = job). A qdesc whose .noise points at its table then loads 16 B per 4 codes
 * instead of running Philox per element (dynamic_fixed_point.py:36).                      */
typedef struct lbt_njob {
  const uint64_t* step;
  uint64_t seed;
  uint32_t qid;
  int32_t pad;
  int64_t n;
  float* out;
} lbt_njob;
int lbt_dfxp_noise_fill(const lbt_njob* jobs, int32_t njobs, int64_t max_n, int64_t* zero, int64_t nzero,
                        void* stream);  /* also zeroes zero[0, nzero) (the step's sums arena) */

/* Quantise a conv / dense weight (HWIO fp32, noise over shape[1:] = [KW,Cin,Cout]) into the
 * layouts the GEMM kernels consume (any output may be NULL):
 *   w_hwio  int8 [KH][KW][Cin][Cout]       (generic kernels)
 *   wf      int8 [Cout][ksf*16]            fwd B operand, k = (tap, ci), zero padded to ksf*16
 *   wd      int8 [Cin][ksd*16]             dgrad B operand, k = (tap, co)
 *   colsum  int32 [Cout]  sum_k w[k][co]   (offset-input correction)                      */
int lbt_dfxp_quantize_weight(const float* w, int32_t KH, int32_t KW, int32_t Cin, int32_t Cout,
                             lbt_qdesc q, int8_t* w_hwio, int8_t* wf, int32_t ksf, int8_t* wd,
                             int32_t ksd, int32_t* colsum, void* stream);

/* ---------------------------------------------------------------- integer GEMMs ------ */

/* Conv2d_q forward y = conv(Xq, Wq) (dynamic_fixed_point.py:287-291, tf.nn.conv2d) as an
 * int8 implicit GEMM on v_mfma_i32_16x16x64_i8.  xq: NHWC int8 codes (x_u8off: unsigned
 * 9-bit offset encoding, else signed 8-bit); wf/wcolsum from lbt_dfxp_quantize_weight.
 * Epilogue: acc -> fp32 * 2^-(ex+ew); written to y (fp32 NHWC) if y != NULL and/or
 * quantised with qout into yq (int8 NHWC) with per-channel sums into ychsum; a stochastic
 * qout must carry its noise table (qout.noise, lbt_dfxp_noise_fill), else LBT_EINVAL.
 * Requires Cin % 16 == 0 and Cout % 16 == 0.                                               */
int lbt_conv_fwd_i8(const int8_t* xq, int32_t x_u8off, const int8_t* wf, int32_t ksf,
                    const int32_t* wcolsum, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw,
                    float* y, int8_t* yq, lbt_qdesc qout, int64_t* ychsum, void* stream);

/* Two lbt_conv_fwd_i8 calls in ONE launch: a projection ResidualBlock_q's first conv (3x3, stride
 * 2; dynamic_fixed_point.py:772-795 -> 860) and its shortcut conv (1x1, stride 2; :831-846 -> 861)
 * read the same input codes and produce same-shaped outputs. Each job is exactly the arguments of
 * lbt_conv_fwd_i8 (w4: wf is the packed 4-bit image, as lbt_conv_fwd_i8w4); both jobs need equal
 * Cin, Cout, N*Ho*Wo and w4, with (Cin, Cout) in {(16,32), (32,64)}, else LBT_EINVAL. Results
 * are bit-identical to the two single calls.                                                    */
typedef struct lbt_conv_fwd_job {
  const int8_t* xq; int32_t x_u8off; int32_t w4; const int8_t* wf; int32_t ksf; const int32_t* wcolsum;
  lbt_conv_desc d; lbt_qdesc qx; lbt_qdesc qw; float* y; int8_t* yq; lbt_qdesc qout; int64_t* ychsum;
} lbt_conv_fwd_job;
int lbt_conv_fwd_pair_i8(const lbt_conv_fwd_job* j0, const lbt_conv_fwd_job* j1, void* stream);

/* Conv2d_q backward dX = tf.gradients(y, X, gradq) (dynamic_fixed_point.py:305): int8
 * implicit GEMM over (tap, co) of the quantised grad.  dx (fp32 NHWC [N,H,W,Cin]) =
 * acc * 2^-(eg+ew) (+ add_src[e] if add_src != NULL).  Requires Cin%16 == 0, Cout%16 == 0. */
int lbt_conv_dgrad_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                      lbt_qdesc qg, lbt_qdesc qw, float* dx, const float* add_src, void* stream);
/* Wide layers (ResNet-50 shapes): LDS-tiled int8-MFMA implicit GEMM, 128 x 128 workgroup tiles,
 * k-blocks of one tap x 64 channels (gathered channels % 64 == 0, output channels % 16 == 0),
 * same weight images and the same results bit for bit as the generic kernels.
 * fwd a_kind: 0 int8 codes, 1 offset int8 (q - 128), 2 int16 codes (9..16-bit; split into two
 * int8 MFMA passes, a = 256 hi + lo' + 128). dgrad g_i16: int16 gradient codes (config 4).
 * colsum is unused (the kernel forms sum_k W itself) and may be NULL.                        */
int lbt_conv_fwd_igemm(const void* xq, int32_t a_kind, const int8_t* wf, int32_t ksf, const int32_t* colsum,
                       lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y, void* stream);
int lbt_conv_dgrad_igemm(const void* gq, int32_t g_i16, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                         lbt_qdesc qg, lbt_qdesc qw, float* dx, const float* add_src, void* stream);
/* Wide-layer weight gradient: x offset int8 codes (post-ReLU 9-bit, q - 128), g int8 or int16
 * (g_i16) codes; Cin, Cout % 64 == 0; adds exact int64 partials into a ZEROED slab
 * [nshard][KH*KW*Cin][Cout] (pixel split b -> shard b % nshard; reduce: lbt_conv_wgrad_reduce64). */
/* Wide forward whose epilogue is the consuming Normalization_q's input quantiser (Conv2d_q.forward
 * :291 then Normalization_q :584-588): int8 codes yq [N*Ho*Wo][Cout] of qout (<= 8 bits), its
 * overflow counters and exact per-channel sums chsum[NSHARD][2*Cout] (sum q, sum q^2) -- the
 * same as lbt_conv_fwd_igemm followed by lbt_dfxp_quantize(y, qout, chsum), without y.
 * a_kind 0 / 1 (int8 / offset int8 codes).                                                   */
int lbt_conv_fwd_igemm_q(const void* xq, int32_t a_kind, const int8_t* wf, int32_t ksf, lbt_conv_desc d, lbt_qdesc qx,
                         lbt_qdesc qw, int8_t* yq, lbt_qdesc qout, int64_t* chsum, void* stream);
/* The same fwd / dgrad with a caller-owned workspace: GEMMs whose row tiles leave the 256 CUs
 * short of work split K over workgroups (exact int32 partials + one reduce launch, bit-identical);
 * lbt_igemm_workspace_bytes(d, mode 0 fwd | 1 dgrad, a16) = the bytes needed (0: no split).   */
int64_t lbt_igemm_workspace_bytes(lbt_conv_desc d, int32_t mode, int32_t a16);
int lbt_conv_fwd_igemm_ws(const void* xq, int32_t a_kind, const int8_t* wf, int32_t ksf, const int32_t* colsum,
                          lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y, void* ws, int64_t ws_bytes,
                          void* stream);
int lbt_conv_dgrad_igemm_ws(const void* gq, int32_t g_i16, const int8_t* wd, int32_t ksd, lbt_conv_desc d,
                            lbt_qdesc qg, lbt_qdesc qw, float* dx, const float* add_src, void* ws, int64_t ws_bytes,
                            void* stream);
/* Selection of the 256-row x BN-column LDS-DMA GEMM that the fwd / dgrad calls above use for
 * large GEMMs (8 waves, S-stage global->LDS DMA ring; bit-identical results to the 128-row kernel
 * and the generic ones). Process-wide, read by every call made after a set (not captured into a
 * graph already recorded). big: 0 never, 1 when the GEMM has >= min_tiles 256-row tiles at the
 * chosen width and is not split-K / a strided dgrad parity class; max_bn: widest column tile
 * (64, 128, or 256 = A8 without the quantising epilogue); stages 2..4 (A16: 2 or 3).
 * Defaults: {1, 200, 2, 128}, or the LBT_IGEMM_BIG / _MIN / _S / _BN256 environment at first use.
 * halo: 3x3 / stride-1 / pad-1 GEMMs (fwd, unit-stride dgrad, W <= 63) stage one A window per
 * 64-channel block for all 9 taps; bit 0: int8 codes, bit 1: 16-bit codes (default 1, LBT_IGEMM_HALO).
 * fwdq_perm: lbt_conv_fwd_igemm_q (and lbt_conv_dgrad_igemm_bna) on the 256-row kernels tile rows 16
 * pixels x 16 samples. 1: the quantiser / pass A runs from an LDS-staged tile, one noise draw per
 * position per 8 samples; 2 (default, LBT_FWDQ_PERM): the same, except the one-k-block forward GEMMs
 * (1x1, K = 64), which take a persistent kernel (one workgroup per CU, an LDS-DMA ring across its row
 * tiles, the quantiser on the accumulators, the tile's noise table DMA'd with its operands; table noise
 * or nearest rounding, 256 % (Cout / column tile) == 0); > 2: the persistent forward and dgrad + pass A
 * kernels wherever they apply, on that many workgroups (tests; slower on the longer-K shapes);
 * 0: row-major tiles. stages 3 / 4 set the persistent ring's depth (2: LBT_FWDQ_S, default 4).
 * launches (get only; set ignores it): 256-row GEMM launches issued by this process so far.      */
typedef struct lbt_igemm_tuning {
  int32_t big, min_tiles, stages, max_bn, halo, fwdq_perm;
  int64_t launches;
} lbt_igemm_tuning;
int lbt_igemm_get_tuning(lbt_igemm_tuning* out);
int lbt_igemm_set_tuning(const lbt_igemm_tuning* t);
/* A 16-bit-gradient dgrad (lbt_conv_dgrad_igemm_ws, g_i16 = 1, no add_src) whose dx is the incoming
 * gradient of a ReLU_q + BN (Rescale_q :686-691, Normalization_q :620-623): ResidualBottleneck_q's bn1 /
 * bn2 behind conv-2 / conv-3. Produces what lbt_bn_bwd_a_wide_masked(dx, mask_r = 1, ...) would from
 * that dx -- the G codes, the four channel sums, both quantisers' overflow counters -- and, when the
 * 256-row GEMM takes the dgrad (unit stride, enough tiles) and each stochastic quantiser carries its
 * noise table (lbt_qdesc.noise over inner = H*W*Cin), evaluates it in the GEMM epilogue: no fp32 dx
 * is stored or read. Otherwise dx (scratch, N*H*W*Cin floats, required) is stored and pass A runs
 * after. Bit-identical either way. bna.sums accumulates (zero it per step); qrg / qng <= 16 bits.
 * Reference: Conv2d_q.backward :299-310 followed by ReLU_q / Rescale_q / Normalization_q backward.   */
typedef struct lbt_dgrad_bna {
  lbt_qdesc qr;          /* Rescale_q input quantiser: the ReLU mask ((float)R * s_qr) * gb[c] + gb[C+c] > 0 */
  const int8_t* R;       /* Rescale_q input codes [rows][Cin]                                     */
  const float* gb;       /* [gamma_q | beta_q] dequantised (2 Cin); gamma_q also scales the rescale  */
  lbt_qdesc qrg;         /* Rescale_q gradient quantiser                                           */
  lbt_qdesc qng;         /* Normalization_q gradient quantiser                                      */
  const int8_t* qn;      /* Normalization_q input codes [rows][Cin]                                */
  int16_t* gout;         /* G codes out [rows][Cin]                                                */
  int64_t* sums;         /* [LBT_NSHARD][4 Cin]: S(G2 R), S(G2), S(G), S(G qn) added in          */
} lbt_dgrad_bna;
int lbt_conv_dgrad_igemm_bna(const int16_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                             lbt_qdesc qw, const lbt_dgrad_bna* bna, float* dx, void* ws, int64_t ws_bytes,
                             void* stream);
/* The same for the gradient ENTERING a bottleneck block from the next one (ResidualBlock_q.backward
 * :865-869 + ReLU_q): dx of the next block's conv-1 plus g2 (the next block's other branch),
 * masked by y_bits (lbt_chain_fwd.ybits of this block's output), optionally stored (gmask_out: the
 * identity shortcut's gradient), then pass A of each BN it feeds -- bn3, and the projection
 * shortcut's BN when nbn = 2 -- as lbt_bn_bwd_a_wide_masked(dx, g2, y_bits, gmask_out, ...) per BN.
 * Fused into the dgrad epilogue on the same conditions as lbt_conv_dgrad_igemm_bna; else through dx.  */
typedef struct lbt_bna_bn {
  lbt_qdesc qrg; const int8_t* R; const float* gamma_q;   /* Rescale_q: grad quantiser, X codes, gamma_q */
  lbt_qdesc qng; const int8_t* qn;                        /* Normalization_q: grad quantiser, X codes    */
  int16_t* gout; int64_t* sums;                           /* G codes, [LBT_NSHARD][4 Cin] sums          */
} lbt_bna_bn;
typedef struct lbt_dgrad_bn3 {
  const float* g2;        /* [rows][Cin] second summand (required)                 */
  const uint8_t* y_bits;  /* [rows * Cin / 4] ReLU mask, bit k of byte e/4 = channel quad k */
  float* gmask_out;       /* optional [rows][Cin]                                   */
  int32_t nbn, pad;       /* 1 or 2                                                 */
  lbt_bna_bn bn[2];
} lbt_dgrad_bn3;
int lbt_conv_dgrad_igemm_bn3(const int16_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                             lbt_qdesc qw, const lbt_dgrad_bn3* b, float* dx, void* ws, int64_t ws_bytes,
                             void* stream);
int lbt_conv_wgrad_igemm(const int8_t* xq, const void* gq, int32_t g_i16, lbt_conv_desc d, int64_t* slab,
                         int32_t nsplit, int32_t nshard, void* stream);
/* ... storing one partial per pixel split: slab [nsplit][KH*KW*Cin][Cout] is fully WRITTEN (no
 * zeroing, no atomics); (N*Ho*Wo)/nsplit <= 2^19 pixels. Reduce with lbt_conv_wgrad_reduce64. */
int lbt_conv_wgrad_igemm_store(const int8_t* xq, const void* gq, int32_t g_i16, lbt_conv_desc d, int64_t* slab,
                               int32_t nsplit, void* stream);

/* 4-bit weights (W 4-bit / A 8-bit): the same GEMMs with the weight
 * image packed two signed 4-bit codes per byte (lbt_pack_int4 of lbt_dfxp_quantize_weight's wf /
 * wd at qw.bits <= 4; ksf / ksd still count 16-element k-slices, 8 bytes each). gfx950 has no
 * int4 MFMA: the kernels unpack to int8 in registers -- half the weight bytes from HBM.        */
int lbt_conv_fwd_i8w4(const int8_t* xq, int32_t x_u8off, const uint8_t* wf4, int32_t ksf, const int32_t* wcolsum,
                      lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw, float* y, int8_t* yq, lbt_qdesc qout,
                      int64_t* ychsum, void* stream);
int lbt_conv_dgrad_i8w4(const int8_t* gq, const uint8_t* wd4, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg, lbt_qdesc qw,
                        float* dx, const float* add_src, void* stream);
/* dst[i] = (src[2i] & 15) | (src[2i+1] << 4), n even: pack signed 4-bit codes held in int8.   */
int lbt_pack_int4(const int8_t* src, uint8_t* dst, int64_t n, void* stream);

/* Conv2d_q backward dW = tf.gradients(y, W, gradq) (dynamic_fixed_point.py:302), pass 1:
 * the pixels are split into `nsplit` ranges (x Cout/16 column slices x taps = the grid); the
 * exact int32 partial of range s is ADDED into shard s % nshard of slab[nshard][KH*KW][Cin][Cout],
 * which the caller zeroes (integer atomics: order-independent). Requires every shard to cover
 * <= 65536 pixels (int32 exactness). x_u8off: xq in the unsigned-9-bit offset encoding; the
 * offset is undone in pass 2 (lbt_conv_wgrad_reduce, nsplit = nshard).                       */
int lbt_conv_wgrad_i8(const int8_t* xq, int32_t x_u8off, const int8_t* gq, lbt_conv_desc d,
                      int32_t* slab, int32_t nsplit, int32_t nshard, void* stream);

/* pass 2: dW = float(sum_split slab + 128*x_u8off*gcolsum[co]) * 2^-(ex+eg) + wd2 * W,
 * written HWIO into dw (wd2 = 2*weight_decay as fp32, the "+ 2*wd*W" of :302).
 * gcolsum is the sharded per-channel sum buffer [LBT_NSHARD][2*Cout] of the grad codes.   */
int lbt_conv_wgrad_reduce(const int32_t* slab, int32_t nsplit, int32_t K, int32_t Cout,
                          int32_t x_u8off, const int64_t* gcolsum, lbt_qdesc qx, lbt_qdesc qg,
                          const float* w, float wd2, float* dw, void* stream);

/* Generic (any-shape) integer conv on the VALU, for signed 9-bit inputs and channel counts
 * that are not multiples of 16 (conv1 3->16, Dense_q as a 1x1 conv).  x codes are int16 when
 * x_i16 != 0, else int8; w is int8 HWIO; g is int8.                                        */
int lbt_conv_fwd_generic(const void* xq, int32_t x_i16, const int8_t* w_hwio, lbt_conv_desc d,
                         lbt_qdesc qx, lbt_qdesc qw, float* y, void* stream);
int lbt_conv_dgrad_generic(const int8_t* gq, const int8_t* w_hwio, lbt_conv_desc d,
                           lbt_qdesc qg, lbt_qdesc qw, float* dx, const float* add_src, void* stream);
int lbt_conv_wgrad_generic(const void* xq, int32_t x_i16, const int8_t* gq, lbt_conv_desc d,
                           int32_t* slab, int32_t nsplit, void* stream);
/* 9..16-bit gradient codes ("16-bit grad DFP"): the same
 * generic dgrad / wgrad with int16 codes and int64 accumulation (int16 x int8 sums overflow
 * int32), an int64 wgrad slab [nsplit][K][Cout], and its reduce (same dequant + 2*wd*W formula
 * as lbt_conv_wgrad_reduce, x_u8off = 0).                                                    */
int lbt_conv_dgrad_generic16(const int16_t* gq, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qg, lbt_qdesc qw,
                             float* dx, const float* add_src, void* stream);
int lbt_conv_wgrad_generic16(const void* xq, int32_t x_i16, const int16_t* gq, lbt_conv_desc d, int64_t* slab,
                             int32_t nsplit, void* stream);
int lbt_conv_wgrad_reduce64(const int64_t* slab, int32_t nsplit, int32_t K, int32_t Cout, lbt_qdesc qx, lbt_qdesc qg,
                            const float* w, float wd2, float* dw, void* stream);
/* Many lbt_conv_wgrad_reduce64 in ONE launch (dynamic_fixed_point.py:302, each conv's dW = dequant(sum) +
 * 2 wd W): job k owns the 64-output blocks [first_block, first_block + ceil(K*Cout/64)), jobs in
 * ascending first_block from 0, nblocks the total. The layer-wise Trainer defers every conv's reduce of
 * the backward into one such launch at its end (each job's slab is the layer's own). Same int64 totals and
 * the same fp32 epilogue as the single-job launch: bit-identical. Job array in device memory.            */
typedef struct lbt_r64job {
  const int64_t* slab; int32_t nsplit, K, Cout, first_block;
  lbt_qdesc qx, qg; const float* w; float wd2; float* dw;
} lbt_r64job;
int lbt_conv_wgrad_reduce64_many(const lbt_r64job* jobs, int32_t njobs, int32_t nblocks, void* stream);

/* Stem convolution (conv1 of the CIFAR ResNets, models.py:387-391): input = the image's SIGNED
 * (bits+1)-bit codes as int16 (|x| <= 2048), patch K = KH*KW*Cin <= 32, Cout % 16 == 0.
 * Runs on fp16 MFMA, which is exact here (every code and product is an fp16/fp32-exact
 * integer and every partial sum < 2^24), i.e. bit-identical to lbt_conv_fwd_generic /
 * lbt_conv_wgrad_generic (dynamic_fixed_point.py:287-305).
 * fwd: exactly one of y (fp32, Cout <= 128) / yq (int8 codes of qout, + counters, + optional
 *      sharded channel sums ychsum; a stochastic qout needs its noise table, as
 *      lbt_conv_fwd_i8) is non-NULL.
 * wgrad: ADDS exact int32 partials into slab[nshard][K][Cout] (zeroed by the caller; workgroup w of
 *      LBT_STEM_WG_PIXELS pixels adds into shard w % nshard), Cout <= 64; requires
 *      ceil(ceil(N*Ho*Wo / LBT_STEM_WG_PIXELS) / nshard) <= 31 (int32 exactness). Finish with
 *      lbt_conv_wgrad_reduce(_many) over nsplit = nshard (x_u8off = 0, gcolsum = NULL).    */
#define LBT_STEM_WG_PIXELS 256
int lbt_conv_stem_fwd(const int16_t* x, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw,
                      float* y, int8_t* yq, lbt_qdesc qout, int64_t* ychsum, void* stream);
int lbt_conv_stem_wgrad(const int16_t* x, const int8_t* gq, lbt_conv_desc d, int32_t* slab, int32_t nshard,
                        void* stream);

/* The ImageNet ResNet's conv1 (7x7/2, 3 -> 64; dynamic_fixed_point.py:287-305)
 * on v_mfma_f32_16x16x32_f16 (stem_wide.hip): signed <= 9-bit int16 image codes, K = KH*KW*Cin
 * <= 480 patch elements, Cout % 16 == 0; exact (integer partial sums < 2^24), bit-identical to
 * lbt_conv_fwd_generic / lbt_conv_wgrad_generic16.
 * fwd: y fp32 [N*Ho*Wo][Cout]; rejects K * 2^(qx.bits-1) * 2^(qw.bits-1) > 2^24.
 * wgrad: g = int8 (g16 = 0) or int16 (g16 = 1, 9..16-bit gradient codes) [N*Ho*Wo][Cout]; WRITES
 *      every element of the int64 slab[nsplit][K][Cout] (nsplit = lbt_stem_wide_nsplit(d)); finish
 *      with lbt_conv_wgrad_reduce64. x_bits <= 9.                                              */
int lbt_conv_stem_wide_fwd(const int16_t* x, const int8_t* w_hwio, lbt_conv_desc d, lbt_qdesc qx, lbt_qdesc qw,
                           float* y, void* stream);
int lbt_stem_wide_nsplit(lbt_conv_desc d);  /* returns nsplit (> 0) */
int lbt_conv_stem_wide_wgrad(const int16_t* x, int32_t x_bits, const void* g, int32_t g16, lbt_conv_desc d,
                             int64_t* slab, int32_t nsplit, void* stream);

/* ---------------------------------------------------------------- batch norm -------- */

/* The statistics of one Normalization_q (dynamic_fixed_point.py:584-616): its input codes q
 * (quantiser qn), the sharded integer sums S1 = sum q, S2 = sum q^2 per channel (chsum,
 * [LBT_NSHARD][2C], produced by the quantiser or by the conv epilogue), n elements/channel.
 * Moments (biased, as tf.nn.moments): mu = S1*s/n, var = S2*s^2/n - mu^2 in double,
 * sigma = sqrtf((float)var + eps).  The first workgroup writes ms = [mu[C], sigma[C]] and,
 * if run_mean != NULL, the running averages avg = momentum*avg + one_minus_momentum*x
 * (:601-612).
 * frozen != 0: the testing branch of the tf.cond (:590-600, set_testing, models.py:15): mu and
 * var are the running averages (chsum unused), sigma = sqrtf(run_var + eps), nothing updated.
 * ms_in != 0 (lbt_bn_chain_fwd only): ms already holds this step's [mu | sigma] (lbt_bn_moments ran
 * on this descriptor): the chain reads its channels' two floats instead of reducing the sums in
 * every workgroup, and updates nothing. Either every normalising branch of a chain sets ms_in or
 * none does (a mixed two-branch chain returns LBT_EINVAL).                                        */
typedef struct lbt_bn_norm {
  const int8_t* q; lbt_qdesc qn; const int64_t* chsum; int64_t n;
  float eps, momentum, one_minus_momentum;
  float* ms; float* run_mean; float* run_var;
  int32_t frozen, ms_in;
} lbt_bn_norm;
/* The moments above, once: ms = [mu | sigma] and the running averages (the first-workgroup writes of
 * the chains), one thread per channel. Bit-identical to what the chains compute.                  */
int lbt_bn_moments(const lbt_bn_norm* nrm, int32_t C, void* stream);

/* One branch of the forward element chain:
 *   v = xin[e]                          if nrm.q == NULL
 *     = ((float)q*s - mu) / sigma       else                          (Normalization_q :616)
 *   if qr.bits: R = Q(v, qr) -> rout; v = ((float)R*sr)*gb[c] + gb[C+c]  (Rescale_q :677-683)
 * gb = [gamma_q[C], beta_q[C]] dequantised (lbt_dfxp_quantize with LBT_OUT_F32).           */
typedef struct lbt_chain_branch {
  lbt_bn_norm nrm; const float* xin;
  lbt_qdesc qr; int8_t* rout; const float* gb;
} lbt_chain_branch;

/* Forward element chain over [rows, inner] (inner = H*W*C, channel = index % C):
 *   v = b1 (+ b2 if has_b2) (+ res[e] if res) ; if relu: v = max(0, v)
 *   (ResidualBlock_q :858-863: relu(y1 + y2))
 *   y = v (fp32, if y != NULL); o1 = Q(v, qo1) and o2 = Q(v, qo2) in o*_kind if != NULL
 *   (the next layers' input quantisers, e.g. Conv2d_q X at bits+1 in LBT_OUT_U8OFF).
 *   ybits (optional, C % 4 == 0, only together with y -- else LBT_EINVAL): ybits[e / 4] bit k =
 *   (v[e + k] > 0) for every channel quad e = 4j -- the ReLU mask of y in 1/32 of y's bytes
 *   (lbt_bn_bwd_a_wide_masked's y_bits).                                                          */
typedef struct lbt_chain_fwd {
  lbt_chain_branch b1, b2; int32_t has_b2;
  const float* res; int32_t relu;
  float* y;
  void* o1; int32_t o1_kind; lbt_qdesc qo1;
  void* o2; int32_t o2_kind; lbt_qdesc qo2;
  int64_t rows, inner; int32_t C;
  uint8_t* ybits;
} lbt_chain_fwd;
int lbt_bn_chain_fwd(const lbt_chain_fwd* a, void* stream);

/* Backward pass A of one BN (Rescale_q.backward :686-691, then the first half of
 * Normalization_q.backward :620-623) on the masked incoming gradient g':
 *   if qrg.bits: G2 = Q(g', qrg); sums[0:C) += G2*R, sums[C:2C) += G2; d = ((float)G2*sg2)*gamma_q
 *   else         d = g'
 *   if qng.bits: G = Q(d, qng) -> gout (int8); sums[2C:3C) += G, sums[3C:4C) += G*qn_codes
 *   else         dout = d (fp32)
 * sums is sharded [LBT_NSHARD][4C].                                                         */
typedef struct lbt_bwd_branch {
  lbt_qdesc qrg; const int8_t* R; lbt_qdesc qr; const float* gb;
  lbt_qdesc qng; const int8_t* qn_codes;
  int8_t* gout; float* dout; int64_t* sums;
} lbt_bwd_branch;

/* g' = g * mask, mask = (y_mask[e] > 0) if y_mask (ReLU_q backward, TF _MaximumGrad), or the
 * recomputed branch-1 Rescale_q output ((float)R*sr*gamma_q + beta_q > 0) if mask_from_r,
 * else 1.  gmask_out = g' (the identity-shortcut gradient) if != NULL.  Both branches see
 * the same g' (ResidualBlock_q.backward :865-869).                                         */
typedef struct lbt_chain_bwd_a {
  const float* g; const float* y_mask; int32_t mask_from_r;
  float* gmask_out;
  lbt_bwd_branch b1, b2; int32_t has_b2;
  int64_t rows, inner; int32_t C;
} lbt_chain_bwd_a;
int lbt_bn_chain_bwd_a(const lbt_chain_bwd_a* a, void* stream);

/* Conv2d_q backward dX (as lbt_conv_dgrad_i8) fused with the pass A that consumes it: the
 * dgrad output is never written; each output element e of [N,H,W,Cin] enters chain a as
 * g[e] = dx[e] (+ add_src[e], the residual gradient, if add_src != NULL), with a->g ignored
 * and a->rows = N, a->inner = H*W*Cin, a->C = Cin. Bit-identical to lbt_conv_dgrad_i8 followed
 * by lbt_bn_chain_bwd_a. Supported chains (else LBT_EINVAL -- run the pair): 1 or 2 branches,
 * each with both (stochastic, noise-table) quantisers, int8 G codes and sums; ReLU mask from
 * y_mask or from branch-1 R; optional gmask_out.                                          */
int lbt_conv_dgrad_chain_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                            lbt_qdesc qw, const float* add_src, const lbt_chain_bwd_a* a, void* stream);

/* A projection ResidualBlock_q's input gradient in one launch: the 3x3/2 conv's dgrad (gq, wd,
 * d, qg, qw) plus the 1x1/2 shortcut conv's (gq2, wd2, d2, qg2, qw2; dynamic_fixed_point.py:866-869,
 * each Conv2d_q.backward :305) summed as fp32 dx + dx2, then pass A of a (as
 * lbt_conv_dgrad_chain_i8). Bit-identical to lbt_conv_dgrad_i8(gq2 ...) into a buffer followed by
 * lbt_conv_dgrad_chain_i8(gq ..., add_src = that buffer). Both descriptors must share N, H, W, Cin,
 * Cout, Ho, Wo with Cout = 2 Cin (16 -> 32, 32 -> 64); w4: wd / wd2 are packed 4-bit images. */
int lbt_conv_dgrad2_chain_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                             lbt_qdesc qw, const int8_t* gq2, const int8_t* wd2, int32_t ksd2,
                             lbt_conv_desc d2, lbt_qdesc qg2, lbt_qdesc qw2, int32_t w4,
                             const lbt_chain_bwd_a* a, void* stream);
/* ... with the 4-bit packed weight image (see lbt_conv_fwd_i8w4). */
int lbt_conv_dgrad_chain_i8w4(const int8_t* gq, const uint8_t* wd4, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                              lbt_qdesc qw, const float* add_src, const lbt_chain_bwd_a* a, void* stream);
/* lbt_conv_dgrad_chain_i8 and lbt_conv_wgrad_i8(xq, x_u8off, gq, d, slab, nsplit, nshard) of the
 * SAME conv in ONE launch (the two read the same gradient codes and are independent): the
 * workgroups of the wgrad grid come first, then the dgrad tiles. Results identical to the two
 * separate calls. (Conv2d_q.backward dynamic_fixed_point.py:302-305 -- dW and dX of one layer.) */
int lbt_conv_dgrad_chain_wgrad_i8(const int8_t* gq, const int8_t* wd, int32_t ksd, lbt_conv_desc d, lbt_qdesc qg,
                                  lbt_qdesc qw, const float* add_src, const lbt_chain_bwd_a* a, const int8_t* xq,
                                  int32_t x_u8off, int32_t* slab, int32_t nsplit, int32_t nshard, void* stream);
int lbt_conv_dgrad_chain_wgrad_i8w4(const int8_t* gq, const uint8_t* wd4, int32_t ksd, lbt_conv_desc d,
                                    lbt_qdesc qg, lbt_qdesc qw, const float* add_src, const lbt_chain_bwd_a* a,
                                    const int8_t* xq, int32_t x_u8off, int32_t* slab, int32_t nsplit,
                                    int32_t nshard, void* stream);

/* Pass B (the rest of Normalization_q.backward): with SG = sum G, SGQ = sum G*q from pass A,
 *   mg = sg*SG/n, mgx = sg*(s*SGQ - mu*SG)/(n*sigma)   (double -> fp32)
 *   dx = (((float)G*sg - mg) - xhat*mgx) / sigma,  xhat = ((float)q*s - mu)/sigma
 * Outputs dx (fp32) if != NULL and/or gq = Q(dx, qo) (int8, the next Conv2d_q grad
 * quantiser) with sharded per-channel sums of gq into gcolsum [LBT_NSHARD][2C].           */
typedef struct lbt_chain_bwd_b {
  const int8_t* G; lbt_qdesc qng; const int8_t* qn_codes; lbt_qdesc qn; const float* ms;
  const int64_t* sums; int64_t n;
  float* dx; int8_t* gq; lbt_qdesc qo; int64_t* gcolsum;
  int64_t rows, inner; int32_t C;
} lbt_chain_bwd_b;
int lbt_bn_chain_bwd_b(const lbt_chain_bwd_b* a, void* stream);
/* The stem's whole backward in one launch (replaces lbt_bn_chain_bwd_b + lbt_conv_stem_wgrad of the
 * fused plan; dynamic_fixed_point.py:620-623 pass B of the stem BN, :299-302 conv1's quantised
 * gradient and dW): pass B of b (C = 16, 8-bit qo, no dx / gcolsum; b->gq optional -- the codes are
 * only written when it is non-NULL) evaluated straight into the weight gradient's operand, then
 * lbt_conv_stem_wgrad's exact partials into slab[nshard][K][16]. Shapes: 3x3 / stride 1 / SAME,
 * Cout 16, W in {8,16,32,64}, (H*W) % LBT_STEM_WG_PIXELS == 0. Bit-identical to the two launches. */
int lbt_conv_stem_bwd(const lbt_chain_bwd_b* b, const int16_t* x, lbt_conv_desc d, int32_t* slab, int32_t nshard,
                      void* stream);
/* Two pass-B chains of the same shape (rows, inner, C) and flags in one launch: a projection
 * block's shortcut-BN and first-BN backward (dynamic_fixed_point.py:620-623 for ns and n1 of
 * :746-875), both feeding strided convs whose dgrad has no pass-B prologue. Bit-identical to two
 * lbt_bn_chain_bwd_b calls; mismatched shapes / flags -> LBT_EINVAL.                         */
int lbt_bn_chain_bwd_b_pair(const lbt_chain_bwd_b* a, const lbt_chain_bwd_b* b, void* stream);

/* The weight gradient of one conv (the arguments of lbt_conv_wgrad_i8), as a job another launch
 * carries out; slab == NULL: no job.                                                        */
typedef struct lbt_wgrad_job {
  const int8_t* xq; int32_t x_u8off; const int8_t* gq; lbt_conv_desc d;
  int32_t* slab; int32_t nsplit, nshard;
} lbt_wgrad_job;

/* lbt_conv_wgrad_i8 for njobs convs in ONE launch (Conv2d_q.backward's dW pass 1,
 * dynamic_fixed_point.py:302, of every conv of a step): jobs is a HOST array, each entry exactly
 * the arguments of one lbt_conv_wgrad_i8 call (Cin = 16, 32 or 64; slab != NULL); the results are
 * those of the njobs calls (integer atomics into each job's slab). Every job is checked before
 * anything is queued.                                                                          */
int lbt_conv_wgrad_many_i8(const lbt_wgrad_job* jobs, int32_t njobs, void* stream);
/* lbt_conv_wgrad_many_i8(jobs, njobs) followed by lbt_conv_stem_bwd(b, x, d, slab, nshard) as ONE
 * launch (the stem BN's pass B + conv1's dW of dynamic_fixed_point.py:620-623 / :302 need only the
 * first block's dgrad output, like every batched wgrad job): the stem's 256-pixel row blocks run two
 * per workgroup as the batched launch's first workgroups (LBT_STEM_FIRST=0: its last). Same arguments, checks and results as the two
 * calls (integer atomics); a batch of more than 24 jobs or an odd number of stem row blocks is run as
 * the two calls.                                                                               */
int lbt_conv_wgrad_many_stem_i8(const lbt_wgrad_job* jobs, int32_t njobs, const lbt_chain_bwd_b* b, const int16_t* x,
                                lbt_conv_desc d, int32_t* slab, int32_t nshard, void* stream);

/* One stride-1 3x3 Conv2d_q's backward in ONE launch, with the BN backward passes on either side
 * (Conv2d_q.backward dynamic_fixed_point.py:299-305 between Normalization_q.backward :620-623 of
 * the BN it feeds and the BN it consumes):
 *   gq = pass B of the BN AFTER the conv (b, exactly lbt_bn_chain_bwd_b; b.gq is required and
 *        stored -- it is this conv's weight-gradient operand -- b.dx must be NULL)
 *   dx = dgrad(gq, wd)  (as lbt_conv_dgrad_i8 with qg = b.qo, qw; never stored)
 *   pass A of the BN BEFORE the conv on g = dx (+ add_src)  (a, as lbt_conv_dgrad_chain_i8)
 * plus, in the same grid, the weight-gradient workgroups of job w (typically the deferred wgrad of
 * the previous such launch, whose gq is complete when this launch starts).
 * Each dgrad workgroup owns 4 image rows and recomputes pass B over its rows plus a one-pixel
 * halo into LDS (no inter-workgroup exchange); gq, its channel sums and its overflow counters are
 * produced by the owning workgroup only. Every output is bit-identical to lbt_bn_chain_bwd_b,
 * lbt_conv_dgrad_chain_i8 (and lbt_conv_wgrad_i8 for w) run one after another.
 * Shapes: KH = KW = 3, strides 1, pads 1, Cin = Cout = C in {16, 32, 64}, H % 4 == 0,
 * (W + 2) * C <= 704 and W * C <= 512 (CIFAR ResNet stages); chains as lbt_conv_dgrad_chain_i8;
 * w4 != 0: wd is the packed 4-bit image (lbt_conv_dgrad_i8w4). Else LBT_EINVAL.              */
typedef struct lbt_conv_bwd {
  lbt_chain_bwd_b b;
  const int8_t* wd; int32_t ksd; int32_t w4; lbt_conv_desc d; lbt_qdesc qw;
  const float* add_src;
  lbt_chain_bwd_a a;
  lbt_wgrad_job w;
} lbt_conv_bwd;
int lbt_conv_bwd_fused_i8(const lbt_conv_bwd* p, void* stream);

/* A projection block's strided convs' backward in ONE launch (the stage transition of the CIFAR
 * ResNets: ResidualBlock_q :772-795 / :831-846 backward): pass B of BOTH BNs after the strided
 * convs (b1: the 3x3/2 conv-1's BN, bs: the 1x1/2 shortcut's; each exactly lbt_bn_chain_bwd_b with
 * gq required and stored, dx NULL), dx = dgrad(d1, wd1 on b1.gq) + dgrad(ds, wds on bs.gq) summed in
 * fp32, and pass A of the BN that consumes dx (a) -- bit-identical to lbt_bn_chain_bwd_b_pair(bs, b1)
 * followed by lbt_conv_dgrad2_chain_i8. Shapes: d1 3x3 stride 2 SAME (pads 0 / 1), ds 1x1 stride 2,
 * Cin = C in {16, 32}, Cout = 2C, W * C = 512, H % (C == 16 ? 8 : 4) == 0; w4 != 0: packed 4-bit
 * weight images. Else LBT_EINVAL.                                                              */
typedef struct lbt_conv_bwd2 {
  lbt_chain_bwd_b b1, bs;
  const int8_t* wd1; int32_t ksd1; const int8_t* wds; int32_t ksds; int32_t w4;
  lbt_conv_desc d1, ds; lbt_qdesc qw1, qws;
  lbt_chain_bwd_a a;
} lbt_conv_bwd2;
int lbt_conv_bwd2_fused_i8(const lbt_conv_bwd2* p, void* stream);

/* One stride-1 3x3 Conv2d_q's forward in ONE launch, with the BN element chain that produces its
 * input (ResidualBlock_q :858-863 / BatchNorm_q :584-616,677-683 -> Conv2d_q.forward :287-291):
 *   X  = chain c (exactly lbt_bn_chain_fwd; c.o1 = this conv's input codes, LBT_OUT_U8OFF, stored:
 *        they are the weight gradient's operand; c.o2 must be NULL)
 *   y  = conv(X, wf)  (as lbt_conv_fwd_i8 with x_u8off = 1, qx = c.qo1, qw)
 *   yq = Q(y, qout) with the channel sums of yq into ychsum (the quantising epilogue of
 *        lbt_conv_fwd_i8: the next Normalization_q's input quantiser)
 * Each workgroup owns 4 image rows and recomputes the chain over its rows plus a one-pixel halo
 * into LDS; the chain's stored outputs (R codes, y, X codes), counters and the BN running-average
 * update (workgroup 0) come from the owning workgroup only: every output is bit-identical to
 * lbt_bn_chain_fwd followed by lbt_conv_fwd_i8. Shapes as lbt_conv_bwd_fused_i8; chains: int8
 * Normalization_q inputs, Rescale_q codes stored, ReLU, stochastic noise tables, 1 or 2 branches,
 * optional residual and y; w4: wf is the packed 4-bit image. Else LBT_EINVAL.                    */
typedef struct lbt_conv_fwd {
  lbt_chain_fwd c;
  const int8_t* wf; int32_t ksf; int32_t w4; const int32_t* wcolsum; lbt_conv_desc d; lbt_qdesc qw;
  int8_t* yq; lbt_qdesc qout; int64_t* ychsum;
} lbt_conv_fwd;
int lbt_conv_fwd_fused_i8(const lbt_conv_fwd* p, void* stream);

/* BN backward passes A and B for 9..16-bit gradient quantisers (config 4): the arithmetic of
 * lbt_bn_chain_bwd_a / _b (one branch, no mask) with int16 grad codes and int64 channel sums.
 * Rows here are pixels: g / R / qn / gout / dout / dx are [rows][C]; inner = the per-sample
 * element count (noise period). A: qrg.bits == 0 skips the rescale part, qng.bits == 0 writes
 * dout instead of norm codes; sums [NSHARD][4C] as lbt_chain_bwd_a's. B: dx from gout, qn, the
 * forward's ms and pass A's sums (n = elements per channel).                                */
int lbt_bn_bwd_a_wide(const float* g, lbt_qdesc qrg, const int8_t* R, const float* gamma_q, lbt_qdesc qng,
                      const int8_t* qn, int16_t* gout, float* dout, int64_t* sums, int64_t rows, int64_t inner,
                      int32_t C, void* stream);
int lbt_bn_bwd_b_wide(const int16_t* G, lbt_qdesc qng, const int8_t* qn, lbt_qdesc qn_q, const float* ms,
                      const int64_t* sums, int64_t n, float* dx, int64_t rows, int32_t C, void* stream);

/* The same passes as one bottleneck block's fused backward runs them (ResidualBottleneck_q,
 * SURVEY 8(f) rank 1): pass A with the ReLU_q mask folded in -- y_mask > 0, or mask_r: the
 * forward chain's pre-ReLU value ((float)R * s_qr) * gb[c] + gb[C+c] > 0 recomputed from the R
 * codes (gb = [gamma_q | beta_q], also the gamma_q of the rescale part) -- and the masked fp32
 * gradient optionally stored (gmask_out: the identity shortcut's gradient); pass B with dx fed
 * straight into the consuming conv's 9..16-bit gradient quantiser qo (int16 codes gq, overflow
 * counters, noise period inner) instead of storing dx. g2 (optional): the incoming gradient is
 * g + g2 (the block's two branch gradients, ResidualBlock_q.backward :865-869, summed here
 * instead of in their own pass). y_bits (instead of y_mask): the mask as lbt_chain_fwd's ybits
 * (one byte per channel quad). Bit-identical to the unfused sequence.                         */
int lbt_bn_bwd_a_wide_masked(const float* g, const float* g2, const float* y_mask, const uint8_t* y_bits,
                             int32_t mask_r, lbt_qdesc qr,
                             const float* gb,
                             float* gmask_out, lbt_qdesc qrg, const int8_t* R, lbt_qdesc qng, const int8_t* qn,
                             int16_t* gout, float* dout, int64_t* sums, int64_t rows, int64_t inner, int32_t C,
                             void* stream);
int lbt_bn_bwd_b_wide_q(const int16_t* G, lbt_qdesc qng, const int8_t* qn, lbt_qdesc qn_q, const float* ms,
                        const int64_t* sums, int64_t n, int16_t* gq, lbt_qdesc qo, int64_t rows, int64_t inner,
                        int32_t C, void* stream);

/* Rescale_q parameter gradients (:689-690) from pass-A sums:
 * dgamma = (float)((double)sum(G2*R) * sg2*sr) + wd2*gamma,  dbeta = (float)((double)sum G2 * sg2). */
int lbt_bn_param_grads(const int64_t* sums, int32_t C, lbt_qdesc qrg, lbt_qdesc qr,
                       const float* gamma, float wd2, float* dgamma, float* dbeta, void* stream);

/* ---------------------------------------------------------------- glue ---------------- */

/* ReLU_q forward (:986, tf.maximum(0,x)) and backward (TF _MaximumGrad: g where x > 0). */
int lbt_relu_fwd(const float* x, float* y, int64_t n, void* stream);
int lbt_relu_bwd(const float* g, const float* x, float* dx, int64_t n, void* stream);
/* elementwise a + b (ResidualBlock_q :862 / :869). */
int lbt_add(const float* a, const float* b, float* y, int64_t n, void* stream);
/* AvgPool_q over the whole HxW map (:1017): y[n,c] = (sequential fp32 sum) * (1/(H*W)). */
int lbt_avgpool_fwd(const float* x, float* y, int32_t N, int32_t HW, int32_t C, void* stream);
int lbt_avgpool_bwd(const float* g, float* dx, int32_t N, int32_t HW, int32_t C, void* stream);
/* AvgPool_q with any window (:1009-1022, tf.nn.avg_pool, SAME or VALID): y = (fp32 sum of the window's
 * valid inputs in (kh, kw) order) / count, count = valid positions (TF SAME excludes padding);
 * backward: each input sums g[o] / count[o] over the windows holding it, ascending output order.
 * d as for lbt_maxpool_fwd.                                                                      */
int lbt_avgpool_gen_fwd(const float* x, float* y, lbt_conv_desc d, void* stream);
int lbt_avgpool_gen_bwd(const float* g, float* dx, lbt_conv_desc d, void* stream);
/* MaxPool_q (:993-1006, tf.nn.max_pool; TF SAME pads with -inf): y = window max (first maximum in
 * (kh, kw) order wins), amax = its window position (one byte per output); backward (TF MaxPoolGrad)
 * routes each output gradient to its argmax input, summed per input in ascending output order.
 * d: N, H, W, Cin (= channels), KH, KW, SH, SW, PT, PL, Ho, Wo; Cout, PB, PR unused.           */
int lbt_maxpool_fwd(const float* x, float* y, uint8_t* amax, lbt_conv_desc d, void* stream);
int lbt_maxpool_bwd(const float* g, const uint8_t* amax, float* dx, lbt_conv_desc d, void* stream);
/* The preceding ReLU_q's backward (:983-990, mask x > 0) folded in: y = this pool's forward output
 * (the pool input is the ReLU output, so an input that receives gradient has x > 0 <=> y[o] > 0);
 * dx = relu_bwd(maxpool_bwd(g)) bit for bit, in one pass. C % 4 == 0.                           */
/* ... and its forward: y = maxpool(relu(x)) from the ReLU's input x (relu(max) = max(relu)); amax
 * differs from lbt_maxpool_fwd's where the window max is <= 0: there it is 255 (route nothing),
 * so lbt_maxpool_relu_bwd may be given y = NULL for this amax. C % 4 == 0, KH*KW <= 255.
 * HARD PRECONDITION of y == NULL: amax must come from lbt_maxpool_relu_fwd (masked codes). The
 * library cannot tell the two amax encodings apart; an amax from plain lbt_maxpool_fwd with
 * y == NULL routes gradient to windows whose max is <= 0 -- silently wrong. With amax from
 * lbt_maxpool_fwd always pass that pool's y.                                                       */
int lbt_maxpool_relu_fwd(const float* x, float* y, uint8_t* amax, lbt_conv_desc d, void* stream);
int lbt_maxpool_relu_bwd(const float* g, const uint8_t* amax, const float* y, float* dx, lbt_conv_desc d,
                         void* stream);
/* mean sparse softmax cross-entropy (models.py:30-32) -> loss[0] (fp32, device), dz = d loss / d z. */
int lbt_softmax_xent(const float* z, const int32_t* labels, int32_t N, int32_t K, float* loss,
                     float* dz, void* stream);
/* The classifier head of CIFAR10_Resnet20, fwd AND bwd, per sample in ONE launch (a workgroup
 * per sample) -- replaces lbt_avgpool_fwd, lbt_dfxp_quantize (pooled, Dense_q X),
 * lbt_conv_fwd_generic (Dense_q y = Xq Wq), lbt_softmax_xent, lbt_dfxp_quantize (Dense_q grad),
 * lbt_conv_dgrad_generic and lbt_avgpool_bwd with the same arithmetic bit for bit:
 *   AvgPool_q   dynamic_fixed_point.py:1009-1022, Dense_q :319-395 (fwd) / :441-466 (bwd),
 *   loss        models.py:30-32 (mean sparse softmax cross-entropy).
 * x [N][HW][C] fp32 (last block output) -> logits, dz, gx [N][HW][C] = d loss / d x, and per
 * sample a record (pq, gq, loss term) in scratch (lbt_head_scratch_bytes(N, C, K) bytes) from
 * which lbt_step_reduce later forms the two batch reductions: the Dense_q weight gradient
 * dw = dequant(sum_n pq^T gq) + wd2*w (lbt_conv_wgrad_reduce's formula) and loss[0].
 * wq is the Dense_q weight codes [C][K] (lbt_dfxp_quantize_weights' w_hwio of a C x 1 x 1 x K job,
 * 4-byte aligned). qx / qg are the stochastic X / grad quantisers (noise tables of C / K values,
 * or Philox inline). pooled, pq, gq are optional outputs (NULL = not stored).
 * Limits: C <= 256, C % 8 == 0, 1 <= K <= 64, HW >= 1, x 16-byte aligned.
 * loss_n: the batch the mean is over (0 = N). A data-parallel rank passes the GLOBAL batch, so its
 * dz rows and its loss share are exactly those of one process running the whole batch.       */
typedef struct lbt_head {
  const float* x; int32_t N, HW, C, K;
  float* pooled; int8_t* pq; lbt_qdesc qx;
  const int8_t* wq; lbt_qdesc qw;
  const int32_t* labels; float* logits; float* loss; float* dz;
  int8_t* gq; lbt_qdesc qg;
  const float* w; float wd2; float* dw;
  float* gx;
  void* scratch;
  int32_t loss_n;
  /* optional: pass A of the last block's output BatchNorm chain (one branch, ReLU mask from
   * y_mask, gmask_out, stochastic quantisers; a.g unused) run per sample on the un-pooled gradient
   * inside this launch -- then gx is not written. Bit-identical to lbt_bn_chain_bwd_a(a) on gx. */
  const lbt_chain_bwd_a* pa;
  /* optional (with pa): the last block's END CHAIN (lbt_bn_chain_fwd of a one-branch chain with int8
   * Normalization_q codes in, stochastic Rescale_q with its noise table, residual add and ReLU, no
   * output quantisers; C == this C, HW * C == 4096) evaluated per sample inside this launch: the
   * block output the head pools and pass A's ReLU mask / R codes come from registers, so x is not
   * read and the chain's y / R / ybits are not written (its ms and running statistics are, by
   * workgroup 0). Bit-identical to lbt_bn_chain_fwd(chain) followed by this head on x = chain.y.    */
  const lbt_chain_fwd* chain;
} lbt_head;
/* scratch: the records transposed, NP = N rounded up to 16: pqT [C][NP] int8 | gqT [64][NP] int8 |
 * loss terms [N] double (lbt_step_reduce sums them 4 samples per v_dot4)                         */
int lbt_head_scratch_bytes(int32_t N, int32_t C, int32_t K);  /* = (C + 64) * NP + 8 * N */
int lbt_head_fwd_bwd(const lbt_head* h, void* stream);

/* MomentumOptimizer.apply_gradients (trainer.py:81-82): a = mu*a + g*gscale; w -= lr*a. */
int lbt_sgd_momentum(float* w, float* a, const float* g, int64_t n, float lr, float mu,
                     float gscale, void* stream);

/* Conv2d_q / Dense_q bias (use_bias=True, dynamic_fixed_point.py:198-201,293-296,390-393):
 * y[e] += bq[e % C] (bq dequantised by lbt_dfxp_quantize), and db[c] = sum_e gq * 2^-eg from
 * the grad quantiser's sharded per-channel sums chsum [LBT_NSHARD][2C] (:209, :459).       */
int lbt_bias_add(float* y, const float* bq, int64_t n, int32_t C, void* stream);
int lbt_bias_grad(const int64_t* chsum, int32_t C, lbt_qdesc qg, float* db, void* stream);

/* ---------------------------------------------------------------- batched (one launch per step)
 * Job arrays live in DEVICE memory (uploaded once by the caller); grid.y = job index.          */

/* lbt_dfxp_quantize_weight for many weights. */
typedef struct lbt_wjob {
  const float* w; int32_t KH, KW, Cin, Cout; lbt_qdesc q;
  int8_t* w_hwio; int8_t* wf; int32_t ksf; int8_t* wd; int32_t ksd; int32_t* colsum;
} lbt_wjob;
int lbt_dfxp_quantize_weights(const lbt_wjob* jobs, int32_t njobs, int32_t max_cout, void* stream);

/* The same for wide layers, element-parallel (coalesced float4 loads, one Philox call per 4
 * noise indices): every job's Cout % 4 == 0, w 16-byte aligned, colsum unused (NULL). Block
 * ranges: job j owns blocks [starts[j], starts[j+1]) of the 1-D grid (starts in device memory,
 * starts[0] = 0, starts[njobs] = total_blocks), lbt_flat_weight_blocks(KH*KW*Cin*Cout) each. */
int lbt_flat_weight_blocks(int64_t n);
int lbt_dfxp_quantize_weights_flat(const lbt_wjob* jobs, const int32_t* starts, int32_t njobs, int32_t total_blocks,
                                   void* stream);

/* lbt_dfxp_quantize (generic path) for many small tensors (Rescale_q gamma / beta, :679-682). */
typedef struct lbt_qjob {
  const float* x; void* out; int32_t out_kind; int64_t n, inner; lbt_qdesc q;
} lbt_qjob;
int lbt_dfxp_quantize_many(const lbt_qjob* jobs, int32_t njobs, void* stream);

/* lbt_conv_wgrad_reduce for many layers: one 1-D launch of total_blocks = sum over the jobs of
 * lbt_rjob_blocks(K*Cout) workgroups (jobs[] in device memory).                            */
int lbt_rjob_blocks(int64_t n);  /* workgroups of one reduce job of n = K*Cout outputs (1024 each) */
typedef struct lbt_rjob {
  const int32_t* slab; int32_t nsplit, K, Cout, x_u8off; const int64_t* gcolsum;
  lbt_qdesc qx, qg; const float* w; float wd2; float* dw;
} lbt_rjob;
/* (a job with x_u8off and gcolsum -- the 128 * sum_p g[co] offset correction -- needs Cout <= 256) */
int lbt_conv_wgrad_reduce_many(const lbt_rjob* jobs, int32_t njobs, int32_t total_blocks, void* stream);

/* lbt_bn_param_grads for many Rescale_q layers. */
typedef struct lbt_pjob {
  const int64_t* sums; int32_t C; lbt_qdesc qrg, qr; const float* gamma; float wd2; float* dgamma; float* dbeta;
} lbt_pjob;
int lbt_bn_param_grads_many(const lbt_pjob* jobs, int32_t njobs, int32_t max_c, void* stream);

/* The start of a step in ONE launch: lbt_dfxp_noise_fill's jobs (+ the arena clear),
 * lbt_dfxp_quantize_weights' jobs, lbt_dfxp_quantize_many's jobs and, if input is not NULL, the
 * step's input images quantised to int16 codes (input->out_kind == LBT_OUT_I16, n and inner
 * multiples of 4, Philox noise inline -- the input quantiser needs no table). Independent parts:
 * nothing here reads another part's output. Job arrays in device memory, *input in host memory. */
/* snap_n > 0: the launch also copies snap_src[0, snap_n) to snap_dst (the step's exponents, read by
 * lbt_step_reduce_update's dequantisations while its range-update blocks rewrite the live ones).  */
int lbt_step_prologue(const lbt_njob* njobs, int32_t nn, int64_t max_n, int64_t* zero, int64_t nzero,
                      const lbt_wjob* wjobs, int32_t nw, int32_t max_cout, const lbt_qjob* qjobs, int32_t nq,
                      const lbt_qjob* input, const int32_t* snap_src, int32_t* snap_dst, int32_t snap_n,
                      void* stream);

/* The end of a step's backward in ONE launch: lbt_conv_wgrad_reduce_many's jobs (r_blocks =
 * sum of lbt_rjob_blocks(K*Cout)), lbt_bn_param_grads_many's jobs (Cout <= max_c) and, if head is not
 * NULL, the head's batch reductions (Dense_q dw and loss[0], from lbt_head_fwd_bwd's records:
 * the loss summed in softmax_xent's order). Job arrays in device memory, *head in host memory.  */
int lbt_step_reduce(const lbt_rjob* rjobs, int32_t nr, int32_t r_blocks, const lbt_pjob* pjobs, int32_t np,
                    int32_t max_c, const lbt_head* head, void* stream);

/* lbt_step_reduce and lbt_step_update in ONE launch (single process): every block that forms a
 * gradient element also applies MomentumOptimizer to it (acc = mu*acc + g; w -= lr*acc,
 * trainer.py:81-82, lbt_sgd_momentum's arithmetic, gscale 1) -- the job's dw / dgamma / dbeta and the
 * head's dw lie inside the flat gradient buffer g, their parameter and accumulator at the same
 * offset in w and a -- and (nslots + 3) / 4 more blocks run update_range on every slot and advance
 * step (lbt_dfxp_range_update). Those rewrite the exponents while other blocks dequantise, so
 * every job / head descriptor must read its exponents from a copy taken earlier in the step
 * (lbt_step_prologue's snapshot). Results bit-identical to lbt_step_reduce + lbt_step_update.   */
typedef struct lbt_update {
  float* w; float* a; const float* g; float lr, mu;
  int32_t* exps; int32_t* counts; const int32_t* bits; const float* target; const float* nelem;
  uint64_t* step; int32_t nslots; int32_t pad;
} lbt_update;
int lbt_step_reduce_update(const lbt_rjob* rjobs, int32_t nr, int32_t r_blocks, const lbt_pjob* pjobs, int32_t np,
                           int32_t max_c, const lbt_head* head, const lbt_update* u, void* stream);

/* lbt_sgd_momentum and lbt_dfxp_range_update in ONE launch (independent: the optimiser reads no
 * exponent; the range update reads only the step's counters).                              */
int lbt_step_update(float* w, float* a, const float* g, int64_t n, float lr, float mu, float gscale,
                    int32_t* exps, int32_t* counts, const int32_t* bits, const float* target,
                    const float* nelem, int32_t nslots, uint64_t* step, void* stream);

/* ---------------------------------------------------------------- data-parallel exchange ----
 * SURVEY 8(e) / DESIGN 7. The step's gradients cross ranks as their EXACT integer numerators
 * (the quantised-gradient exchange): lbt_step_reduce_x runs lbt_step_reduce's jobs but, instead of
 * dequantising, writes each gradient element's int64 numerator into xbuf at its flat index
 * (dw - gbase): a weight gradient's slab sum + 128 * its grad-code column sum (:302), a Rescale_q's
 * sum G2*R and sum G2 (:689-690), the head's sum pq^T gq (:457); every quantiser's overflow counts
 * (shards summed and ZEROED) at buf[cnt_off + 2*slot + {0,1}]; and the head's loss-term sum in
 * 2^-32 fixed point at buf[loss_off]. One int64 SUM all-reduce over the ranks is exact and
 * order-independent; lbt_step_finish then dequantises the totals with the single-process formulas
 * (so a data-parallel step equals the one-process step whenever the per-sample work does), runs
 * SGD-momentum, and lbt_dfxp_range_update_x applies update_range to the summed counts (a separate
 * launch: the dequantisation reads the exponents the range update rewrites).
 * pjob_scale multiplies the gamma / beta numerators: 1, or under SyncBN -- whose pass-A sums were
 * already all-reduced -- 1 on one rank and 0 on the others.                                     */
typedef struct lbt_xchg {
  int64_t* buf; const float* gbase; int32_t pjob_scale; int32_t nslots;
  int32_t* counts; int64_t cnt_off; int64_t loss_off;
} lbt_xchg;
int lbt_step_reduce_x(const lbt_rjob* rjobs, int32_t nr, int32_t r_blocks, const lbt_pjob* pjobs, int32_t np,
                      int32_t max_c, const lbt_head* head, const lbt_xchg* x, void* stream);
/* One parameter tensor of the flat buffers, [off, off + n): kind 0 = conv / dense weight
 * (g = (float)S * 2^-(ex+eg) + wd2*w), 1 = Rescale_q gamma (g = (float)((double)S * 2^-eg * 2^-ex)
 * + wd2*w; qx = its X quantiser, qg = its grad quantiser), 2 = Rescale_q beta (g = (float)((double)S
 * * 2^-eg)). Blocks: ceil(n / 256) per segment in order (total_blocks = their sum).             */
typedef struct lbt_fseg {
  int64_t off, n; int32_t kind; lbt_qdesc qx, qg; float wd2;
} lbt_fseg;
/* g[i] (if g != NULL) = the dequantised gradient of xbuf[i]; a = mu*a + g; w -= lr*a (gscale 1);
 * loss[0] = (float)(xbuf[loss_off] * 2^-32 / loss_n) if loss != NULL.                          */
int lbt_step_finish(const lbt_fseg* segs, int32_t nseg, int32_t total_blocks, const int64_t* xbuf, float* w,
                    float* a, float* g, float lr, float mu, float* loss, int64_t loss_off, int32_t loss_n,
                    void* stream);
int lbt_dfxp_range_update_x(int32_t* exps, const int64_t* xbuf, int64_t cnt_off, const int32_t* bits,
                            const float* target, const float* nelem, int32_t nslots, uint64_t* step, void* stream);

/* ---------------------------------------------------------------- either side of the path ---
 * GradientBuffer_q.backward (dynamic_fixed_point.py:473-509): total = pad(g, n_buf) + buffer;
 * gq = Q(total) (dequantised fp32; noise index i % inner, inner = prod(buffer.shape[1:]));
 * buffer = total - gq; gq[0 : n_g] out. q.bits == 32: the reference's bypass (gq = total).    */
int lbt_grad_buffer_bwd(const float* g, int64_t n_g, float* buffer, int64_t n_buf, int64_t inner, lbt_qdesc q,
                        float* gq, void* stream);
/* Dense_q._pre_dense_func (:397-439, dormant in the reference): grad [rows][cols] updated in place
 * against the per-element state accu / init_flag / rem_flag [state_rows][state_cols] (initially
 * 0.001 / 1 / 0, :364-366,449), eps = 2^-(bits - I_grad) (:444). rows <= state_rows.          */
int lbt_pre_dense(float* grad, int32_t rows, int32_t cols, int32_t state_rows, int32_t state_cols, lbt_qdesc qg,
                  float* accu, int32_t* init_flag, int32_t* rem_flag, void* stream);
/* preprocess_image (trainer.py:24-28): per sample a random left-right flip and a random crop of
 * the zero-padded (pad on each side) image back to H x W; the draws are Philox4x32-10 of
 * (sample, "AUG!", counter; seed): flip = r0 & 1, oy = r1 % (2pad+1), ox = r2 % (2pad+1).    */
int lbt_augment_flip_crop(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C, int32_t pad,
                          uint64_t seed, uint64_t counter, void* stream);

/* Diagnostics: counts (atomically into *bad) the i < n where the BN kernels' division by a
 * reused divisor (div_by(x, recip(y)), dfxp_device.h) differs in any bit from x / y; if qa
 * is not NULL also writes x / y to qa and div_by to qb.                                      */
int lbt_selftest_div(const float* x, const float* y, int64_t n, int32_t* bad, float* qa, float* qb, void* stream);

/* Dense_q for wide classifier heads (dynamic_fixed_point.py:319-395, 441-466; ResNet-50's
 * 2048 -> 1000 fc) on int8 MFMA (dense.hip); exact, bit-identical to the generic kernels.
 * lbt_dense_pack: HWIO codes W[in][out] -> wf [out][kf] and wd [in][up] (zero-padded; kf, up
 *      multiples of 64 >= in, out).
 * lbt_dense_gemm: out[rows][cols] = a[rows][:kvalid] . b[cols][:kb]^T * 2^-(e_a + e_b); a int8
 *      codes (a16 = 0) or int16 9..16-bit codes (a16 = 1); kvalid, lda multiples of 8. fwd: a = xq,
 *      b = wf; dgrad: a = gq, b = wd.
 * lbt_dense_wgrad: dw[in][out] = (float)(sum_n x[n][k] g[n][u]) * 2^-(e_x + e_g) + wd2 * w (the
 *      reduce of lbt_conv_wgrad_reduce64 fused in); g int8 / int16; out % 4 == 0.
 * lbt_softmax_xent_wide: lbt_softmax_xent for wide K (one wave per row).                      */
int lbt_dense_pack(const int8_t* w_hwio, int32_t in_units, int32_t units, int8_t* wf, int32_t kf, int8_t* wd,
                   int32_t up, void* stream);
int lbt_dense_gemm(const void* a, int32_t a16, int32_t lda, int32_t kvalid, const int8_t* b, int32_t kb, int32_t rows,
                   int32_t cols, lbt_qdesc qa, lbt_qdesc qb, float* out, void* stream);
int lbt_dense_wgrad(const int8_t* xq, const void* g, int32_t g16, int32_t N, int32_t in_units, int32_t units,
                    lbt_qdesc qx, lbt_qdesc qg, const float* w, float wd2, float* dw, void* stream);
int lbt_softmax_xent_wide(const float* z, const int32_t* labels, int32_t N, int32_t K, float* loss, float* dz,
                          void* stream);

/* ---------------------------------------------------------------- 17..32-bit quantisers --------
 * The top of weight_quantization's domain (1 <= bits <= 32, dynamic_fixed_point.py:21-23): a 17..31-
 * bit quantiser's codes no longer fit the int8 / int16 GEMM operands, so it writes fake-quantised fp32
 * values (lbt_dfxp_quantize, LBT_OUT_F32 -- the reference's own STE output), and bits == 32 is the
 * full-precision bypass. The layers then contract fp32 operands as TF does (fp32.hip), accumulating
 * in double in a fixed order (deterministic):
 *   conv fwd / dgrad (dx += add_src if not NULL) / wgrad (pixels split nsplit ways into a double slab
 *   [nsplit][KH*KW*Cin][Cout], then reduce: dw = (float)sum + wd2 * w); Dense_q = a 1x1 conv on a 1x1 map;
 *   chan_sums: part[split][c] = sum a, part[split][C + c] = sum a*b (b NULL: a*a) over [rows][C];
 *   bn_f32_fwd: biased moments from those sums, sigma = sqrtf(var + eps), y = (x - mu) / sigma, running
 *   averages and ms = [mu | sigma] as lbt_bn_norm (frozen: testing mode, the running averages);
 *   bn_f32_bwd: part = chan sums of (g, x); dx = ((g - mg) - xhat*mgx) / sigma (frozen: g / sigma);
 *   affine: y = x*gb[c] + gb[C + c] (bwd != 0: y = x*gb[c]); affine_grads: dgamma = (float)sum g*x + wd2*gamma,
 *   dbeta = (float)sum g, from chan sums of (g, x).                                                   */
int lbt_conv_fwd_f32(const float* x, const float* w, lbt_conv_desc d, float* y, void* stream);
int lbt_conv_dgrad_f32(const float* g, const float* w, lbt_conv_desc d, float* dx, const float* add_src, void* stream);
int lbt_conv_wgrad_f32(const float* x, const float* g, lbt_conv_desc d, double* slab, int32_t nsplit, void* stream);
int lbt_conv_wgrad_reduce_f32(const double* slab, int32_t nsplit, int64_t total, const float* w, float wd2, float* dw,
                              void* stream);
int lbt_chan_sums_f32(const float* a, const float* b, int64_t rows, int32_t C, int32_t nsplit, double* part,
                      void* stream);
int lbt_bn_f32_fwd(const float* x, const double* part, int32_t nsplit, int64_t rows, int32_t C, float eps,
                   float momentum, float one_minus_momentum, float* ms, float* run_mean, float* run_var, int32_t frozen,
                   float* y, void* stream);
int lbt_bn_f32_bwd(const float* g, const float* x, const float* ms, const double* part, int32_t nsplit, int64_t rows,
                   int32_t C, int32_t frozen, float* dx, void* stream);
int lbt_affine_f32(const float* x, const float* gb, int64_t n, int32_t C, int32_t bwd, float* y, void* stream);
int lbt_affine_grads_f32(const double* part, int32_t nsplit, int32_t C, const float* gamma, float wd2, float* dgamma,
                         float* dbeta, void* stream);

/* ---- The exact data-parallel exchange of the layer-wise models (ResNet-50, configs[3] at N GPUs;
 * SURVEY 8(e)). Each of these writes the INTEGER numerator of a gradient where its dequantising twin
 * (same name without _x) writes dW = (float)S * 2^-(ex+eg) + wd2 * W (dynamic_fixed_point.py:302,
 * :457-460) or dgamma / dbeta (:689-691): num[i] = S (int64, exact). The trainer points num into
 * the int64 exchange buffer at the gradient's offset in the flat gradient buffer, all-reduces it
 * (RCCL, SUM: exact and order-independent) and dequantises once with lbt_step_finish -- so a step
 * on N ranks equals the oracle's N-shard step (oracle/resnet.py dp_train_step) bit for bit.
 * lbt_softmax_xent_n: lbt_softmax_xent(_wide) with the mean over `norm` >= N rows (the GLOBAL
 * batch of a shard) and, if loss_fx != NULL, the ordered double sum of the loss terms in 2^-32 fixed
 * point (the exchange's loss slot). */
int lbt_conv_wgrad_reduce_x(const int32_t* slab, int32_t nsplit, int32_t K, int32_t Cout, int32_t x_u8off,
                            const int64_t* gcolsum, int64_t* num, void* stream);
int lbt_conv_wgrad_reduce64_x(const int64_t* slab, int32_t nsplit, int32_t K, int32_t Cout, int64_t* num,
                              void* stream);
int lbt_dense_wgrad_x(const int8_t* xq, const void* g, int32_t g16, int32_t N, int32_t in_units, int32_t units,
                      int64_t* num, void* stream);
int lbt_bn_param_grads_x(const int64_t* sums, int32_t C, int64_t* num_g, int64_t* num_b, void* stream);
int lbt_softmax_xent_n(const float* z, const int32_t* labels, int32_t N, int32_t K, int32_t norm, float* loss,
                       float* dz, int64_t* loss_fx, void* stream);
int lbt_softmax_xent_wide_n(const float* z, const int32_t* labels, int32_t N, int32_t K, int32_t norm, float* loss,
                            float* dz, int64_t* loss_fx, void* stream);

/* A stage transition's forward in ONE launch (the last identity block's end chain, ResidualBlock_q
 * :858-863 with BatchNorm_q :584-616,677-683, feeding a projection block's 3x3/2 conv and 1x1/2
 * shortcut :772-795 / :831-846): the chain c (exactly lbt_bn_chain_fwd; NB 1, residual, y stored,
 * o1 = the 3x3/2 conv's input codes and o2 = the shortcut's, both LBT_OUT_U8OFF and stored) evaluated
 * into LDS, both convs from there (as lbt_conv_fwd_pair_i8: wf1 / wfs, their wcolsum offset
 * corrections), and each conv's quantising epilogue (yq1 / qout1 / ychsum1, yqs / qouts / ychsums).
 * Bit-identical to lbt_bn_chain_fwd followed by lbt_conv_fwd_pair_i8. Shapes: d1 3x3 stride 2 SAME
 * (pads 0 / 1), ds 1x1 stride 2, Cin = C in {16, 32}, Cout = 2C, W * C = 512, Ho % 4 == 0. */
typedef struct lbt_conv_fwd2 {
  lbt_chain_fwd c;
  const int8_t* wf1; int32_t ksf1; const int32_t* wcolsum1;
  const int8_t* wfs; int32_t ksfs; const int32_t* wcolsums;
  int32_t w4;
  lbt_conv_desc d1, ds; lbt_qdesc qw1, qws;
  int8_t* yq1; lbt_qdesc qout1; int64_t* ychsum1;
  int8_t* yqs; lbt_qdesc qouts; int64_t* ychsums;
} lbt_conv_fwd2;
int lbt_conv_fwd2_fused_i8(const lbt_conv_fwd2* p, void* stream);

/* ABI version for the Python loader. */
int lbt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LBT_DFXP_H */

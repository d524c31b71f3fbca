// bn.hip -- BatchNorm_q = Normalization_q + Rescale_q (dynamic_fixed_point.py:539-743) and the
// ReLU / residual glue around it, as element chains fused with the neighbouring DFXP quantisers.
//
// All three kernels are HBM-bound element passes over [rows, inner] (inner = H*W*C): each
// thread owns 4 consecutive elements of one row (one channel quad, one Philox call per
// quantiser, reused over `rpt` rows of the batch since the noise is shared over dim 0) and
// reads / writes them with 4- or 16-byte vector accesses.  Per-channel statistics are exact
// integer sums (moments of the quantised input; G*R, G, G*q for the backward), reduced
// wave -> LDS -> one atomic per workgroup into a shard, so they are deterministic and
// independent of the launch geometry.
#include <cstdio>
#include <cstdlib>

#include "bn_moments.h"
#include "chain_flags.h"
#include "pk2.h"

using namespace lbt;

namespace {

constexpr int kThreads = 256;

LBT_DEV void load4_i8(const int8_t* p, int64_t i, int v[4]) {
  const char4 c = *reinterpret_cast<const char4*>(p + i);
  v[0] = c.x; v[1] = c.y; v[2] = c.z; v[3] = c.w;
}
LBT_DEV void unpack4_i8(int w, int v[4]) {
  v[0] = (int8_t)(w & 0xff); v[1] = (int8_t)((w >> 8) & 0xff);
  v[2] = (int8_t)((w >> 16) & 0xff); v[3] = (int8_t)(w >> 24);
}
LBT_DEV int ld_i8x4(const int8_t* p, int64_t i) { return *reinterpret_cast<const int*>(p + i); }
LBT_DEV float4 ld_f32x4(const float* p, int64_t i) { return *reinterpret_cast<const float4*>(p + i); }
LBT_DEV void f4(const float4& c, float v[4]) { v[0] = c.x; v[1] = c.y; v[2] = c.z; v[3] = c.w; }

// Rows are processed in batches of kRB: every load of a batch is issued before any of its
// arithmetic (stores may alias the inputs as far as the compiler knows, so it would not hoist
// them itself) -- one HBM round trip per batch instead of one per row.
constexpr int kRB = 4;
// The forward chains' batch: 4 rows per thread by default for every chain. The 3-byte-per-element chains
// (int8 codes in, two int8 code sets out) can take LBT_FWD_RB rows instead, a build-time option: 16 / 8
// were measured against 4 and gained nothing -- those chains are VALU-bound, not bound by the loads in
// flight (profiles/round5/elem_batch_ab.txt). The ones with an fp32 operand (20 bytes a row) always stay
// at 4: 8 rows cost 50+ VGPRs, i.e. half the waves. The host guard inner * (LBT_FWD_RB + 1) follows it.
#ifndef LBT_FWD_RB
#define LBT_FWD_RB 4
#endif
template <int F>
constexpr int fwd_rb() {
  return ((F & kRt) || (F & kFRes) || !(F & kFQ)) ? 4 : LBT_FWD_RB;
}

LBT_DEV void load4_f32(const float* p, int64_t i, float v[4]) {
  const float4 c = *reinterpret_cast<const float4*>(p + i);
  v[0] = c.x; v[1] = c.y; v[2] = c.z; v[3] = c.w;
}
LBT_DEV void store4_i8(int8_t* p, int64_t i, const int v[4], int off) {
  char4 c;
  c.x = (int8_t)(v[0] - off); c.y = (int8_t)(v[1] - off); c.z = (int8_t)(v[2] - off); c.w = (int8_t)(v[3] - off);
  *reinterpret_cast<char4*>(p + i) = c;
}
LBT_DEV void store4_f32(float* p, int64_t i, const float v[4]) {
  *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
}
LBT_DEV void store4_code(void* out, int kind, int64_t i, const int c[4], float inv_m) {
  if (kind == LBT_OUT_I8) {
    store4_i8((int8_t*)out, i, c, 0);
  } else if (kind == LBT_OUT_U8OFF) {
    int t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = c[k] < 0 ? 0 : c[k];
    store4_i8((int8_t*)out, i, t, 128);
  } else if (kind == LBT_OUT_I16) {
    short4 s; s.x = (short)c[0]; s.y = (short)c[1]; s.z = (short)c[2]; s.w = (short)c[3];
    *reinterpret_cast<short4*>((int16_t*)out + i) = s;
  } else {
    float f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = (float)c[k] * inv_m;
    store4_f32((float*)out, i, f);
  }
}

LBT_DEV Noise4 noise_for(const lbt_qdesc& q, const QState& s, int64_t g) {
  Noise4 n = {{0.f, 0.f, 0.f, 0.f}};
  if (s.active && q.stochastic) n = qnoise4(q, s.step, (uint64_t)g);
  return n;
}

// ============================================================================ forward chain
// Kernel variants: F holds the chain's configuration as compile-time flags for the combinations
// the fused ResNet plan launches (no per-element branches, constant rounding mode and output
// encoding); kRt selects the variant that reads everything from the descriptor at run time.

template <int B>
LBT_DEV const lbt_chain_branch& fbranch(const lbt_chain_fwd& a) { return B == 0 ? a.b1 : a.b2; }

template <int NB, int F>
__global__ __launch_bounds__(kThreads) void chain_fwd_kernel(lbt_chain_fwd a, int rpt) {
  extern __shared__ float shf[];  // per branch: mu, sigma, gq, bq [C each]; then long long tmp[2C]
  __shared__ int sh_cnt[8 * kThreads / 64];
  constexpr int ST = (F & kRt) ? -1 : ((F & kFStoch) ? 1 : 0);
  constexpr int RB = fwd_rb<F>();
  LBT_TS(0);
  const int C = a.C;
  long long* tmp = reinterpret_cast<long long*>(shf + 8 * C);
  const int64_t groups = a.inner >> 2;
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool live = g < groups;
  const int64_t gl = live ? g : 0;
  const int c0 = (int)(((uint32_t)gl << 2) % (uint32_t)C);
  const int64_t r0 = (int64_t)blockIdx.y * rpt;
  const int64_t rend = r0 + rpt < a.rows ? r0 + rpt : a.rows;
  const bool q_in[2] = {LBT_FL(kFQ, a.b1.nrm.q != nullptr), LBT_FL(kFQ, a.b2.nrm.q != nullptr)};
  const bool res = LBT_FL(kFRes, a.res != nullptr);

  // ---- the first rows and the noise go out before the moment prologue (their latency overlaps it)
  int qv[NB][RB];
  float4 xv[NB][RB], rv[RB];
  // addresses: a uniform 64-bit row-batch base + a 32-bit lane offset (j * inner + 4 g < 2^31, checked on
  // the host) -- per-row 64-bit addresses of every operand held ~7 VGPRs a row
  const uint32_t inner32 = (uint32_t)a.inner, lo32 = (uint32_t)(gl << 2);
  auto load_batch = [&](int64_t rb) {
    const int64_t eb = rb * a.inner;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const uint32_t oj = (uint32_t)(rb + j < rend ? j : 0) * inner32 + lo32;  // clamped: never branch
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const lbt_chain_branch& Bb = b == 0 ? fbranch<0>(a) : fbranch<NB - 1>(a);
        if (q_in[b]) qv[b][j] = ld_i8x4(Bb.nrm.q + eb, oj);
        else xv[b][j] = ld_f32x4(Bb.xin + eb, oj);
      }
      if (res) rv[j] = ld_f32x4(a.res + eb, oj);
    }
  };
  load_batch(r0);
  QState qr[2];
  Noise4 nr[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_chain_branch& Bb = b == 0 ? fbranch<0>(a) : fbranch<NB - 1>(a);
    qr[b] = qstate(Bb.qr);
    nr[b] = noise_for(Bb.qr, qr[b], gl);
  }
  const QState so1 = qstate(a.qo1), so2 = qstate(a.qo2);
  const bool o1 = LBT_FL(kFO1, a.o1 && so1.active), o2 = LBT_FL(kFO2, a.o2 && so2.active);
  const Noise4 no1 = noise_for(a.qo1, so1, gl);
  const Noise4 no2 = noise_for(a.qo2, so2, gl);

  // ms_in (lbt_bn_moments ran): every branch's [mu | sigma] is in nrm.ms -- no LDS, no moment prologue
  bool msall = true;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_chain_branch& Bb = b == 0 ? fbranch<0>(a) : fbranch<NB - 1>(a);
    msall = msall && (!q_in[b] || Bb.nrm.ms_in);
  }
  float sn[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_chain_branch& Bb = b == 0 ? fbranch<0>(a) : fbranch<NB - 1>(a);
    float* P = shf + 4 * C * b;
    sn[b] = 0.f;
    if (q_in[b]) {
      sn[b] = qscale(Bb.nrm.qn);
      if (!msall) {
        bn_moments(Bb.nrm, C, P, P + C, tmp);
        __syncthreads();
      }
    }
    if (qr[b].active && !msall)
      for (int c = threadIdx.x; c < C; c += kThreads) { P[2 * C + c] = Bb.gb[c]; P[3 * C + c] = Bb.gb[C + c]; }
  }
  if (!msall) __syncthreads();
  LBT_TS(1);
  // this thread's channel quad is fixed: its per-channel constants live in registers
  float pm[NB][4], pg[NB][4], pb[NB][4];
  Recip ps[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_chain_branch& Bb = b == 0 ? fbranch<0>(a) : fbranch<NB - 1>(a);
    const float* P = shf + 4 * C * b;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (msall) {
        pm[b][k] = q_in[b] ? Bb.nrm.ms[c0 + k] : 0.f;
        ps[b][k] = recip(q_in[b] ? Bb.nrm.ms[C + c0 + k] : 1.f);
        pg[b][k] = qr[b].active ? Bb.gb[c0 + k] : 0.f;
        pb[b][k] = qr[b].active ? Bb.gb[C + c0 + k] : 0.f;
      } else {
        pm[b][k] = P[c0 + k];
        ps[b][k] = recip(P[C + c0 + k]);
        pg[b][k] = P[2 * C + c0 + k];
        pb[b][k] = P[3 * C + c0 + k];
      }
    }
  }
  // ... and as channel pairs for the packed math
  pf2 pmv[NB][2], psy[NB][2], psr[NB][2], pgv[NB][2], pbv[NB][2], nr2[NB][2];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      pmv[b][h] = pk(pm[b][2 * h], pm[b][2 * h + 1]);
      psy[b][h] = pk(ps[b][2 * h].y, ps[b][2 * h + 1].y);
      psr[b][h] = pk(ps[b][2 * h].rc, ps[b][2 * h + 1].rc);
      pgv[b][h] = pk(pg[b][2 * h], pg[b][2 * h + 1]);
      pbv[b][h] = pk(pb[b][2 * h], pb[b][2 * h + 1]);
      nr2[b][h] = pk(nr[b].u[2 * h], nr[b].u[2 * h + 1]);
    }
  int ovr[2][2] = {{0, 0}, {0, 0}};  // wave totals (quant_w)
  int ovo[2][2] = {{0, 0}, {0, 0}};
  const bool relu = LBT_FL(kFRelu, a.relu != 0), ystore = LBT_FL(kFY, a.y != nullptr);
  const bool u8 = LBT_FL(kFU8, a.o1_kind == LBT_OUT_U8OFF && (!o2 || a.o2_kind == LBT_OUT_U8OFF));

  for (int64_t rb = r0; rb < rend; rb += RB) {
    if (rb != r0) load_batch(rb);
    if (live) {
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        if (rb + j >= rend) break;
        const int64_t e = rb * a.inner + (int64_t)((uint32_t)j * inner32 + lo32);
        pf2 v2[2] = {pk(0.f, 0.f), pk(0.f, 0.f)};
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const lbt_chain_branch& Bb = b == 0 ? fbranch<0>(a) : fbranch<NB - 1>(a);
          pf2 t2[2];
          if (q_in[b]) {
            int q[4];
            unpack4_i8(qv[b][j], q);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const pf2 x1 = pcvt(q[2 * h], q[2 * h + 1]) * pk(sn[b], sn[b]);
              const pf2 x2 = x1 - pmv[b][h];
              t2[h] = pdiv_nz(x2, psy[b][h], psr[b][h]);  // == x2 / sigma (x2 is never -0: see pdiv_nz)
            }
          } else {
            float t[4];
            f4(xv[b][j], t);
            t2[0] = pk(t[0], t[1]);
            t2[1] = pk(t[2], t[3]);
          }
          if ((F & kRt) ? qr[b].active : !(F & kFNoR)) {
            int R[4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              quant_w2<ST>(qr[b], Bb.qr.stochastic, t2[h], nr2[b][h], ovr[b][0], ovr[b][1], R[2 * h], R[2 * h + 1]);
              const pf2 xr = pcvt(R[2 * h], R[2 * h + 1]) * pk(qr[b].inv_m, qr[b].inv_m);
              const pf2 m1 = xr * pgv[b][h];
              t2[h] = m1 + pbv[b][h];
            }
            if (LBT_FL(kFRout, Bb.rout != nullptr)) store4_i8(Bb.rout, e, R, 0);
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) v2[h] = b ? v2[h] + t2[h] : t2[h];
        }
        if (res) {
          float rr[4];
          f4(rv[j], rr);
          v2[0] = v2[0] + pk(rr[0], rr[1]);
          v2[1] = v2[1] + pk(rr[2], rr[3]);
        }
        float v[4] = {v2[0].x, v2[0].y, v2[1].x, v2[1].y};
        if (relu) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
        }
        if (ystore) store4_f32(a.y, e, v);
        if (ystore && a.ybits)  // uniform; ybits travels with y (host check), so y-less variants compile it out
          a.ybits[e >> 2] = (uint8_t)((v[0] > 0.f) | ((v[1] > 0.f) << 1) | ((v[2] > 0.f) << 2) | ((v[3] > 0.f) << 3));
        if (o1) {
          int c[4];
#pragma unroll
          for (int h = 0; h < 2; ++h)
            quant_w2<ST>(so1, a.qo1.stochastic, pk(v[2 * h], v[2 * h + 1]), pk(no1.u[2 * h], no1.u[2 * h + 1]),
                         ovo[0][0], ovo[0][1], c[2 * h], c[2 * h + 1]);
          if (u8 && relu) store4_i8((int8_t*)a.o1, e, c, 128);  // after the ReLU every code is >= 0
          else if (u8) store4_code(a.o1, LBT_OUT_U8OFF, e, c, 0.f);
          else store4_code(a.o1, a.o1_kind, e, c, so1.inv_m);
        }
        if (o2) {
          int c[4];
#pragma unroll
          for (int h = 0; h < 2; ++h)
            quant_w2<ST>(so2, a.qo2.stochastic, pk(v[2 * h], v[2 * h + 1]), pk(no2.u[2 * h], no2.u[2 * h + 1]),
                         ovo[1][0], ovo[1][1], c[2 * h], c[2 * h + 1]);
          if (u8 && relu) store4_i8((int8_t*)a.o2, e, c, 128);
          else if (u8) store4_code(a.o2, LBT_OUT_U8OFF, e, c, 0.f);
          else store4_code(a.o2, a.o2_kind, e, c, so2.inv_m);
        }
        // one row at a time: interleaving the batch's rows (the scheduler's default) doubles the VGPRs
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  LBT_TS(2);
  // every quantiser's counters behind one barrier
  const bool st[4] = {qr[0].active && a.b1.qr.counts, NB > 1 && qr[NB - 1].active && a.b2.qr.counts,
                      o1 && a.qo1.counts, o2 && a.qo2.counts};
  if (st[0]) counts_stage_w(0, 4, ovr[0][0], ovr[0][1], sh_cnt);
  if (st[1]) counts_stage_w(1, 4, ovr[NB - 1][0], ovr[NB - 1][1], sh_cnt);
  if (st[2]) counts_stage_w(2, 4, ovo[0][0], ovo[0][1], sh_cnt);
  if (st[3]) counts_stage_w(3, 4, ovo[1][0], ovo[1][1], sh_cnt);
  if (!(st[0] || st[1] || st[2] || st[3])) return;
  __syncthreads();
  if (st[0]) counts_publish(0, 4, a.b1.qr, sh_cnt);
  if (st[1]) counts_publish(1, 4, a.b2.qr, sh_cnt);
  if (st[2]) counts_publish(2, 4, a.qo1, sh_cnt);
  if (st[3]) counts_publish(3, 4, a.qo2, sh_cnt);
  LBT_TS(3);
}

// ============================================================================ backward pass A

template <int NB, int F>
__global__ __launch_bounds__(kThreads) void chain_bwd_a_kernel(lbt_chain_bwd_a a, int rpt) {
  extern __shared__ float shf[];  // per branch: gq, bq [C]; then long long sums[2][4C]
  __shared__ int sh_cnt[8 * kThreads / 64];
  constexpr int ST = (F & kRt) ? -1 : ((F & kAStoch) ? 1 : 0);
  LBT_TS(0);
  const int C = a.C;
  long long* S = reinterpret_cast<long long*>(shf + 4 * C);  // [NB][4C]
  const int64_t groups = a.inner >> 2;
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool live = g < groups;
  const int64_t gl = live ? g : 0;
  const int c0 = (int)(((uint32_t)gl << 2) % (uint32_t)C);
  const int64_t r0 = (int64_t)blockIdx.y * rpt;
  const int64_t rend = r0 + rpt < a.rows ? r0 + rpt : a.rows;
  const bool ymask = LBT_FL(kAYMask, a.y_mask != nullptr);
  const bool maskr = LBT_FL(kAMaskR, a.y_mask == nullptr && a.mask_from_r);
  QState qrg[2], qng[2], qr[2];
  bool arg[2], ang[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& Bb = b == 0 ? a.b1 : a.b2;
    qrg[b] = qstate(Bb.qrg);
    qng[b] = qstate(Bb.qng);
    qr[b] = qstate(Bb.qr);
    arg[b] = LBT_FL(kAFB, qrg[b].active);
    ang[b] = LBT_FL(kAFB, qng[b].active);
  }
  const bool r1 = LBT_FL(kAFB, a.b1.R != nullptr);

  // ---- first rows + noise before the (short) prologue
  float4 gv4[kRB], ym4[kRB];
  int R1v[kRB], R2v[kRB], qnv[2][kRB];
  auto load_batch = [&](int64_t rb) {
#pragma unroll
    for (int j = 0; j < kRB; ++j) {
      const int64_t e = (rb + j < rend ? rb + j : r0) * a.inner + (gl << 2);
      gv4[j] = ld_f32x4(a.g, e);
      R1v[j] = r1 ? ld_i8x4(a.b1.R, e) : 0;
      if (ymask) ym4[j] = ld_f32x4(a.y_mask, e);
      if (NB > 1 && arg[NB - 1]) R2v[j] = ld_i8x4(a.b2.R, e);
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (ang[b]) qnv[b][j] = ld_i8x4(b == 0 ? a.b1.qn_codes : a.b2.qn_codes, e);
    }
  };
  load_batch(r0);
  Noise4 nrg[2], nng[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& Bb = b == 0 ? a.b1 : a.b2;
    nrg[b] = noise_for(Bb.qrg, qrg[b], gl);
    nng[b] = noise_for(Bb.qng, qng[b], gl);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& Bb = b == 0 ? a.b1 : a.b2;
    if (Bb.gb)
      for (int c = threadIdx.x; c < C; c += kThreads) { shf[b * 2 * C + c] = Bb.gb[c]; shf[b * 2 * C + C + c] = Bb.gb[C + c]; }
  }
  for (int i = threadIdx.x; i < NB * 4 * C; i += kThreads) S[i] = 0;
  __syncthreads();
  LBT_TS(1);
  float gam[2][4], bet[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int b = 0; b < NB; ++b) gam[b][k] = shf[b * 2 * C + c0 + k];
    bet[k] = shf[C + c0 + k];
  }
  int ov[2][2][2] = {{{0, 0}, {0, 0}}, {{0, 0}, {0, 0}}};  // [branch][rescale|norm][c1|c2], wave totals
  int acc[2][4][4];  // [branch][sum][k]
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[b][s][k] = 0;
  const bool gmask = LBT_FL(kAGmask, a.gmask_out != nullptr);

  for (int64_t rb = r0; rb < rend; rb += kRB) {
    if (rb != r0) load_batch(rb);
    if (live) {
#pragma unroll
      for (int j = 0; j < kRB; ++j) {
        if (rb + j >= rend) break;
        const int64_t e = (rb + j) * a.inner + (g << 2);
        float gv[4];
        f4(gv4[j], gv);
        int R1[4];
        unpack4_i8(R1v[j], R1);
        if (ymask) {
          float ym[4];
          f4(ym4[j], ym);
#pragma unroll
          for (int k = 0; k < 4; ++k) gv[k] = ym[k] > 0.f ? gv[k] : 0.f;
        } else if (maskr) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float xr = (float)R1[k] * qr[0].inv_m;
            const float m1 = xr * gam[0][k];
            const float yv = m1 + bet[k];
            gv[k] = yv > 0.f ? gv[k] : 0.f;
          }
        }
        if (gmask) store4_f32(a.gmask_out, e, gv);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const lbt_bwd_branch& Bb = b == 0 ? a.b1 : a.b2;
          float d[4] = {gv[0], gv[1], gv[2], gv[3]};
          if (arg[b]) {
            int R[4] = {R1[0], R1[1], R1[2], R1[3]};
            if (b) unpack4_i8(R2v[j], R);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int G2 = quant_w<ST>(qrg[b], Bb.qrg.stochastic, d[k], nrg[b].u[k], ov[b][0][0], ov[b][0][1]);
              acc[b][0][k] += G2 * R[k];
              acc[b][1][k] += G2;
              const float gh = (float)G2 * qrg[b].inv_m;
              d[k] = gh * gam[b][k];
            }
          }
          if (ang[b]) {
            int G[4], qn[4];
            unpack4_i8(qnv[b][j], qn);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              G[k] = quant_w<ST>(qng[b], Bb.qng.stochastic, d[k], nng[b].u[k], ov[b][1][0], ov[b][1][1]);
              acc[b][2][k] += G[k];
              acc[b][3][k] += G[k] * qn[k];
            }
            store4_i8(Bb.gout, e, G, 0);
          } else if (Bb.dout) {
            store4_f32(Bb.dout, e, d);
          }
        }
      }
    }
  }
  LBT_TS(2);
  {
    const int per = chan_period(C);
    if (chan_scatter_ok(per)) {  // uniform: row lane >> 4 ends with channel c0 + (lane >> 4)
      const bool own = chan_scatter_owner(per);
      const int cr = (int)(((uint32_t)g << 2) % (uint32_t)C) + (int)((threadIdx.x & 63) >> 4);  // natural quad (c0 is 0 on dead lanes)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int v = chan_scatter4(acc[b][s], per);
          if (own && v) atomicAdd((unsigned long long*)&S[b * 4 * C + s * C + cr], (unsigned long long)(long long)v);
        }
    } else {
      const bool own = chan_owner(per);
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int v = wave_chan_reduce(acc[b][s][k], per);
            if (own && v) atomicAdd((unsigned long long*)&S[b * 4 * C + s * C + c0 + k], (unsigned long long)(long long)v);
          }
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& Bb = b == 0 ? a.b1 : a.b2;
    if (qrg[b].active && Bb.qrg.counts) counts_stage_w(2 * b, 4, ov[b][0][0], ov[b][0][1], sh_cnt);
    if (qng[b].active && Bb.qng.counts) counts_stage_w(2 * b + 1, 4, ov[b][1][0], ov[b][1][1], sh_cnt);
  }
  __syncthreads();  // the only barrier after the main loop: LDS sums and counters complete
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const lbt_bwd_branch& Bb = b == 0 ? a.b1 : a.b2;
    if (qrg[b].active) counts_publish(2 * b, 4, Bb.qrg, sh_cnt);
    if (qng[b].active) counts_publish(2 * b + 1, 4, Bb.qng, sh_cnt);
    if (Bb.sums) block_flush_sums(S + b * 4 * C, 4 * C, Bb.sums, 4 * C);
  }
  LBT_TS(3);
}

// ============================================================================ backward pass B

// (by: the workgroup's row-block index -- blockIdx.y, or its index within its job of a pair launch)
template <int F>
__device__ __forceinline__ void chain_bwd_b_body(const lbt_chain_bwd_b& a, int rpt, uint32_t by) {
  extern __shared__ float shf[];  // mu, sigma, mg, mgx [C]; then long long tmp[2C], csum[2C]
  __shared__ int sh_cnt[8 * kThreads / 64];
  constexpr int ST = (F & kRt) ? -1 : ((F & kBStoch) ? 1 : 0);
  LBT_TS(0);
  const int C = a.C;
  float* mu = shf;
  float* sg = shf + C;
  float* mg = shf + 2 * C;
  float* mgx = shf + 3 * C;
  long long* tmp = reinterpret_cast<long long*>(shf + 4 * C);
  const int64_t groups = a.inner >> 2;
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool live = g < groups;
  const int64_t gl = live ? g : 0;
  const int c0 = (int)(((uint32_t)gl << 2) % (uint32_t)C);
  const int64_t r0 = (int64_t)by * rpt;
  const int64_t rend = r0 + rpt < a.rows ? r0 + rpt : a.rows;
  // ---- first rows + noise before the moment prologue
  int Gv[kRB], qv[kRB];
  auto load_batch = [&](int64_t rb) {
#pragma unroll
    for (int j = 0; j < kRB; ++j) {
      const int64_t e = (rb + j < rend ? rb + j : r0) * a.inner + (gl << 2);
      Gv[j] = ld_i8x4(a.G, e);
      qv[j] = ld_i8x4(a.qn_codes, e);
    }
  };
  load_batch(r0);
  const QState sgq = qstate(a.qng), sn = qstate(a.qn), so = qstate(a.qo);
  const bool want_q = LBT_FL(kBQ, a.gq && so.active);
  const Noise4 no = noise_for(a.qo, so, gl);
  // SG at sums[2C:3C), SGQ at sums[3C:4C) of each shard
  sum_shards(a.sums + 2 * C, 2 * C, 4 * C, tmp);
  long long* csum = tmp + 2 * C;  // this block's gq channel sums [2C]
  for (int i = threadIdx.x; i < 2 * C; i += kThreads) csum[i] = 0;
  __syncthreads();
  {
    const double s = (double)sn.inv_m, gsc = (double)sgq.inv_m, n = (double)a.n;
    for (int c = threadIdx.x; c < C; c += kThreads) {
      const float m = a.ms[c], sig = a.ms[C + c];
      mu[c] = m;
      sg[c] = sig;
      const double SG = (double)tmp[c], SGQ = (double)tmp[C + c];
      mg[c] = (float)(gsc * SG / n);
      mgx[c] = (float)(gsc * (s * SGQ - (double)m * SG) / (n * (double)sig));
    }
  }
  __syncthreads();
  LBT_TS(1);
  float rmu[4], rmg[4], rmgx[4];
  Recip rsg[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rmu[k] = mu[c0 + k];
    rsg[k] = recip(sg[c0 + k]);
    rmg[k] = mg[c0 + k];
    rmgx[k] = mgx[c0 + k];
  }
  int ov1 = 0, ov2 = 0;  // wave totals
  int s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  const bool dxo = LBT_FL(kBDx, a.dx != nullptr);
  for (int64_t rb = r0; rb < rend; rb += kRB) {
    if (rb != r0) load_batch(rb);
    if (live) {
#pragma unroll
      for (int j = 0; j < kRB; ++j) {
        if (rb + j >= rend) break;
        const int64_t e = (rb + j) * a.inner + (g << 2);
        int G[4], q[4];
        unpack4_i8(Gv[j], G);
        unpack4_i8(qv[j], q);
        float dx[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float x1 = (float)q[k] * sn.inv_m;
          const float x2 = x1 - rmu[k];
          const float xh = div_by(x2, rsg[k]);  // == x2 / sigma
          const float gh = (float)G[k] * sgq.inv_m;
          const float t1 = gh - rmg[k];
          const float t2 = xh * rmgx[k];
          dx[k] = div_by(t1 - t2, rsg[k]);      // == (t1 - t2) / sigma
        }
        if (dxo) store4_f32(a.dx, e, dx);
        if (want_q) {
          int c[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            c[k] = quant_w<ST>(so, a.qo.stochastic, dx[k], no.u[k], ov1, ov2);
            s1[k] += c[k];
            s2[k] += c[k] * c[k];
          }
          store4_i8(a.gq, e, c, 0);
        }
      }
    }
  }
  LBT_TS(2);
  const bool gcol = LBT_FL(kBGcol, a.gcolsum != nullptr);
  if (want_q && gcol) {
    const int per = chan_period(C);
    if (chan_scatter_ok(per)) {  // uniform: row lane >> 4 ends with channel c0 + (lane >> 4)
      const bool own = chan_scatter_owner(per);
      const int cr = (int)(((uint32_t)g << 2) % (uint32_t)C) + (int)((threadIdx.x & 63) >> 4);  // natural quad (c0 is 0 on dead lanes)
      const int v1 = chan_scatter4(s1, per), v2 = chan_scatter4(s2, per);
      if (own && v1) atomicAdd((unsigned long long*)&csum[cr], (unsigned long long)(long long)v1);
      if (own && v2) atomicAdd((unsigned long long*)&csum[C + cr], (unsigned long long)(long long)v2);
    } else {
      const bool own = chan_owner(per);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int v1 = wave_chan_reduce(s1[k], per), v2 = wave_chan_reduce(s2[k], per);
        if (own && v1) atomicAdd((unsigned long long*)&csum[c0 + k], (unsigned long long)(long long)v1);
        if (own && v2) atomicAdd((unsigned long long*)&csum[C + c0 + k], (unsigned long long)(long long)v2);
      }
    }
  }
  if (!want_q) return;
  if (a.qo.counts) counts_stage_w(0, 1, ov1, ov2, sh_cnt);
  __syncthreads();
  counts_publish(0, 1, a.qo, sh_cnt);
  if (gcol) block_flush_sums(csum, 2 * C, a.gcolsum, 2 * C);
  LBT_TS(3);
}

template <int F>
__global__ __launch_bounds__(kThreads) void chain_bwd_b_kernel(lbt_chain_bwd_b a, int rpt) {
  chain_bwd_b_body<F>(a, rpt, blockIdx.y);
}

// two same-shaped pass-B chains in one grid: row blocks [0, ny) of job a, then those of job b
template <int F>
__global__ __launch_bounds__(kThreads) void chain_bwd_b2_kernel(lbt_chain_bwd_b a, lbt_chain_bwd_b b, int rpt,
                                                                uint32_t ny) {
  if (blockIdx.y < ny)
    chain_bwd_b_body<F>(a, rpt, blockIdx.y);
  else
    chain_bwd_b_body<F>(b, rpt, blockIdx.y - ny);
}

// num_g / num_b (the exact exchange): the integer sums instead, dequantised after the all-reduce
__global__ void param_grads_kernel(const int64_t* sums, int C, lbt_qdesc qrg, lbt_qdesc qr, const float* gamma,
                                   float wd2, float* dgamma, float* dbeta, long long* num_g, long long* num_b) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  long long sgr = 0, sg = 0;
  for (int k = 0; k < LBT_NSHARD; ++k) {
    sgr += sums[(int64_t)k * 4 * C + c];
    sg += sums[(int64_t)k * 4 * C + C + c];
  }
  if (num_g) {
    num_g[c] = sgr;
    num_b[c] = sg;
    return;
  }
  const double g2 = ldexp(1.0, -frac_exp(qrg)), r = ldexp(1.0, -frac_exp(qr));
  const float a = (float)((double)sgr * (g2 * r));
  const float b = wd2 * gamma[c];
  dgamma[c] = a + b;
  dbeta[c] = (float)((double)sg * g2);
}

// grid over [groups, rows/rpt] with >= ~2048 workgroups
// target: the workgroup count aimed for (LBT_CHAIN_BLOCKS overrides every chain's). The forward chain
// aims at 2048 (ResNet-50: 5.40 -> 5.16 ms per step against 512, 1024: 5.22, 4096: 5.33;
// profiles/round5/chain_blocks_ab.txt), the backward chains keep 512.
bool grid_for(int64_t rows, int64_t inner, dim3& grid, int& rpt, int64_t dflt = 512) {
  const int64_t groups = inner / 4;
  const int64_t gblocks = (groups + kThreads - 1) / kThreads;
  static const int64_t env_target = [] {
    const char* e = getenv("LBT_CHAIN_BLOCKS");
    return (int64_t)(e ? atoi(e) : 0);
  }();
  const int64_t target = env_target > 0 ? env_target : dflt;
  // a workgroup's fixed costs (moment prologue, counter / channel-sum flush) must amortise over
  // enough rows: at least min_rpt per thread even if that leaves fewer than `target` workgroups
  static const int64_t min_rpt = [] {
    const char* e = getenv("LBT_CHAIN_MINRPT");
    return (int64_t)(e ? atoi(e) : 1);
  }();
  int64_t r = (gblocks * rows) / target;
  if (r < min_rpt) r = min_rpt;
  if (r > rows) r = rows;
  if (r < 1) r = 1;
  if (r > 64) r = 64;
  const int64_t yb = (rows + r - 1) / r;
  if (gblocks > 0x7fffffff || yb > 65535) return false;
  grid = dim3((unsigned)gblocks, (unsigned)yb);
  rpt = (int)r;
  return true;
}

bool shape_ok(int64_t rows, int64_t inner, int C) {
  return rows > 0 && inner > 0 && C > 0 && C % 4 == 0 && inner % C == 0 && inner % 4 == 0;
}

// Dynamic LDS above the default 64 KiB (BN layers with C > ~680; gfx950 gives one workgroup up to
// 160 KiB): raise the kernel's limit before launching it.
template <typename K>
void allow_shm(K kernel, size_t shm) {
  if (shm > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)shm);
}
#define LBT_LAUNCH(KERNEL, GRID, SHM, ST, ...)                                  \
  do {                                                                          \
    allow_shm(KERNEL, SHM);                                                     \
    hipLaunchKernelGGL(KERNEL, GRID, dim3(kThreads), SHM, ST, __VA_ARGS__);     \
  } while (0)

}  // namespace

namespace {
// lbt_bn_moments: bn_moments' arithmetic (bn_moments.h), one thread per channel
__global__ __launch_bounds__(256) void bn_moments_kernel(lbt_bn_norm b, int C) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  if (b.frozen) {
    const float m = b.run_mean[c], sigma = sqrtf(b.run_var[c] + b.eps);
    b.ms[c] = m;
    b.ms[C + c] = sigma;
    return;
  }
  long long v1[LBT_NSHARD], v2[LBT_NSHARD];
#pragma unroll
  for (int k = 0; k < LBT_NSHARD; ++k) {
    v1[k] = b.chsum[(int64_t)k * 2 * C + c];
    v2[k] = b.chsum[(int64_t)k * 2 * C + C + c];
  }
  long long s1 = 0, s2 = 0;
#pragma unroll
  for (int k = 0; k < LBT_NSHARD; ++k) {
    s1 += v1[k];
    s2 += v2[k];
  }
  const double s = ldexp(1.0, -frac_exp(b.qn));
  const double mean_d = (double)s1 * s / (double)b.n;
  const double var_d = (double)s2 * (s * s) / (double)b.n - mean_d * mean_d;
  const float m = (float)mean_d, v = (float)var_d;
  const float sigma = sqrtf(v + b.eps);
  b.ms[c] = m;
  b.ms[C + c] = sigma;
  if (b.run_mean) {
    b.run_mean[c] = b.momentum * b.run_mean[c] + b.one_minus_momentum * m;
    b.run_var[c] = b.momentum * b.run_var[c] + b.one_minus_momentum * v;
  }
}
}  // namespace

extern "C" int lbt_bn_moments(const lbt_bn_norm* nrm, int32_t C, void* stream) {
  if (!nrm || C <= 0 || !nrm->ms || (nrm->frozen ? (!nrm->run_mean || !nrm->run_var) : !nrm->chsum)) return LBT_EINVAL;
  hipLaunchKernelGGL(bn_moments_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *nrm,
                     (int)C);
  return (int)hipGetLastError();
}

LBT_TRACE_SETTER(bn)

// ---- host-side variant selection (flag words: chain_flags.h)
namespace {

constexpr int kFwdBlk = kFQ | kFRout | kFRelu | kFStoch;  // every fused-plan forward chain

}  // namespace

extern "C" int lbt_bn_chain_fwd(const lbt_chain_fwd* a, void* stream) {
  if (!shape_ok(a->rows, a->inner, a->C)) return LBT_EINVAL;
  if (a->inner * (LBT_FWD_RB + 1) >= ((int64_t)1 << 31)) return LBT_EINVAL;  // 32-bit lane offsets of a row batch
  if (a->ybits && !a->y) return LBT_EINVAL;  // the ReLU mask bytes are written beside the fp32 block output
  dim3 grid;
  int rpt;
  if (!grid_for(a->rows, a->inner, grid, rpt, 2048)) return LBT_EINVAL;
  // moments precomputed (nrm.ms_in) on every normalising branch: no dynamic LDS (the 48 C bytes of the
  // in-kernel reduction held wide layers to 1-3 workgroups per CU)
  const bool msall = (!a->b1.nrm.q || a->b1.nrm.ms_in) && (!a->has_b2 || !a->b2.nrm.q || a->b2.nrm.ms_in);
  if ((a->b1.nrm.ms_in && !a->b1.nrm.ms) || (a->has_b2 && a->b2.nrm.ms_in && !a->b2.nrm.ms)) return LBT_EINVAL;
  // all or none: a mixed chain would re-run the moments (and the running-average update) of its ms_in branch
  const bool msany = (a->b1.nrm.q && a->b1.nrm.ms_in) || (a->has_b2 && a->b2.nrm.q && a->b2.nrm.ms_in);
  if (msany && !msall) return LBT_EINVAL;
  const size_t shm = msall ? 0 : sizeof(float) * 8 * a->C + sizeof(long long) * 2 * a->C;
  hipStream_t st = (hipStream_t)stream;
  const int f = fwd_flags(*a);
#define LBT_CF(NB, FL)                                                                            \
  if (a->has_b2 == (NB == 2) && f == (FL)) {                                                      \
    LBT_LAUNCH((chain_fwd_kernel<NB, FL>), grid, shm, st, *a, rpt);       \
    return (int)hipGetLastError();                                                                \
  }
  LBT_CF(1, kFwdBlk | kFY | kFO1 | kFU8)                  // stem: bn0 -> relu -> X0 + block-0 input
  LBT_CF(1, kFwdBlk | kFO1 | kFU8)                        // block, first BN: -> conv-2 input
  LBT_CF(1, kFwdBlk | kFRes | kFY | kFO1 | kFU8)          // block end, identity shortcut
  LBT_CF(1, kFwdBlk | kFRes | kFY | kFO1 | kFO2 | kFU8)   // ... next block downsamples
  LBT_CF(1, kFwdBlk | kFRes | kFY)                        // last block
  LBT_CF(2, kFwdBlk | kFY | kFO1 | kFU8)                  // block end, projection shortcut
  LBT_CF(2, kFwdBlk | kFY | kFO1 | kFO2 | kFU8)
  LBT_CF(1, kFQ | kFNoR | kFY)                            // layer-path Normalization_q (ResNet-50 stem)
  LBT_CF(1, kFRout | kFStoch | kFY)                       // ... and its Rescale_q
#undef LBT_CF
  if (getenv("LBT_CHAIN_DEBUG"))
    fprintf(stderr, "chain_fwd kRt: f=%d nb=%d q=%d,%d rout=%d,%d qr=%d/%d,%d/%d o1=%d/%d/%d o2=%d/%d/%d relu=%d res=%d y=%d\n", f,
            a->has_b2 ? 2 : 1, a->b1.nrm.q != nullptr, a->b2.nrm.q != nullptr, a->b1.rout != nullptr, a->b2.rout != nullptr,
            a->b1.qr.bits, a->b1.qr.stochastic, a->b2.qr.bits, a->b2.qr.stochastic, a->o1 != nullptr, a->qo1.bits,
            a->qo1.stochastic, a->o2 != nullptr, a->qo2.bits, a->qo2.stochastic, a->relu, a->res != nullptr, a->y != nullptr);
  if (a->has_b2)
    LBT_LAUNCH((chain_fwd_kernel<2, kRt>), grid, shm, st, *a, rpt);
  else
    LBT_LAUNCH((chain_fwd_kernel<1, kRt>), grid, shm, st, *a, rpt);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_chain_bwd_a(const lbt_chain_bwd_a* a, void* stream) {
  if (!shape_ok(a->rows, a->inner, a->C)) return LBT_EINVAL;
  dim3 grid;
  int rpt;
  if (!grid_for(a->rows, a->inner, grid, rpt)) return LBT_EINVAL;
  const size_t shm = sizeof(float) * 4 * a->C + sizeof(long long) * (a->has_b2 ? 8 : 4) * a->C;
  hipStream_t st = (hipStream_t)stream;
  const int f = bwd_a_flags(*a);
#define LBT_CA(NB, FL)                                                                            \
  if (a->has_b2 == (NB == 2) && f == (FL)) {                                                      \
    LBT_LAUNCH((chain_bwd_a_kernel<NB, FL>), grid, shm, st, *a, rpt);     \
    return (int)hipGetLastError();                                                                \
  }
  LBT_CA(1, kAFB | kAStoch | kAYMask | kAGmask)  // block end, identity shortcut
  LBT_CA(1, kAFB | kAStoch | kAYMask)            // stem
  LBT_CA(1, kAFB | kAStoch | kAMaskR)            // block, first BN (mask recomputed from R)
  LBT_CA(2, kAFB | kAStoch | kAYMask)            // block end, projection shortcut
#undef LBT_CA
  if (a->has_b2)
    LBT_LAUNCH((chain_bwd_a_kernel<2, kRt>), grid, shm, st, *a, rpt);
  else
    LBT_LAUNCH((chain_bwd_a_kernel<1, kRt>), grid, shm, st, *a, rpt);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_chain_bwd_b(const lbt_chain_bwd_b* a, void* stream) {
  if (!shape_ok(a->rows, a->inner, a->C)) return LBT_EINVAL;
  dim3 grid;
  int rpt;
  if (!grid_for(a->rows, a->inner, grid, rpt)) return LBT_EINVAL;
  const size_t shm = sizeof(float) * 4 * a->C + sizeof(long long) * 4 * a->C;
  hipStream_t st = (hipStream_t)stream;
  const int f = bwd_b_flags(*a);
  if (f == (kBQ | kBStoch | kBGcol))
    LBT_LAUNCH((chain_bwd_b_kernel<kBQ | kBStoch | kBGcol>), grid, shm, st, *a, rpt);
  else if (f == (kBQ | kBStoch))
    LBT_LAUNCH((chain_bwd_b_kernel<kBQ | kBStoch>), grid, shm, st, *a, rpt);
  else
    LBT_LAUNCH((chain_bwd_b_kernel<kRt>), grid, shm, st, *a, rpt);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_chain_bwd_b_pair(const lbt_chain_bwd_b* a, const lbt_chain_bwd_b* b, void* stream) {
  if (!a || !b || !shape_ok(a->rows, a->inner, a->C)) return LBT_EINVAL;
  if (a->rows != b->rows || a->inner != b->inner || a->C != b->C) return LBT_EINVAL;
  const int f = bwd_b_flags(*a);
  if (f != bwd_b_flags(*b)) return LBT_EINVAL;
  dim3 grid;
  int rpt;
  if (!grid_for(a->rows, a->inner, grid, rpt)) return LBT_EINVAL;
  const uint32_t ny = grid.y;
  if ((uint64_t)ny * 2 > 65535) return LBT_EINVAL;
  grid.y = 2 * ny;
  const size_t shm = sizeof(float) * 4 * a->C + sizeof(long long) * 4 * a->C;
  hipStream_t st = (hipStream_t)stream;
  if (f == (kBQ | kBStoch | kBGcol))
    LBT_LAUNCH((chain_bwd_b2_kernel<kBQ | kBStoch | kBGcol>), grid, shm, st, *a, *b, rpt, ny);
  else if (f == (kBQ | kBStoch))
    LBT_LAUNCH((chain_bwd_b2_kernel<kBQ | kBStoch>), grid, shm, st, *a, *b, rpt, ny);
  else
    LBT_LAUNCH((chain_bwd_b2_kernel<kRt>), grid, shm, st, *a, *b, rpt, ny);
  return (int)hipGetLastError();
}

extern "C" int lbt_bn_param_grads(const int64_t* sums, int32_t C, lbt_qdesc qrg, lbt_qdesc qr, const float* gamma,
                                  float wd2, float* dgamma, float* dbeta, void* stream) {
  hipLaunchKernelGGL(param_grads_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, C, qrg, qr,
                     gamma, wd2, dgamma, dbeta, nullptr, nullptr);
  return (int)hipGetLastError();
}
extern "C" int lbt_bn_param_grads_x(const int64_t* sums, int32_t C, int64_t* num_g, int64_t* num_b, void* stream) {
  if (!num_g || !num_b || C <= 0) return LBT_EINVAL;
  hipLaunchKernelGGL(param_grads_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, C, lbt_qdesc{},
                     lbt_qdesc{}, nullptr, 0.f, nullptr, nullptr, (long long*)num_g, (long long*)num_b);
  return (int)hipGetLastError();
}

// pk2.h -- channel pairs on packed fp32 for the element-chain kernels (bn.hip, bn_wide.hip).
#pragma once
#include "dfxp_device.h"

namespace lbt {

// The quantisers' last steps for an ACTIVE quantiser (L >= 1) and a non-NaN operand -- every caller of the
// packed helpers below: the clip is one v_med3_f32 (fminf(fmaxf(v, -L), L - 1) needs two; the fused conv
// kernels' qfloor2 already clips this way), and floor + conversion is one v_cvt_flr_i32_f32 (exact: |v|
// <= 2^15). The element chains are VALU-bound (profiles/round5/chain_pmc.txt).
LBT_DEV float clip_q(const QState& s, float v) { return __builtin_amdgcn_fmed3f(v, -s.L, s.Lm1); }

// v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32: each half rounded exactly as the scalar op. The element
// chains are VALU-heavy on the wide layers (ResNet-50: ~30-40 VALU ops per element against 3-12 bytes),
// so their multiplies / adds / fmas run two channels per instruction; compares, clamps, floors and
// conversions stay scalar.
typedef float pf2 __attribute__((ext_vector_type(2)));
LBT_DEV pf2 pk(float a, float b) { return pf2{a, b}; }
LBT_DEV pf2 pcvt(int a, int b) { return pf2{(float)a, (float)b}; }
// div_by on a pair (the same operations, so the same bits as '/')
LBT_DEV pf2 pdiv(pf2 x, pf2 y, pf2 rc) {
  const pf2 q = x * rc;
  const pf2 r = __builtin_elementwise_fma(-y, q, x);
  const pf2 q1 = __builtin_elementwise_fma(r, rc, q);
  const pf2 r1 = __builtin_elementwise_fma(-y, q1, x);
  return __builtin_elementwise_copysign(__builtin_elementwise_fma(r1, rc, q1), x);
}
// pdiv for dividends that are never -0 (the copysign only restores x = -0; the BN normalisation's
// q s - mu is q s for q = 0, i.e. +0, or a difference of two equal values, +0): one VALU fewer per element
LBT_DEV pf2 pdiv_nz(pf2 x, pf2 y, pf2 rc) {
  const pf2 q = x * rc;
  const pf2 r = __builtin_elementwise_fma(-y, q, x);
  const pf2 q1 = __builtin_elementwise_fma(r, rc, q);
  const pf2 r1 = __builtin_elementwise_fma(-y, q1, x);
  return __builtin_elementwise_fma(r1, rc, q1);
}
// quant_w on a pair: the codes of x.x / x.y into c0 / c1, wave-total overflow counts. The predicates
// x m >= T or x m < -T (T = L, Lh: powers of two) as ONE compare each on max(x m, -x m (1 - 2^-24)) (see
// quant4_w below): one packed multiply and two max for the pair instead of a second compare and an OR per
// element and threshold -- the ResNet-50 forward chains are VALU-bound (profiles/round5/chain_pmc.txt).
template <int STOCH>
LBT_DEV void quant_w2(const QState& s, int stochastic, pf2 x, pf2 u, int& ov1w, int& ov2w, int& c0, int& c1) {
  const pf2 xm = x * pk(s.m, s.m);
  const pf2 ng = xm * pk(-0x1.fffffep-1f, -0x1.fffffep-1f);
  const float a0 = fmaxf(xm.x, ng.x), a1 = fmaxf(xm.y, ng.y);
  ov1w += __popcll(__ballot(a0 >= s.L)) + __popcll(__ballot(a1 >= s.L));
  ov2w += __popcll(__ballot(a0 >= s.Lh)) + __popcll(__ballot(a1 >= s.Lh));
  const bool st = STOCH < 0 ? stochastic != 0 : STOCH == 1;
  const pf2 v = st ? xm + u : xm;
  const float v0 = clip_q(s, v.x), v1 = clip_q(s, v.y);
  if (STOCH == 1) {
    c0 = floor_i(v0);
    c1 = floor_i(v1);
  } else {
    c0 = (int)(st ? floorf(v0) : rintf(v0));
    c1 = (int)(st ? floorf(v1) : rintf(v1));
  }
}

// Four consecutive elements (one float4) through a stochastic (ST) or round-to-nearest quantiser: codes
// c[0..3] and the overflow counts as WAVE totals added to ov1w / ov2w in every active lane (quant_w's
// convention). One v_cmp per element and predicate: the asymmetric x*m >= T or x*m < -T (T a power of two)
// equals max(x*m, -x*m (1 - 2^-24)) >= T (x*m < 0: the product rounds to >= T exactly when -x*m > T; NaN
// compares false either way); the multiplies / adds run on packed pairs, each half rounded as the scalar
// op, and the stochastic / nearest choice is compile time -- bit-identical to quant1 / quant_w per element
// at about half their VALU count.
template <bool ST>
LBT_DEV void quant4_w(const QState& s, const float4& x, const float4& u, int (&c)[4], int& ov1w, int& ov2w) {
  const pf2 m2 = pk(s.m, s.m), k2 = pk(-0x1.fffffep-1f, -0x1.fffffep-1f);
  const pf2 xm[2] = {pk(x.x, x.y) * m2, pk(x.z, x.w) * m2};
  const pf2 ng[2] = {xm[0] * k2, xm[1] * k2};
  const float a[4] = {fmaxf(xm[0].x, ng[0].x), fmaxf(xm[0].y, ng[0].y), fmaxf(xm[1].x, ng[1].x),
                      fmaxf(xm[1].y, ng[1].y)};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ov1w += __popcll(__ballot(a[e] >= s.L));
    ov2w += __popcll(__ballot(a[e] >= s.Lh));
  }
  pf2 v[2] = {xm[0], xm[1]};
  if constexpr (ST) {
    v[0] = v[0] + pk(u.x, u.y);
    v[1] = v[1] + pk(u.z, u.w);
  }
  const float w[4] = {v[0].x, v[0].y, v[1].x, v[1].y};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float vv = clip_q(s, w[e]);
    c[e] = ST ? floor_i(vv) : (int)rintf(vv);
  }
}

}  // namespace lbt

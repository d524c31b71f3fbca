// chain_flags.h -- configuration words of the element-chain kernels (bn.hip) and of the GEMM
// epilogues that run the same chains (conv_mfma.hip): each launch's descriptor is reduced to a
// flag word on the host, and the combinations the fused ResNet plan uses are compiled as their
// own kernel variants (no per-element branches); kRt selects the run-time-descriptor variant.
#pragma once
#include "dfxp_device.h"

namespace lbt {

enum : int {
  kRt = 1 << 20,
  // forward
  kFQ = 1,       // branch inputs are int8 Normalization_q codes (else fp32 xin)
  kFRout = 2,    // store the Rescale_q codes R
  kFRes = 4,     // residual add
  kFRelu = 8,
  kFY = 16,      // store fp32 y
  kFO1 = 32,     // first output quantiser
  kFO2 = 64,     // second output quantiser
  kFStoch = 128, // every quantiser stochastic
  kFU8 = 256,    // outputs in the unsigned 9-bit offset encoding
  kFNoR = 512,   // no Rescale_q part (a layer-path Normalization_q alone)
};

enum : int {
  kAYMask = 1,   // ReLU mask from the fp32 forward output y_mask
  kAMaskR = 2,   // ReLU mask recomputed from the Rescale_q codes of branch 1
  kAGmask = 4,   // store the masked fp32 gradient
  kAStoch = 8,   // every quantiser stochastic
  kAFB = 16,     // every branch: both quantisers active, int8 G codes and sums out
};

enum : int {
  kBQ = 1,      // quantised gq output (else fp32 dx)
  kBGcol = 2,   // per-channel sums of gq
  kBStoch = 4,  // stochastic output quantiser
  kBDx = 8,     // fp32 dx output
};

#define LBT_FL(bit, rt) ((F & kRt) ? (rt) : ((F & (bit)) != 0))

// ---- host side: the descriptor's configuration as a flag word, or kRt when it is not uniform
// across branches / quantisers.
inline int tri(bool all, bool none) { return all ? 1 : (none ? 0 : -1); }

inline int fwd_flags(const lbt_chain_fwd& a) {
  const int nb = a.has_b2 ? 2 : 1;
  const lbt_chain_branch* br[2] = {&a.b1, &a.b2};
  bool q_all = true, q_none = true, r_all = true, r_none = true, act = true, act_none = true;
  bool st_all = true, st_none = true;
  for (int b = 0; b < nb; ++b) {
    q_all &= br[b]->nrm.q != nullptr; q_none &= br[b]->nrm.q == nullptr;
    r_all &= br[b]->rout != nullptr; r_none &= br[b]->rout == nullptr;
    act &= br[b]->qr.bits > 0;
    act_none &= br[b]->qr.bits <= 0;
    st_all &= br[b]->qr.stochastic != 0; st_none &= br[b]->qr.stochastic == 0;
  }
  const bool o1 = a.o1 && a.qo1.bits > 0, o2 = a.o2 && a.qo2.bits > 0;
  if (o1) { st_all &= a.qo1.stochastic != 0; st_none &= a.qo1.stochastic == 0; }
  if (o2) { st_all &= a.qo2.stochastic != 0; st_none &= a.qo2.stochastic == 0; }
  const int q = tri(q_all, q_none), r = tri(r_all, r_none), st = tri(st_all, st_none);
  if (q < 0 || r < 0 || st < 0 || !(act || (act_none && r == 0))) return kRt;
  int f = act ? 0 : kFNoR;
  if (q) f |= kFQ;
  if (r) f |= kFRout;
  if (a.res) f |= kFRes;
  if (a.relu) f |= kFRelu;
  if (a.y) f |= kFY;
  if (o1) f |= kFO1;
  if (o2) f |= kFO2;
  if (st) f |= kFStoch;
  if ((o1 || o2) && (!o1 || a.o1_kind == LBT_OUT_U8OFF) && (!o2 || a.o2_kind == LBT_OUT_U8OFF)) f |= kFU8;
  return f;
}

inline int bwd_a_flags(const lbt_chain_bwd_a& a) {
  const int nb = a.has_b2 ? 2 : 1;
  const lbt_bwd_branch* br[2] = {&a.b1, &a.b2};
  bool fb = a.b1.R != nullptr, st_all = true, st_none = true;
  for (int b = 0; b < nb; ++b) {
    const lbt_bwd_branch& B = *br[b];
    fb &= B.qrg.bits > 0 && B.qng.bits > 0 && B.gout && B.sums && B.R && !B.dout && B.qn_codes;
    st_all &= B.qrg.stochastic != 0 && B.qng.stochastic != 0;
    st_none &= B.qrg.stochastic == 0 && B.qng.stochastic == 0;
  }
  if (!fb) return kRt;
  int f = kAFB;
  if (a.y_mask) f |= kAYMask;
  else if (a.mask_from_r) f |= kAMaskR;
  if (a.gmask_out) f |= kAGmask;
  if (st_all) f |= kAStoch;
  else if (!st_none) return kRt;
  return f;
}

inline int bwd_b_flags(const lbt_chain_bwd_b& a) {
  int f = 0;
  if (a.gq && a.qo.bits > 0) f |= kBQ | (a.qo.stochastic ? kBStoch : 0);
  if (a.gcolsum) f |= kBGcol;
  if (a.dx) f |= kBDx;
  return f;
}

}  // namespace lbt

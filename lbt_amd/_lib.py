"""ctypes binding of ``include/lbt_dfxp.h`` -- the C-ABI of the gfx950 DFXP kernels.

This is the only place Python touches the native library. There is no CPU fallback: if
``liblbt_dfxp.so`` is missing or fails to load, every op raises. ``torch`` is imported first
so that the HIP runtime the library binds to (``libamdhip64.so.7``) is the one PyTorch-ROCm
already loaded -- device pointers and streams are then shared with torch.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime before the kernels library)

HERE = os.path.dirname(os.path.abspath(__file__))
# LBT_LIBRARY: an alternative build of the same C-ABI (e.g. instrumented scratch builds for kernel
# studies); the default is the in-tree build.
LIB_PATH = os.environ.get("LBT_LIBRARY") or os.path.join(HERE, "liblbt_dfxp.so")

NSHARD = 32
STEM_WG_PIXELS = 256  # LBT_STEM_WG_PIXELS
CSTRIDE = 32  # int32 stride between overflow-counter shards (LBT_CSTRIDE)
OUT_I8, OUT_U8OFF, OUT_I16, OUT_F32 = 0, 1, 2, 3
ABI_VERSION = 21

c_void_p, c_int32, c_int64, c_uint32, c_uint64, c_float = (
    ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float)


class QDesc(ctypes.Structure):
    _fields_ = [("exps", c_void_p), ("counts", c_void_p), ("step", c_void_p), ("seed", c_uint64),
                ("qid", c_uint32), ("slot", c_int32), ("bits", c_int32), ("stochastic", c_int32),
                ("noise", c_void_p)]


NO_Q = QDesc()  # bits == 0: inactive quantiser


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("N", "H", "W", "Cin", "Cout", "KH", "KW", "SH", "SW",
                                       "PT", "PB", "PL", "PR", "Ho", "Wo")]


class BnNorm(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("qn", QDesc), ("chsum", c_void_p), ("n", c_int64),
                ("eps", c_float), ("momentum", c_float), ("one_minus_momentum", c_float),
                ("ms", c_void_p), ("run_mean", c_void_p), ("run_var", c_void_p), ("frozen", c_int32),
                ("ms_in", c_int32)]


class ChainBranch(ctypes.Structure):
    _fields_ = [("nrm", BnNorm), ("xin", c_void_p), ("qr", QDesc), ("rout", c_void_p), ("gb", c_void_p)]


class ChainFwd(ctypes.Structure):
    _fields_ = [("b1", ChainBranch), ("b2", ChainBranch), ("has_b2", c_int32),
                ("res", c_void_p), ("relu", c_int32), ("y", c_void_p),
                ("o1", c_void_p), ("o1_kind", c_int32), ("qo1", QDesc),
                ("o2", c_void_p), ("o2_kind", c_int32), ("qo2", QDesc),
                ("rows", c_int64), ("inner", c_int64), ("C", c_int32), ("ybits", c_void_p)]


class BwdBranch(ctypes.Structure):
    _fields_ = [("qrg", QDesc), ("R", c_void_p), ("qr", QDesc), ("gb", c_void_p),
                ("qng", QDesc), ("qn_codes", c_void_p), ("gout", c_void_p), ("dout", c_void_p),
                ("sums", c_void_p)]


class ChainBwdA(ctypes.Structure):
    _fields_ = [("g", c_void_p), ("y_mask", c_void_p), ("mask_from_r", c_int32), ("gmask_out", c_void_p),
                ("b1", BwdBranch), ("b2", BwdBranch), ("has_b2", c_int32),
                ("rows", c_int64), ("inner", c_int64), ("C", c_int32)]


class ChainBwdB(ctypes.Structure):
    _fields_ = [("G", c_void_p), ("qng", QDesc), ("qn_codes", c_void_p), ("qn", QDesc), ("ms", c_void_p),
                ("sums", c_void_p), ("n", c_int64),
                ("dx", c_void_p), ("gq", c_void_p), ("qo", QDesc), ("gcolsum", c_void_p),
                ("rows", c_int64), ("inner", c_int64), ("C", c_int32)]


class WgradJob(ctypes.Structure):
    _fields_ = [("xq", c_void_p), ("x_u8off", c_int32), ("gq", c_void_p), ("d", ConvDesc), ("slab", c_void_p),
                ("nsplit", c_int32), ("nshard", c_int32)]


class ConvBwd(ctypes.Structure):
    _fields_ = [("b", ChainBwdB), ("wd", c_void_p), ("ksd", c_int32), ("w4", c_int32), ("d", ConvDesc),
                ("qw", QDesc), ("add_src", c_void_p), ("a", ChainBwdA), ("w", WgradJob)]


class ConvBwd2(ctypes.Structure):
    _fields_ = [("b1", ChainBwdB), ("bs", ChainBwdB), ("wd1", c_void_p), ("ksd1", c_int32), ("wds", c_void_p),
                ("ksds", c_int32), ("w4", c_int32), ("d1", ConvDesc), ("ds", ConvDesc), ("qw1", QDesc),
                ("qws", QDesc), ("a", ChainBwdA)]


class ConvFwd(ctypes.Structure):
    _fields_ = [("c", ChainFwd), ("wf", c_void_p), ("ksf", c_int32), ("w4", c_int32), ("wcolsum", c_void_p),
                ("d", ConvDesc), ("qw", QDesc), ("yq", c_void_p), ("qout", QDesc), ("ychsum", c_void_p)]


class ConvFwd2(ctypes.Structure):
    _fields_ = [("c", ChainFwd), ("wf1", c_void_p), ("ksf1", c_int32), ("wcolsum1", c_void_p), ("wfs", c_void_p),
                ("ksfs", c_int32), ("wcolsums", c_void_p), ("w4", c_int32), ("d1", ConvDesc), ("ds", ConvDesc),
                ("qw1", QDesc), ("qws", QDesc), ("yq1", c_void_p), ("qout1", QDesc), ("ychsum1", c_void_p),
                ("yqs", c_void_p), ("qouts", QDesc), ("ychsums", c_void_p)]


class ConvFwdJob(ctypes.Structure):
    _fields_ = [("xq", c_void_p), ("x_u8off", c_int32), ("w4", c_int32), ("wf", c_void_p), ("ksf", c_int32),
                ("wcolsum", c_void_p), ("d", ConvDesc), ("qx", QDesc), ("qw", QDesc), ("y", c_void_p),
                ("yq", c_void_p), ("qout", QDesc), ("ychsum", c_void_p)]


class WJob(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("KH", c_int32), ("KW", c_int32), ("Cin", c_int32), ("Cout", c_int32),
                ("q", QDesc), ("w_hwio", c_void_p), ("wf", c_void_p), ("ksf", c_int32), ("wd", c_void_p),
                ("ksd", c_int32), ("colsum", c_void_p)]


class QJob(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("out", c_void_p), ("out_kind", c_int32), ("n", c_int64), ("inner", c_int64),
                ("q", QDesc)]


class NJob(ctypes.Structure):
    _fields_ = [("step", c_void_p), ("seed", c_uint64), ("qid", c_uint32), ("pad", c_int32), ("n", c_int64),
                ("out", c_void_p)]


class RJob(ctypes.Structure):
    _fields_ = [("slab", c_void_p), ("nsplit", c_int32), ("K", c_int32), ("Cout", c_int32), ("x_u8off", c_int32),
                ("gcolsum", c_void_p), ("qx", QDesc), ("qg", QDesc), ("w", c_void_p), ("wd2", c_float),
                ("dw", c_void_p)]


class R64Job(ctypes.Structure):
    _fields_ = [("slab", c_void_p), ("nsplit", c_int32), ("K", c_int32), ("Cout", c_int32), ("first_block", c_int32),
                ("qx", QDesc), ("qg", QDesc), ("w", c_void_p), ("wd2", c_float), ("dw", c_void_p)]


class PJob(ctypes.Structure):
    _fields_ = [("sums", c_void_p), ("C", c_int32), ("qrg", QDesc), ("qr", QDesc), ("gamma", c_void_p),
                ("wd2", c_float), ("dgamma", c_void_p), ("dbeta", c_void_p)]


class Head(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("N", c_int32), ("HW", c_int32), ("C", c_int32), ("K", c_int32),
                ("pooled", c_void_p), ("pq", c_void_p), ("qx", QDesc),
                ("wq", c_void_p), ("qw", QDesc),
                ("labels", c_void_p), ("logits", c_void_p), ("loss", c_void_p), ("dz", c_void_p),
                ("gq", c_void_p), ("qg", QDesc),
                ("w", c_void_p), ("wd2", c_float), ("dw", c_void_p),
                ("gx", c_void_p),
                ("scratch", c_void_p), ("loss_n", c_int32), ("pa", c_void_p), ("chain", c_void_p)]


class Xchg(ctypes.Structure):
    _fields_ = [("buf", c_void_p), ("gbase", c_void_p), ("pjob_scale", c_int32), ("nslots", c_int32),
                ("counts", c_void_p), ("cnt_off", c_int64), ("loss_off", c_int64)]


class IgemmTuning(ctypes.Structure):
    _fields_ = [("big", c_int32), ("min_tiles", c_int32), ("stages", c_int32), ("max_bn", c_int32),
                ("halo", c_int32), ("fwdq_perm", c_int32), ("launches", c_int64)]


class Update(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("a", c_void_p), ("g", c_void_p), ("lr", c_float), ("mu", c_float),
                ("exps", c_void_p), ("counts", c_void_p), ("bits", c_void_p), ("target", c_void_p),
                ("nelem", c_void_p), ("step", c_void_p), ("nslots", c_int32), ("pad", c_int32)]


class DgradBna(ctypes.Structure):
    _fields_ = [("qr", QDesc), ("R", c_void_p), ("gb", c_void_p), ("qrg", QDesc), ("qng", QDesc), ("qn", c_void_p),
                ("gout", c_void_p), ("sums", c_void_p)]


class BnaBn(ctypes.Structure):
    _fields_ = [("qrg", QDesc), ("R", c_void_p), ("gamma_q", c_void_p), ("qng", QDesc), ("qn", c_void_p),
                ("gout", c_void_p), ("sums", c_void_p)]


class DgradBn3(ctypes.Structure):
    _fields_ = [("g2", c_void_p), ("y_bits", c_void_p), ("gmask_out", c_void_p), ("nbn", c_int32), ("pad", c_int32),
                ("bn", BnaBn * 2)]


class FSeg(ctypes.Structure):
    _fields_ = [("off", c_int64), ("n", c_int64), ("kind", c_int32), ("qx", QDesc), ("qg", QDesc), ("wd2", c_float)]


_P = c_void_p
_SIGS = {
    "lbt_abi_version": [],
    "lbt_dfxp_quantize": [_P, _P, c_int32, c_int64, c_int64, QDesc, _P, c_int32, _P],
    "lbt_dfxp_range_update": [_P, _P, _P, _P, _P, c_int32, _P, _P],
    "lbt_dfxp_counts_fold": [_P, c_int32, _P, _P],
    "lbt_dfxp_range_update_folded": [_P, _P, _P, _P, _P, c_int32, _P, _P],
    "lbt_dfxp_quantize_weight": [_P, c_int32, c_int32, c_int32, c_int32, QDesc, _P, _P, c_int32, _P, c_int32,
                                 _P, _P],
    "lbt_conv_fwd_i8": [_P, c_int32, _P, c_int32, _P, ConvDesc, QDesc, QDesc, _P, _P, QDesc, _P, _P],
    "lbt_conv_dgrad_i8": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P],
    "lbt_conv_fwd_i8w4": [_P, c_int32, _P, c_int32, _P, ConvDesc, QDesc, QDesc, _P, _P, QDesc, _P, _P],
    "lbt_conv_dgrad_i8w4": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P],
    "lbt_pack_int4": [_P, _P, c_int64, _P],
    "lbt_conv_fwd_igemm": [_P, c_int32, _P, c_int32, _P, ConvDesc, QDesc, QDesc, _P, _P],
    "lbt_conv_dgrad_igemm": [_P, c_int32, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P],
    "lbt_conv_wgrad_igemm": [_P, _P, c_int32, ConvDesc, _P, c_int32, c_int32, _P],
    "lbt_igemm_workspace_bytes": [ConvDesc, c_int32, c_int32],
    "lbt_igemm_get_tuning": [_P],
    "lbt_igemm_set_tuning": [_P],
    "lbt_conv_fwd_igemm_q": [_P, c_int32, _P, c_int32, ConvDesc, QDesc, QDesc, _P, QDesc, _P, _P],
    "lbt_conv_fwd_igemm_ws": [_P, c_int32, _P, c_int32, _P, ConvDesc, QDesc, QDesc, _P, _P, c_int64, _P],
    "lbt_conv_dgrad_igemm_ws": [_P, c_int32, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P, c_int64, _P],
    "lbt_conv_dgrad_igemm_bna": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, ctypes.POINTER(DgradBna), _P, _P, c_int64,
                                 _P],
    "lbt_bn_moments": [ctypes.POINTER(BnNorm), c_int32, _P],
    "lbt_conv_dgrad_igemm_bn3": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, ctypes.POINTER(DgradBn3), _P, _P, c_int64,
                                 _P],
    "lbt_conv_wgrad_igemm_store": [_P, _P, c_int32, ConvDesc, _P, c_int32, _P],
    "lbt_conv_dgrad_chain_i8w4": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P],
    "lbt_conv_dgrad_chain_i8": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P],
    "lbt_conv_dgrad_chain_wgrad_i8": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P, c_int32, _P, c_int32,
                                      c_int32, _P],
    "lbt_conv_dgrad_chain_wgrad_i8w4": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, _P, c_int32, _P, c_int32,
                                        c_int32, _P],
    "lbt_conv_wgrad_i8": [_P, c_int32, _P, ConvDesc, _P, c_int32, c_int32, _P],
    "lbt_conv_wgrad_many_i8": [_P, c_int32, _P],
    "lbt_conv_wgrad_many_stem_i8": [_P, c_int32, _P, _P, ConvDesc, _P, c_int32, _P],
    "lbt_conv_wgrad_reduce": [_P, c_int32, c_int32, c_int32, c_int32, _P, QDesc, QDesc, _P, c_float, _P, _P],
    "lbt_conv_fwd_generic": [_P, c_int32, _P, ConvDesc, QDesc, QDesc, _P, _P],
    "lbt_conv_dgrad_generic": [_P, _P, ConvDesc, QDesc, QDesc, _P, _P, _P],
    "lbt_conv_wgrad_generic": [_P, c_int32, _P, ConvDesc, _P, c_int32, _P],
    "lbt_conv_dgrad_generic16": [_P, _P, ConvDesc, QDesc, QDesc, _P, _P, _P],
    "lbt_conv_wgrad_generic16": [_P, c_int32, _P, ConvDesc, _P, c_int32, _P],
    "lbt_conv_wgrad_reduce64": [_P, c_int32, c_int32, c_int32, QDesc, QDesc, _P, c_float, _P, _P],
    "lbt_conv_wgrad_reduce64_many": [_P, c_int32, c_int32, _P],
    "lbt_conv_stem_fwd": [_P, _P, ConvDesc, QDesc, QDesc, _P, _P, QDesc, _P, _P],
    "lbt_conv_stem_wgrad": [_P, _P, ConvDesc, _P, c_int32, _P],
    "lbt_conv_stem_bwd": [_P, _P, ConvDesc, _P, c_int32, _P],
    "lbt_conv_bwd2_fused_i8": [_P, _P],
    "lbt_conv_fwd2_fused_i8": [_P, _P],
    "lbt_conv_wgrad_reduce_x": [_P, c_int32, c_int32, c_int32, c_int32, _P, _P, _P],
    "lbt_conv_wgrad_reduce64_x": [_P, c_int32, c_int32, c_int32, _P, _P],
    "lbt_dense_wgrad_x": [_P, _P, c_int32, c_int32, c_int32, c_int32, _P, _P],
    "lbt_bn_param_grads_x": [_P, c_int32, _P, _P, _P],
    "lbt_softmax_xent_n": [_P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P],
    "lbt_softmax_xent_wide_n": [_P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P],
    "lbt_conv_stem_wide_fwd": [_P, _P, ConvDesc, QDesc, QDesc, _P, _P],
    "lbt_stem_wide_nsplit": [ConvDesc],
    "lbt_conv_stem_wide_wgrad": [_P, c_int32, _P, c_int32, ConvDesc, _P, c_int32, _P],
    "lbt_dense_pack": [_P, c_int32, c_int32, _P, c_int32, _P, c_int32, _P],
    "lbt_flat_weight_blocks": [c_int64],
    "lbt_dfxp_quantize_weights_flat": [_P, _P, c_int32, c_int32, _P],
    "lbt_bn_bwd_a_wide_masked": [_P, _P, _P, _P, c_int32, QDesc, _P, _P, QDesc, _P, QDesc, _P, _P, _P, _P, c_int64, c_int64,
                                 c_int32, _P],
    "lbt_bn_bwd_b_wide_q": [_P, QDesc, _P, QDesc, _P, _P, c_int64, _P, QDesc, c_int64, c_int64, c_int32, _P],
    "lbt_dense_gemm": [_P, c_int32, c_int32, c_int32, _P, c_int32, c_int32, c_int32, QDesc, QDesc, _P, _P],
    "lbt_dense_wgrad": [_P, _P, c_int32, c_int32, c_int32, c_int32, QDesc, QDesc, _P, c_float, _P, _P],
    "lbt_softmax_xent_wide": [_P, _P, c_int32, c_int32, _P, _P, _P],
    "lbt_bn_chain_fwd": [_P, _P],
    "lbt_bn_chain_bwd_a": [_P, _P],
    "lbt_bn_chain_bwd_b": [_P, _P],
    "lbt_bn_chain_bwd_b_pair": [_P, _P, _P],
    "lbt_conv_fwd_pair_i8": [_P, _P, _P],
    "lbt_conv_dgrad2_chain_i8": [_P, _P, c_int32, ConvDesc, QDesc, QDesc, _P, _P, c_int32, ConvDesc, QDesc, QDesc,
                                 c_int32, _P, _P],
    "lbt_conv_bwd_fused_i8": [_P, _P],
    "lbt_conv_fwd_fused_i8": [_P, _P],
    "lbt_bn_bwd_a_wide": [_P, QDesc, _P, _P, QDesc, _P, _P, _P, _P, c_int64, c_int64, c_int32, _P],
    "lbt_bn_bwd_b_wide": [_P, QDesc, _P, QDesc, _P, _P, c_int64, _P, c_int64, c_int32, _P],
    "lbt_bn_param_grads": [_P, c_int32, QDesc, QDesc, _P, c_float, _P, _P, _P],
    "lbt_relu_fwd": [_P, _P, c_int64, _P],
    "lbt_relu_bwd": [_P, _P, _P, c_int64, _P],
    "lbt_add": [_P, _P, _P, c_int64, _P],
    "lbt_maxpool_fwd": [_P, _P, _P, ConvDesc, _P],
    "lbt_maxpool_bwd": [_P, _P, _P, ConvDesc, _P],
    "lbt_maxpool_relu_bwd": [_P, _P, _P, _P, ConvDesc, _P],
    "lbt_maxpool_relu_fwd": [_P, _P, _P, ConvDesc, _P],
    "lbt_avgpool_fwd": [_P, _P, c_int32, c_int32, c_int32, _P],
    "lbt_avgpool_bwd": [_P, _P, c_int32, c_int32, c_int32, _P],
    "lbt_avgpool_gen_fwd": [_P, _P, ConvDesc, _P],
    "lbt_conv_fwd_f32": [_P, _P, ConvDesc, _P, _P],
    "lbt_conv_dgrad_f32": [_P, _P, ConvDesc, _P, _P, _P],
    "lbt_conv_wgrad_f32": [_P, _P, ConvDesc, _P, c_int32, _P],
    "lbt_conv_wgrad_reduce_f32": [_P, c_int32, c_int64, _P, c_float, _P, _P],
    "lbt_chan_sums_f32": [_P, _P, c_int64, c_int32, c_int32, _P, _P],
    "lbt_bn_f32_fwd": [_P, _P, c_int32, c_int64, c_int32, c_float, c_float, c_float, _P, _P, _P, c_int32, _P, _P],
    "lbt_bn_f32_bwd": [_P, _P, _P, _P, c_int32, c_int64, c_int32, c_int32, _P, _P],
    "lbt_affine_f32": [_P, _P, c_int64, c_int32, c_int32, _P, _P],
    "lbt_affine_grads_f32": [_P, c_int32, c_int32, _P, c_float, _P, _P, _P],
    "lbt_avgpool_gen_bwd": [_P, _P, ConvDesc, _P],
    "lbt_softmax_xent": [_P, _P, c_int32, c_int32, _P, _P, _P],
    "lbt_sgd_momentum": [_P, _P, _P, c_int64, c_float, c_float, c_float, _P],
    "lbt_bias_add": [_P, _P, c_int64, c_int32, _P],
    "lbt_bias_grad": [_P, c_int32, QDesc, _P, _P],
    "lbt_dfxp_quantize_weights": [_P, c_int32, c_int32, _P],
    "lbt_dfxp_quantize_many": [_P, c_int32, _P],
    "lbt_dfxp_noise_fill": [_P, c_int32, c_int64, _P, c_int64, _P],
    "lbt_selftest_div": [_P, _P, c_int64, _P, _P, _P, _P],
    "lbt_conv_wgrad_reduce_many": [_P, c_int32, c_int32, _P],
    "lbt_bn_param_grads_many": [_P, c_int32, c_int32, _P],
    "lbt_head_scratch_bytes": [c_int32, c_int32, c_int32],
    "lbt_rjob_blocks": [c_int64],
    "lbt_head_fwd_bwd": [_P, _P],
    "lbt_step_prologue": [_P, c_int32, c_int64, _P, c_int64, _P, c_int32, c_int32, _P, c_int32, _P, _P, _P, c_int32,
                          _P],
    "lbt_step_reduce": [_P, c_int32, c_int32, _P, c_int32, c_int32, _P, _P],
    "lbt_step_reduce_x": [_P, c_int32, c_int32, _P, c_int32, c_int32, _P, _P, _P],
    "lbt_step_reduce_update": [_P, c_int32, c_int32, _P, c_int32, c_int32, _P, _P, _P],
    "lbt_step_finish": [_P, c_int32, c_int32, _P, _P, _P, _P, c_float, c_float, _P, c_int64, c_int32, _P],
    "lbt_dfxp_range_update_x": [_P, _P, c_int64, _P, _P, _P, c_int32, _P, _P],
    "lbt_grad_buffer_bwd": [_P, c_int64, _P, c_int64, c_int64, QDesc, _P, _P],
    "lbt_pre_dense": [_P, c_int32, c_int32, c_int32, c_int32, QDesc, _P, _P, _P, _P],
    "lbt_augment_flip_crop": [_P, _P, c_int32, c_int32, c_int32, c_int32, c_int32, c_uint64, c_uint64, _P],
    "lbt_step_update": [_P, _P, _P, c_int64, c_float, c_float, c_float, _P, _P, _P, _P, _P, c_int32, _P, _P],
}
EXPORTED = sorted(_SIGS)

_lib = None


class LbtError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load (once) and type the native library. Raises if it is missing -- no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError("lbt_amd native library not built: %s (run `python -m lbt_amd._build`)" % path)
    lib = ctypes.CDLL(path)
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = c_int32
    lib.lbt_igemm_workspace_bytes.restype = c_int64  # the one int64-valued query
    if lib.lbt_abi_version() != ABI_VERSION:
        raise ImportError("lbt_amd ABI mismatch: library %d, bindings %d" % (lib.lbt_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def call(name, *args):
    """Invoke a C-ABI entry point; raise LbtError on a non-zero status."""
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise LbtError("%s failed with status %d%s" % (name, rc, " (LBT_EINVAL)" if rc == 1001 else ""))


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

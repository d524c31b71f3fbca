"""CPU: lbt_amd.roofline.family maps device symbols (rocprofv3 / PMC summaries) onto the labels
lbt_amd.dfxp.ops times launches with, so bench.py's roofline and the committed traffic files agree."""
from lbt_amd.roofline import family

NS = "void (anonymous namespace)::"


def test_family_gemm_symbols():
    assert family(NS + "igemm_big_kernel<0, false, false, 128, 2, 4, false>(IgArgs)") == "igemm_kernel<fwd>"
    assert family(NS + "igemm_big_kernel<1, true, false, 64, 2, 1, false>(IgArgs)") == "igemm_kernel<dgrad+bn_a>"
    assert family(NS + "igemm_big_kernel<1, true, false, 64, 2, 3, false>(IgArgs)") == "igemm_kernel<dgrad+bn3_a>"
    assert family(NS + "igemm_big_kernel<1, true, false, 64, 2, 0, false>(IgArgs)") == "igemm_kernel<dgrad>"
    assert family(NS + "igemm_fwdq_kernel<128, 4, true>(IgArgs, int)") == "igemm_kernel<fwd>"
    assert family(NS + "igemm_dgrada_kernel<4>(IgArgs)") == "igemm_kernel<dgrad+bn_a>"
    assert family("igemm_kernel<dgrad+bn_a>") == "igemm_kernel<dgrad+bn_a>"  # a label stays a label


def test_family_other_symbols():
    for k in ("wgrad1_kernel<2, 3>(signed char const*)", "wgrad3_kernel<true, 1, 4>(x)", "wgrad_wide_kernel<true, true>(x)"):
        assert family(NS + k) == "wgrad_wide_kernel"
    assert family(NS + "stem_wide_fwd_tiles_kernel<4>(short const*)") == "stem_wide_fwd_kernel"
    assert family(NS + "stem_wide_fwd_kernel<4>(short const*)") == "stem_wide_fwd_kernel"
    assert family("(anonymous namespace)::bn_bwd_b_wide_kernel((anonymous namespace)::WideB)") == "bn_bwd_b_wide_kernel"
    assert family(NS + "conv_gemm_kernel<0, 1, 4, 0, 1>(x)") == "conv_gemm_kernel<0> (fwd)"
    assert family(NS + "conv_gemm_kernel<1, 1, 4, 2, 1>(x)") == "conv_gemm_kernel<1> (dgrad+A)"

"""The all-taps 3x3 weight gradient (igemm.hip wgrad3_kernel, behind lbt_conv_wgrad_igemm_store) against
an exact float64 reference of dynamic_fixed_point.py:302's integer sum  dW[kh,kw,ci,co] =
sum_{n,oh,ow} x[n, oh+kh-1, ow+kw-1, ci] * g[n, oh, ow, co]  (x = 0 outside the image; x offset int8
codes x' = x - 128, g int16 or int8 codes). Bit-exact: every partial is an integer below 2^53."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _expected(x, g):
    """x [N,H,W,Ci] float64 (0..255), g [N,H,W,Co] float64 -> [9*Ci, Co] (tap-major)."""
    N, H, W, Ci = x.shape
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1))
    out = []
    for kh in range(3):
        for kw in range(3):
            xs = xp[:, kh:kh + H, kw:kw + W, :].reshape(-1, Ci)
            out.append(xs.t() @ g.reshape(-1, g.shape[-1]))
    return torch.cat(out, 0)


@pytest.mark.parametrize("N,H,W,Ci,Co,g16", [(2, 56, 56, 64, 64, True), (4, 14, 14, 64, 128, True),
                                             (3, 7, 7, 128, 64, True), (2, 28, 28, 64, 64, False),
                                             (5, 14, 14, 128, 64, False), (2, 20, 20, 64, 64, True)])
def test_wgrad3_exact(N, H, W, Ci, Co, g16):
    from lbt_amd.dfxp import ops
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device="cpu").manual_seed(N * 1000 + H + Ci + Co + g16)
    x = torch.randint(0, 256, (N, H, W, Ci), generator=gen)
    lim = 32768 if g16 else 128
    g = torch.randint(-lim, lim, (N, H, W, Co), generator=gen)
    d = ops.conv_desc(N, H, W, Ci, Co, 3, 3, 1, 1, "SAME")
    assert ops.wgrad3_ok(d)
    ns = ops.wgrad_store_nsplit(d)
    xq = (x - 128).to(torch.int8).to(dev)
    gq = g.to(torch.int16 if g16 else torch.int8).to(dev)
    slab = torch.full((ns, 9 * Ci, Co), 7, dtype=torch.int64, device=dev)  # every element must be written
    ops.conv_wgrad_igemm_store(xq, gq, 1 if g16 else 0, d, slab, ns)
    torch.cuda.synchronize()
    got = slab.sum(0).cpu()
    exp = _expected(x.double(), g.double()).to(torch.int64)
    assert torch.equal(got, exp)


@pytest.mark.parametrize("N,H,Ci,Co,s", [(2, 14, 128, 128, 1), (3, 9, 64, 256, 1), (2, 10, 256, 64, 1),
                                         (2, 15, 128, 256, 2), (3, 7, 256, 128, 1), (4, 56, 64, 256, 1),
                                         (1, 8, 512, 512, 2)])
def test_wgrad1_exact(N, H, Ci, Co, s):
    """The 1x1 16-bit-gradient weight gradient (igemm.hip wgrad1_kernel: raw int16 G images read
    transposed as (lo, hi) byte columns) against the float64 sum dW[ci, co] = sum_{n,oh,ow}
    x[n, oh*s, ow*s, ci] * g[n, oh, ow, co]; ragged pixel counts (P % 64 != 0), every tile shape
    (wci 1 / 2 / 4), strided shortcuts, several splits."""
    from lbt_amd.dfxp import ops
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device="cpu").manual_seed(N * 1000 + H + Ci + Co + s)
    d = ops.conv_desc(N, H, H, Ci, Co, 1, 1, s, s, "SAME")
    assert ops.wgrad1_wci(d)
    x = torch.randint(0, 256, (N, H, H, Ci), generator=gen)
    g = torch.randint(-32768, 32768, (N, d.Ho, d.Wo, Co), generator=gen)
    ns = ops.wgrad_store_nsplit(d, 1)
    xq = (x - 128).to(torch.int8).to(dev)
    slab = torch.full((ns, Ci, Co), 7, dtype=torch.int64, device=dev)  # every element must be written
    ops.conv_wgrad_igemm_store(xq, g.to(torch.int16).to(dev), 1, d, slab, ns)
    torch.cuda.synchronize()
    xs = x[:, ::s, ::s, :][:, :d.Ho, :d.Wo, :].reshape(-1, Ci).double()
    exp = (xs.t() @ g.reshape(-1, Co).double()).to(torch.int64)
    assert torch.equal(slab.sum(0).cpu(), exp)

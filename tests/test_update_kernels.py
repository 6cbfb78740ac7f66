"""The PPO update's elementwise / reduction kernels (mjl_tanh_bwd_colsum, mjl_slice_sum,
mjl_tanh_inplace) against float64 torch references of the same ops, and the tanh-fused layers
(_TanhSplitKLinear) against torch autograd through nn.Linear + tanh (reference: jax.value_and_grad
through src/networks.py:22-61 in train_ppo.py:204-252)."""
import pytest
import torch

from mjx_amd import ppo
from mjx_amd.config import reference_ppo_config

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d", [(65536, 256), (8192, 256), (4133, 256), (300, 64), (129, 8)])
def test_tanh_bwd_colsum_matches_float64(n, d):
    """mjl_tanh_bwd_colsum: dz = g (1 - y^2) to an ulp (the kernel may contract 1 - y y into an fma),
    its column sums (fixed order) within fp32 summation error, bit-identical run to run."""
    g = torch.Generator(device="cuda").manual_seed(n + d)
    gy = torch.randn((n, d), generator=g, device="cuda")
    y = torch.tanh(torch.randn((n, d), generator=g, device="cuda"))
    dz, db = ppo.tanh_bwd_colsum_native(gy, y)
    torch.testing.assert_close(dz.double(), gy.double() * (1 - y.double() ** 2), rtol=1e-6, atol=1e-7)
    zr = gy.double() * (1 - y.double() ** 2)
    torch.testing.assert_close(db.double(), zr.sum(0), rtol=0, atol=1e-6 * float(zr.abs().sum(0).max()))
    dz2, db2 = ppo.tanh_bwd_colsum_native(gy, y)
    assert torch.equal(dz, dz2) and torch.equal(db, db2)


@pytest.mark.parametrize("net", ["policy", "value"])
def test_tanh_fused_layers_match_torch_autograd(net):
    """The update's default path (_TanhSplitKLinear: tanh backward + bias-gradient column sum in one
    pass, split-K weight gradient) against nn.Linear + torch.tanh autograd at a 65,536-row minibatch."""
    cfg = reference_ppo_config()
    gen = torch.Generator().manual_seed(3)
    if net == "policy":
        m = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, 0.0, gen).cuda()
    else:
        m = ppo.ValueNet(54, cfg.value_hidden_layer_specs, gen).cuda()
    x = torch.randn((65536, 54), generator=torch.Generator(device="cuda").manual_seed(4), device="cuda")
    res, prev = {}, (ppo.TANH_FUSED, ppo.UPDATE_MIN_ROWS)
    for mode in ("tanh_fused", "torch"):
        ppo.TANH_FUSED = mode == "tanh_fused"
        ppo.UPDATE_MIN_ROWS = 4096 if mode == "tanh_fused" else 1 << 30  # torch: plain nn.Linear
        try:
            for p in m.parameters():
                p.grad = None
            out = m(x)
            y = out[0] if net == "policy" else out
            w = torch.randn(y.shape, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
            (y * w).sum().backward()
            res[mode] = (y.detach().clone(), [p.grad.clone() for p in m.parameters() if p.grad is not None])
        finally:
            ppo.TANH_FUSED, ppo.UPDATE_MIN_ROWS = prev
    torch.testing.assert_close(res["tanh_fused"][0], res["torch"][0], rtol=1e-5, atol=1e-5)
    assert len(res["tanh_fused"][1]) == len(res["torch"][1])
    for a, b in zip(res["tanh_fused"][1], res["torch"][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))


@pytest.mark.parametrize("ns,shape", [(32, (256, 256)), (4, (256, 54)), (64, (21, 32)), (3, (1, 4))])
def test_slice_sum_matches_ordered_sum(ns, shape):
    """mjl_slice_sum: the slices added in order 0, 1, ... (bit-equal to that loop) and within fp32
    summation error of the float64 sum."""
    x = torch.randn((ns,) + shape, generator=torch.Generator(device="cuda").manual_seed(ns), device="cuda")
    out = ppo.slice_sum_native(x)
    ref = x[0].clone()
    for s in range(1, ns):
        ref = ref + x[s]
    assert torch.equal(out, ref)
    torch.testing.assert_close(out.double(), x.double().sum(0), rtol=1e-5, atol=1e-5)


def test_tanh_inplace_matches_torch():
    x = torch.randn((4096, 256), generator=torch.Generator(device="cuda").manual_seed(1), device="cuda") * 3
    ref = torch.tanh(x)
    y = ppo.tanh_inplace_native(x.clone())
    torch.testing.assert_close(y, ref, rtol=2e-7, atol=2e-7)


@pytest.mark.parametrize("nb,rows,n,mask", [(2, 3001, 256, 3), (2, 3001, 256, 1), (2, 8192, 256, 2), (2, 77, 21, 1),
                                             (1, 5, 8, 0)])
def test_bias_act_matches_torch(nb, rows, n, mask):
    """mjl_bias_act (a float4 per thread; the scalar form for odd widths): x + bias, tanh on the
    matrices whose act_mask bit is set. (Four float4 per thread measured slower: 7.5 -> 9.8 us at the
    twin update's [2, 8192, 256], profiles/r4/bias_act_u4_kernels.txt.)"""
    from mjx_amd._lib import check, lib
    g = torch.Generator(device="cuda").manual_seed(rows + n)
    x = torch.randn((nb, rows, n), generator=g, device="cuda") * 2
    b = torch.randn((nb, n), generator=g, device="cuda")
    ref = x + b[:, None, :]
    for k in range(nb):
        if (mask >> k) & 1:
            ref[k] = torch.tanh(ref[k])
    y = x.clone()
    check(lib().mjl_bias_act(y.data_ptr(), b.data_ptr(), nb, rows, n, mask, torch.cuda.current_stream().cuda_stream))
    torch.testing.assert_close(y, ref, rtol=2e-6, atol=2e-6)

"""The PPO update's dense-layer kernels (mjl_mlp_fwd / mjl_mlp_bwd, csrc/mlp_kernels.hip) against
float64 torch references of the same ops, and the fused MLP (ppo._FusedMLP) against torch autograd
through nn.Linear + tanh (reference: jax.value_and_grad through src/networks.py:22-61 in
train_ppo.py:204-252). fp32 on the matrix cores: tolerances relative to the magnitudes summed."""
import ctypes

import pytest
import torch

from mjx_amd import ppo
from mjx_amd._lib import MjlError, check, lib
from mjx_amd.config import reference_ppo_config

pytestmark = pytest.mark.gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("M,N,K,act", [(4096, 256, 256, 1), (4133, 256, 54, 1), (1000, 21, 256, 1),
                                       (4096, 1, 256, 0), (300, 256, 256, 0), (1, 128, 8, 1)])
def test_mlp_fwd_matches_float64(M, N, K, act):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn((M, K), generator=g, device="cuda")
    w = torch.randn((N, K), generator=g, device="cuda") * (2.0 / (N + K)) ** 0.5
    b = torch.randn(N, generator=g, device="cuda") * 0.1
    y = torch.empty((M, N), device="cuda")
    check(lib().mjl_mlp_fwd(_p(x), K, _p(w), _p(b), M, N, K, act, _p(y), _st()))
    ref = x.double() @ w.double().T + b.double()
    scale = (x.double().abs() @ w.double().abs().T + b.double().abs())
    if act:
        ref = torch.tanh(ref)
    err = (y.double() - ref).abs()
    assert float((err / (scale + 1e-30)).max()) < 1e-5, float(err.max())


@pytest.mark.parametrize("M,N,K,act,dx", [(4096, 256, 256, 1, True), (4133, 21, 256, 1, True),
                                          (4096, 1, 256, 0, True), (4133, 256, 54, 1, False),
                                          (257, 256, 256, 1, True)])
def test_mlp_bwd_matches_float64(M, N, K, act, dx):
    g = torch.Generator(device="cuda").manual_seed(7 * M + N + K)
    gy = torch.randn((M, N), generator=g, device="cuda")
    y = torch.tanh(torch.randn((M, N), generator=g, device="cuda"))
    w = torch.randn((N, K), generator=g, device="cuda") * 0.1
    dz = torch.empty((M, N), device="cuda")
    rows = int(lib().mjl_mlp_colpart_rows(M))
    part = torch.empty((rows, N), device="cuda")
    dX = torch.empty((M, K), device="cuda") if dx else None
    check(lib().mjl_mlp_bwd(_p(gy), _p(y), M, N, _p(w) if dx else None, K, act, _p(dz), _p(dX), _p(part), _st()))
    zr = gy.double() * (1 - y.double() ** 2) if act else gy.double()
    torch.testing.assert_close(dz.double(), zr, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(part.double().sum(0), zr.sum(0), rtol=1e-5, atol=1e-5 * float(zr.abs().sum(0).max()))
    if dx:
        ref = zr @ w.double()
        scale = zr.abs() @ w.double().abs()
        assert float(((dX.double() - ref).abs() / (scale + 1e-30)).max()) < 1e-5


def test_mlp_bwd_rejects_misaligned_dx():
    M, N, K = 64, 256, 54
    gy, y = torch.zeros((M, N), device="cuda"), torch.zeros((M, N), device="cuda")
    w, dz = torch.zeros((N, K), device="cuda"), torch.zeros((M, N), device="cuda")
    part = torch.zeros((1, N), device="cuda")
    dX = torch.zeros((M, K), device="cuda")
    with pytest.raises(MjlError):  # K % 4 != 0 with dx requested
        check(lib().mjl_mlp_bwd(_p(gy), _p(y), M, N, _p(w), K, 1, _p(dz), _p(dX), _p(part), _st()))


@pytest.mark.parametrize("net", ["policy", "value"])
def test_fused_mlp_matches_torch_autograd(net):
    """65,536-row minibatch through the reference-size nets: outputs and every parameter gradient of
    the fused path against torch's nn.Linear + tanh autograd (rtol 1e-4 on the gradient scale)."""
    cfg = reference_ppo_config()
    gen = torch.Generator().manual_seed(3)
    if net == "policy":
        m = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, 0.0, gen).cuda()
    else:
        m = ppo.ValueNet(54, cfg.value_hidden_layer_specs, gen).cuda()
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn((65536, 54), generator=g, device="cuda")
    res, prev, prev_t = {}, ppo.FUSED_MLP, ppo.TANH_FUSED
    for fused in (True, False):
        ppo.FUSED_MLP = fused
        ppo.TANH_FUSED = False  # the reference: nn.Linear + torch.tanh autograd
        try:
            for p in m.parameters():
                p.grad = None
            out = m(x)
            y = out[0] if net == "policy" else out
            w = torch.randn(y.shape, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
            (y * w).sum().backward()
            res[fused] = (y.detach().clone(), [p.grad.clone() if p.grad is not None else None for p in m.parameters()])
        finally:
            ppo.FUSED_MLP, ppo.TANH_FUSED = prev, prev_t
    torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-5, atol=1e-5)
    for a, b in zip(res[True][1], res[False][1]):
        if b is None:
            continue
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))


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
    res, prev = {}, (ppo.FUSED_MLP, ppo.TANH_FUSED, ppo.UPDATE_MIN_ROWS)
    for mode in ("tanh_fused", "torch"):
        ppo.FUSED_MLP = False
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
            ppo.FUSED_MLP, ppo.TANH_FUSED, ppo.UPDATE_MIN_ROWS = prev
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

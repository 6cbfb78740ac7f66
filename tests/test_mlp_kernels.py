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
    res, prev = {}, ppo.FUSED_MLP
    for fused in (True, False):
        ppo.FUSED_MLP = fused
        try:
            for p in m.parameters():
                p.grad = None
            out = m(x)
            y = out[0] if net == "policy" else out
            w = torch.randn(y.shape, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
            (y * w).sum().backward()
            res[fused] = (y.detach().clone(), [p.grad.clone() if p.grad is not None else None for p in m.parameters()])
        finally:
            ppo.FUSED_MLP = prev
    torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-5, atol=1e-5)
    for a, b in zip(res[True][1], res[False][1]):
        if b is None:
            continue
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))

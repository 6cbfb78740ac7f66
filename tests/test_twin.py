"""The twin PPO update (mjx_amd/twin.py: the policy and value nets' layers as one batched GEMM per layer,
train_ppo.py:233-252) against autograd of the reference's loss formulas in float64
(train_ppo.py:204-220 restated as torch ops, ppo.NATIVE_LOSSES = False): every gradient of both nets to
1e-4 of its scale, at the 8,192-row per-rank minibatch of C5 (8 GPUs) and the 65,536-row one of C3;
and the twin updater against the per-net updater (MJL_TWIN_UPDATE path off) over a whole update."""
import pytest
import torch

from mjx_amd import ppo, twin
from mjx_amd.config import reference_ppo_config

pytestmark = pytest.mark.gpu


def _nets(cfg, seed=0):
    g = torch.Generator().manual_seed(seed)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
    with torch.no_grad():  # non-trivial biases and log_std (the init zeroes them)
        for p in list(pol.parameters()) + list(val.parameters()):
            if p.dim() == 1:
                p.add_(torch.randn(p.shape, generator=g).cuda() * 0.1)
    return pol, val


def _data(n, seed=1):
    gd = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn((n, 54), generator=gd, device="cuda"),
            torch.rand((n, 21), generator=gd, device="cuda") * 1.8 - 0.9,
            torch.randn(n, generator=gd, device="cuda") - 20.0,
            torch.randn(n, generator=gd, device="cuda"), torch.randn(n, generator=gd, device="cuda"))


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("dup", [False, True])
@pytest.mark.parametrize("n", [8192, 65536])
def test_twin_gradients_match_float64_autograd(monkeypatch, n, dup, fused):
    """dup: the observations handed over as the [2, M, K0] block the graphed update's gather writes
    (one copy per net) instead of one [M, K0] matrix read through a batch-stride-0 view. fused: the
    update's thin ends as single launches (at these shapes the whole head as mjl_twin_head, 32-row
    chunks: one per workgroup at 8,192 rows, eight at 65,536), or the library GEMM path (twin.FUSED_ENDS off)."""
    monkeypatch.setattr(twin, "FUSED_ENDS", fused)
    cfg = reference_ppo_config()
    pol, val = _nets(cfg)
    ref_p = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs).cuda().double()
    ref_v = ppo.ValueNet(54, cfg.value_hidden_layer_specs).cuda().double()
    ref_p.load_state_dict({k: v.double() for k, v in pol.state_dict().items()})
    ref_v.load_state_dict({k: v.double() for k, v in val.state_dict().items()})
    assert twin.TwinNets.eligible(pol, val)
    tw = twin.TwinNets(pol, val)
    o, a, ol, r, ad = _data(n)
    ob = o.unsqueeze(0).expand(2, n, 54).contiguous() if dup else o
    splits = min(64, n // ppo.SPLIT_ROWS)
    # the update's form first (the output layer's bias and tanh folded into the loss launch), then the
    # reporting form (bias + tanh pass, the value loss too): the same gradients to rounding
    tw.forward_backward(ob, a, ol, r, ad, None, cfg.clip_eps, cfg.ent_coef, splits)
    g_fold = [g.clone() for g in tw.grads_p + tw.grads_v]
    lp, lv = tw.forward_backward(ob, a, ol, r, ad, None, cfg.clip_eps, cfg.ent_coef, splits, want_value_loss=True)
    torch.cuda.synchronize()
    for gf, gu in zip(g_fold, tw.grads_p + tw.grads_v):
        assert float((gf - gu).abs().max()) <= 1e-5 * (float(gu.abs().max()) + 1e-12)
    old = ppo.NATIVE_LOSSES
    ppo.NATIVE_LOSSES = False
    try:
        loss_p = ppo.ppo_policy_loss(ref_p, o.double(), a.double(), ol.double(), ad.double(), cfg.clip_eps,
                                     cfg.ent_coef)
        loss_v = ppo.value_loss(ref_v, o.double(), r.double())
        (loss_p + loss_v).backward()
    finally:
        ppo.NATIVE_LOSSES = old
    assert float(lp) == pytest.approx(float(loss_p), rel=1e-5, abs=1e-6)
    assert float(lv) == pytest.approx(float(loss_v), rel=1e-5)
    for got, p in zip(tw.grads_p + tw.grads_v, list(ref_p.parameters()) + list(ref_v.parameters())):
        want = p.grad.float()
        scale = float(want.abs().max()) + 1e-12
        err = float((got - want).abs().max())
        assert err <= 1e-4 * scale, f"{tuple(want.shape)}: max error {err:.3e} of scale {scale:.3e}"
    # the modules' parameters are views of the stacked storage, the value's padded output rows stay 0
    assert tw.owns_storage()
    assert float(tw.W[-1][1, 1:].abs().max()) == 0.0 and float(tw.gW[-1][1, 1:].abs().max()) == 0.0


@pytest.mark.parametrize("n", [10240, 16448])
def test_fused_head_uneven_chunks_match_float64_autograd(monkeypatch, n):
    """The fused head where workgroups take different chunk counts: 10,240 rows = 320 chunks of 32 over
    256 workgroups per net (one or two each), 16,448 rows = 514 chunks (two or three)."""
    test_twin_gradients_match_float64_autograd(monkeypatch, n, False, True)


@pytest.mark.parametrize("n", [8192, 1000])
def test_fused_gather_input_layer_matches_float64(n):
    """mjl_twin_gather_in: the minibatch rows (a permutation with one out-of-range index, which gathers
    NaN as mjl_gather_rows does) and both nets' first hidden layer tanh(o W0^T + b0) against float64;
    n = 1000 leaves a ragged last block of 8 rows."""
    cfg = reference_ppo_config()
    pol, val = _nets(cfg)
    tw = twin.TwinNets(pol, val)
    src = _data(4096)
    assert tw.fused_input_ok(src)
    g = torch.Generator(device="cuda").manual_seed(5)
    idx = torch.randint(0, 4096, (n,), generator=g, device="cuda")
    idx[7] = 4096  # out of range
    o2, a, ol, r, ad, h1 = tw.gather_input(idx, src)
    torch.cuda.synchronize()
    ok = idx < 4096
    for got, x in ((a, src[1]), (ol, src[2]), (r, src[3]), (ad, src[4])):
        assert torch.equal(got[ok], x[idx[ok]]) and bool(torch.isnan(got[~ok]).all())
    for k in range(2):
        assert torch.equal(o2[k][ok], src[0][idx[ok]]) and bool(torch.isnan(o2[k][~ok]).all())
    x = src[0][idx[ok]].double()
    for k, net in enumerate((pol, val)):
        lin = net.mlp.layers[0]
        want = torch.tanh(x @ lin.weight.double().T + lin.bias.double())
        err = float((h1[k][ok].double() - want).abs().max())
        assert err <= 1e-5, f"net {k}: max error {err:.3e}"


def test_fused_ends_update_matches_library_path(monkeypatch):
    """The whole twin forward + backward with the fused thin ends (gather + input layer, output backward
    + last tanh backward) against the same minibatch through the library GEMM path: every gradient of
    both nets to 1e-5 of its scale."""
    cfg = reference_ppo_config()
    pol, val = _nets(cfg)
    tw = twin.TwinNets(pol, val)
    src = _data(16384)
    idx = torch.randperm(16384, generator=torch.Generator(device="cuda").manual_seed(3), device="cuda")[:8192]
    splits = 8192 // ppo.SPLIT_ROWS
    o2, a, ol, r, ad, h1 = tw.gather_input(idx, src)
    tw.forward_backward(o2, a, ol, r, ad, None, cfg.clip_eps, cfg.ent_coef, splits, h1=h1)
    got = [g.clone() for g in tw.grads_p + tw.grads_v]
    monkeypatch.setattr(twin, "FUSED_ENDS", False)
    o, a, ol, r, ad = (x[idx] for x in src)
    tw.forward_backward(o, a, ol, r, ad, None, cfg.clip_eps, cfg.ent_coef, splits)
    torch.cuda.synchronize()
    for g1, g0 in zip(got, tw.grads_p + tw.grads_v):
        scale = float(g0.abs().max()) + 1e-12
        assert float((g1 - g0).abs().max()) <= 1e-5 * scale


def test_twin_update_matches_per_net_update():
    """One update (2 minibatches of 8,192 rows x 2 epochs) through PPOUpdater with and without the
    twin path: parameters and Adam moments agree to rounding (the batched GEMMs round like the single
    ones up to the library's kernel choice)."""
    cfg = reference_ppo_config()
    cfg.minibatch_size, cfg.epochs = 8192, 2
    runs = []
    for use_twin in (True, False):
        pol, val = _nets(cfg)
        op, ov = ppo._adam(pol.parameters(), cfg.lr_policy), ppo._adam(val.parameters(), cfg.lr_value)
        saved = twin.TWIN_UPDATE
        twin.TWIN_UPDATE = use_twin
        try:
            up = ppo.PPOUpdater(pol, val, op, ov, cfg, use_graph=False)
        finally:
            twin.TWIN_UPDATE = saved
        assert (up.twin is not None) == use_twin
        idx = ppo.make_index_batches(2 * 8192, 8192, 2, torch.Generator(device="cuda").manual_seed(5), "cuda")
        up.run(*_data(2 * 8192), idx)
        torch.cuda.synchronize()
        runs.append([t.detach().clone() for t in list(pol.parameters()) + list(val.parameters())])
    for a, b in zip(*runs):
        # 4 Adam steps of lr 3e-4: all but 1e-3 of the entries to 2e-6 + 2e-5 relative; an entry whose
        # gradient is at rounding-noise level may take a different O(lr) step, so every entry within
        # 2 lr per step
        err = (a - b).abs()
        off = err > 2e-6 + 2e-5 * b.abs()
        assert off.float().mean().item() <= 1e-3, f"{int(off.sum())} of {off.numel()} entries off"
        assert err.max().item() <= 2 * 3e-4 * 4


def test_deep_nets_take_the_per_net_path():
    """the twin step's fused launches have caps (mjl_adam_multi 24 tensors, the pair needs
    4 nl + 1; mjl_slice_sum_multi 16 segments, the pair needs 2 nl + 2). Five hidden layers (nl = 6)
    exceed them: the pair is not eligible, and an update over them runs on the per-net path."""
    cfg = reference_ppo_config()
    cfg.policy_hidden_layer_specs = cfg.value_hidden_layer_specs = [(64, "tanh")] * 5
    cfg.minibatch_size, cfg.epochs = 8192, 1
    pol, val = _nets(cfg)
    assert not twin.TwinNets.eligible(pol, val)
    op, ov = ppo._adam(pol.parameters(), cfg.lr_policy), ppo._adam(val.parameters(), cfg.lr_value)
    up = ppo.PPOUpdater(pol, val, op, ov, cfg, use_graph=False)
    assert up.twin is None
    before = [p.detach().clone() for p in pol.parameters()]
    idx = ppo.make_index_batches(8192, 8192, 1, torch.Generator(device="cuda").manual_seed(3), "cuda")
    up.run(*_data(8192), idx)
    torch.cuda.synchronize()
    assert all(torch.isfinite(p).all() for p in pol.parameters())
    assert any(float((p - b).abs().max()) > 0 for p, b in zip(pol.parameters(), before))


def test_twin_storage_reused_and_repointing_detected():
    """a second updater over the same modules reuses their TwinNets (no re-stacking that
    would strand the first holder), and re-pointing any value parameter ends ownership."""
    cfg = reference_ppo_config()
    pol, val = _nets(cfg)
    a = twin.twin_for(pol, val)
    b = twin.twin_for(pol, val)
    assert a is b and a.owns_storage()
    with torch.no_grad():
        val.mlp.layers[1].bias.data = val.mlp.layers[1].bias.data.clone()
    assert not a.owns_storage()
    c = twin.twin_for(pol, val)
    assert c is not a and c.owns_storage()

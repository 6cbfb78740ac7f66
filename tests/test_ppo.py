"""PPO trainer (mjx_amd/ppo.py) against the reference formulas (train_ppo.py, src/networks.py,
src/training_utils.py) and its data-parallel path (world size 2, gloo, CPU).

No reference outputs can be captured (jax is absent), so the formulas are pinned by
closed forms and hand-computed recurrences; the distributed path is pinned by equality with the
single-process computation over the union of the ranks' data.
"""
import json
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

from mjx_amd import ppo
from mjx_amd.config import reference_ppo_config


class PointEnv:
    """CPU stand-in with the HumanoidEnv interface (reset / step with auto-reset): a damped 3-D
    point pushed by a 2-D action; reward -|x|; terminates outside |x| < 2, truncates at 20 steps."""

    def __init__(self, num_envs, seed=0):
        self.num_envs, self.obs_dim, self.act_dim = num_envs, 6, 2
        self.g = torch.Generator().manual_seed(seed)
        self.x = torch.zeros(num_envs, 3)
        self.v = torch.zeros(num_envs, 3)
        self.t = torch.zeros(num_envs)

    def _obs(self):
        return torch.cat([self.x, self.v], 1)

    def reset(self, mask=None):
        m = torch.ones(self.num_envs, dtype=torch.bool) if mask is None else mask > 0.5
        self.x[m] = torch.rand((int(m.sum()), 3), generator=self.g) - 0.5
        self.v[m] = 0.0
        self.t[m] = 0.0
        return self._obs()

    def step(self, act):
        a = torch.clamp(act, -1, 1)
        self.v = 0.9 * self.v + 0.1 * torch.cat([a, -a[:, :1]], 1)
        self.x = self.x + 0.1 * self.v
        self.t += 1
        r = -self.x.norm(dim=1)
        term = (self.x.abs().max(1).values > 2.0).float()
        trunc = (self.t >= 20).float() * (1 - term)
        done = torch.maximum(term, trunc)
        if done.any():
            self.reset(done)
        return self._obs(), r, term, trunc


def small_cfg(**kw):
    cfg = reference_ppo_config()
    cfg.policy_hidden_layer_specs = [(32, "tanh"), (32, "tanh")]
    cfg.value_hidden_layer_specs = [(32, "tanh"), (32, "tanh")]
    cfg.rollout_length, cfg.minibatch_size, cfg.epochs = 8, 32, 2
    cfg.eval_interval, cfg.checkpoint_every, cfg.log_interval = 1, 1, 1
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


# --------------------------------------------------------------------------------- formulas
def test_param_counts_and_glorot_init():
    cfg = reference_ppo_config()
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, torch.Generator().manual_seed(0))
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, torch.Generator().manual_seed(1))
    assert sum(p.numel() for p in pol.parameters()) == 151082
    assert sum(p.numel() for p in val.parameters()) == 145921
    w = pol.mlp.layers[1].weight.detach()
    assert abs(w.std().item() - math.sqrt(2.0 / 512)) < 0.003
    assert all(float(l.bias.detach().abs().max()) == 0.0 for l in pol.mlp.layers)
    assert float(pol.log_std.detach().abs().max()) == 0.0


def test_logprob_and_entropy_closed_forms():
    g = torch.Generator().manual_seed(3)
    mean, act = torch.randn(5, 21, generator=g), torch.randn(5, 21, generator=g)
    log_std = torch.randn(21, generator=g) * 0.3
    ref = torch.distributions.Normal(mean, torch.exp(log_std)).log_prob(act).sum(-1)
    torch.testing.assert_close(ppo.gaussian_logprob(mean, log_std, act), ref, rtol=1e-5, atol=1e-5)
    ent = torch.distributions.Normal(torch.zeros(21), torch.exp(log_std)).entropy().sum() / 21
    torch.testing.assert_close(ppo.gaussian_entropy(log_std, 21), ent, rtol=1e-6, atol=1e-6)


def test_gae_matches_hand_recurrence():
    rng = np.random.default_rng(0)
    T, B, gam, lam = 7, 3, 0.99, 0.95
    r, v = rng.normal(size=(T, B)), rng.normal(size=(T + 1, B))
    te = (rng.uniform(size=(T, B)) < 0.2).astype(float)
    tr = (rng.uniform(size=(T, B)) < 0.2).astype(float) * (1 - te)
    adv = np.zeros((T, B))
    for b in range(B):
        nxt = 0.0
        for t in reversed(range(T)):
            delta = r[t, b] + gam * v[t + 1, b] * (1 - te[t, b]) - v[t, b]
            nxt = delta + gam * lam * (1 - max(te[t, b], tr[t, b])) * nxt
            adv[t, b] = nxt
    a, ret = ppo.compute_gae(*(torch.tensor(x) for x in (r, v, te, tr)), gam, lam)
    np.testing.assert_allclose(a.numpy(), adv, atol=1e-12)
    np.testing.assert_allclose(ret.numpy(), adv + v[:-1], atol=1e-12)


def test_rms_merge_formula():
    rng = np.random.default_rng(1)
    rms = ppo.RunningMeanStd(4)
    mean, var, count = np.zeros(4), np.ones(4), 1e-4
    for _ in range(3):
        x = rng.normal(2.0, 3.0, size=(50, 4))
        rms.update(torch.tensor(x, dtype=torch.float32))
        bm, bv, n = x.mean(0), x.var(0), x.shape[0]
        d, tot = bm - mean, count + n
        mean, var, count = mean + d * n / tot, np.maximum((var * count + bv * n + d * d * count * n / tot) / tot, 1e-4), tot
    np.testing.assert_allclose(rms.mean.numpy(), mean, rtol=1e-5)
    np.testing.assert_allclose(rms.var.numpy(), var, rtol=1e-4)
    x = torch.tensor(rng.normal(size=(3, 4)), dtype=torch.float32)
    torch.testing.assert_close(rms.normalize(x), torch.clamp((x - rms.mean) / torch.sqrt(rms.var + 1e-8), -10, 10))


def test_adam_matches_optax_formula():
    """optax.adam (b1 .9, b2 .999, eps 1e-8, eps_root 0): u = -lr m_hat / (sqrt(v_hat) + eps)."""
    p = torch.nn.Parameter(torch.tensor([1.0, -2.0, 0.5]))
    opt = torch.optim.Adam([p], lr=3e-4, betas=(0.9, 0.999), eps=1e-8)
    x = p.detach().clone().double()
    m = torch.zeros(3, dtype=torch.float64)
    v = torch.zeros(3, dtype=torch.float64)
    for t in range(1, 6):
        g = torch.tensor([0.3, -1.0, 2.0]) * t
        p.grad = g.clone()
        opt.step()
        m = 0.9 * m + 0.1 * g.double()
        v = 0.999 * v + 0.001 * g.double() ** 2
        x = x - 3e-4 * (m / (1 - 0.9 ** t)) / (torch.sqrt(v / (1 - 0.999 ** t)) + 1e-8)
    np.testing.assert_allclose(p.detach().numpy(), x.numpy(), rtol=1e-6)


def test_adam_state_dict_conversion_round_trip():
    """NativeAdam's checkpoint layout is torch.optim.Adam's: the conversion helpers
    round-trip torch's own state dict, accept the round-2 layout, and refuse mismatched shapes."""
    params = [torch.nn.Parameter(torch.randn(3, 2)), torch.nn.Parameter(torch.randn(4))]
    opt = torch.optim.Adam(params, lr=1e-3, betas=(0.9, 0.99), eps=1e-7)
    for _ in range(3):
        for p in params:
            p.grad = torch.randn_like(p)
        opt.step()
    sd = opt.state_dict()
    step, m, v, lr, betas, eps = ppo.adam_state_from_torch(sd, [p.shape for p in params])
    assert (step, lr, betas, eps) == (3.0, 1e-3, (0.9, 0.99), 1e-7)
    back = ppo.adam_state_to_torch(step, m, v, lr, betas, eps)
    opt2 = torch.optim.Adam([torch.nn.Parameter(p.detach().clone()) for p in params], lr=5.0)
    opt2.load_state_dict(back)
    for i in range(2):
        assert torch.equal(opt2.state_dict()["state"][i]["exp_avg"], sd["state"][i]["exp_avg"])
    old = {"t": 3, "lr": 1e-3, "betas": [0.9, 0.99], "eps": 1e-7, "m": m, "v": v}
    assert ppo.adam_state_from_torch(old, [p.shape for p in params])[0] == 3.0
    with pytest.raises(ValueError):
        ppo.adam_state_from_torch(sd, [params[0].shape])
    with pytest.raises(ValueError):
        ppo.adam_state_from_torch(sd, [(3, 2), (5,)])


def test_index_batches_drop_partial():
    idx = ppo.make_index_batches(100, 32, 2, torch.Generator().manual_seed(0), "cpu")
    assert idx.shape == (6, 32)
    for e in range(2):
        assert len(set(idx[3 * e:3 * e + 3].reshape(-1).tolist())) == 96


# ------------------------------------------------------------------------ trainer end to end
def test_trainer_end_to_end_cpu(tmp_path):
    cfg = small_cfg(total_iterations=3)
    tr = ppo.PPOTrainer(cfg, PointEnv(16, 0), PointEnv(8, 1), device="cpu", out_dir=str(tmp_path))
    tr.evaluate = lambda it=0, steps=500: ppo.PPOTrainer.evaluate(tr, it, 20)
    hist = tr.train(verbose=False)
    assert len(hist) == 3 and all(np.isfinite(h["train_return_avg"]) for h in hist)
    lines = [json.loads(l) for l in open(tmp_path / "logs" / "metrics.jsonl")]
    keys = {"step", "train_return_avg", "train_return_max", "train_eplen_avg", "env_steps_per_sec",
            "total_env_steps", "elapsed_time", "eval_return"}
    assert keys <= set(lines[0]) and lines[-1]["total_env_steps"] == 3 * 16 * 8
    assert json.load(open(tmp_path / "config.json"))["rollout_length"] == 8
    ck = sorted(os.listdir(tmp_path / "checkpoints"))
    assert ck[-1] == "checkpoint_000002.pt"
    tr2 = ppo.PPOTrainer(cfg, PointEnv(16, 0), None, device="cpu")
    assert tr2.load_checkpoint(str(tmp_path / "checkpoints" / ck[-1])) == 2
    for a, b in zip(tr.policy.parameters(), tr2.policy.parameters()):
        torch.testing.assert_close(a, b)


# ------------------------------------------------------------------- data parallel (gloo, ws 2)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _synthetic(n, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, 6, generator=g), torch.randn(n, 2, generator=g), torch.randn(n, generator=g) - 3,
            torch.randn(n, generator=g), torch.randn(n, generator=g))


def _dp_worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=2)
    torch.manual_seed(0)
    cfg = small_cfg()
    pol = ppo.GaussianPolicy(6, 2, cfg.policy_hidden_layer_specs, 0.0, torch.Generator().manual_seed(5))
    val = ppo.ValueNet(6, cfg.value_hidden_layer_specs, torch.Generator().manual_seed(6))
    op = torch.optim.Adam(pol.parameters(), lr=1e-3)
    ov = torch.optim.Adam(val.parameters(), lr=1e-3)
    data = _synthetic(64, 10 + rank)
    idx = torch.arange(64).view(4, 16)  # 4 minibatches, 16 local rows each
    ppo.ppo_update(pol, val, op, ov, *data, idx, cfg, tdist, 2)
    rms = ppo.RunningMeanStd(6)
    rms.update(data[0], tdist)
    # trainer on two ranks: identical parameters after training
    tr = ppo.PPOTrainer(small_cfg(total_iterations=2), PointEnv(8, 100 + rank), None, device="cpu", dist=tdist)
    tr.train(verbose=False)
    flat = torch.cat([p.detach().reshape(-1) for p in tr.policy.parameters()])
    if rank == 0:
        torch.save({"pol": pol.state_dict(), "val": val.state_dict(), "rms": rms.state_dict(), "trainer": flat}, out[0])
    else:
        torch.save({"trainer": flat}, out[1])
    tdist.destroy_process_group()


def test_data_parallel_update_equals_single_process(tmp_path):
    out = [str(tmp_path / "r0.pt"), str(tmp_path / "r1.pt")]
    mp.spawn(_dp_worker, args=(_free_port(), out), nprocs=2, join=True)
    got = torch.load(out[0], weights_only=True)
    cfg = small_cfg()
    pol = ppo.GaussianPolicy(6, 2, cfg.policy_hidden_layer_specs, 0.0, torch.Generator().manual_seed(5))
    val = ppo.ValueNet(6, cfg.value_hidden_layer_specs, torch.Generator().manual_seed(6))
    op = torch.optim.Adam(pol.parameters(), lr=1e-3)
    ov = torch.optim.Adam(val.parameters(), lr=1e-3)
    d0, d1 = _synthetic(64, 10), _synthetic(64, 11)
    data = tuple(torch.cat([a, b]) for a, b in zip(d0, d1))
    idx = torch.cat([torch.arange(64).view(4, 16), torch.arange(64, 128).view(4, 16)], 1)  # union minibatches
    ppo.ppo_update(pol, val, op, ov, *data, idx, cfg)
    for k, v in pol.state_dict().items():
        torch.testing.assert_close(got["pol"][k], v, rtol=2e-5, atol=2e-6)
    for k, v in val.state_dict().items():
        torch.testing.assert_close(got["val"][k], v, rtol=2e-5, atol=2e-6)
    rms = ppo.RunningMeanStd(6)
    rms.update(data[0])
    torch.testing.assert_close(got["rms"]["mean"], rms.mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(got["rms"]["var"], rms.var, rtol=1e-4, atol=1e-5)
    t1 = torch.load(out[1], weights_only=True)["trainer"]
    torch.testing.assert_close(got["trainer"], t1, rtol=0, atol=0)


@pytest.mark.gpu
def test_native_gae_bit_identical_to_formula():
    """mjl_gae (one reverse-scan launch) vs the elementwise torch restatement on the same device:
    bit-identical, at the PPO size (T 256, B 2048) and at a ragged one (T 13, B 37: unroll tail)."""
    for T, B in ((256, 2048), (13, 37), (1, 1)):
        g = torch.Generator(device="cuda").manual_seed(T * 1000 + B)
        r = torch.randn((T, B), generator=g, device="cuda")
        v = torch.randn((T + 1, B), generator=g, device="cuda")
        te = (torch.rand((T, B), generator=g, device="cuda") < 0.05).float()
        tr = (torch.rand((T, B), generator=g, device="cuda") < 0.05).float() * (1 - te)
        a, ret = ppo.compute_gae(r, v, te, tr, 0.99, 0.95)
        a_ref, ret_ref = ppo.compute_gae_torch(r, v, te, tr, 0.99, 0.95)
        assert torch.equal(a, a_ref) and torch.equal(ret, ret_ref)


@pytest.mark.gpu
def test_native_rollout_head_matches_formulas():
    """mjl_obs_normalize matches RunningMeanStd.normalize to fp32 rounding (ragged size too);
    mjl_policy_head (tanh head, sampling, log-prob) matches the torch formulas to fp32 rounding, with
    log_std outside the [-20, 2] clip on some entries."""
    g = torch.Generator(device="cuda").manual_seed(3)
    for n, dim in ((2048, 54), (37, 5)):
        x = torch.randn((n, dim), generator=g, device="cuda") * 20
        rms = ppo.RunningMeanStd(dim, "cuda")
        rms.mean.copy_(torch.randn(dim, generator=g, device="cuda"))
        rms.var.copy_(torch.rand(dim, generator=g, device="cuda") + 1e-3)
        out = torch.empty_like(x)
        ppo.obs_normalize_native(x, rms.mean, rms.var, 10.0, out)
        torch.testing.assert_close(out, rms.normalize(x), rtol=2e-7, atol=1e-6)
    for B, A in ((2048, 21), (5, 3)):
        z = torch.randn((B, A), generator=g, device="cuda") * 2
        ls = torch.randn(A, generator=g, device="cuda")
        ls[0] = -25.0
        ls[-1] = 3.0
        eps = torch.randn((B, A), generator=g, device="cuda")
        act, lp = torch.empty_like(z), torch.empty(B, device="cuda")
        ppo.policy_head_native(z, ls, eps, act, lp)
        mean, s = torch.tanh(z), torch.clamp(ls, -20.0, 2.0)
        act_ref = mean + torch.exp(s) * eps
        torch.testing.assert_close(act, act_ref, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(lp, ppo.gaussian_logprob(mean, s, act), rtol=1e-5, atol=1e-3)


def test_policy_pack_layout():
    """mjl_policy_fwd's parameter layout (pack_policy_params): WP[k // 4, n, k % 4] = weight[n, k]
    zero-padded to multiples of 16, bias after each layer; length = mjl_policy_param_floats."""
    import ctypes as C
    from mjx_amd._lib import lib
    g = torch.Generator().manual_seed(9)
    pol = ppo.GaussianPolicy(54, 21, [(256, "tanh"), (256, "tanh"), (256, "tanh")], 0.0, g)
    for lin in pol.mlp.layers:
        with torch.no_grad():
            lin.bias.normal_(generator=g)
    dims = ppo.policy_fused_dims(pol)
    assert dims == [54, 256, 256, 256, 21]
    flat = ppo.pack_policy_params(pol)
    assert flat.numel() == lib().mjl_policy_param_floats(len(dims) - 1, (C.c_int * len(dims))(*dims))
    off = 0
    for lin in pol.mlp.layers:
        n, k = lin.weight.shape
        kp, np_ = -(-k // 16) * 16, -(-n // 16) * 16
        wp = flat[off:off + kp * np_].reshape(kp // 4, np_, 4)
        w = torch.zeros(kp, np_)
        w[:k, :n] = lin.weight.detach().t()
        for kk in (0, 1, k - 1):
            for nn_ in (0, 7, n - 1):
                assert wp[kk // 4, nn_, kk % 4] == lin.weight[nn_, kk]
        assert torch.equal(wp.permute(0, 2, 1).reshape(kp, np_), w)
        b = flat[off + kp * np_:off + kp * np_ + np_]
        assert torch.equal(b[:n], lin.bias.detach()) and torch.all(b[n:] == 0)
        off += kp * np_ + np_
    assert ppo.policy_fused_dims(ppo.GaussianPolicy(54, 21, [(300, "tanh")], 0.0, g)) is None   # > 256
    assert ppo.policy_fused_dims(ppo.GaussianPolicy(54, 21, [(64, "relu")], 0.0, g)) is None    # not tanh


@pytest.mark.gpu
def test_fused_rollout_policy_matches_torch_path():
    """mjl_policy_fwd (normalisation + MLP on the matrix cores + head + sampling + log-prob, one
    launch) = obs_normalize_native -> policy.mlp (torch GEMMs) -> policy_head_native up to the GEMMs'
    fp32 accumulation order; the reference-size policy at 2048 envs, a ragged batch, and a
    different shape (obs 17, hidden 64 / 48, act 6)."""
    g = torch.Generator().manual_seed(4)
    gd = torch.Generator(device="cuda").manual_seed(4)
    for obs_dim, hid, act_dim, B in ((54, [256, 256, 256], 21, 2048), (54, [256, 256, 256], 21, 37),
                                     (17, [64, 48], 6, 100)):
        pol = ppo.GaussianPolicy(obs_dim, act_dim, [(h, "tanh") for h in hid], 0.0, g)
        with torch.no_grad():
            for lin in pol.mlp.layers:
                lin.bias.normal_(0.0, 0.3, generator=g)
            pol.log_std.copy_(torch.linspace(-1.0, 0.5, act_dim))
        pol = pol.cuda()
        x = torch.randn((B, obs_dim), generator=gd, device="cuda") * 3
        rms = ppo.RunningMeanStd(obs_dim, "cuda")
        rms.mean.copy_(torch.randn(obs_dim, generator=gd, device="cuda"))
        rms.var.copy_(torch.rand(obs_dim, generator=gd, device="cuda") + 0.5)
        eps = torch.randn((B, act_dim), generator=gd, device="cuda")
        dims = ppo.policy_fused_dims(pol)
        params = ppo.pack_policy_params(pol)
        act, lp = torch.empty((B, act_dim), device="cuda"), torch.empty(B, device="cuda")
        ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps, act, lp)
        xn = torch.empty_like(x)
        ppo.obs_normalize_native(x, rms.mean, rms.var, 10.0, xn)
        with torch.no_grad():
            z = pol.mlp(xn)
        act_ref, lp_ref = torch.empty_like(act), torch.empty_like(lp)
        ppo.policy_head_native(z, pol.log_std, eps, act_ref, lp_ref)
        torch.testing.assert_close(act, act_ref, rtol=0, atol=2e-5)
        torch.testing.assert_close(lp, lp_ref, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_native_colsum_matches_torch():
    """mjl_colsum (bias gradients, split-K sums of the update) equals x.sum(0) in fp64 to fp32
    accumulation error: the update's shapes, one-chunk and two-stage sizes, ragged and
    single-column ones, and n = 0; a repeat run is bit-identical (fixed summation order)."""
    g = torch.Generator(device="cuda").manual_seed(5)
    for n, d in ((65536, 256), (65536, 21), (65536, 1), (32, 65536), (32, 13824), (1000, 3), (257, 300),
                 (7, 5), (0, 4)):
        x = torch.randn((n, d), generator=g, device="cuda")
        out = ppo.colsum_native(x)
        ref = x.double().sum(0)
        tol = 1e-5 * math.sqrt(max(n, 1)) + 1e-6
        assert out.shape == (d,)
        scale = max(1.0, float(x.abs().max())) if n else 1.0
        assert float((out.double() - ref).abs().max()) <= tol * scale, (n, d)
        assert torch.equal(out, ppo.colsum_native(x)), (n, d)


@pytest.mark.gpu
def test_minibatch_logprob_backward_matches_autograd():
    """The update-size log-prob (hand-written backward, native column sum for d/d log_std) equals
    autograd of the reference's elementwise formula (train_ppo.py:121-126) to fp32 rounding."""
    g = torch.Generator(device="cuda").manual_seed(8)
    mean = torch.randn((65536, 21), generator=g, device="cuda").requires_grad_()
    ls = (0.3 * torch.randn(21, generator=g, device="cuda")).requires_grad_()
    act = torch.randn((65536, 21), generator=g, device="cuda")
    gout = torch.randn(65536, generator=g, device="cuda")
    lp = ppo.gaussian_logprob(mean, ls, act)
    ref = torch.sum((act - mean) ** 2 / torch.exp(2.0 * ls) + 2.0 * ls + ppo.LOG2PI, dim=-1) * -0.5
    torch.testing.assert_close(lp, ref, rtol=1e-5, atol=1e-4)
    gm, gs = torch.autograd.grad(lp, (mean, ls), gout)
    gm_r, gs_r = torch.autograd.grad(ref, (mean, ls), gout)
    torch.testing.assert_close(gm, gm_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gs, gs_r, rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
def test_splitk_linear_backward_matches_autograd():
    """The split-K linear's backward (weight gradient as batched GEMMs + column sums, bias gradient
    as a column sum) matches nn.Linear's autograd gradients on the update's minibatch shape."""
    g = torch.Generator(device="cuda").manual_seed(6)
    lin = torch.nn.Linear(54, 256).cuda()
    x = torch.randn((65536, 54), generator=g, device="cuda", requires_grad=True)
    gy = torch.randn((65536, 256), generator=g, device="cuda")
    y = ppo._linear(lin, x)
    gx, gw, gb = torch.autograd.grad(y, (x, lin.weight, lin.bias), gy)
    gx_r, gw_r, gb_r = torch.autograd.grad(torch.nn.functional.linear(x, lin.weight, lin.bias), (x, lin.weight, lin.bias), gy)
    torch.testing.assert_close(gx, gx_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gw, gw_r, rtol=1e-4, atol=5e-2)
    torch.testing.assert_close(gb, gb_r, rtol=1e-4, atol=5e-2)


@pytest.mark.gpu
def test_graph_rollout_bit_identical_to_eager():
    """The hipGraph replay of the T-step rollout (policy, sampling, log-prob, fused env step with
    auto-reset) reproduces the eager loop bit for bit, including the env's reset RNG draws (device
    counter base) and observation statistics updated in place between rollouts."""
    import mjx_amd
    from mjx_amd import mjx
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    m = mjx_amd.load_model("humanoid_mjx")
    cfg = small_cfg(num_envs=256, rollout_length=24)
    cfg.env_config.max_episode_steps = 10  # truncations -> auto-resets inside the captured steps
    ecfg = resolve_ids(m, cfg.env_config)
    trs = [ppo.PPOTrainer(cfg, HumanoidEnv(mjx.put_model(m), ecfg, cfg.num_envs, seed=11), None, device="cuda",
                          use_graph=g, jax_keys=jk) for g, jk in ((False, False), (True, False))]
    trs += [ppo.PPOTrainer(cfg, HumanoidEnv(mjx.put_model(m), ecfg, cfg.num_envs, seed=11), None, device="cuda",
                           use_graph=g, jax_keys=True) for g in (False, True)]
    # the first two pool their auto-resets (reset_pool, default 16); these two reset in place only
    trs += [ppo.PPOTrainer(cfg, HumanoidEnv(mjx.put_model(m), ecfg, cfg.num_envs, seed=11), None, device="cuda",
                           use_graph=g, jax_keys=False, reset_pool=0) for g in (False, True)]
    assert trs[0]._pool_n is not None and trs[2]._pool_n is None and trs[4]._pool_n is None
    for it in range(3):
        outs = []
        for tr in trs:
            bufs = [x.clone() for x in tr.collect_rollout()]
            tr.rms.update(bufs[0])
            outs.append(bufs)
        assert (trs[1]._graph is not None and trs[3]._graph is not None) or it == 0
        for a, b in zip(outs[0], outs[1]):
            assert torch.equal(a, b), f"rollout {it}"
        for a, b in zip(outs[2], outs[3]):  # jax-key resets: keys split inside the captured steps
            assert torch.equal(a, b), f"rollout {it} (jax keys)"
        for a, b in zip(outs[4], outs[5]):
            assert torch.equal(a, b), f"rollout {it} (in-place resets)"
        assert outs[0][5].sum() > 0  # truncations happened


@pytest.mark.gpu
def test_split_k_linear_gradients():
    """The minibatch-size Linear (split-K weight gradient) matches nn.Linear's gradients within fp32
    summation noise, for every layer shape of the reference nets."""
    g = torch.Generator(device="cuda").manual_seed(0)
    for fin, fout in ((54, 256), (256, 256), (256, 21), (256, 1)):
        lin = torch.nn.Linear(fin, fout).cuda()
        x = torch.randn((65536, fin), generator=g, device="cuda", requires_grad=True)
        gy = torch.randn((65536, fout), generator=g, device="cuda")
        y = ppo._linear(lin, x)
        y.backward(gy)
        got = [x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()]
        x.grad = None
        lin.zero_grad()
        torch.testing.assert_close(y, torch.nn.functional.linear(x, lin.weight, lin.bias), rtol=1e-5, atol=1e-5)
        torch.nn.functional.linear(x, lin.weight, lin.bias).backward(gy)
        for a, b in zip(got, [x.grad, lin.weight.grad, lin.bias.grad]):  # sums of 65,536 terms: scale-relative
            assert (a - b).abs().max() <= 2e-5 * b.abs().max(), (fin, fout)


@pytest.mark.gpu
def test_jax_key_chain_follows_train_ppo():
    """With jax_keys the trainer's reset keys are train_ppo.py's: PRNGKey(seed) -> two init splits ->
    split -> split(key_reset, B) for the initial reset (:88-118); per iteration split -> key_roll
    (:325), per rollout step split (sampling key, :132) then split -> split(key_reset, B) (:150-151).
    Derived independently with the numpy restatement of jax.random (tests/rng_ref.py)."""
    import mjx_amd
    from mjx_amd import mjx
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    from rng_ref import jax_split
    m = mjx_amd.load_model("humanoid_mjx")
    cfg = small_cfg(num_envs=64, rollout_length=5, seed=1234)
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, cfg.env_config), cfg.num_envs, seed=0)
    tr = ppo.PPOTrainer(cfg, env, None, device="cuda", use_graph=False, jax_keys=True)
    rng = np.array([0, 1234], np.uint32)
    rng = jax_split(rng, 2)[0]
    rng = jax_split(rng, 2)[0]
    rng, key_reset = jax_split(rng, 2)
    np.testing.assert_array_equal(tr._env_keys.cpu().numpy().view(np.uint32), jax_split(key_reset, 64))
    tr.collect_rollout()
    rng, roll = jax_split(rng, 2)
    for _ in range(5):
        roll = jax_split(jax_split(roll, 2)[0], 2)
        keys = jax_split(roll[1], 64)
        roll = roll[0]
    np.testing.assert_array_equal(tr._env_keys.cpu().numpy().view(np.uint32), keys)
    np.testing.assert_array_equal(tr._jax_rng.cpu().numpy().view(np.uint32), rng)


@pytest.mark.gpu
def test_native_update_losses_match_torch_ops():
    """mjl_ppo_surrogate / mjl_mse / mjl_gather_rows against the torch restatement of
    train_ppo.py:204-220 on a 65,536-row minibatch: losses and every parameter gradient of both nets,
    with ratios spread across the clip range (ties, both sides of the bounds)."""
    cfg = reference_ppo_config()
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
    gd = torch.Generator(device="cuda").manual_seed(3)
    N, n = 131072, 65536
    obs = torch.randn((N, 54), generator=gd, device="cuda")
    idx = torch.randperm(N, generator=gd, device="cuda")[:n]
    with torch.no_grad():
        mean, log_std = pol(obs)
        acts = (mean + torch.exp(log_std) * torch.randn((N, 21), generator=gd, device="cuda")).contiguous()
        from mjx_amd.ppo import gaussian_logprob
        logp = gaussian_logprob(mean, log_std, acts) + 0.3 * torch.randn(N, generator=gd, device="cuda")
    ret = torch.randn(N, generator=gd, device="cuda")
    adv = 2.0 * torch.randn(N, generator=gd, device="cuda") + 0.5
    res = []
    for native in (True, False):
        ppo.NATIVE_LOSSES = native
        try:
            o, a, ol, r, ad = (ppo._gather_minibatch(idx, obs, acts, logp, ret, adv) if native else
                               (obs[idx], acts[idx], logp[idx], ret[idx], adv[idx]))
            for p in list(pol.parameters()) + list(val.parameters()):
                p.grad = None
            lp = ppo.ppo_policy_loss(pol, o, a, ol, ad, cfg.clip_eps, cfg.ent_coef)
            lv = ppo.value_loss(val, o, r)
            (lp + lv).backward()
            res.append((float(lp), float(lv), [p.grad.clone() for p in list(pol.parameters()) + list(val.parameters())],
                        (o, a, ol, r, ad)))
        finally:
            ppo.NATIVE_LOSSES = True
    (lp1, lv1, g1, d1), (lp2, lv2, g2, d2) = res
    for x, y in zip(d1, d2):
        assert torch.equal(x, y)
    assert lp1 == pytest.approx(lp2, rel=1e-5, abs=1e-6) and lv1 == pytest.approx(lv2, rel=1e-5)
    for x, y in zip(g1, g2):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_native_adam_matches_torch_adam():
    """NativeAdam (mjl_adam) against torch.optim.Adam(fused=True) over 6 steps on the policy's
    parameter shapes, one tensor without a gradient; state_dict round trip."""
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [(256, 54), (256,), (256, 256), (256,), (21, 256), (21,), (21,)]
    a = [torch.randn(s, generator=g, device="cuda") for s in shapes]
    b = [x.clone() for x in a]
    oa = ppo.NativeAdam(a, lr=3e-4)
    ob = torch.optim.Adam(b, lr=3e-4, betas=(0.9, 0.999), eps=1e-8, fused=True)
    for step in range(6):
        grads = [torch.randn(s, generator=g, device="cuda") * (10.0 ** (k % 3 - 1)) for k, s in enumerate(shapes)]
        for k, (x, y) in enumerate(zip(a, b)):
            x.grad = None if k == 3 else grads[k].clone()
            y.grad = None if k == 3 else grads[k].clone()
        oa.step()
        ob.step()
        for x, y in zip(a, b):
            torch.testing.assert_close(x, y, rtol=2e-6, atol=1e-7)
    sd = oa.state_dict()
    oc = ppo.NativeAdam([x.clone() for x in a], lr=1.0)
    oc.load_state_dict(sd)
    assert oc.t == 6 and oc.lr == pytest.approx(3e-4) and all(torch.equal(x, y) for x, y in zip(oc.m, oa.m))


@pytest.mark.gpu
def test_native_surrogate_with_global_advantage_stats():
    """The data-parallel form of the native surrogate (advantage statistics all-reduced over the
    ranks, passed in) equals the single-process form on a one-rank group (gloo over 127.0.0.1)."""
    import os
    cfg = reference_ppo_config()
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    gd = torch.Generator(device="cuda").manual_seed(5)
    n = 65536
    o = torch.randn((n, 54), generator=gd, device="cuda")
    with torch.no_grad():
        m, s = pol(o)
        a = (m + torch.exp(s) * torch.randn((n, 21), generator=gd, device="cuda")).contiguous()
        from mjx_amd.ppo import gaussian_logprob
        lp = gaussian_logprob(m, s, a) + 0.3 * torch.randn(n, generator=gd, device="cuda")
    adv = 1.5 * torch.randn(n, generator=gd, device="cuda") - 0.4
    port = _free_port()
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        out = []
        for dist in (None, tdist):
            for p in pol.parameters():
                p.grad = None
            loss = ppo.ppo_policy_loss(pol, o, a, lp, adv, cfg.clip_eps, cfg.ent_coef, dist)
            loss.backward()
            out.append((float(loss), [p.grad.clone() for p in pol.parameters()]))
    finally:
        tdist.destroy_process_group()
    assert out[0][0] == pytest.approx(out[1][0], rel=1e-5)
    for x, y in zip(out[0][1], out[1][1]):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_gather_rows_bounds():
    """mjl_gather_rows: rows gathered exactly; an index outside the source rows gives a NaN row
    instead of an out-of-bounds read."""
    g = torch.Generator(device="cuda").manual_seed(0)
    a, b = torch.randn((100, 7), generator=g, device="cuda"), torch.randn(100, generator=g, device="cuda")
    idx = torch.tensor([3, 99, 0, 100, -1, 50], dtype=torch.int64, device="cuda")
    oa, ob = ppo._gather_minibatch(idx, a, b)
    ok = torch.tensor([True, True, True, False, False, True], device="cuda")
    assert torch.equal(oa[ok], a[idx[ok]]) and torch.equal(ob[ok], b[idx[ok]])
    assert bool(torch.isnan(oa[~ok]).all()) and bool(torch.isnan(ob[~ok]).all())


@pytest.mark.gpu
@pytest.mark.parametrize("cols", [(54, 54, 21, 1, 1, 1), (200,), (150, 60)])
def test_gather_rows_indexed_wide_and_twice(cols):
    """mjl_gather_rows_indexed through both kernels (a wave per row up to 192 total columns, an
    element per thread beyond), row *idx_row of an index table; and the twin update's form (the
    first array written twice into one [2, rows, ...] block)."""
    g = torch.Generator(device="cuda").manual_seed(len(cols))
    arrs = [torch.randn((300, c) if c > 1 else (300,), generator=g, device="cuda") for c in cols]
    table = torch.randint(0, 300, (3, 77), generator=g, device="cuda", dtype=torch.int64)
    table[1, 5] = 300  # out of range: a NaN row
    row = torch.tensor([1], dtype=torch.int32, device="cuda")
    outs = ppo._gather_minibatch(table, *arrs, row=row)
    idx = table[1]
    ok = idx < 300
    for o, a in zip(outs, arrs):
        assert torch.equal(o[ok], a[idx[ok]]) and bool(torch.isnan(o[~ok]).all())
    if len(arrs) + 1 <= 8:
        tw = ppo._gather_minibatch(table, *arrs, row=row, twice_first=True)
        assert tw[0].shape == (2,) + outs[0].shape
        assert torch.equal(tw[0][0][ok], tw[0][1][ok]) and torch.equal(tw[0][0][ok], outs[0][ok])
        assert bool(torch.isnan(tw[0][:, ~ok]).all())
        for o, t in zip(outs[1:], tw[1:]):
            assert torch.equal(o[ok], t[ok])

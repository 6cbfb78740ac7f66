"""The PPO update as hipGraph replays (PPOUpdater, mjx_amd/ppo.py) against the eager update, bit for bit
(the round-2 whole-update capture drifted ~2e-3 from eager from its second replay on; the
cause was NativeAdam's host step count, baked into the captured launch's bias corrections — the step
count is now device state, advanced inside the capture).

Reference: run_ppo_updates, one compiled lax.scan over the minibatches (train_ppo.py:233-252).
* single process: one graph per minibatch step (both nets, value on the side stream), 2 epochs x 2
  minibatches of 65,536 rows, 1 eager run then 3 runs of replays;
* data-parallel path (gloo, one rank, on the GPU): graph A (forward + backward + flattened gradients),
  the eager all-reduce, graph B (mean + both Adam steps), at the 8,192-row per-rank minibatch of C5 on
  8 GPUs.
"""
import socket

import pytest
import torch
import torch.distributed as tdist

from mjx_amd import ppo
from mjx_amd.config import reference_ppo_config

pytestmark = pytest.mark.gpu


def _nets_and_data(cfg, n, seed=0):
    g = torch.Generator().manual_seed(seed)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
    op, ov = ppo._adam(pol.parameters(), cfg.lr_policy), ppo._adam(val.parameters(), cfg.lr_value)
    assert isinstance(op, ppo.NativeAdam) and isinstance(ov, ppo.NativeAdam)
    gd = torch.Generator(device="cuda").manual_seed(seed + 1)
    data = (torch.randn((n, 54), generator=gd, device="cuda"),
            torch.rand((n, 21), generator=gd, device="cuda") * 1.8 - 0.9,
            torch.randn(n, generator=gd, device="cuda") - 20.0,
            torch.randn(n, generator=gd, device="cuda"), torch.randn(n, generator=gd, device="cuda"))
    return pol, val, op, ov, data


def _state(pol, val, op, ov):
    return [t.detach().clone() for t in list(pol.parameters()) + list(val.parameters()) + op.m + op.v + ov.m + ov.v
            + [op.step_t, ov.step_t]]


def _compare(a, b, run):
    for k, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), f"run {run}: tensor {k} differs (max {float((x - y).abs().max()):.3e})"


def _run_pair(cfg, n, dist=None):
    """Two identical (nets, optimisers, data): one through PPOUpdater with graphs, one eager; 4 runs
    with the same permutations; compared after every run."""
    A = _nets_and_data(cfg, n)
    B = _nets_and_data(cfg, n)
    ua = ppo.PPOUpdater(*A[:4], cfg, dist, 1, use_graph=True)
    ub = ppo.PPOUpdater(*B[:4], cfg, dist, 1, use_graph=False)
    assert ua.graph_ok and not ub.graph_ok
    for run in range(4):  # run 0 eager in both (warm-up), runs 1-3 replay the graphs
        idx = ppo.make_index_batches(n, cfg.minibatch_size, cfg.epochs,
                                     torch.Generator(device="cuda").manual_seed(100 + run), "cuda")
        ua.run(*A[4], idx)
        ub.run(*B[4], idx)
        torch.cuda.synchronize()
        _compare(_state(*A[:4]), _state(*B[:4]), run)
    assert ua._ga is not None  # the graphs were captured and replayed
    assert float(A[2].step_t) == 4 * idx.shape[0]


def test_update_graph_replay_bit_identical_to_eager():
    cfg = reference_ppo_config()
    cfg.epochs = 2
    _run_pair(cfg, 2 * cfg.minibatch_size)  # 2 epochs x 2 minibatches of 65,536 rows


def test_data_parallel_update_graph_bit_identical_to_eager():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        cfg = reference_ppo_config()
        cfg.minibatch_size, cfg.epochs = 8192, 2  # the per-rank minibatch of C5 on 8 GPUs
        _run_pair(cfg, 4 * 8192, tdist)
    finally:
        tdist.destroy_process_group()


def _one_rank_group(backend):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    tdist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, **kw)


def test_data_parallel_bucketed_update_graph_bit_identical_to_eager(monkeypatch):
    """The bucketed data-parallel step (the gradient all-reduced in two buckets, the first in flight
    while the lower layers' backward runs; graph A in two parts around it) equals its eager run bit for
    bit (gloo, one rank, buckets forced on: by default they are on only with more than one rank)."""
    monkeypatch.setattr(ppo, "DP_BUCKETS", "1")
    _one_rank_group("gloo")
    try:
        cfg = reference_ppo_config()
        cfg.minibatch_size, cfg.epochs = 8192, 2
        _run_pair(cfg, 4 * 8192, tdist)
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("buckets", ["0", "1"])
def test_rccl_captured_step_graph_bit_identical_to_eager(monkeypatch, buckets):
    """Over RCCL the data-parallel minibatch step is ONE graph with its all-reduce(s) captured inside
    (ppo.DP_CAPTURE): the replays equal the eager update (collectives between eager bodies) bit for bit,
    one rank on cuda:0, one bucket and two."""
    monkeypatch.setattr(ppo, "DP_BUCKETS", buckets)
    _one_rank_group("nccl")
    try:
        cfg = reference_ppo_config()
        cfg.minibatch_size, cfg.epochs = 8192, 2
        A = _nets_and_data(cfg, 4 * 8192)
        B = _nets_and_data(cfg, 4 * 8192)
        ua = ppo.PPOUpdater(*A[:4], cfg, tdist, 1, use_graph=True)
        ub = ppo.PPOUpdater(*B[:4], cfg, tdist, 1, use_graph=False)
        for run in range(3):
            idx = ppo.make_index_batches(4 * 8192, cfg.minibatch_size, cfg.epochs,
                                         torch.Generator(device="cuda").manual_seed(200 + run), "cuda")
            ua.run(*A[4], idx)
            ub.run(*B[4], idx)
            torch.cuda.synchronize()
            _compare(_state(*A[:4]), _state(*B[:4]), run)
        assert ua._gstep is not None and ua.collectives_last_run == idx.shape[0] * (2 if buckets == "1" else 1)
    finally:
        tdist.destroy_process_group()


def test_native_adam_state_dict_is_torch_layout():
    """NativeAdam checkpoints use torch.optim.Adam's state-dict layout, both ways, and a
    mismatched parameter count is refused."""
    cfg = reference_ppo_config()
    pol, val, op, ov, data = _nets_and_data(cfg, 65536)
    for p in pol.parameters():
        p.grad = torch.randn_like(p)
    op.step()
    op.step()
    sd = op.state_dict()
    tad = torch.optim.Adam(pol.parameters(), lr=cfg.lr_policy)
    tad.load_state_dict(sd)  # torch accepts it
    assert float(tad.state_dict()["state"][0]["step"]) == 2.0
    op2 = ppo.NativeAdam(list(pol.parameters()), lr=1.0)
    op2.load_state_dict(tad.state_dict())  # and NativeAdam takes torch's
    assert op2.lr == cfg.lr_policy and float(op2.step_t) == 2.0
    for a, b in zip(op.m + op.v, op2.m + op2.v):
        assert torch.equal(a, b)
    with pytest.raises(ValueError):
        ppo.NativeAdam(list(val.parameters()), lr=1.0).load_state_dict(sd)

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
    assert ua._ga is not None or ua._gstep is not None  # the graphs were captured and replayed
    assert float(A[2].step_t) == 4 * idx.shape[0]


@pytest.mark.parametrize("whole", [True, False])
def test_update_graph_replay_bit_identical_to_eager(monkeypatch, whole):
    """One graph per update (ppo.WHOLE_UPDATE_GRAPH) and one per minibatch step, both against eager."""
    monkeypatch.setattr(ppo, "WHOLE_UPDATE_GRAPH", whole)
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


@pytest.mark.parametrize("buckets,whole", [("0", True), ("1", True), ("0", False), ("1", False)])
def test_rccl_captured_step_graph_bit_identical_to_eager(monkeypatch, buckets, whole):
    """Over RCCL the data-parallel minibatch step is ONE graph with its all-reduce(s) captured inside
    (ppo.DP_CAPTURE) — and, with ppo.WHOLE_UPDATE_GRAPH, every minibatch step of the update in one
    graph: the replays equal the eager update (collectives between eager bodies) bit for bit, one rank
    on cuda:0, one bucket and two."""
    monkeypatch.setattr(ppo, "DP_BUCKETS", buckets)
    monkeypatch.setattr(ppo, "WHOLE_UPDATE_GRAPH", whole)
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
        assert ua._gstep_n == (idx.shape[0] if whole else 1)
    finally:
        tdist.destroy_process_group()


def _refuse_capture(monkeypatch):
    """all_reduce raises while the current stream captures (a capture this RCCL build refuses);
    eager calls go through."""
    orig = tdist.all_reduce

    def refusing(t, *a, **k):
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("collective capture refused (test)")
        return orig(t, *a, **k)
    monkeypatch.setattr(tdist, "all_reduce", refusing)


@pytest.mark.parametrize("buckets", ["0", "1"])
def test_rccl_capture_refused_falls_back_to_eager_bit_identical(monkeypatch, buckets):
    """VERDICT r5 item 5 / ADVICE r5: when the in-graph collective capture is refused, the updater
    agrees on it across ranks (one eager all-reduce of a failure flag), replays nothing captured, and
    runs the eager collectives between captured bodies — equal to the eager update bit for bit."""
    monkeypatch.setattr(ppo, "DP_BUCKETS", buckets)
    _one_rank_group("nccl")
    _refuse_capture(monkeypatch)
    try:
        cfg = reference_ppo_config()
        cfg.minibatch_size, cfg.epochs = 8192, 2
        A = _nets_and_data(cfg, 4 * 8192)
        B = _nets_and_data(cfg, 4 * 8192)
        ua = ppo.PPOUpdater(*A[:4], cfg, tdist, 1, use_graph=True)
        ub = ppo.PPOUpdater(*B[:4], cfg, tdist, 1, use_graph=False)
        with pytest.warns(UserWarning, match="capture failed"):
            for run in range(3):
                idx = ppo.make_index_batches(4 * 8192, cfg.minibatch_size, cfg.epochs,
                                             torch.Generator(device="cuda").manual_seed(300 + run), "cuda")
                ua.run(*A[4], idx)
                ub.run(*B[4], idx)
                torch.cuda.synchronize()
                _compare(_state(*A[:4]), _state(*B[:4]), run)
        assert ua._gstep is None and not ua.captured_last_run
        assert "refused" in ua.capture_fallback_reason and ua._ga is not None  # the eager-collective graphs ran
        assert ua.dp_buckets == (2 if buckets == "1" else 1)
    finally:
        tdist.destroy_process_group()


def test_c5_line_reports_the_capture_fallback(monkeypatch):
    """The bench's C5 keys say which path ran: with the capture refused, allreduce_captured_in_graph
    is false, dp_capture_fallback_reason names the refusal and the eager all-reduces are timed; a
    one-rank RCCL PPOTrainer over a 64-env humanoid shard, 8,192 rows per update."""
    import importlib.util
    import os
    import mjx_amd
    from mjx_amd import mjx
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    _one_rank_group("nccl")
    _refuse_capture(monkeypatch)
    try:
        cfg = reference_ppo_config()
        cfg.num_envs, cfg.rollout_length, cfg.minibatch_size, cfg.epochs = 64, 128, 4096, 2
        cfg.eval_interval, cfg.checkpoint_every, cfg.log_interval = 10 ** 9, 10 ** 9, 1
        m = mjx_amd.load_model("humanoid_mjx")
        env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, cfg.env_config), 64, device=0, seed=3)
        tr = ppo.PPOTrainer(cfg, env, None, device="cuda:0", dist=tdist)
        with pytest.warns(UserWarning, match="capture failed"):
            res = bench.ppo_leg(tr, 1, 2, tdist, "cuda:0")
        line = bench.c5_fields(res, 1, tdist.get_backend(), bench.grad_numel(tr))
        assert line["allreduce_captured_in_graph"] is False and line["rccl_ranks"] == 1
        assert "refused" in line["dp_capture_fallback_reason"] and line["dp_buckets"] == 1
        assert line["allreduces_per_iteration"] == 4 and line["allreduce_ms_per_minibatch"] > 0
        assert len(line["ppo_c5_update_ms_per_rank"]) == 1 and line["ppo_c5_update_ms_per_rank"][0] > 0
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

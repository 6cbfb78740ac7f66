"""The data-parallel PPO path (BASELINE C5, train_ppo.py:233-252) on the HIP path: two ranks on the
one GPU of the test box, over gloo (RCCL refuses two ranks on one device; the collective calls are
the same ones the RCCL run makes).

* `ppo_update` with each rank holding half of every minibatch (native surrogate / MSE / gather
  kernels, global advantage statistics all-reduced) equals one process over the union of the data
  (the CPU version is tests/test_ppo.py::test_data_parallel_update_equals_single_process);
* two `PPOTrainer` ranks over their own HumanoidEnv shards (fused env step, captured rollout graph)
  end with bit-identical parameters and finite metrics.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

import mjx_amd
from mjx_amd import mjx, ppo
from mjx_amd.config import reference_ppo_config
from mjx_amd.envs import HumanoidEnv, resolve_ids

pytestmark = pytest.mark.gpu

N, OBS, ACT = 1024, 54, 21


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    cfg = reference_ppo_config()
    cfg.rollout_length, cfg.minibatch_size, cfg.epochs = 16, 512, 2
    cfg.num_envs = 128
    cfg.eval_interval, cfg.checkpoint_every, cfg.log_interval = 10 ** 9, 10 ** 9, 1
    return cfg


def _nets(cfg):
    pol = ppo.GaussianPolicy(OBS, ACT, cfg.policy_hidden_layer_specs, 0.0, torch.Generator().manual_seed(5)).cuda()
    val = ppo.ValueNet(OBS, cfg.value_hidden_layer_specs, torch.Generator().manual_seed(6)).cuda()
    return pol, val, torch.optim.Adam(pol.parameters(), lr=3e-4), torch.optim.Adam(val.parameters(), lr=3e-4)


def _data(seed):
    g = torch.Generator().manual_seed(seed)
    d = (torch.randn(N, OBS, generator=g), torch.rand(N, ACT, generator=g) * 1.8 - 0.9,
         torch.randn(N, generator=g) - 20.0, torch.randn(N, generator=g), torch.randn(N, generator=g))
    return tuple(x.cuda() for x in d)


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    tdist.init_process_group("gloo", rank=rank, world_size=2)
    cfg = _cfg()
    pol, val, op, ov = _nets(cfg)
    idx = torch.arange(N, device="cuda").view(4, N // 4)  # 4 minibatches, a quarter of the local rows each
    ppo.ppo_update(pol, val, op, ov, *_data(10 + rank), idx, cfg, tdist, 2)
    # two trainer ranks, each over its own 64-env shard of the humanoid
    m = mjx_amd.load_model("humanoid_mjx")
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, cfg.env_config), cfg.num_envs // 2, device=0,
                      seed=cfg.seed * 7919 + rank)
    tr = ppo.PPOTrainer(cfg, env, None, device="cuda", dist=tdist)
    hist = [tr.iteration(it) for it in range(3)]
    flat = torch.cat([p.detach().reshape(-1) for p in list(tr.policy.parameters()) + list(tr.value.parameters())])
    torch.save({"pol": {k: v.cpu() for k, v in pol.state_dict().items()},
                "val": {k: v.cpu() for k, v in val.state_dict().items()},
                "trainer": flat.cpu(), "returns": [h["train_return_avg"] for h in hist]}, out[rank])
    tdist.destroy_process_group()


def _close_adam(got, want, lr=3e-4, steps=4):
    """Parameters after `steps` Adam steps from the same start: all but 1e-3 of the entries to
    rtol 2e-5 / atol 2e-6 (the all-reduced gradient sums in another order), and every entry within
    2 lr steps — Adam's step m / (sqrt(v) + eps) is O(lr) whatever the gradient's size, so an entry
    whose gradient is at rounding-noise level may step differently (seen: 1 of 65,536, 1e-5)."""
    err = (got - want).abs()
    off = err > 2e-6 + 2e-5 * want.abs()
    assert off.float().mean().item() <= 1e-3, f"{int(off.sum())} of {off.numel()} entries off"
    assert err.max().item() <= 2 * lr * steps


def test_data_parallel_ppo_on_gpu(tmp_path):
    out = [str(tmp_path / "r0.pt"), str(tmp_path / "r1.pt")]
    mp.spawn(_worker, args=(_port(), out), nprocs=2, join=True)
    r0, r1 = (torch.load(p, weights_only=True) for p in out)
    # single process over the union: minibatch k = rank 0's quarter k, then rank 1's
    cfg = _cfg()
    pol, val, op, ov = _nets(cfg)
    d0, d1 = _data(10), _data(11)
    data = tuple(torch.cat([a, b]) for a, b in zip(d0, d1))
    idx = torch.cat([torch.arange(N).view(4, N // 4), torch.arange(N, 2 * N).view(4, N // 4)], 1).cuda()
    ppo.ppo_update(pol, val, op, ov, *data, idx, cfg)
    for k, v in pol.state_dict().items():
        _close_adam(r0["pol"][k], v.cpu())
        torch.testing.assert_close(r1["pol"][k], r0["pol"][k], rtol=0, atol=0)
    for k, v in val.state_dict().items():
        _close_adam(r0["val"][k], v.cpu())
    # the trainer ranks stay in lockstep
    torch.testing.assert_close(r0["trainer"], r1["trainer"], rtol=0, atol=0)
    assert torch.isfinite(r0["trainer"]).all()
    assert all(np.isfinite(r) for r in r0["returns"] + r1["returns"])


# ------------------------------------------------------------------------------------------------
# BASELINE configs[4] (C5) at its real per-rank shape: 8 ranks x 1024 envs, T = 256, 4 epochs, global
# minibatch 65,536 = 8,192 rows per rank, 128 all-reduces per iteration. All 8 ranks share the one GPU
# of the test box over gloo: a rehearsal of the collective pattern, not RCCL over xGMI (the driver's
# 8-GPU node runs that through bench.py --gpus 8).
C5_WORLD, C5_ENVS, C5_MB_ROWS = 8, 1024, 65536 // 8


def _c5_cfg():
    cfg = reference_ppo_config()  # src/config.json: T 256, 4 epochs, minibatch 65,536
    cfg.num_envs = C5_ENVS * C5_WORLD
    cfg.eval_interval, cfg.checkpoint_every, cfg.log_interval = 10 ** 9, 10 ** 9, 1
    return cfg


def _c5_data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    d = (torch.randn(C5_MB_ROWS, OBS, generator=g), torch.rand(C5_MB_ROWS, ACT, generator=g) * 1.8 - 0.9,
         torch.randn(C5_MB_ROWS, generator=g) - 20.0, torch.randn(C5_MB_ROWS, generator=g),
         torch.randn(C5_MB_ROWS, generator=g))
    return tuple(x.cuda() for x in d)


def _c5_worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    tdist.init_process_group("gloo", rank=rank, world_size=C5_WORLD)
    cfg = _c5_cfg()
    # (1) one minibatch: this rank's 8,192 rows of a 65,536-row minibatch
    pol, val, op, ov = _nets(cfg)
    idx = torch.arange(C5_MB_ROWS, device="cuda").view(1, C5_MB_ROWS)
    ppo.ppo_update(pol, val, op, ov, *_c5_data(rank), idx, cfg, tdist, C5_WORLD)
    # (2) the trainer at the C5 shape: iteration 0 eager, iteration 1 replays the update graphs A / B
    m = mjx_amd.load_model("humanoid_mjx")
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, cfg.env_config), C5_ENVS, device=0,
                      seed=cfg.seed * 7919 + rank)
    tr = ppo.PPOTrainer(cfg, env, None, device="cuda", dist=tdist)
    counts, hist = [], []
    for it in range(2):
        tr.allreduce_events = []
        hist.append(tr.iteration(it))
        counts.append(len(tr.allreduce_events))
    tr.allreduce_events = None
    flat = torch.cat([p.detach().reshape(-1) for p in list(tr.policy.parameters()) + list(tr.value.parameters())])
    torch.save({"pol": {k: v.cpu() for k, v in pol.state_dict().items()},
                "val": {k: v.cpu() for k, v in val.state_dict().items()},
                "trainer": flat.cpu(), "returns": [h["train_return_avg"] for h in hist],
                "allreduces": counts, "mb_rows": cfg.minibatch_size // C5_WORLD,
                "graph_used": tr.updater._ga is not None}, out[rank])
    tdist.destroy_process_group()


def test_c5_eight_ranks_at_full_per_rank_shape(tmp_path):
    """C5 (train_ppo.py:233-252, BASELINE configs[4]) with 8 ranks at 1024 envs each: every rank ends
    bit-identical; 4 * 256 * 8192 / 65,536 = 128 all-reduces per iteration, eager and graph-replayed;
    one 65,536-row minibatch split 8 ways equals one process over the union."""
    out = [str(tmp_path / f"r{r}.pt") for r in range(C5_WORLD)]
    mp.spawn(_c5_worker, args=(_port(), out), nprocs=C5_WORLD, join=True)
    rs = [torch.load(p, weights_only=True) for p in out]
    for r in rs:
        assert r["mb_rows"] == C5_MB_ROWS
        assert r["allreduces"] == [128, 128], r["allreduces"]
        assert r["graph_used"]
        torch.testing.assert_close(r["trainer"], rs[0]["trainer"], rtol=0, atol=0)
        for k in rs[0]["pol"]:
            torch.testing.assert_close(r["pol"][k], rs[0]["pol"][k], rtol=0, atol=0)
        assert all(np.isfinite(x) for x in r["returns"])
    assert torch.isfinite(rs[0]["trainer"]).all()
    # one process over the union of the 8 shares, in rank order
    cfg = _c5_cfg()
    pol, val, op, ov = _nets(cfg)
    data = tuple(torch.cat(parts) for parts in zip(*[_c5_data(r) for r in range(C5_WORLD)]))
    idx = torch.arange(C5_MB_ROWS * C5_WORLD, device="cuda").view(1, -1)
    ppo.ppo_update(pol, val, op, ov, *data, idx, cfg)
    for k, v in pol.state_dict().items():
        _close_adam(rs[0]["pol"][k], v.cpu(), steps=1)
    for k, v in val.state_dict().items():
        _close_adam(rs[0]["val"][k], v.cpu(), steps=1)

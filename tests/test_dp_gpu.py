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

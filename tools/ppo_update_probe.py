"""Diagnostic: wall time of one PPO update (4 epochs x 8 minibatches of 65,536 at 2048 envs x 256
steps) on synthetic rollout data, for optimizer / split-K variants. Not product code."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

from mjx_amd import ppo  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402


def run(fused: bool, splits: int, reps: int = 3):
    cfg = reference_ppo_config()
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
    kw = {"fused": True} if fused else {}
    op = torch.optim.Adam(pol.parameters(), lr=3e-4, **kw)
    ov = torch.optim.Adam(val.parameters(), lr=3e-4, **kw)
    N = 2048 * 256
    gd = torch.Generator(device="cuda").manual_seed(1)
    obs = torch.randn((N, 54), generator=gd, device="cuda")
    act = torch.randn((N, 21), generator=gd, device="cuda").clamp(-1, 1)
    logp = torch.randn(N, generator=gd, device="cuda") - 20
    ret = torch.randn(N, generator=gd, device="cuda")
    adv = torch.randn(N, generator=gd, device="cuda")
    ppo.SPLIT_ROWS = 65536 // splits
    ts = []
    for r in range(reps + 1):
        idx = ppo.make_index_batches(N, cfg.minibatch_size, cfg.epochs, torch.Generator().manual_seed(r), "cuda")
        torch.cuda.synchronize()
        t0 = time.time()
        ppo.ppo_update(pol, val, op, ov, obs, act, logp, ret, adv, idx, cfg)
        torch.cuda.synchronize()
        if r:
            ts.append(time.time() - t0)
    return sum(ts) / len(ts)


def enqueue_vs_wall():
    """Host enqueue time of one update vs its synced wall time (CPU-bound if they are close)."""
    cfg = reference_ppo_config()
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
    op = torch.optim.Adam(pol.parameters(), lr=3e-4, fused=True)
    ov = torch.optim.Adam(val.parameters(), lr=3e-4, fused=True)
    N = 2048 * 256
    gd = torch.Generator(device="cuda").manual_seed(1)
    obs, act = torch.randn((N, 54), generator=gd, device="cuda"), torch.randn((N, 21), generator=gd, device="cuda")
    logp, ret, adv = (torch.randn(N, generator=gd, device="cuda") for _ in range(3))
    for r in range(3):
        idx = ppo.make_index_batches(N, cfg.minibatch_size, cfg.epochs, torch.Generator(device="cuda").manual_seed(r), "cuda")
        torch.cuda.synchronize()
        t0 = time.time()
        ppo.ppo_update(pol, val, op, ov, obs, act, logp, ret, adv, idx, cfg)
        t1 = time.time()
        torch.cuda.synchronize()
        t2 = time.time()
        print(f"enqueue {1e3 * (t1 - t0):.1f} ms, wall {1e3 * (t2 - t0):.1f} ms", flush=True)


def two_stream(envs: int, reps: int = 8):
    """Synced wall time of one update with the value net on a side stream vs sequential,
    interleaved, with the trainer's NativeAdam."""
    cfg = reference_ppo_config()
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
    op, ov = ppo._adam(pol.parameters(), 3e-4), ppo._adam(val.parameters(), 3e-4)
    N = envs * 256
    gd = torch.Generator(device="cuda").manual_seed(1)
    obs, act = torch.randn((N, 54), generator=gd, device="cuda"), torch.randn((N, 21), generator=gd, device="cuda").clamp(-1, 1)
    logp, ret, adv = (torch.randn(N, generator=gd, device="cuda") for _ in range(3))
    ts = {True: [], False: []}
    for r in range(reps + 1):
        for mode in (True, False):
            ppo.TWO_STREAM_UPDATE = mode
            idx = ppo.make_index_batches(N, cfg.minibatch_size, cfg.epochs, torch.Generator().manual_seed(r), "cuda")
            torch.cuda.synchronize()
            t0 = time.time()
            ppo.ppo_update(pol, val, op, ov, obs, act, logp, ret, adv, idx, cfg)
            t1 = time.time()
            torch.cuda.synchronize()
            t2 = time.time()
            if r:
                ts[mode].append((t1 - t0, t2 - t0))
    for mode in (True, False):
        e = sorted(x[0] for x in ts[mode]); w = sorted(x[1] for x in ts[mode])
        print(f"envs={envs} two_stream={mode}: wall median {1e3 * w[len(w) // 2]:.2f} ms min {1e3 * w[0]:.2f} "
              f"max {1e3 * w[-1]:.2f}; enqueue median {1e3 * e[len(e) // 2]:.2f} ms", flush=True)


class _NoComm:
    """A one-rank stand-in for torch.distributed in the probe: all_reduce is the identity."""

    @staticmethod
    def all_reduce(t, op=None, async_op=False):
        return None

    @staticmethod
    def get_world_size():
        return 1


def shard_twin(reps: int = 5, envs: int = 1024):
    """Graph-replayed updates, twin path (mjx_amd/twin.py) vs per-net two-stream path, interleaved:
    C5's per-rank shard (8,192-row minibatches through the data-parallel bodies, identity
    collective, 128 steps) and C3's single-process update (65,536-row minibatches, 16 steps)."""
    from mjx_amd import twin
    cfg = reference_ppo_config()
    N = envs * 256
    gd = torch.Generator(device="cuda").manual_seed(1)
    obs, act = torch.randn((N, 54), generator=gd, device="cuda"), torch.randn((N, 21), generator=gd, device="cuda").clamp(-1, 1)
    logp, ret, adv = (torch.randn(N, generator=gd, device="cuda") for _ in range(3))
    for mb, dist in ((8192, _NoComm()), (65536, None)):
        cfg.minibatch_size = mb
        ups = {}
        for tw in (True, False):
            g = torch.Generator().manual_seed(0)
            pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
            val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
            op, ov = ppo._adam(pol.parameters(), 3e-4), ppo._adam(val.parameters(), 3e-4)
            twin.TWIN_UPDATE = tw
            ups[tw] = ppo.PPOUpdater(pol, val, op, ov, cfg, dist, 1, use_graph=True)
            assert (ups[tw].twin is not None) == tw
        ts = {True: [], False: []}
        for r in range(reps + 2):
            idx = ppo.make_index_batches(N, mb, cfg.epochs, torch.Generator(device="cuda").manual_seed(r), "cuda")
            for tw in (True, False):
                torch.cuda.synchronize()
                t0 = time.time()
                ups[tw].run(obs, act, logp, ret, adv, idx)
                torch.cuda.synchronize()
                if r >= 2:
                    ts[tw].append(time.time() - t0)
        for tw in (True, False):
            w = sorted(ts[tw])
            print(f"{'dp-shard' if dist is not None else 'single'} minibatch={mb} steps={idx.shape[0]} twin={tw}: "
                  f"wall median {1e3 * w[len(w) // 2]:.2f} ms (min {1e3 * w[0]:.2f}, max {1e3 * w[-1]:.2f})", flush=True)


def twin_chunk(reps: int = 5, envs: int = 1024, chunks=(128, 64, 32), mbs=(8192, 65536), attr="COLSUM_CHUNK"):
    """Graph-replayed twin updates at several values of a twin-module setting (attr: twin.COLSUM_CHUNK,
    the column-sum partial chunk; read when a minibatch step is captured), interleaved:
    C5's per-rank shard and C3's single-process update."""
    from mjx_amd import twin
    cfg = reference_ppo_config()
    N = envs * 256
    gd = torch.Generator(device="cuda").manual_seed(1)
    obs, act = torch.randn((N, 54), generator=gd, device="cuda"), torch.randn((N, 21), generator=gd, device="cuda").clamp(-1, 1)
    logp, ret, adv = (torch.randn(N, generator=gd, device="cuda") for _ in range(3))
    for mb, dist in ((8192, _NoComm()), (65536, None)):
        if mb not in mbs:
            continue
        cfg.minibatch_size = mb
        ups = {}
        for c in chunks:
            g = torch.Generator().manual_seed(0)
            pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
            val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
            op, ov = ppo._adam(pol.parameters(), 3e-4), ppo._adam(val.parameters(), 3e-4)
            ups[c] = ppo.PPOUpdater(pol, val, op, ov, cfg, dist, 1, use_graph=True)
        ts = {c: [] for c in chunks}
        for r in range(reps + 2):
            idx = ppo.make_index_batches(N, mb, cfg.epochs, torch.Generator(device="cuda").manual_seed(r), "cuda")
            for c in chunks:
                setattr(twin, attr, c)
                torch.cuda.synchronize()
                t0 = time.time()
                ups[c].run(obs, act, logp, ret, adv, idx)
                torch.cuda.synchronize()
                if r >= 2:
                    ts[c].append(time.time() - t0)
        for c in chunks:
            w = sorted(ts[c])
            print(f"{'dp-shard' if dist is not None else 'single'} minibatch={mb} steps={idx.shape[0]} {attr}={c}: "
                  f"wall median {1e3 * w[len(w) // 2]:.2f} ms (min {1e3 * w[0]:.2f}, max {1e3 * w[-1]:.2f})", flush=True)


def shard(reps: int = 5, minibatch: int = 8192, envs: int = 1024):
    """One rank's update in the C5 configuration on 8 GPUs (1024 envs x 256 steps, 4 epochs of
    8,192-row minibatches: 128 minibatch steps) through PPOUpdater's data-parallel bodies with the
    collective replaced by the identity: eager vs hipGraph replays, interleaved; and the single-process
    C3 update (65,536-row minibatches) eager vs graph."""
    cfg = reference_ppo_config()
    N = envs * 256
    gd = torch.Generator(device="cuda").manual_seed(1)
    obs, act = torch.randn((N, 54), generator=gd, device="cuda"), torch.randn((N, 21), generator=gd, device="cuda").clamp(-1, 1)
    logp, ret, adv = (torch.randn(N, generator=gd, device="cuda") for _ in range(3))
    for mb, dist in ((minibatch, _NoComm()), (cfg.minibatch_size, None)):
        cfg.minibatch_size = mb
        ups = {}
        for mode in (False, True):
            g = torch.Generator().manual_seed(0)
            pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
            val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
            op, ov = ppo._adam(pol.parameters(), 3e-4), ppo._adam(val.parameters(), 3e-4)
            ups[mode] = ppo.PPOUpdater(pol, val, op, ov, cfg, dist, 1, use_graph=mode)
        ts = {False: [], True: []}
        for r in range(reps + 2):
            idx = ppo.make_index_batches(N, mb, cfg.epochs, torch.Generator(device="cuda").manual_seed(r), "cuda")
            for mode in (False, True):
                torch.cuda.synchronize()
                t0 = time.time()
                ups[mode].run(obs, act, logp, ret, adv, idx)
                t1 = time.time()
                torch.cuda.synchronize()
                t2 = time.time()
                if r >= 2:
                    ts[mode].append((t1 - t0, t2 - t0))
        for mode in (False, True):
            w = sorted(x[1] for x in ts[mode]); e = sorted(x[0] for x in ts[mode])
            print(f"{'dp-shard' if dist is not None else 'single'} minibatch={mb} steps={idx.shape[0]} "
                  f"graph={mode}: wall median {1e3 * w[len(w) // 2]:.2f} ms (min {1e3 * w[0]:.2f}, max "
                  f"{1e3 * w[-1]:.2f}); host enqueue median {1e3 * e[len(e) // 2]:.2f} ms", flush=True)


def graph_update(envs: int = 2048, reps: int = 4):
    """The single-process update as the trainer runs it (PPOUpdater, hipGraph replays) at `envs` x 256
    steps, for a rocprofv3 kernel trace: per-kernel time of GEMMs vs elementwise vs losses / Adam."""
    cfg = reference_ppo_config()
    N = envs * 256
    gd = torch.Generator(device="cuda").manual_seed(1)
    obs, act = torch.randn((N, 54), generator=gd, device="cuda"), torch.randn((N, 21), generator=gd, device="cuda").clamp(-1, 1)
    logp, ret, adv = (torch.randn(N, generator=gd, device="cuda") for _ in range(3))
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).cuda()
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).cuda()
    op, ov = ppo._adam(pol.parameters(), 3e-4), ppo._adam(val.parameters(), 3e-4)
    up = ppo.PPOUpdater(pol, val, op, ov, cfg, None, 1, use_graph=True)
    for r in range(reps):
        idx = ppo.make_index_batches(N, cfg.minibatch_size, cfg.epochs, torch.Generator(device="cuda").manual_seed(r), "cuda")
        torch.cuda.synchronize()
        t0 = time.time()
        up.run(obs, act, logp, ret, adv, idx)
        torch.cuda.synchronize()
        print(f"update {r}: {1e3 * (time.time() - t0):.2f} ms ({'graph' if r else 'eager'})", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "graph":
        graph_update(int(sys.argv[2]) if len(sys.argv) > 2 else 2048)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "shard":
        shard()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "thin":  # split-K slices of the thin layers' weight gradients
        twin_chunk(reps=6, chunks=(None, 8, 16), attr="THIN_SPLITS", mbs=(8192,))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "splits":  # split-K slices of the hidden layers' weight gradients
        twin_chunk(reps=6, chunks=(None, 2, 8), attr="HIDDEN_SPLITS", mbs=(8192,))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "fold":  # the head's bias + tanh folded into the loss launch or not
        twin_chunk(reps=8, chunks=(True, False), attr="FOLD_HEAD")
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "twinonly":  # the twin update alone at C5's and C3's shapes
        twin_chunk(chunks=(128,))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "c5twin":  # the C5-shape twin update alone (for kernel traces)
        twin_chunk(chunks=(128,), mbs=(8192,))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "chunk":
        twin_chunk()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "twin":
        shard_twin()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "two":
        two_stream(2048)
        two_stream(1024)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "enqueue":
        enqueue_vs_wall()
        sys.exit(0)
    for fused in (False, True):
        for splits in (32, 64):
            print(f"fused={fused} splits={splits}: {run(fused, splits) * 1e3:.1f} ms per update", flush=True)

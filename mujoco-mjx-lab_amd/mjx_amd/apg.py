"""APG (analytic policy gradients) over the native env step and its VJP (reference train_apg.py).

Intended semantics of train_apg.py:161-209 (the shipped script is broken):
  * every update resets all envs (v_reset), then rolls out `horizon` steps with no reset merge;
  * obs = [qpos, qvel] (nq + nv), normalised after `obs_warmup_steps` updates as
    clip((obs - mean) / (sqrt(var) + 1e-8), -10, 10) (train_apg.py:171-176);
  * loss = -mean_envs sum_t disc_t r_t, disc_0 = 1, disc_{t+1} = disc_t gamma (1 - done_t);
  * gradients flow through the policy and through every env step (jax.grad through mjx.step with
    per-step remat, train_apg.py:187-189); clip_by_global_norm(0.3) then Adam(lr);
  * observation statistics are updated every `rms_update_every` updates from the rollout's obs.

Here the forward rollout records the pre-step state of every step (the remat tape); the backward
sweeps the tape in reverse, restoring each state into the batch and calling `mjl_env_step_vjp`,
whose action cotangent is pulled back through the policy by torch autograd. Data-parallel: each
rank rolls out its own envs; gradients (one all-reduce) and observation statistics are averaged.
"""
from __future__ import annotations

import ctypes
import json
import os
import time
from typing import Optional

import torch

from .ppo import APGPolicy, RunningMeanStd, _flat_grads, _jsonable, _set_grads, graph_capture


def _u8(t: torch.Tensor):
    """Device pointer of a contiguous uint8 CUDA tensor (alive flags of the native bookkeeping)."""
    if not t.is_cuda or t.dtype != torch.uint8 or not t.is_contiguous():
        raise ValueError("alive flags must be a contiguous uint8 CUDA tensor")
    return ctypes.c_void_p(t.data_ptr())


class NativeAPGPolicy:
    """APGPolicy's per-step passes on the native small-MLP kernels (mjl_small_mlp_fwd /
    mjl_small_mlp_bwd_input, include/mjx355.h): the forward keeps every layer's tanh output, the
    backward returns the input cotangent only (the parameter gradient is one torch pass over all
    H x B policy inputs at the end of the sweep). One launch each per rollout step where torch ran
    six. Reads the parameters in place (Adam updates them in place). MJL_APG_NATIVE_POLICY=0
    keeps torch."""

    def __init__(self, policy):
        layers = list(policy.mlp.layers)
        self.k0 = layers[0].in_features
        self.widths = [lin.out_features for lin in layers]
        self.params = [(lin.weight, lin.bias) for lin in layers]
        nl = len(layers)
        self._widths = (ctypes.c_int * nl)(*self.widths)

    @staticmethod
    def eligible(policy, device) -> bool:
        mlp = getattr(policy, "mlp", None)
        if (torch.device(device).type != "cuda" or not isinstance(policy, APGPolicy) or mlp is None
                or os.environ.get("MJL_APG_NATIVE_POLICY", "1") == "0"):
            return False
        from .ppo import ACTIVATIONS
        layers = list(mlp.layers)
        acts = list(mlp.acts)
        if not 1 <= len(layers) <= 4 or acts[-1] not in ("linear", "none"):
            return False
        if any(ACTIVATIONS.get(a, torch.tanh) is not torch.tanh for a in acts[:-1]):
            return False
        dims = [layers[0].in_features] + [lin.out_features for lin in layers]
        return all(1 <= d <= 64 for d in dims) and all(
            lin.weight.dtype == torch.float32 and lin.weight.is_contiguous() and lin.bias is not None
            for lin in layers)

    def _ptrs(self, ts):
        return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])

    def forward(self, x: torch.Tensor, ys) -> torch.Tensor:
        """ys[l]: [B, widths[l]] outputs (written); returns ys[-1], the action mean (tanh-squashed)."""
        from ._lib import check, lib
        x = x.contiguous()
        check(lib().mjl_small_mlp_fwd(x.data_ptr(), x.shape[0], self.k0, len(self.widths), self._widths,
                                      self._ptrs([w for w, _ in self.params]), self._ptrs([b for _, b in self.params]),
                                      self._ptrs(ys), torch.cuda.current_stream(x.device).cuda_stream))
        return ys[-1]

    def forward_obs(self, env, alive, rms, use_norm, o, on, snap, ys) -> torch.Tensor:
        """HumanoidAPGEnv.apg_obs, then forward(on, ys), as one launch (mjl_apg_obs_policy_fwd)."""
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        check(lib().mjl_apg_obs_policy_fwd(env.env.data.handle, _u8(alive), _ptr(rms.mean), _ptr(rms.var),
                                           int(use_norm), _ptr(o), _ptr(on), _u8(snap), len(self.widths),
                                           self._widths, self._ptrs([w for w, _ in self.params]),
                                           self._ptrs([b for _, b in self.params]), self._ptrs(ys), _stream()))
        return ys[-1]

    def transposed_weights(self):
        """The layers' weights as [k_l, n_l] copies (mjl_env_step_record_apg_next reads k rows coalesced)."""
        return [w.t().contiguous() for w, _ in self.params]

    def record_next(self, env, slot, act, gamma, diverge_qvel, alive, disc, ret, dropped, grew, rfin, rms, use_norm,
                    o, on, snap, ys, w_t):
        """HumanoidAPGEnv.step_record_apg, then forward_obs for the next step from its state, as one launch
        (mjl_env_step_record_apg_next); returns ys[-1], the next action mean."""
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        e = env.env
        act = act.to(e.obs.device, torch.float32).contiguous()
        check(lib().mjl_env_step_record_apg_next(
            e.data.handle, int(slot), _ptr(act), _ptr(e.obs), _ptr(e.rew), _ptr(e.term), _ptr(e.trunc), float(gamma),
            float(diverge_qvel), _u8(alive), _ptr(disc), _ptr(ret), _ptr(dropped), _ptr(grew), _ptr(rfin),
            _ptr(rms.mean), _ptr(rms.var), int(use_norm), _ptr(o), _ptr(on), _u8(snap), len(self.widths), self._widths,
            self._ptrs(w_t), self._ptrs([b for _, b in self.params]), self._ptrs(ys), _stream()))
        return ys[-1]

    def replay_bwd(self, env, slot, act, gq, gv, gws, grew, gaux, nonfinite, ys, o, snap, rms, use_norm):
        """HumanoidAPGEnv.step_vjp_replay, then backward_obs_vjp on its action cotangent, as one launch
        (mjl_env_step_vjp_replay_apg): returns the replay's (gq, gv, gws, ga, gaux) with the policy's
        observation path added to gq / gv."""
        from . import abi
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        B, dev = env.num_envs, env.env.obs.device
        f = lambda x, *shape: x.to(dev, torch.float32).reshape(B, *shape).contiguous()  # noqa: E731
        act, gq, gv, gr = f(act, env.act_dim), f(gq, env.nq), f(gv, env.nv), f(grew)
        ga = torch.zeros((B, abi.AUX_DIM), device=dev) if gaux is None else f(gaux, abi.AUX_DIM)
        gw = None if gws is None else f(gws, env.nv)
        oq, ov, oa, oaux = torch.empty_like(gq), torch.empty_like(gv), torch.empty_like(act), torch.empty_like(ga)
        ow = None if gws is None else torch.empty_like(gw)
        check(lib().mjl_env_step_vjp_replay_apg(
            env.env.data.handle, int(slot), _ptr(act), _ptr(gq), _ptr(gv), _ptr(gw), _ptr(gr), _ptr(ga), _ptr(oq),
            _ptr(ov), _ptr(ow), _ptr(oa), _ptr(oaux), _ptr(nonfinite), len(self.widths), self._widths,
            self._ptrs([w for w, _ in self.params]), self._ptrs(ys), _ptr(o), _u8(snap), _ptr(rms.mean),
            _ptr(rms.var), int(use_norm), _stream()))
        return oq, ov, ow, oa, oaux

    def backward_obs_vjp(self, env, g_out, ys, o, snap, rms, use_norm, gq, gv):
        """backward_input(g_out, ys), then HumanoidAPGEnv.apg_obs_vjp on its result, as one launch
        (mjl_apg_policy_bwd_obs_vjp): gq / gv accumulate the observation's cotangent."""
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        g_out = g_out.contiguous()
        check(lib().mjl_apg_policy_bwd_obs_vjp(_ptr(g_out), env.num_envs, env.nq, env.nv, len(self.widths),
                                               self._widths, self._ptrs([w for w, _ in self.params]),
                                               self._ptrs(ys), _ptr(o), _u8(snap), _ptr(rms.mean), _ptr(rms.var),
                                               int(use_norm), _ptr(gq), _ptr(gv), _stream()))

    def backward_input(self, g_out: torch.Tensor, ys) -> torch.Tensor:
        from ._lib import check, lib
        g_out = g_out.contiguous()
        gx = torch.empty((g_out.shape[0], self.k0), device=g_out.device)
        check(lib().mjl_small_mlp_bwd_input(g_out.data_ptr(), g_out.shape[0], self.k0, len(self.widths), self._widths,
                                            self._ptrs([w for w, _ in self.params]), self._ptrs(ys), gx.data_ptr(),
                                            torch.cuda.current_stream(g_out.device).cuda_stream))
        return gx


def apg_normalize(rms: RunningMeanStd, x: torch.Tensor) -> torch.Tensor:
    """train_apg.py:171-176 (note sqrt(var) + 1e-8, unlike PPO's sqrt(var + 1e-8))."""
    return torch.clamp((x - rms.mean) / (torch.sqrt(rms.var) + 1e-8), -10.0, 10.0)


class APGTrainer:
    """`env` exposes reset(), step(act, auto_reset=False) -> (obs, rew, term, trunc), step_vjp(...),
    get_state() / set_state(tape entry), qpos_qvel() and num_envs, act_dim, nq, nv (HumanoidEnv
    through `HumanoidAPGEnv`, or the differentiable stand-in of the CPU tests)."""

    def __init__(self, cfg, env, device="cuda", dist=None, out_dir: Optional[str] = None, use_graph: bool = True,
                 vjp_tape: bool = True):
        """vjp_tape: the forward rollout records each step's workspace in HBM (mjl_env_step_record,
        ~50 KB per env-step: 6 GB at 2048 x 128) and the reverse sweep replays it
        (mjl_env_step_vjp_replay) instead of restoring the state and recomputing the step."""
        self.cfg, self.env, self.dist = cfg, env, dist
        self.use_graph = bool(use_graph)
        self.vjp_tape = bool(vjp_tape)
        self._graphs, self._warm = {}, set()
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.device = torch.device(device)
        self.obs_dim = env.nq + env.nv
        g = torch.Generator().manual_seed(int(cfg.seed))
        self.policy = APGPolicy(self.obs_dim, env.act_dim, cfg.hidden_size, cfg.hidden_depth, None, g).to(self.device)
        if dist is not None:
            for p in self.policy.parameters():
                dist.broadcast(p.data, 0)
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=cfg.lr, betas=(0.9, 0.999), eps=1e-8)
        # MJL_APG_NATIVE_POLICY=0 (or native_policy = None): the policy's per-step passes through torch,
        # so the torch restatement (_loss_and_grad_torch) checks the native kernels independently
        use_nat = os.environ.get("MJL_APG_NATIVE_POLICY", "1") != "0"
        self.native_policy = (NativeAPGPolicy(self.policy)
                              if use_nat and NativeAPGPolicy.eligible(self.policy, self.device) else None)
        self.rms = RunningMeanStd(self.obs_dim, self.device)
        self.diag = None  # a dict: the eager native sweep adds per-env action-cotangent energy (probes)
        self.last_reverse_inputs = None
        self.total_env_steps = 0.0
        self.start = time.time()
        self.out_dir = out_dir if self.rank == 0 else None
        if self.out_dir:
            for sub in ("checkpoints", "logs"):
                os.makedirs(os.path.join(self.out_dir, sub), exist_ok=True)
            with open(os.path.join(self.out_dir, "config.json"), "w") as f:
                json.dump(_jsonable(cfg), f, indent=2)

    def _obs(self, use_norm: bool, alive: torch.Tensor):
        o = self.env.qpos_qvel().detach().clone().requires_grad_(True)
        # envs out of the loss (past termination, or non-finite) see a zero input: their actions
        # cannot matter, and where() keeps their non-finite values out of the policy gradient
        x = torch.where(alive[:, None], o, torch.zeros_like(o))
        return o, (apg_normalize(self.rms, x) if use_norm else x)

    def loss_and_grad(self, use_norm: bool, per_step_param_grad: bool = False):
        """_loss_and_grad_graphed under the tuned GEMM table (mjx_amd/tunable.py: on only here)."""
        from .tunable import tuned_gemms
        with tuned_gemms(self.device):
            return self._loss_and_grad_graphed(use_norm, per_step_param_grad)

    def _loss_and_grad_graphed(self, use_norm: bool, per_step_param_grad: bool = False):
        """One rollout + backward (see _loss_and_grad). On the GPU the second and later calls per
        `use_norm` replay one hipGraph of the whole thing: ~60 launches per rollout step (env step,
        VJP, the policy's forward and backward, the guard's elementwise ops) with no host in between;
        the env's reset counter comes from its device counter base, so a replay is bit-identical to
        the eager call (tests/test_apg.py)."""
        env = self.env
        if per_step_param_grad or not self.use_graph or self.device.type != "cuda" or not hasattr(env, "ctr_base"):
            return self._loss_and_grad(use_norm, per_step_param_grad)
        key = bool(use_norm)
        if key not in self._graphs:
            if key not in self._warm:  # first call eager: library handles, allocator pools, GEMM choices
                self._warm.add(key)
                return self._loss_and_grad(use_norm, False)
            graph = torch.cuda.CUDAGraph()
            c0 = env.counter
            self.opt.zero_grad(set_to_none=True)
            with graph_capture(graph):
                out = self._loss_and_grad(use_norm, False, graph=True)
            # the counters the eager call takes: the host code's during capture, plus the reset's own
            # (passed explicitly, relative to the base, under capture)
            used = env.counter - c0 + 1
            env.counter = c0  # capture ran nothing; the replay below draws the reset
            self._graphs[key] = (graph, out, [p.grad for p in self.policy.parameters()], used,
                                 self.last_reverse_inputs)
        graph, out, grads, used, self.last_reverse_inputs = self._graphs[key]
        env.ctr_base.fill_(env.counter)
        graph.replay()
        env.counter += used
        env.ctr_base.zero_()
        for p, g in zip(self.policy.parameters(), grads):  # the graph's gradient buffers
            p.grad = g
        return out

    def _loss_and_grad(self, use_norm: bool, per_step_param_grad: bool = False, graph: bool = False):
        if getattr(self.env, "native_apg", False) and not per_step_param_grad:
            return self._loss_and_grad_native(use_norm, graph)
        return self._loss_and_grad_torch(use_norm, per_step_param_grad, graph)

    def _loss_and_grad_native(self, use_norm: bool, graph: bool = False):
        """_loss_and_grad_torch with its per-step bookkeeping as three native launches
        (mjl_apg_obs / mjl_apg_post / mjl_apg_obs_vjp, include/mjx355.h: the same guard, discount,
        return and observation derivative): ~50 torch ops per rollout step become 2, and the
        reverse sweep's observation backward 1. The policy input `on` is the autograd leaf."""
        cfg, env = self.cfg, self.env
        H, B, gamma, dev = cfg.horizon, env.num_envs, cfg.gamma, self.device
        w = env.nq + env.nv
        if graph:
            env.reset(counter=1)  # relative to ctr_base = the counter before the call
        else:
            env.reset()
        o_all, on_all = torch.empty((H, B, w), device=dev), torch.empty((H, B, w), device=dev)
        snap = torch.empty((H, B), dtype=torch.uint8, device=dev)
        grew_all, rfin = torch.empty((H, B), device=dev), torch.empty((H, B), device=dev)
        alive = torch.ones(B, dtype=torch.uint8, device=dev)
        disc, ret = torch.ones(B, device=dev), torch.zeros(B, device=dev)
        dropped_e = torch.zeros(B, device=dev)
        dq = float(getattr(cfg, "diverge_qvel", None) or 0.0)
        taped = self.vjp_tape and hasattr(env, "step_record")
        if taped and getattr(env, "tape_slots", 0) < H:
            env.enable_vjp_tape(H)
        tape, acts, leaves = [], [], []
        nat = self.native_policy
        ys_all = [torch.empty((H, B, n), device=dev) for n in nat.widths] if nat is not None else None
        # the observation and the policy forward as one launch (and their backward as one), when the env
        # is the native one (HumanoidAPGEnv); MJL_APG_FUSED_OBS=0 keeps the separate launches
        fused = nat is not None and isinstance(env, HumanoidAPGEnv) and os.environ.get("MJL_APG_FUSED_OBS", "1") != "0"
        # the record and the post-step update as one launch (MJL_APG_FUSED_POST=0: the two launches), and
        # with it the next step's observation + policy forward (MJL_APG_FUSED_NEXT=0: their own launch)
        fused_post = taped and hasattr(env, "step_record_apg") and os.environ.get("MJL_APG_FUSED_POST", "1") != "0"
        fused_next = (fused_post and fused and env.supports_record_next()
                      and os.environ.get("MJL_APG_FUSED_NEXT", "1") != "0")
        w_t = nat.transposed_weights() if fused_next else None
        a_next = None
        for t in range(H):
            if not taped:
                tape.append(env.get_state())
            if a_next is not None:  # written by the previous step's record launch
                a, a_next = a_next, None
            elif fused:
                a = nat.forward_obs(env, alive, self.rms, use_norm, o_all[t], on_all[t], snap[t], [y[t] for y in ys_all])
            elif nat is not None:  # one launch; the layers' outputs kept for the reverse
                env.apg_obs(alive, self.rms, use_norm, o_all[t], on_all[t], snap[t])
                a = nat.forward(on_all[t], [y[t] for y in ys_all])
            else:
                env.apg_obs(alive, self.rms, use_norm, o_all[t], on_all[t], snap[t])
                on = on_all[t].detach().requires_grad_(True)
                a = self.policy(on)
                leaves.append(on)
            acts.append(a)
            if fused_next and t + 1 < H:  # the step, slot t, the post-step update and step t + 1's policy
                a_next = nat.record_next(env, t, a.detach(), gamma, dq, alive, disc, ret, dropped_e, grew_all[t],
                                         rfin[t], self.rms, use_norm, o_all[t + 1], on_all[t + 1], snap[t + 1],
                                         [y[t + 1] for y in ys_all], w_t)
                continue
            if fused_post:  # the step, its tape slot t and the post-step update in one launch
                env.step_record_apg(t, a.detach(), gamma, dq, alive, disc, ret, dropped_e, grew_all[t], rfin[t])
                continue
            if taped:  # the step, leaving its forward workspace in tape slot t
                _, r, te, tr = env.step_record(t, a.detach())
            else:
                _, r, te, tr = env.step(a.detach(), auto_reset=False)
            env.apg_post(r, te, tr, gamma, dq, alive, disc, ret, dropped_e, grew_all[t], rfin[t])
        loss = -ret.mean()
        final = None if taped else env.get_state()
        self.opt.zero_grad(set_to_none=True)
        gq = torch.zeros((B, env.nq), device=dev)
        gv = torch.zeros((B, env.nv), device=dev)
        gaux = None
        nonfinite = torch.zeros(1, device=dev)
        gws = torch.zeros((B, env.nv), device=dev) if getattr(env, "vjp_carries_ws", False) else None
        gas = [None] * H
        # the policy + observation backward in the replay launch (MJL_APG_FUSED_BWD=0: their own launch)
        fused_bwd = taped and fused and os.environ.get("MJL_APG_FUSED_BWD", "1") != "0"
        for t in range(H - 1, -1, -1):
            if fused_bwd:  # slot t's reverse passes, then the policy's and the observation's backward
                gq, gv, gws, ga, gaux = nat.replay_bwd(env, t, acts[t].detach(), gq, gv, gws, grew_all[t], gaux,
                                                       nonfinite, [y[t] for y in ys_all], o_all[t], snap[t], self.rms,
                                                       use_norm)
                gas[t] = ga
                if self.diag is not None and not graph:
                    e = (ga.double() ** 2).sum(1)
                    self.diag["ga_sq"] = e if t == H - 1 else self.diag["ga_sq"] + e
                continue
            if taped:  # the reverse passes from slot t: no state restore, no recompute
                gq, gv, gws, ga, gaux = env.step_vjp_replay(t, acts[t].detach(), gq, gv, gws, grew_all[t], gaux,
                                                            nonfinite)
            else:
                env.set_state(tape[t], tape[t + 1] if t + 1 < H else final)
                if gws is not None:
                    gq, gv, gws, ga, gaux = env.step_vjp_full(acts[t].detach(), gq, gv, gws, grew_all[t], gaux,
                                                              nonfinite)
                else:
                    gq, gv, ga, gaux = env.step_vjp(acts[t].detach(), gq, gv, grew_all[t], gaux, nonfinite)
            if fused:
                nat.backward_obs_vjp(env, ga, [y[t] for y in ys_all], o_all[t], snap[t], self.rms, use_norm, gq, gv)
            else:
                if nat is not None:
                    og = nat.backward_input(ga, [y[t] for y in ys_all])
                else:
                    og, = torch.autograd.grad(acts[t], leaves[t], grad_outputs=ga)
                env.apg_obs_vjp(o_all[t], snap[t], self.rms, use_norm, og, gq, gv)
            gas[t] = ga
            if self.diag is not None and not graph:  # sum over steps of |d loss / d a_t|^2 per env
                e = (ga.double() ** 2).sum(1)
                self.diag["ga_sq"] = e if t == H - 1 else self.diag["ga_sq"] + e
        torch.autograd.backward(self.policy(on_all.reshape(H * B, w)), grad_tensors=torch.cat(gas))
        dropped = torch.stack([dropped_e.sum(), nonfinite[0]])  # (forward guard, reverse guard)
        # the reward cotangents and actions of the last rollout (graph-owned under capture: they hold
        # the last replay's values), for timing the replay VJP on the trainer's own workload (bench.py)
        self.last_reverse_inputs = (grew_all, [a.detach() for a in acts]) if taped else None
        return loss.detach(), (rfin.mean(1).sum() / H).detach(), (o_all, snap), dropped

    def _loss_and_grad_torch(self, use_norm: bool, per_step_param_grad: bool = False, graph: bool = False):
        """One rollout + backward. Returns (loss, mean reward, (obs trajectory [H, B, nq + nv], in-loss
        mask [H, B]: the env was alive at that step), envs dropped as non-finite); grads in .grad.

        An env whose state or reward turns non-finite, or whose max |qvel| passes cfg.diverge_qvel,
        is treated as terminated from that step on (its reward at that step is dropped); an env whose
        cotangents overflow in the reverse sweep is cut from the gradient at that step. The reference has no such guard: one such env makes its
        loss NaN and train_apg.py:278-287 stops the run; here the run continues and the count of
        dropped envs is reported."""
        cfg, env = self.cfg, self.env
        H, B, gamma = cfg.horizon, env.num_envs, cfg.gamma
        if graph:
            env.reset(counter=1)  # relative to ctr_base = the counter before the call
        else:
            env.reset()
        tape, obs_leaves, acts, discs, pol_in = [], [], [], [], []
        nat = self.native_policy  # the same policy numerics as the native sweep (rollouts amplify ulps)
        ons, ys_steps = [], []
        disc = ret = rsum = None  # created from the first reward (dtype follows the env)
        alive = torch.ones(B, dtype=torch.bool, device=self.device)
        dropped = torch.zeros((), device=self.device)
        rev_dropped = torch.zeros((), device=self.device)
        obs_traj, in_loss = [], []
        for _ in range(H):
            tape.append(env.get_state())
            o, on = self._obs(use_norm, alive)
            if nat is not None:
                ys = [torch.empty((B, n), device=self.device) for n in nat.widths]
                a = nat.forward(on.detach(), ys)
                ys_steps.append(ys)
                ons.append(on)
            else:
                a = self.policy(on)
            pol_in.append(on.detach())
            obs_leaves.append(o)
            acts.append(a)
            obs_traj.append(o.detach())
            in_loss.append(alive.clone())
            _, r, te, tr = env.step(a.detach(), auto_reset=False)
            if disc is None:
                disc, ret, rsum = torch.ones_like(r), torch.zeros_like(r), torch.zeros_like(r[0])
            # a non-finite post-step state must leave the loss at this step: next step its obs would
            # reach the policy, and backward through tanh turns even a zero cotangent into NaN; so does
            # a diverged one (max |qvel| > cfg.diverge_qvel: truncated solves)
            qq = env.qpos_qvel()
            ok = torch.isfinite(r) & torch.isfinite(qq).all(1)
            if getattr(cfg, "diverge_qvel", None):
                ok = ok & (qq[:, env.nq:].abs().amax(1) <= cfg.diverge_qvel)
            bad = alive & ~ok
            dropped = dropped + bad.sum()
            alive = alive & ~bad
            disc = torch.where(alive, disc, torch.zeros_like(disc))
            discs.append(disc)
            ret = ret + torch.where(alive, disc * r, torch.zeros_like(r))
            rsum = rsum + torch.where(torch.isfinite(r), r, torch.zeros_like(r)).mean()  # mean(rewards)
            disc = disc * gamma * (1.0 - torch.maximum(te, tr))
            alive = alive & (disc != 0)
        loss = -ret.mean()
        final = env.get_state()
        # reverse sweep: state cotangents of step t+1 -> step t; action cotangents -> policy
        self.opt.zero_grad(set_to_none=True)
        gq = torch.zeros((B, env.nq), device=self.device)
        gv = torch.zeros((B, env.nv), device=self.device)
        gaux = None
        guarded = getattr(env, "guarded_vjp", False)
        nonfinite = torch.zeros(1, device=self.device) if guarded else None
        # unrolled VJP: the next solve depends on the carried qacc_warmstart, so its cotangent rides along
        gws = torch.zeros((B, env.nv), device=self.device) if getattr(env, "vjp_carries_ws", False) else None
        gas = [None] * H
        for t in range(H - 1, -1, -1):
            # the VJP recomputes the step to find its converged active set; the solution the forward
            # step reached (the next tape entry's qacc_warmstart) seeds that solve: ~1 Newton iteration
            env.set_state(tape[t], tape[t + 1] if t + 1 < H else final)
            grew = -discs[t] / B
            # an env whose cotangents overflow (a state blowing up while still in the loss) is cut from
            # the gradient at this step, like the forward guard above (in the kernel when it can)
            if gws is not None:
                gq, gv, gws, ga, gaux = env.step_vjp_full(acts[t].detach(), gq, gv, gws, grew, gaux, nonfinite)
            else:
                gq, gv, ga, gaux = env.step_vjp(acts[t].detach(), gq, gv, grew, gaux, nonfinite)
            if not guarded:
                ok = torch.isfinite(gq).all(1) & torch.isfinite(gv).all(1) & torch.isfinite(ga).all(1)
                rev_dropped = rev_dropped + (~ok).sum()
                gq = torch.where(ok[:, None], gq, torch.zeros_like(gq))
                gv = torch.where(ok[:, None], gv, torch.zeros_like(gv))
                ga = torch.where(ok[:, None], ga, torch.zeros_like(ga))
            # the chain needs only the observation cotangent here; the parameter gradient (a sum over
            # steps) is taken once below from all steps' action cotangents
            if nat is not None:  # native policy backward to its input, torch for the normalisation
                g_on = nat.backward_input(ga, ys_steps[t])
                og, = torch.autograd.grad(ons[t], obs_leaves[t], grad_outputs=g_on.to(ons[t].dtype))
                if per_step_param_grad:
                    pg = torch.autograd.grad(self.policy(pol_in[t]), list(self.policy.parameters()), grad_outputs=ga)
                    for p_, g_ in zip(self.policy.parameters(), pg):
                        p_.grad = g_ if p_.grad is None else p_.grad + g_
            elif per_step_param_grad:  # the unbatched form (tests): parameter gradient accumulated per step
                og, *pg = torch.autograd.grad(acts[t], [obs_leaves[t]] + list(self.policy.parameters()), grad_outputs=ga)
                for p_, g_ in zip(self.policy.parameters(), pg):
                    p_.grad = g_ if p_.grad is None else p_.grad + g_
            else:
                og, = torch.autograd.grad(acts[t], obs_leaves[t], grad_outputs=ga)
            gas[t] = ga
            gq = gq + og[:, :env.nq]
            gv = gv + og[:, env.nq:]
        # parameter gradient: sum_t (d a_t / d theta)^T ga_t as one forward + backward over the H * B
        # policy inputs of the rollout (the same inputs; per step it was H small backward passes)
        if not per_step_param_grad:
            torch.autograd.backward(self.policy(torch.cat(pol_in)), grad_tensors=torch.cat(gas))
        dropped = torch.stack([dropped.to(torch.float32), (nonfinite[0] if guarded else rev_dropped).to(torch.float32)])
        return loss.detach(), (rsum / H).detach(), (torch.stack(obs_traj), torch.stack(in_loss)), dropped

    def update(self, step: int) -> dict:
        cfg = self.cfg
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t0 = time.time()
        use_norm = step >= cfg.obs_warmup_steps and cfg.normalize_observations
        loss, mean_r, obs_traj, dropped = self.loss_and_grad(use_norm)
        params = list(self.policy.parameters())
        g = _flat_grads(params)
        stats = torch.cat([torch.stack([loss, mean_r]), dropped.to(loss.dtype).reshape(2)])
        if self.dist is not None:
            self.dist.all_reduce(g)
            g /= self.world
            self.dist.all_reduce(stats)
            stats[:2] /= self.world
        gnorm = torch.linalg.vector_norm(g.double())  # fp64: an fp32 sum of squares overflows on blow-ups
        g = g * torch.clamp(cfg.grad_clip / (gnorm + 1e-16), max=1.0).to(g.dtype)  # optax.clip_by_global_norm
        _set_grads(params, g)
        self.opt.step()
        frozen = getattr(cfg, "rms_freeze_after", None) is not None and step > cfg.rms_freeze_after
        if cfg.normalize_observations and step % cfg.rms_update_every == 0 and not frozen:
            obs, in_loss = obs_traj
            flat = obs.reshape(-1, obs.shape[-1])
            keep = torch.isfinite(flat).all(1)
            if cfg.rms_in_loss_only:
                keep = keep & in_loss.reshape(-1).bool()
            self.rms.update(flat[keep], self.dist)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = max(time.time() - t0, 1e-9)
        steps = float(cfg.horizon * self.env.num_envs * self.world)
        self.total_env_steps += steps
        return {"loss": float(stats[0]), "return": float(-stats[0]), "mean_reward": float(stats[1]),
                "grad_norm": float(gnorm), "env_steps_per_sec": steps / dt,
                "nonfinite_envs": int(stats[2]) + int(stats[3]),  # dropped from the loss, either guard
                "forward_dropped_envs": int(stats[2]),  # state / reward non-finite or |qvel| > diverge_qvel
                "reverse_nonfinite_envs": int(stats[3])}  # cotangents overflowed in the VJP sweep

    def train(self, steps: Optional[int] = None, verbose: bool = True):
        n = self.cfg.total_steps if steps is None else steps
        hist = []
        for step in range(n):
            m = self.update(step)
            if not (m["loss"] == m["loss"]):  # NaN guard (train_apg.py:278-287)
                if verbose and self.rank == 0:
                    print(f"NaN loss at step {step}", flush=True)
                break
            m["total_env_steps"] = self.total_env_steps
            m["elapsed_time"] = time.time() - self.start
            if self.out_dir:
                with open(os.path.join(self.out_dir, "logs", "metrics.jsonl"), "a") as f:
                    f.write(json.dumps({"step": step, **m}) + "\n")
                if (step + 1) % self.cfg.checkpoint_every == 0 or step == n - 1:
                    torch.save({"step": step, "params": self.policy.state_dict(), "rms": self.rms.state_dict(),
                                "opt": self.opt.state_dict()},
                               os.path.join(self.out_dir, "checkpoints", f"checkpoint_{step:06d}.pt"))
            if verbose and self.rank == 0 and (step < 10 or step % 10 == 0):
                print(f"Step {step:5d} | Return: {m['return']:8.3f} | Reward: {m['mean_reward']:7.4f} | "
                      f"GradNorm: {m['grad_norm']:8.3f} | Steps/s: {m['env_steps_per_sec']:9.0f}", flush=True)
            hist.append(m)
        return hist


class HumanoidAPGEnv:
    """HumanoidEnv adapter for APGTrainer: tape entries are packed state rows (mjl_get_state).

    vjp="unrolled": the VJP differentiates the constraint solve's iterations as executed, what
    jax.grad through MJX's fixed-count solver computes (train_apg.py:101-105,187-189, CG 4/4); the
    recompute must replay the forward's solve, so it starts from the tape entry's own warm start.
    vjp="implicit": the derivative at the converged active set (exact for a converged solve, e.g.
    the MJCF's Newton 10/20); the recompute is seeded with the forward's solution (~1 iteration)."""

    guarded_vjp = True
    native_apg = True  # APGTrainer's bookkeeping as native launches (apg_obs / apg_post / apg_obs_vjp)

    def __init__(self, env, vjp: str = "implicit"):
        from . import abi
        if vjp not in ("implicit", "unrolled"):
            raise ValueError(f"vjp must be 'implicit' or 'unrolled', not {vjp!r}")
        self.vjp = vjp
        self.vjp_carries_ws = vjp == "unrolled"  # jax.grad also differentiates the carried warm start
        env.data.set_option(abi.OPT_VJP_UNROLLED, int(vjp == "unrolled"))
        self.env = env
        self.num_envs, self.act_dim = env.num_envs, env.act_dim
        self.nq, self.nv = env.sys.nq, env.sys.nv

    def reset(self, counter=None):
        return self.env.reset(counter=counter)

    @property
    def ctr_base(self):
        return self.env.ctr_base

    @property
    def counter(self):
        return self.env.counter

    @counter.setter
    def counter(self, v):
        self.env.counter = v

    def step(self, act, auto_reset=False):
        return self.env.step(act, auto_reset=auto_reset)

    def qpos_qvel(self):
        return torch.cat([self.env.data.get("qpos"), self.env.data.get("qvel")], 1)

    def get_state(self):
        return self.env.get_state()

    def set_state(self, st, warm_from=None):
        """Restore a tape entry; qacc_warmstart from `warm_from` (another entry) when given and the
        VJP is implicit (the unrolled VJP replays the forward's own solve)."""
        self.env.set_state(st, warm_from if self.vjp == "implicit" else None)

    def step_vjp(self, act, gq, gv, grew, gaux, nonfinite=None):
        return self.env.step_vjp(act, gq, gv, grew, gaux, nonfinite)

    def enable_vjp_tape(self, slots: int):
        """Allocate `slots` VJP tape slots (MJL_OPT_VJP_TAPE; outside stream capture)."""
        from . import abi
        self.env.data.set_option(abi.OPT_VJP_TAPE, int(slots))
        self.tape_slots = int(slots)

    def step_record(self, slot: int, act):
        """The env step (no reset merge) that also records slot `slot` of the VJP tape."""
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        e = self.env
        act = act.to(e.obs.device, torch.float32).contiguous()
        check(lib().mjl_env_step_record(e.data.handle, int(slot), _ptr(act), _ptr(e.obs), _ptr(e.rew), _ptr(e.term),
                                        _ptr(e.trunc), _stream()))
        return e.obs, e.rew, e.term, e.trunc

    def supports_record_next(self) -> bool:
        """Whether the record kernel takes the next step's policy forward (mjl_env_step_record_apg_next:
        the implicit record on the humanoid dims)."""
        from ._lib import lib
        return bool(lib().mjl_env_record_fused(self.env.data.handle))

    def step_record_apg(self, slot: int, act, gamma, diverge_qvel, alive, disc, ret, dropped, grew, rfin):
        """step_record then apg_post on its outputs, as one launch where the record kernel allows it
        (mjl_env_step_record_apg)."""
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        e = self.env
        act = act.to(e.obs.device, torch.float32).contiguous()
        check(lib().mjl_env_step_record_apg(e.data.handle, int(slot), _ptr(act), _ptr(e.obs), _ptr(e.rew),
                                            _ptr(e.term), _ptr(e.trunc), float(gamma), float(diverge_qvel), _u8(alive),
                                            _ptr(disc), _ptr(ret), _ptr(dropped), _ptr(grew), _ptr(rfin), _stream()))
        return e.obs, e.rew, e.term, e.trunc

    def step_vjp_replay(self, slot: int, act, gq, gv, gws, grew, gaux, nonfinite=None):
        """VJP of the step recorded in `slot` (mjl_env_step_vjp_replay): returns the cotangents of
        (qpos, qvel, qacc_warmstart or None, action, aux)."""
        from . import abi
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        B, dev = self.num_envs, self.env.obs.device
        f = lambda x, *shape: x.to(dev, torch.float32).reshape(B, *shape).contiguous()  # noqa: E731
        act, gq, gv, gr = f(act, self.act_dim), f(gq, self.nq), f(gv, self.nv), f(grew)
        ga = torch.zeros((B, abi.AUX_DIM), device=dev) if gaux is None else f(gaux, abi.AUX_DIM)
        gw = None if gws is None else f(gws, self.nv)
        oq, ov, oa, oaux = torch.empty_like(gq), torch.empty_like(gv), torch.empty_like(act), torch.empty_like(ga)
        ow = None if gws is None else torch.empty_like(gw)
        check(lib().mjl_env_step_vjp_replay(self.env.data.handle, int(slot), _ptr(act), _ptr(gq), _ptr(gv), _ptr(gw),
                                            _ptr(gr), _ptr(ga), _ptr(oq), _ptr(ov), _ptr(ow), _ptr(oa), _ptr(oaux),
                                            _ptr(nonfinite), _stream()))
        return oq, ov, ow, oa, oaux

    def apg_obs(self, alive, rms, use_norm, o, on, snap):
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        check(lib().mjl_apg_obs(self.env.data.handle, _u8(alive), _ptr(rms.mean), _ptr(rms.var), int(use_norm),
                                _ptr(o), _ptr(on), _u8(snap), _stream()))

    def apg_post(self, r, te, tr, gamma, diverge_qvel, alive, disc, ret, dropped, grew, rfin):
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        check(lib().mjl_apg_post(self.env.data.handle, _ptr(r), _ptr(te), _ptr(tr), float(gamma), float(diverge_qvel),
                                 _u8(alive), _ptr(disc), _ptr(ret), _ptr(dropped), _ptr(grew), _ptr(rfin), _stream()))

    def apg_obs_vjp(self, o, snap, rms, use_norm, go, gq, gv):
        from ._lib import check, lib
        from .mjx import _ptr, _stream
        check(lib().mjl_apg_obs_vjp(self.num_envs, self.nq, self.nv, _ptr(o), _u8(snap), _ptr(rms.mean),
                                    _ptr(rms.var), int(use_norm), _ptr(go.contiguous()), _ptr(gq), _ptr(gv), _stream()))

    def step_vjp_full(self, act, gq, gv, gws, grew, gaux, nonfinite=None):
        return self.env.step_vjp_full(act, gq, gv, gws, grew, gaux, nonfinite)

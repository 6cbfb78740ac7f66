"""PPO trainer over the native env step (reference train_ppo.py, src/networks.py, src/training_utils.py).

Host-side PyTorch: the MLPs are rocBLAS/hipBLASLt GEMMs on the same stream as the env kernels; the
env step (physics + reward + obs + auto-reset) is one `mjl_env_step` launch per rollout step.
Formulas follow the reference line by line (cited per function); data-parallel training over
`torch.distributed` (RCCL on GPUs, gloo on CPU) adds exactly the exchanges SURVEY.md §8e lists:
parameter broadcast at start, one all-reduce of the flattened policy+value gradients per
minibatch, the advantage-normalisation sums per minibatch, and the observation statistics per
iteration. Each rank steps its own envs; nothing in the physics path communicates.
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict, is_dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

ACTIVATIONS = {
    "tanh": torch.tanh, "relu": torch.relu, "elu": nn.functional.elu, "swish": nn.functional.silu,
    "silu": nn.functional.silu, "gelu": nn.functional.gelu, "linear": lambda x: x, "none": lambda x: x,
}


# ----------------------------------------------------------------------------------------- networks
_COLSUM_SCRATCH = {}


def colsum_native(x: torch.Tensor) -> torch.Tensor:
    """x[n, d].sum(0) for a contiguous float32 device matrix as one or two launches of mjl_colsum
    (fixed summation order); torch's sum(0) is 33 us at [65536, 256] and 169 us at [65536, 21]."""
    from ._lib import check, lib
    n, d = x.shape
    if not (x.is_contiguous() and x.dtype == torch.float32 and x.is_cuda):
        raise ValueError("colsum_native: contiguous float32 device matrix expected")
    out = torch.empty(d, dtype=torch.float32, device=x.device)
    ns = int(lib().mjl_colsum_scratch(n, d))
    scratch = None
    if ns:
        key = (x.device, ns, torch.cuda.current_stream(x.device).cuda_stream)  # one per stream (two-stream update)
        scratch = _COLSUM_SCRATCH.get(key)
        if scratch is None:
            scratch = _COLSUM_SCRATCH[key] = torch.empty(ns, dtype=torch.float32, device=x.device)
    check(lib().mjl_colsum(x.data_ptr(), n, d, scratch.data_ptr() if scratch is not None else None, out.data_ptr(),
                           torch.cuda.current_stream(x.device).cuda_stream))
    return out


class _SplitKLinear(torch.autograd.Function):
    """y = x Wᵀ + b whose weight gradient Wᵀ-shaped dY ᵀ X (K = the batch, 65,536 rows in a PPO
    minibatch, output only 256 x 256) runs as `splits` batched GEMMs of K / splits rows plus one
    sum: as a single GEMM the library tiles the small output into 32 workgroups and leaves most
    of the 256 CUs idle (measured 37 TFLOP/s on MI355X). The bias gradient (a column sum over the
    65,536 rows) runs on the native kernel (colsum_native: 14.8 / 11.8 us against torch's 33 / 168
    us at 256 / 21 columns); a single column and the 32-row split sum stay with torch's reduction,
    which is faster there (7.6 / 5.5 us against 11.7 / 8.5)."""

    @staticmethod
    def forward(ctx, x, w, b, splits):
        ctx.save_for_backward(x, w)
        ctx.splits = splits
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        s, n = ctx.splits, x.shape[0]
        gx = gy @ w if ctx.needs_input_grad[0] else None
        gw = slice_sum_native(torch.bmm(gy.reshape(s, n // s, -1).transpose(1, 2), x.reshape(s, n // s, -1)))
        gb = colsum_native(gy.contiguous()) if gy.shape[1] > 1 else gy.sum(0)
        return gx, gw, gb, None


def slice_sum_native(x: torch.Tensor) -> torch.Tensor:
    """x[s, ...].sum(0) for a contiguous float32 device tensor, slices added in order (mjl_slice_sum):
    the split-K weight gradient's sum over its batched GEMMs; torch's sum(0) took 13 us at [32, 256, 256]."""
    m = x[0].numel()
    if not (x.is_cuda and x.is_contiguous() and x.dtype == torch.float32 and m % 4 == 0):
        return x.sum(0)
    from ._lib import check, lib
    out = torch.empty(x.shape[1:], dtype=torch.float32, device=x.device)
    check(lib().mjl_slice_sum(x.data_ptr(), x.shape[0], m, out.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream))
    return out


def tanh_inplace_native(x: torch.Tensor) -> torch.Tensor:
    """x.tanh_() for a contiguous float32 device tensor (mjl_tanh_inplace, float4 per thread)."""
    if not (x.is_cuda and x.is_contiguous() and x.dtype == torch.float32 and x.numel() % 4 == 0):
        return x.tanh_()
    from ._lib import check, lib
    check(lib().mjl_tanh_inplace(x.data_ptr(), x.numel(), torch.cuda.current_stream(x.device).cuda_stream))
    return x


def tanh_bwd_colsum_native(gy: torch.Tensor, y: torch.Tensor):
    """(dz, db) = (gy (1 - y^2), dz.sum(0)) for y = tanh(z) [n, d] in one pass (mjl_tanh_bwd_colsum) plus
    the column sum's small second stage: torch's tanh_backward and then a column sum re-reading dz."""
    from ._lib import check, lib
    n, d = y.shape
    dz = torch.empty_like(y)
    db = torch.empty(d, dtype=torch.float32, device=y.device)
    st = torch.cuda.current_stream(y.device).cuda_stream
    ns = int(lib().mjl_colsum_scratch(n, d))
    scratch = None
    if ns:
        key = (y.device, ns, st)
        scratch = _COLSUM_SCRATCH.get(key)
        if scratch is None:
            scratch = _COLSUM_SCRATCH[key] = torch.empty(ns, dtype=torch.float32, device=y.device)
    check(lib().mjl_tanh_bwd_colsum(gy.data_ptr(), y.data_ptr(), n, d, dz.data_ptr(),
                                    scratch.data_ptr() if scratch is not None else None, db.data_ptr(), st))
    return dz, db


class _TanhSplitKLinear(torch.autograd.Function):
    """y = tanh(x Wᵀ + b) as _SplitKLinear + tanh, whose backward forms dz = dy (1 - y²) and the bias
    gradient's column sums in one pass over dy and y (tanh_bwd_colsum_native) instead of torch's
    tanh_backward followed by a column sum that reads dz again."""

    @staticmethod
    def forward(ctx, x, w, b, splits):
        y = tanh_inplace_native(torch.addmm(b, x, w.t()))
        ctx.save_for_backward(x, w, y)
        ctx.splits = splits
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        s, n = ctx.splits, x.shape[0]
        dz, gb = tanh_bwd_colsum_native(gy.contiguous(), y)
        gx = dz @ w if ctx.needs_input_grad[0] else None
        gw = slice_sum_native(torch.bmm(dz.reshape(s, n // s, -1).transpose(1, 2), x.reshape(s, n // s, -1)))
        return gx, gw, gb, None


SPLIT_ROWS = int(os.environ.get("MJL_SPLIT_ROWS", "2048"))  # rows per split of the split-K weight gradient (32 splits at a 65,536 minibatch)


UPDATE_MIN_ROWS = 4096  # minibatches of at least this many rows take the native / split-K update path


# tanh layers of the update on _TanhSplitKLinear (MJL_TANH_FUSED=0: torch's tanh_backward + colsum)
TANH_FUSED = os.environ.get("MJL_TANH_FUSED", "1") == "1"


def _tanh_linear(lin: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    """tanh(Dense(x)); the update's layers (as _linear's split-K condition, width % 4 == 0) fuse the
    tanh backward with the bias gradient's column sum (_TanhSplitKLinear)."""
    n = x.shape[0] if x.dim() == 2 else 0
    if (TANH_FUSED and x.is_cuda and torch.is_grad_enabled() and n >= UPDATE_MIN_ROWS and n % SPLIT_ROWS == 0
            and lin.out_features % 4 == 0 and x.dtype == torch.float32):
        return _TanhSplitKLinear.apply(x, lin.weight, lin.bias, min(64, n // SPLIT_ROWS))
    return torch.tanh(_linear(lin, x))


def _linear(lin: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    """Dense layer; in the update (grad enabled, >= UPDATE_MIN_ROWS rows) the split-K weight gradient,
    whose fixed batched-GEMM + sum order is also deterministic: the library's single GEMM over K =
    8,192 rows (the per-rank minibatch of C5 at 8 GPUs) was not bit-reproducible run to run."""
    n = x.shape[0] if x.dim() == 2 else 0
    if (x.is_cuda and torch.is_grad_enabled() and n >= UPDATE_MIN_ROWS and n % SPLIT_ROWS == 0
            and x.dtype == torch.float32):
        return _SplitKLinear.apply(x, lin.weight, lin.bias, min(64, n // SPLIT_ROWS))
    return lin(x)


class MLP(nn.Module):
    """src/networks.py:22-61: layers of (features, activation); Glorot-normal weights
    N(0, 2/(in+out)), zero biases (networks.py:32-53). Unknown activations fall back to tanh.
    Batches of >= UPDATE_MIN_ROWS rows on the GPU (the PPO update's minibatches, the value pass over
    the rollout) take the split-K weight gradient and the native tanh-backward + bias-gradient pass
    (_TanhSplitKLinear)."""

    def __init__(self, in_dim: int, layer_specs: Sequence[Tuple[int, str]], generator: Optional[torch.Generator] = None):
        super().__init__()
        self.acts = [str(a).lower() for _, a in layer_specs]
        layers, d = [], in_dim
        for feat, _ in layer_specs:
            lin = nn.Linear(d, int(feat))
            with torch.no_grad():
                lin.weight.normal_(0.0, math.sqrt(2.0 / (d + int(feat))), generator=generator)
                lin.bias.zero_()
            layers.append(lin)
            d = int(feat)
        self.layers = nn.ModuleList(layers)

    def forward(self, x, out_tanh: bool = False):
        """out_tanh: a tanh after the last layer (GaussianPolicy's mean, networks.py:103)."""
        last = len(self.layers) - 1
        for l, (lin, a) in enumerate(zip(self.layers, self.acts)):
            act = ACTIVATIONS.get(a, torch.tanh)
            if act is torch.tanh:
                x = _tanh_linear(lin, x)
            elif l == last and out_tanh and a in ("linear", "none"):  # the mean's tanh on the last Dense
                return _tanh_linear(lin, x)
            else:
                x = act(_linear(lin, x))
        return torch.tanh(x) if out_tanh else x


class GaussianPolicy(nn.Module):
    """networks.py:82-112: mean = tanh(MLP(x)), learnable log_std (init log_std_init), clipped to [-20, 2]."""

    def __init__(self, obs_dim, act_dim, hidden_layer_specs, log_std_init=0.0, generator=None):
        super().__init__()
        self.mlp = MLP(obs_dim, list(hidden_layer_specs) + [(act_dim, "linear")], generator)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))

    def forward(self, x):
        return self.mlp(x, out_tanh=True), torch.clamp(self.log_std, -20.0, 2.0)


class ValueNet(nn.Module):
    """networks.py:114-131: MLP -> scalar."""

    def __init__(self, obs_dim, hidden_layer_specs, generator=None):
        super().__init__()
        self.mlp = MLP(obs_dim, list(hidden_layer_specs) + [(1, "linear")], generator)

    def forward(self, x):
        return self.mlp(x).squeeze(-1)


class APGPolicy(nn.Module):
    """networks.py:63-80: tanh-squashed MLP (hidden_dim x hidden_depth tanh layers)."""

    def __init__(self, obs_dim, act_dim, hidden_dim=64, hidden_depth=2, hidden_layer_specs=None, generator=None):
        super().__init__()
        specs = list(hidden_layer_specs) if hidden_layer_specs is not None else [(hidden_dim, "tanh")] * hidden_depth
        self.mlp = MLP(obs_dim, specs + [(act_dim, "linear")], generator)

    def forward(self, x):
        return self.mlp(x, out_tanh=True)


# ------------------------------------------------------------------------------------- statistics
class RunningMeanStd:
    """training_utils.py:20-56 (RMSState / update_rms / normalize_obs): mean 0, var 1, count 1e-4;
    parallel-variance merge with population batch variance; var floored at 1e-4."""

    def __init__(self, dim: int, device="cpu"):
        self.mean = torch.zeros(dim, device=device)
        self.var = torch.ones(dim, device=device)
        self.count = torch.tensor(1e-4, device=device)

    def update(self, x: torch.Tensor, dist=None):
        x = x.reshape(-1, x.shape[-1]).float()
        n = torch.tensor(float(x.shape[0]), device=x.device)
        s1, s2 = x.sum(0), (x * x).sum(0)
        if dist is not None:  # global batch statistics: sum, sum of squares, count over ranks
            buf = torch.cat([s1, s2, n.reshape(1)])
            dist.all_reduce(buf)
            s1, s2, n = buf[: x.shape[1]], buf[x.shape[1]: 2 * x.shape[1]], buf[-1]
            bmean = s1 / n
            bvar = torch.clamp(s2 / n - bmean * bmean, min=0.0)
        else:
            bmean = x.mean(0)
            bvar = x.var(0, unbiased=False)
        delta = bmean - self.mean
        tot = self.count + n
        new_mean = self.mean + delta * n / tot
        m2 = self.var * self.count + bvar * n + delta * delta * self.count * n / tot
        # in place: a captured rollout graph reads these tensors at replay time
        self.mean.copy_(new_mean)
        self.var.copy_(torch.clamp(m2 / tot, min=1e-4))
        self.count.copy_(tot)

    def normalize(self, x, clip: float = 10.0):
        """normalize_obs + the clip to [-10, 10] the trainers apply (train_ppo.py:134-135)."""
        return torch.clamp((x - self.mean) / torch.sqrt(self.var + 1e-8), -clip, clip)

    def state_dict(self):
        return {"mean": self.mean, "var": self.var, "count": self.count}

    def load_state_dict(self, d):
        self.mean.copy_(d["mean"])
        self.var.copy_(d["var"])
        self.count.copy_(d["count"])


# ---------------------------------------------------------------------------------- PPO formulas
LOG2PI = math.log(2.0 * math.pi)


def obs_normalize_native(x, mean, var, clip, out):
    """RunningMeanStd.normalize on device as one launch (mjl_obs_normalize)."""
    from ._lib import check, lib
    n, dim = x.numel() // x.shape[-1], x.shape[-1]
    check(lib().mjl_obs_normalize(x.data_ptr(), mean.data_ptr(), var.data_ptr(), n, dim, float(clip), out.data_ptr(),
                                  torch.cuda.current_stream(x.device).cuda_stream))
    return out


def policy_head_native(z, log_std, eps, act_out, logp_out):
    """tanh head + sampling + gaussian_logprob of one rollout step as one launch (mjl_policy_head)."""
    from ._lib import check, lib
    B, A = z.shape
    if not (z.is_contiguous() and eps.is_contiguous() and act_out.is_contiguous() and logp_out.is_contiguous()):
        raise ValueError("policy_head_native: contiguous [B, A] / [B] tensors expected")
    check(lib().mjl_policy_head(z.data_ptr(), log_std.detach().contiguous().data_ptr(), eps.data_ptr(), B, A,
                                act_out.data_ptr(), logp_out.data_ptr(), torch.cuda.current_stream(z.device).cuda_stream))


def _ceil16(x: int) -> int:
    return (x + 15) // 16 * 16


def policy_fused_dims(policy) -> Optional[List[int]]:
    """[obs_dim, hidden..., act_dim] when the policy fits mjl_policy_fwd (tanh hidden layers, a linear
    last layer, every size <= 256, at most 6 layers), else None (the rollout keeps the torch MLP)."""
    mlp = policy.mlp
    if len(mlp.layers) > 6 or any(a not in ("tanh",) for a in mlp.acts[:-1]) or mlp.acts[-1] != "linear":
        return None
    dims = [mlp.layers[0].in_features] + [lin.out_features for lin in mlp.layers]
    return dims if max(dims) <= 256 else None


def pack_policy_params(policy, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """mjl_policy_fwd's parameter layout: per layer WP[K/4][N][4] = W^T zero-padded to K, N multiples
    of 16 (WP[k // 4, n, k % 4] = weight[n, k]), then the padded bias [N]."""
    parts = []
    for lin in policy.mlp.layers:
        w = lin.weight.detach()
        n, k = w.shape
        kp, np_ = _ceil16(k), _ceil16(n)
        wt = torch.zeros((kp, np_), device=w.device, dtype=torch.float32)
        wt[:k, :n] = w.t()
        parts.append(wt.reshape(kp // 4, 4, np_).permute(0, 2, 1).reshape(-1))
        b = torch.zeros(np_, device=w.device, dtype=torch.float32)
        b[:n] = lin.bias.detach()
        parts.append(b)
    flat = torch.cat(parts)
    if out is None:
        return flat
    out.copy_(flat)
    return out


def policy_fwd_native(obs, mean, var, clip, params, dims, log_std, eps, act_out, logp_out):
    """The rollout step's normalisation + policy MLP + head + sampling + log-prob as one launch
    (mjl_policy_fwd); same results as obs_normalize_native -> policy.mlp -> policy_head_native up to
    the GEMMs' accumulation order."""
    import ctypes as C
    from ._lib import check, lib
    B = obs.shape[0]
    d = (C.c_int * len(dims))(*dims)
    check(lib().mjl_policy_fwd(obs.data_ptr(), mean.data_ptr(), var.data_ptr(), float(clip), params.data_ptr(),
                               len(dims) - 1, d, log_std.detach().contiguous().data_ptr(), eps.data_ptr(), B,
                               act_out.data_ptr(), logp_out.data_ptr(), torch.cuda.current_stream(obs.device).cuda_stream))


class _GaussianLogprob(torch.autograd.Function):
    """gaussian_logprob for the update's [65,536, 21] minibatch with a hand-written backward:
    d logp / d mean = (act - mean) e^(-2 s), d logp / d s_j = sum_i g_i (q_ij - 1) with
    q = (act - mean)^2 e^(-2 s). Autograd of the elementwise formula reduces the broadcast
    log_std terms over the 65,536 rows with torch's column reduction (66-169 us each, several per
    minibatch); here that is one native column sum (colsum_native)."""

    @staticmethod
    def forward(ctx, mean, log_std, action):
        d = action - mean
        iv = torch.exp(-2.0 * log_std)
        q = d * d * iv
        ctx.save_for_backward(d, iv, q)
        return (q.sum(-1) + (2.0 * log_std + LOG2PI).sum()) * -0.5

    @staticmethod
    def backward(ctx, g):
        d, iv, q = ctx.saved_tensors
        gm = g[:, None] * d * iv
        gs = colsum_native(torch.addcmul(-g[:, None], g[:, None], q).contiguous())
        return gm, gs, (-gm if ctx.needs_input_grad[2] else None)


def gaussian_logprob(mean, log_std, action, out=None):
    """train_ppo.py:121-126: diagonal Gaussian log-density summed over action dims."""
    if (out is None and mean.is_cuda and torch.is_grad_enabled() and mean.dim() == 2 and mean.dtype == torch.float32
            and mean.shape[0] >= UPDATE_MIN_ROWS and log_std.dim() == 1):
        return _GaussianLogprob.apply(mean, log_std, action)
    var = torch.exp(2.0 * log_std)
    s = torch.sum((action - mean) ** 2 / var + 2.0 * log_std + LOG2PI, dim=-1)
    return s.mul_(-0.5) if out is None else torch.mul(s, -0.5, out=out)


def gaussian_entropy(log_std, act_dim):
    """train_ppo.py:215: 0.5 * sum(1 + log 2pi + 2 log_std) / act_dim."""
    return 0.5 * torch.sum(1.0 + LOG2PI + 2.0 * log_std) / act_dim


def compute_gae(rewards, values, terminated, truncated, gamma: float, lam: float):
    """train_ppo.py:171-202: values [T+1, B]; only termination stops the bootstrap, either
    termination or truncation stops the advantage accumulation. Returns (adv, ret) [T, B].
    Device tensors go to the native reverse-scan kernel (mjl_gae, one launch instead of ~8 per
    time step); host tensors (CPU tests) use the same formula in torch."""
    if rewards.is_cuda:
        return _gae_native(rewards, values, terminated, truncated, gamma, lam)
    return compute_gae_torch(rewards, values, terminated, truncated, gamma, lam)


def _gae_native(rewards, values, terminated, truncated, gamma: float, lam: float):
    from ._lib import check, lib
    T, B = rewards.shape
    if values.shape != (T + 1, B) or terminated.shape != (T, B) or truncated.shape != (T, B):
        raise ValueError("compute_gae: rewards/term/trunc [T, B] and values [T+1, B] expected")
    f = lambda x: x.float().contiguous()  # noqa: E731
    r, v, te, tr = f(rewards), f(values), f(terminated), f(truncated)
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    check(lib().mjl_gae(r.data_ptr(), v.data_ptr(), te.data_ptr(), tr.data_ptr(), T, B, float(gamma), float(lam),
                        adv.data_ptr(), ret.data_ptr(), torch.cuda.current_stream(r.device).cuda_stream))
    return adv, ret


def compute_gae_torch(rewards, values, terminated, truncated, gamma: float, lam: float):
    """The elementwise restatement of train_ppo.py:171-202 (reference for mjl_gae)."""
    T = rewards.shape[0]
    adv = torch.empty_like(rewards)
    carry = torch.zeros_like(rewards[0])
    for t in range(T - 1, -1, -1):
        delta = rewards[t] + gamma * values[t + 1] * (1.0 - terminated[t]) - values[t]
        carry = delta + gamma * lam * (1.0 - torch.maximum(terminated[t], truncated[t])) * carry
        adv[t] = carry
    return adv, adv + values[:-1]


def normalize_adv(adv, dist=None):
    """(adv - mean) / (std + 1e-8) over the minibatch (train_ppo.py:209; jnp.std is the population
    std); over the global minibatch when data-parallel."""
    if dist is None:
        return (adv - adv.mean()) / (adv.std(unbiased=False) + 1e-8)
    mu, sd = _global_adv_stats(adv, dist)
    return (adv - mu) / (sd + 1e-8)


_LOSS_SCRATCH = {}


def _loss_scratch(dev, floats: int) -> torch.Tensor:
    key = (dev, floats, torch.cuda.current_stream(dev).cuda_stream)  # one per stream (two-stream update)
    t = _LOSS_SCRATCH.get(key)
    if t is None:
        t = _LOSS_SCRATCH[key] = torch.empty(max(floats, 1), dtype=torch.float32, device=dev)
    return t


class _PPOSurrogate(torch.autograd.Function):
    """ppo_policy_loss's clipped surrogate + entropy on the native kernels (mjl_ppo_surrogate: the
    advantage normalisation, log-prob, ratio, clip, min, mean and entropy with their gradients in
    three launches, where the torch ops were ~60 small kernels per minibatch)."""

    @staticmethod
    def forward(ctx, mean, log_std, act, old_logp, adv, clip_eps, ent_coef, adv_stats=None):
        from ._lib import check, lib
        n, A = mean.shape
        loss = torch.empty((), dtype=torch.float32, device=mean.device)
        gm, gs = torch.empty_like(mean), torch.empty_like(log_std)
        scr = _loss_scratch(mean.device, int(lib().mjl_ppo_loss_scratch(n, A)))
        check(lib().mjl_ppo_surrogate(mean.data_ptr(), log_std.data_ptr(), act.data_ptr(), old_logp.data_ptr(),
                                      adv.data_ptr(), None if adv_stats is None else adv_stats.data_ptr(), n, A, float(clip_eps), float(ent_coef), scr.data_ptr(),
                                      loss.data_ptr(), gm.data_ptr(), gs.data_ptr(),
                                      torch.cuda.current_stream(mean.device).cuda_stream))
        ctx.save_for_backward(gm, gs)
        return loss

    @staticmethod
    def backward(ctx, g):
        gm, gs = ctx.saved_tensors
        return gm * g, gs * g, None, None, None, None, None, None


class _MSE(torch.autograd.Function):
    """value_loss's mean squared error on the native kernels (mjl_mse, two launches)."""

    @staticmethod
    def forward(ctx, v, r):
        from ._lib import check, lib
        n = v.numel()
        loss = torch.empty((), dtype=torch.float32, device=v.device)
        gv = torch.empty_like(v)
        scr = _loss_scratch(v.device, n // 256 + 1)
        check(lib().mjl_mse(v.data_ptr(), r.data_ptr(), n, scr.data_ptr(), loss.data_ptr(), gv.data_ptr(),
                            torch.cuda.current_stream(v.device).cuda_stream))
        ctx.save_for_backward(gv)
        return loss

    @staticmethod
    def backward(ctx, g):
        gv, = ctx.saved_tensors
        return gv * g, None


NATIVE_LOSSES = True  # tests switch the torch restatement back on


def _native_loss_ok(x: torch.Tensor) -> bool:
    return NATIVE_LOSSES and x.is_cuda and torch.is_grad_enabled() and x.shape[0] >= UPDATE_MIN_ROWS


def _global_adv_stats(adv, dist) -> torch.Tensor:
    """(mean, population std) of the advantages over every rank's share of the minibatch."""
    buf = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(adv.numel()), device=adv.device)])
    dist.all_reduce(buf)
    mu = buf[0] / buf[2]
    return torch.stack([mu, torch.sqrt(torch.clamp(buf[1] / buf[2] - mu * mu, min=0.0))]).contiguous()


def ppo_policy_loss(policy, obs, acts, old_logp, adv, clip_eps, ent_coef, dist=None, adv_stats=None):
    """train_ppo.py:204-216. Data-parallel, the advantages are normalised by the global minibatch's
    (mean, population std): `adv_stats` when given (a device [2]), else all-reduced here."""
    mean, log_std = policy(obs)
    if _native_loss_ok(mean) and mean.dim() == 2 and log_std.dim() == 1 and mean.shape[1] <= 32:
        f = lambda x: x.float().contiguous()  # noqa: E731
        st = adv_stats if adv_stats is not None else (None if dist is None else _global_adv_stats(f(adv), dist))
        return _PPOSurrogate.apply(f(mean), log_std.contiguous(), f(acts), f(old_logp), f(adv), float(clip_eps),
                                   float(ent_coef), st)
    ratio = torch.exp(gaussian_logprob(mean, log_std, acts) - old_logp)
    if adv_stats is not None:
        adv_n = (adv - adv_stats[0]) / (adv_stats[1] + 1e-8)
    else:
        adv_n = normalize_adv(adv, dist)
    surr = torch.minimum(ratio * adv_n, torch.clamp(ratio, 1.0 - clip_eps, 1.0 + clip_eps) * adv_n)
    return -surr.mean() - ent_coef * gaussian_entropy(log_std, acts.shape[-1])


def value_loss(value, obs, returns):
    """train_ppo.py:218-220 (vf_coef is unused by the reference)."""
    v = value(obs)
    if _native_loss_ok(v) and v.shape == returns.shape:
        return _MSE.apply(v.contiguous(), returns.float().contiguous())
    return torch.mean((v - returns) ** 2)


def _gather_minibatch(idx, *arrays, row: Optional[torch.Tensor] = None, twice_first: bool = False):
    """arrays[k][idx] for every k, as one native launch (mjl_gather_rows) on the GPU. With `row` (a
    device int32), idx is an [n_minibatches, rows] table and the launch gathers row *row of it, read
    when the launch runs (a captured minibatch step; mjl_gather_rows_indexed). twice_first (with
    row): the first array's rows are written twice, as one [2, rows, ...] block (the twin update's
    observations, one copy per net)."""
    if row is not None:
        import ctypes
        from ._lib import check, lib
        n = idx.shape[1]
        outs = [torch.empty((n,) + tuple(a.shape[1:]), dtype=a.dtype, device=a.device) for a in arrays]
        dsts, srcs = list(outs), list(arrays)
        if twice_first:
            a0 = arrays[0]
            outs[0] = torch.empty((2, n) + tuple(a0.shape[1:]), dtype=a0.dtype, device=a0.device)
            dsts = [outs[0][0], outs[0][1]] + outs[1:]
            srcs = [a0] + list(arrays)
        k = len(srcs)
        check(lib().mjl_gather_rows_indexed(idx.data_ptr(), ctypes.c_void_p(row.data_ptr()), n,
                                            min(a.shape[0] for a in arrays), k,
                                            (ctypes.c_void_p * k)(*[a.data_ptr() for a in srcs]),
                                            (ctypes.c_void_p * k)(*[o.data_ptr() for o in dsts]),
                                            (ctypes.c_int * k)(*[max(1, a[0].numel()) for a in srcs]),
                                            torch.cuda.current_stream(idx.device).cuda_stream))
        return tuple(outs)
    if not (idx.is_cuda and idx.dtype == torch.int64 and len(arrays) <= 8
            and all(a.is_cuda and a.dtype == torch.float32 and a.is_contiguous() for a in arrays)):
        return tuple(a[idx] for a in arrays)
    import ctypes
    from ._lib import check, lib
    idx = idx.contiguous()
    n = idx.numel()
    outs = tuple(torch.empty((n,) + tuple(a.shape[1:]), dtype=a.dtype, device=a.device) for a in arrays)
    k = len(arrays)
    src = (ctypes.c_void_p * k)(*[a.data_ptr() for a in arrays])
    dst = (ctypes.c_void_p * k)(*[o.data_ptr() for o in outs])
    cols = (ctypes.c_int * k)(*[max(1, a[0].numel()) for a in arrays])
    nsrc = min(a.shape[0] for a in arrays)
    check(lib().mjl_gather_rows(idx.data_ptr(), n, nsrc, k, src, dst, cols,
                                torch.cuda.current_stream(idx.device).cuda_stream))
    return outs


def make_index_batches(total: int, minibatch: int, epochs: int, generator: torch.Generator, device):
    """train_ppo.py:222-231: a fresh permutation per epoch, the last partial minibatch dropped."""
    per = total // minibatch
    out = [torch.randperm(total, generator=generator, device=generator.device)[: per * minibatch].view(per, minibatch)
           for _ in range(epochs)]
    return torch.cat(out, 0).to(device)


def _torch_adam_groups(n: int, lr: float, betas, eps: float) -> list:
    """torch.optim.Adam's param_groups entry for n parameters with these hyper-parameters (taken from
    a throwaway torch Adam, so the keys are exactly this torch version's)."""
    dummy = torch.optim.Adam([torch.zeros(1, requires_grad=True) for _ in range(n)], lr=lr, betas=tuple(betas), eps=eps)
    return dummy.state_dict()["param_groups"]


def adam_state_to_torch(step: float, m: list, v: list, lr: float, betas, eps: float) -> dict:
    """torch.optim.Adam.state_dict() layout: state[i] = {step, exp_avg, exp_avg_sq}, param_groups."""
    state = {} if step <= 0 else {
        i: {"step": torch.tensor(float(step)), "exp_avg": a.detach().clone(), "exp_avg_sq": b.detach().clone()}
        for i, (a, b) in enumerate(zip(m, v))}
    return {"state": state, "param_groups": _torch_adam_groups(len(m), lr, betas, eps)}


def adam_state_from_torch(d: dict, shapes: list):
    """(step, m list or None, v list or None, lr, betas, eps) from a torch.optim.Adam state dict (or a
    round-2 NativeAdam one: t / m / v); raises ValueError when it does not fit `shapes`."""
    if "t" in d:  # round-2 NativeAdam layout
        m, v, step, lr, betas, eps = list(d["m"]), list(d["v"]), float(d["t"]), d["lr"], d["betas"], d["eps"]
    else:
        if "state" not in d or "param_groups" not in d or len(d["param_groups"]) != 1:
            raise ValueError("Adam state dict: expected torch.optim.Adam's layout with one parameter group")
        g = d["param_groups"][0]
        if len(g["params"]) != len(shapes):
            raise ValueError(f"Adam state dict: {len(g['params'])} parameters, optimiser has {len(shapes)}")
        lr, betas, eps = g["lr"], g["betas"], g["eps"]
        st = d["state"]
        if not st:
            return 0.0, None, None, float(lr), (float(betas[0]), float(betas[1])), float(eps)
        ids = list(g["params"])
        if any(i not in st for i in ids):
            raise ValueError("Adam state dict: state missing for some parameters")
        m = [st[i]["exp_avg"] for i in ids]
        v = [st[i]["exp_avg_sq"] for i in ids]
        step = float(st[ids[0]]["step"])
    if len(m) != len(shapes) or len(v) != len(shapes):
        raise ValueError(f"Adam state dict: {len(m)} moment tensors, optimiser has {len(shapes)} parameters")
    for a, b, sh in zip(m, v, shapes):
        if tuple(a.shape) != tuple(sh) or tuple(b.shape) != tuple(sh):
            raise ValueError(f"Adam state dict: moment shape {tuple(a.shape)} does not match parameter {tuple(sh)}")
    return step, m, v, float(lr), (float(betas[0]), float(betas[1])), float(eps)


class NativeAdam:
    """torch.optim.Adam (betas, eps; no weight decay) for CUDA float32 parameters as one native
    launch per step (mjl_adam_multi: the fused update of every tensor), where torch's fused Adam took
    ≈42 µs for the 151K-parameter policy. The step count lives on the device and is advanced on the
    device after the step, so a hipGraph that captured step() takes each replay's own bias corrections
    (a host int baked into the capture made replays drift from eager). adam_steps() takes
    several optimisers' steps in one launch. state_dict / load_state_dict use torch.optim.Adam's
    layout (checkpoints interchange)."""

    def __init__(self, params, lr: float, betas=(0.9, 0.999), eps: float = 1e-8):
        self.params = [p for p in params]
        if len(self.params) > 16 or any((not p.is_cuda) or p.dtype != torch.float32 or not p.is_contiguous()
                                        for p in self.params):
            raise ValueError("NativeAdam: at most 16 contiguous float32 CUDA tensors")
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.step_t = torch.zeros(1, dtype=torch.float32, device=self.params[0].device)

    @property
    def t(self) -> int:
        return int(self.step_t.item())

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    @torch.no_grad()
    def step(self, grads: Optional[List[torch.Tensor]] = None):
        """One Adam step with `grads` (default: the parameters' .grad)."""
        adam_steps([(self, grads)])

    def state_dict(self):
        return adam_state_to_torch(float(self.step_t.item()), self.m, self.v, self.lr, self.betas, self.eps)

    def load_state_dict(self, d):
        step, m, v, self.lr, self.betas, self.eps = adam_state_from_torch(d, [p.shape for p in self.params])
        self.step_t.fill_(step)
        for dst, src in zip(self.m + self.v, (m + v) if m is not None else [torch.zeros_like(x) for x in self.m + self.v]):
            dst.copy_(src)


@torch.no_grad()
def adam_steps(pairs, gscale: float = 1.0, ctr: Optional[torch.Tensor] = None, advanced: bool = False):
    """One Adam step of each (NativeAdam, grads or None for the parameters' .grad) in ONE launch
    (mjl_adam_multi, up to 2 optimisers with the same betas / eps; plus a one-thread launch advancing
    the step counters), gradients scaled by gscale; `ctr` (device int32, optional) is advanced with
    the step counters. advanced: the counters (and ctr) were already advanced in this minibatch step
    (the twin update's loss launch does it in the captured graphs): no counter launch."""
    import ctypes
    from ._lib import check, lib
    o0 = pairs[0][0]
    if len(pairs) > 2 or any(o.betas != o0.betas or o.eps != o0.eps for o, _ in pairs):
        raise ValueError("adam_steps: at most 2 optimisers with equal betas and eps")
    ps, gs, ms, vs, ns, grp = [], [], [], [], [], []
    for gi, (opt, grads) in enumerate(pairs):
        src = [p.grad for p in opt.params] if grads is None else list(grads)
        if len(src) != len(opt.params):
            raise ValueError("adam_steps: one gradient per parameter")
        for p, g, m, v in zip(opt.params, src, opt.m, opt.v):
            ps.append(p); gs.append(None if g is None else g.contiguous()); ms.append(m); vs.append(v)
            ns.append(p.numel()); grp.append(gi)
    k = len(ps)
    vp = ctypes.c_void_p * k
    dev = o0.params[0].device
    check(lib().mjl_adam_multi(k, vp(*[p.data_ptr() for p in ps]), vp(*[None if g is None else g.data_ptr() for g in gs]),
                               vp(*[x.data_ptr() for x in ms]), vp(*[x.data_ptr() for x in vs]),
                               (ctypes.c_longlong * k)(*ns), (ctypes.c_int * k)(*grp), len(pairs),
                               (ctypes.c_float * len(pairs))(*[o.lr for o, _ in pairs]), o0.betas[0], o0.betas[1],
                               o0.eps, float(gscale), (ctypes.c_void_p * len(pairs))(*[o.step_t.data_ptr() for o, _ in pairs]),
                               None if ctr is None else ctypes.c_void_p(ctr.data_ptr()), int(advanced),
                               torch.cuda.current_stream(dev).cuda_stream))
    for opt, _ in pairs:
        opt._keep = gs  # the launch reads the gradients asynchronously


def _adam(params, lr):
    """optax.adam defaults (b1 .9, b2 .999, eps 1e-8) = torch.optim.Adam defaults; on the GPU one
    native launch per step (NativeAdam), on the CPU torch's."""
    params = list(params)
    if params and all(p.is_cuda for p in params) and len(params) <= 16:
        return NativeAdam(params, lr=lr, betas=(0.9, 0.999), eps=1e-8)
    return torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), eps=1e-8)


def _flat_grads(params: List[torch.Tensor]) -> torch.Tensor:
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params])


def _set_grads(params: List[torch.Tensor], flat: torch.Tensor):
    o = 0
    for p in params:
        n = p.numel()
        p.grad = flat[o:o + n].view_as(p).clone()
        o += n


TWO_STREAM_UPDATE = os.environ.get("MJL_TWO_STREAM", "1") != "0"  # value net on a side stream in ppo_update
def graph_capture(graph, pool=None):
    """torch.cuda.graph with capture_error_mode="thread_local": RCCL's watchdog thread queries its
    collectives' events while this thread captures, and under the default "global" mode such a query
    invalidates the capture (measured: an eager bucketed update followed by the rollout capture failed
    with hipErrorStreamCaptureInvalidated). Only this thread's own calls are checked."""
    return torch.cuda.graph(graph, pool=pool, capture_error_mode="thread_local")


# data-parallel twin update: the gradient all-reduce in two buckets, the top layers' (and log_std's) in
# flight while the lower layers' backward runs (PPOUpdater._allreduce_buckets). MJL_DP_BUCKETS: "auto"
# (default) = with more than one rank (one rank has no link time to hide, and the second collective
# costs 0.85 ms per C5 update there), "1" always, "0" never
DP_BUCKETS = os.environ.get("MJL_DP_BUCKETS", "auto")
# data-parallel update over RCCL: the minibatch step's collective(s) captured in its graph, one replay
# per minibatch step (MJL_DP_CAPTURE=0: eager collectives between the graphs). One-rank RCCL, C5's
# per-rank update (128 steps of 8,192 rows): 33.1 ms eager -> 30.0 ms captured (profiles/r5/)
DP_CAPTURE = os.environ.get("MJL_DP_CAPTURE", "1") != "0"
# the twin update's minibatch steps captured as ONE graph per update (single process, and
# data-parallel with the collectives captured): one replay per update instead of one per minibatch
# step — a graph boundary idled the GPU ~8.7 us per replay (rocprofv3, C5's 8,192-row steps);
# MJL_WHOLE_UPDATE_GRAPH=0: one graph per minibatch step, replayed per step
WHOLE_UPDATE_GRAPH = os.environ.get("MJL_WHOLE_UPDATE_GRAPH", "1") != "0"
_SIDE_STREAMS = {}


def _side_stream(dev):
    s = _SIDE_STREAMS.get(dev)
    if s is None:
        s = _SIDE_STREAMS[dev] = torch.cuda.Stream(dev)
    return s


def minibatch_adv_stats(adv, index_batches, dist) -> torch.Tensor:
    """(mean, population std) of the advantages of every minibatch over all ranks' shares, as
    [n_minibatches, 2], with ONE all-reduce per update instead of one per minibatch (the reference
    normalises per minibatch, train_ppo.py:209; data-parallel, the minibatch is the union of the
    ranks' shares)."""
    a = adv.reshape(-1)[index_batches]  # [nmb, mb]
    loc = torch.stack([a.sum(1), (a * a).sum(1), torch.full((a.shape[0],), float(a.shape[1]), device=a.device,
                                                              dtype=a.dtype)], 1)
    dist.all_reduce(loc)
    mu = loc[:, 0] / loc[:, 2]
    return torch.stack([mu, torch.sqrt(torch.clamp(loc[:, 1] / loc[:, 2] - mu * mu, min=0.0))], 1).contiguous()


class _HostTimer:
    """A (start, end) pair like two CUDA events, for the all-reduce timing on CPU (gloo)."""

    def __init__(self):
        self.t = [0.0, 0.0]

    def record(self, i):
        self.t[i] = time.perf_counter()

    def ms(self) -> float:
        return (self.t[1] - self.t[0]) * 1e3


def event_ms(ev) -> float:
    """Milliseconds of one all-reduce timing pair collected by PPOUpdater (CUDA events or host)."""
    if isinstance(ev, _HostTimer):
        return ev.ms()
    return ev[0].elapsed_time(ev[1])


class PPOUpdater:
    """run_ppo_updates (train_ppo.py:233-252): per minibatch a policy Adam step and a value Adam step
    over 4 epochs of minibatches. The reference compiles the whole loop as one lax.scan; here:

    * single process on the GPU: the minibatch step (gather, both nets' forward + backward through the
      native losses, both Adam steps; the value net on a second stream) is captured once as a
      hipGraph and replayed per minibatch, the minibatch's indices copied into the graph's static
      index buffer before each replay;
    * data-parallel: the advantage statistics of every minibatch in one all-reduce up front, then per
      minibatch graph A (gather, forward, backward, both nets' gradients flattened into one buffer),
      the RCCL all-reduce of that buffer (eager: the one exchange of the update), and
      graph B (divide by the world size, both Adam steps);
    * eager (CPU, torch optimisers, or use_graph=False): the same bodies without capture.

    The graphs need NativeAdam (its step count is device state). The first run is eager (library
    handles, allocator pools, GEMM choices); the second captures. Replays equal the eager bodies bit
    for bit (tests/test_ppo_graph.py).

    With NativeAdam on the GPU and the reference's network pair (same tanh hidden layers), the two
    nets run as one batched pass per layer (twin.TwinNets, MJL_TWIN_UPDATE=0 disables): their
    parameters become views of stacked storage, the gradients land in one flat buffer that is also
    the data-parallel all-reduce buffer, and no second stream is needed."""

    def __init__(self, policy, value, opt_p, opt_v, cfg, dist=None, world=1, use_graph=True):
        self.policy, self.value, self.opt_p, self.opt_v, self.cfg = policy, value, opt_p, opt_v, cfg
        self.dist, self.world = dist, world
        self.pp, self.vp = list(policy.parameters()), list(value.parameters())
        dev = self.pp[0].device
        self.cuda = dev.type == "cuda"
        self.graph_ok = (bool(use_graph) and self.cuda and isinstance(opt_p, NativeAdam)
                         and isinstance(opt_v, NativeAdam))
        # the value net's forward / backward (and, single-process, its Adam step) on a second stream beside
        # the policy's: independent within a minibatch, and one net's GEMMs leave CUs idle — at the
        # 8,192-row per-rank minibatch of C5 on 8 GPUs a 256-wide layer is 64 row tiles for 256 CUs
        self.side = _side_stream(dev) if (self.cuda and TWO_STREAM_UPDATE) else None
        self.flat = None
        if dist is not None:
            n = sum(p.numel() for p in self.pp + self.vp)
            self.flat = torch.zeros(n, device=dev)
            views, o = [], 0
            for p in self.pp + self.vp:
                views.append(self.flat[o:o + p.numel()].view_as(p))
                o += p.numel()
            self.views_p, self.views_v = views[:len(self.pp)], views[len(self.pp):]
        self.twin = None
        if self.cuda and isinstance(opt_p, NativeAdam) and isinstance(opt_v, NativeAdam):
            from .twin import twin_for
            self.twin = twin_for(policy, value)
        self._tw = False  # this run takes the twin path (minibatch shape permitting)
        self.runs = 0
        self._src = self._idx = self._st = None
        self._ga = self._gb = self._gstep = None
        # data-parallel observability (bench line): gradient buckets per minibatch step (0 single
        # process), whether the last run replayed the step graph with its collectives captured, and why
        # the capture was given up (None: not attempted or succeeded)
        self.dp_buckets = 0
        self.captured_last_run = False
        self.capture_fallback_reason: Optional[str] = None
        self._gstep_n = 0

    def _twin_ok(self, rows: int, act_dim: int) -> bool:
        return (self.twin is not None and rows >= UPDATE_MIN_ROWS and rows % SPLIT_ROWS == 0 and rows % 128 == 0
                and act_dim == self.twin.A and self.twin.owns_storage())

    def _grad_buffer(self):
        """The data-parallel all-reduce buffer of this run: the twin's flat gradients or self.flat."""
        return self.twin.grad if self._tw else self.flat

    def allreduce_numel(self) -> int:
        """Floats per all-reduce (the twin layout pads the value's output layer to the policy's width)."""
        if self.twin is not None:
            return int(self.twin.grad.numel())
        return sum(p.numel() for p in self.pp + self.vp)

    # ------------------------------------------------------------------ bodies
    def _body_a(self, idx, src, st, row: Optional[torch.Tensor] = None):
        """Gather the minibatch; forward + backward of both nets (and, single-process, both Adam
        steps). Data-parallel: leaves both nets' gradients in the all-reduce buffer. With `row` (twin
        graphs), idx and st are the whole update's [n_minibatches, ...] tables, read at row *row, which
        the Adam launch advances: the replays need no per-minibatch host copies."""
        cfg, opt_p, opt_v = self.cfg, self.opt_p, self.opt_v
        o, a, ol, r, ad, h1 = self._gather(idx, src, row)
        dp = self.dist is not None
        if self._tw:
            tw = self.twin
            # captured (row given): the backward's final reduction launch advances the step counters
            # and the row, Adam takes them as they are
            ctrs = (opt_p.step_t, opt_v.step_t, row) if row is not None else None
            tw.forward_backward(o, a, ol, r, ad, st, cfg.clip_eps, cfg.ent_coef, min(64, o.shape[-2] // SPLIT_ROWS),
                                stats_row=row, counters=ctrs, h1=h1)
            if not dp:  # both nets' Adam steps in one launch
                adam_steps([(opt_p, tw.grads_p), (opt_v, tw.grads_v)], advanced=ctrs is not None)
            return
        if self.side is not None:
            cur = torch.cuda.current_stream(o.device)
            self.side.wait_stream(cur)
            # o and r (allocated on cur, read on side) are released at the next gather, after the
            # cur.wait_stream(side) below, so their blocks are not reused early (no record_stream)
            with torch.cuda.stream(self.side):
                opt_v.zero_grad(set_to_none=True)
                value_loss(self.value, o, r).backward()
                if not dp:
                    opt_v.step()
            opt_p.zero_grad(set_to_none=True)
            ppo_policy_loss(self.policy, o, a, ol, ad, cfg.clip_eps, cfg.ent_coef, adv_stats=st).backward()
            if not dp:
                opt_p.step()
            cur.wait_stream(self.side)
        else:
            opt_p.zero_grad(set_to_none=True)
            opt_v.zero_grad(set_to_none=True)
            ppo_policy_loss(self.policy, o, a, ol, ad, cfg.clip_eps, cfg.ent_coef, adv_stats=st).backward()
            value_loss(self.value, o, r).backward()
        if dp:
            torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in self.pp + self.vp],
                      out=self.flat)
        elif self.side is None:
            opt_p.step()
            opt_v.step()

    def _gather(self, idx, src, row=None):
        """The minibatch's rows (+ h1, the first hidden layer of both nets, when the twin path's fused
        gather + input layer launch applies — eager and captured alike, so replays equal eager runs)."""
        if self._tw and self.twin.fused_input_ok(src):
            return self.twin.gather_input(idx, src, row)
        return _gather_minibatch(idx, *src, row=row, twice_first=self._tw and row is not None) + (None,)

    def _bucketed(self) -> bool:
        """Data-parallel twin runs all-reduce the gradient in two buckets, the first overlapping the
        lower layers' backward (DP_BUCKETS; needs a hidden-hidden layer below the top two)."""
        if DP_BUCKETS == "0" or self.dist is None or not self._tw or self.twin.nl <= 2:
            return False
        return DP_BUCKETS == "1" or self.world > 1

    def _body_a_phases(self, idx, src, st, row: Optional[torch.Tensor] = None):
        """_body_a of the data-parallel twin path in two phases (a generator): the gather, forward, loss
        head and the top two layers' backward, after which bucket 1 of the gradient is final (yield);
        then the layers below, finishing bucket 2 (and advancing the captured counters)."""
        cfg, opt_p, opt_v = self.cfg, self.opt_p, self.opt_v
        o, a, ol, r, ad, h1 = self._gather(idx, src, row)
        ctrs = (opt_p.step_t, opt_v.step_t, row) if row is not None else None
        gen = self.twin.forward_backward_phases(o, a, ol, r, ad, st, cfg.clip_eps, cfg.ent_coef,
                                                min(64, o.shape[-2] // SPLIT_ROWS), stats_row=row, counters=ctrs,
                                                h1=h1)
        next(gen)
        yield
        next(gen)
        self._keep_phase = (o, a, ol, r, ad, h1, gen)

    def _allreduce_buckets(self, run_phase2, events):
        """Bucket 1's all-reduce in flight while run_phase2() enqueues the lower layers' backward, then
        bucket 2's; both joined into the current stream. `events` gets one pair per minibatch around the
        exposed part: from the end of phase 2's compute to the end of both collectives."""
        b1, b2 = self.twin.buckets()
        w1 = self.dist.all_reduce(b1, async_op=True)
        run_phase2()
        ev = None
        if events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        w2 = self.dist.all_reduce(b2, async_op=True)
        for w in (w1, w2):
            if w is not None and hasattr(w, "wait"):
                w.wait()
        if ev is not None:
            ev[1].record()
            events.append(ev)

    def _body_b(self, row: Optional[torch.Tensor] = None):
        """Data-parallel: the all-reduced gradient sum -> mean, then both Adam steps (advancing the
        twin graphs' minibatch row)."""
        if isinstance(self.opt_p, NativeAdam) and isinstance(self.opt_v, NativeAdam):
            # the all-reduced sum -> mean inside the one Adam launch of both nets
            gp, gv = (self.twin.grads_p, self.twin.grads_v) if self._tw else (self.views_p, self.views_v)
            if row is not None and self._tw:  # (the twin backward advanced the counters and the row)
                adam_steps([(self.opt_p, gp), (self.opt_v, gv)], gscale=1.0 / self.world, advanced=True)
            else:
                adam_steps([(self.opt_p, gp), (self.opt_v, gv)], gscale=1.0 / self.world, ctr=row)
            return
        self.flat.div_(self.world)
        if isinstance(self.opt_p, NativeAdam):
            self.opt_p.step(grads=self.views_p)
            self.opt_v.step(grads=self.views_v)
        else:
            _set_grads(self.pp + self.vp, self.flat)
            self.opt_p.step()
            self.opt_v.step()

    def _allreduce(self, events):
        ev = None
        if events is not None:
            if self.cuda:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            else:
                ev = _HostTimer()
                ev.record(0)
        self.dist.all_reduce(self._grad_buffer())
        if ev is not None:
            if self.cuda:
                ev[1].record()
            else:
                ev.record(1)
            events.append(ev)

    # ------------------------------------------------------------------ driver
    def run(self, obs, acts, logp, ret, adv, index_batches, events: Optional[list] = None):
        """One update over `index_batches` [n_minibatches, rows] of the flattened rollout arrays.
        `events` (a list) collects one timing pair per all-reduce (event_ms). The update's GEMMs run
        under the tuned GEMM table (mjx_amd/tunable.py: on only inside this call)."""
        from .tunable import tuned_gemms
        with tuned_gemms(self.pp[0].device if self.cuda else None):
            self._run(obs, acts, logp, ret, adv, index_batches, events)

    def _run(self, obs, acts, logp, ret, adv, index_batches, events):
        src = (obs, acts, logp, ret, adv)
        stats = minibatch_adv_stats(adv, index_batches, self.dist) if self.dist is not None else None
        tw = self._twin_ok(int(index_batches.shape[1]), int(acts.shape[1]) if acts.dim() == 2 else -1)
        if tw != self._tw:
            self._ga = self._gb = self._gstep = None  # the captured bodies belong to the other path
        self._tw = tw
        self.dp_buckets = (2 if self._bucketed() else 1) if self.dist is not None else 0
        self.captured_last_run = False
        use_graph = self.graph_ok and self.runs > 0
        self.runs += 1
        if not use_graph:
            for i in range(index_batches.shape[0]):
                if self._bucketed():
                    gen = self._body_a_phases(index_batches[i], src, None if stats is None else stats[i])
                    next(gen)
                    self._allreduce_buckets(lambda: next(gen, None), events)
                    self._body_b()
                    continue
                self._body_a(index_batches[i], src, None if stats is None else stats[i])
                if self.dist is not None:
                    self._allreduce(events)
                    self._body_b()
            return
        mb = index_batches.shape[1]
        if self._src is None or any(a.shape != b.shape for a, b in zip(self._src, src)) or self._idx.shape[0] != mb:
            self._src = tuple(torch.empty_like(x, memory_format=torch.contiguous_format) for x in src)
            self._idx = torch.empty(mb, dtype=index_batches.dtype, device=index_batches.device)
            self._st = torch.zeros(2, device=adv.device)
            self._ga = self._gb = self._gstep = None
        for dst, x in zip(self._src, src):  # the graphs read the static copies
            dst.copy_(x)
        if self._tw:  # the twin graphs read the update's index / statistics tables at a device row
            self._run_twin_graphs(index_batches, stats, events)
            return
        for i in range(index_batches.shape[0]):
            self._idx.copy_(index_batches[i])
            if stats is not None:
                self._st.copy_(stats[i])
            if self._ga is None:
                self._ga = torch.cuda.CUDAGraph()
                with graph_capture(self._ga):
                    self._body_a(self._idx, self._src, None if stats is None else self._st)
                if self.dist is not None:
                    self._gb = torch.cuda.CUDAGraph()
                    with graph_capture(self._gb):
                        self._body_b()
            self._ga.replay()
            if self.dist is not None:
                self._allreduce(events)
                self._gb.replay()


    def _run_twin_graphs(self, index_batches, stats, events):
        """The twin path's replays: the whole update's index table (and, data-parallel, its advantage
        statistics) copied once, a device row counter that the captured Adam launch advances, so a
        minibatch step is graph A (+ the all-reduce + graph B) with no host copy in between."""
        nmb = index_batches.shape[0]
        if getattr(self, "_idx_all", None) is None or self._idx_all.shape != index_batches.shape:
            self._idx_all = torch.empty_like(index_batches, memory_format=torch.contiguous_format)
            self._st_all = torch.zeros((nmb, 2), device=index_batches.device)
            self._row = torch.zeros(1, dtype=torch.int32, device=index_batches.device)
            self._ga = self._gb = self._gstep = None
        self._idx_all.copy_(index_batches)
        if stats is not None:
            self._st_all.copy_(stats)
        self._row.zero_()
        st = self._st_all if stats is not None else None
        bucketed = self._bucketed()
        whole = self.dist is None or self._capture_collectives()
        if whole and self.capture_fallback_reason is None:
            k = nmb if WHOLE_UPDATE_GRAPH else 1  # minibatch steps per captured graph
            if nmb % k:
                k = 1
            if self._gstep is None or self._gstep_n != k:
                self._capture_steps(st, bucketed, k)
            if self.capture_fallback_reason is None:
                for _ in range(nmb // k):  # replay errors propagate (no eager re-run of applied steps)
                    self._gstep.replay()
                if self.dist is not None:
                    self.collectives_last_run = nmb * self.dp_buckets
                    self.captured_last_run = True
                return
        for _ in range(nmb):
            if self._ga is None:
                self._ga = torch.cuda.CUDAGraph()
                if bucketed:  # graph A in two parts around bucket 1's all-reduce, one memory pool
                    pool = torch.cuda.graph_pool_handle()
                    with graph_capture(self._ga, pool=pool):
                        gen = self._body_a_phases(self._idx_all, self._src, st, row=self._row)
                        next(gen)
                    self._ga2 = torch.cuda.CUDAGraph()
                    with graph_capture(self._ga2, pool=pool):
                        next(gen, None)
                    self._gen_keep = gen  # phase 1's tensors, read by phase 2's replays
                else:
                    with graph_capture(self._ga):
                        self._body_a(self._idx_all, self._src, st, row=self._row)
                if self.dist is not None:
                    self._gb = torch.cuda.CUDAGraph()
                    with graph_capture(self._gb):
                        self._body_b(row=self._row)
            self._ga.replay()
            if bucketed:
                self._allreduce_buckets(self._ga2.replay, events)
                self._gb.replay()
            elif self.dist is not None:
                self._allreduce(events)
                self._gb.replay()


    def _capture_collectives(self) -> bool:
        """The data-parallel minibatch step as ONE graph with its RCCL all-reduce(s) captured inside
        (DP_CAPTURE, RCCL process groups only): no host round trip and no eager cross-stream
        synchronisation between the backward, the collective and the Adam step."""
        if not (DP_CAPTURE and self.dist is not None and self._tw):
            return False
        try:  # RCCL, or bench's one-rank identity stand-in (the same captured structure, no link)
            return self.dist.get_backend() in ("nccl", "identity")
        except Exception:  # a stand-in without backends
            return False

    def _step_body(self, st, bucketed):
        """One minibatch step as captured: single process, graph A's body (both Adam steps inside);
        data-parallel, the body with its collective(s) and the Adam launch."""
        if self.dist is None:
            self._body_a(self._idx_all, self._src, st, row=self._row)
            return
        if bucketed:
            gen = self._body_a_phases(self._idx_all, self._src, st, row=self._row)
            next(gen)
            b1, b2 = self.twin.buckets()
            w1 = self.dist.all_reduce(b1, async_op=True)
            next(gen, None)
            w2 = self.dist.all_reduce(b2, async_op=True)
            for w in (w1, w2):
                if w is not None:
                    w.wait()
            self._gen_keep = gen
        else:
            self._body_a(self._idx_all, self._src, st, row=self._row)
            self.dist.all_reduce(self._grad_buffer())
        self._body_b(row=self._row)

    def _capture_steps(self, st, bucketed, k):
        """Capture k consecutive minibatch steps as ONE graph (WHOLE_UPDATE_GRAPH: k = the update's
        minibatch count, so an update is one replay; the steps read the device row counter, so they
        differ only in the row they gather). Data-parallel, only the capture is guarded: a
        capture refused on any rank (this RCCL build, a collective the capture does not take) sends
        EVERY rank to the eager collectives — the ranks agree through one eager all-reduce of a
        failure flag, so no rank replays captured collectives that another rank issues eagerly.
        Nothing captured has run: the replays come only after the agreement."""
        self._gstep = None
        g = torch.cuda.CUDAGraph()
        if self.dist is None:
            with graph_capture(g):
                for _ in range(k):
                    self._step_body(st, bucketed)
            self._gstep, self._gstep_n = g, k
            return
        reason = None
        try:
            with graph_capture(g):
                for _ in range(k):
                    self._step_body(st, bucketed)
        except RuntimeError as e:
            reason = f"{type(e).__name__}: {e}"[:300]
            g = None
            torch.cuda.synchronize()
        flag = torch.tensor([0.0 if reason is None else 1.0], device=self._row.device)
        self.dist.all_reduce(flag)  # eager, outside any capture: how many ranks failed
        nfail = int(flag.item())
        if nfail:
            import warnings
            self.capture_fallback_reason = reason or f"capture refused on {nfail} other rank(s)"
            warnings.warn(f"PPOUpdater: RCCL collective capture failed ({self.capture_fallback_reason}); "
                          "eager collectives between the captured bodies instead")
            self._gstep = None
            self._ga = self._gb = None
        else:
            self._gstep, self._gstep_n = g, k


def ppo_update(policy, value, opt_p, opt_v, obs, acts, logp, ret, adv, index_batches, cfg, dist=None, world=1,
               events: Optional[list] = None):
    """train_ppo.py:233-252 as one eager pass of PPOUpdater (no graphs): per minibatch, a policy Adam
    step then a value Adam step; data-parallel, each rank takes its share of every minibatch and both
    nets' gradients travel in one all-reduce."""
    PPOUpdater(policy, value, opt_p, opt_v, cfg, dist, world, use_graph=False).run(obs, acts, logp, ret, adv,
                                                                                  index_batches, events)


# ----------------------------------------------------------------------------------------- trainer
def _jsonable(cfg):
    d = asdict(cfg) if is_dataclass(cfg) else dict(cfg)
    return json.loads(json.dumps(d, default=str))


class PPOTrainer:
    """train_ppo.py:64-441 over any env exposing reset() -> obs, step(act) -> (obs, rew, term, trunc)
    with auto-reset (HumanoidEnv, or a stand-in in CPU tests), obs_dim, act_dim, num_envs."""

    def __init__(self, cfg, env, eval_env=None, device="cuda", dist=None, out_dir: Optional[str] = None,
                 use_graph: bool = True, jax_keys: bool = False, fused_policy: bool = True,
                 reset_pool: int = 16, update_graph: bool = True):
        """jax_keys: draw every env reset (initial, auto-reset, eval) from the jax.random key chain
        train_ppo.py derives from cfg.seed (:88-118, :132/:150-151 per rollout step, :325, :359,
        :419, eval :268-293), so the reset stream equals the reference's for the same seed.
        fused_policy: the rollout's normalisation + policy MLP + head as one launch (mjl_policy_fwd)
        when the network fits it; False keeps normalisation launch + torch MLP + head launch.
        reset_pool: up to this many auto-resets per env and rollout are computed in bulk before the
        rollout (mjl_env_fill_reset_pool; as many as the busiest env used last rollout, + 1) and
        merged by the env steps, instead of each finishing env resetting at the end of its step;
        0 = in place only. Not with jax_keys (those resets are drawn per step).
        update_graph: the update's minibatch steps replay hipGraphs (PPOUpdater) from the second
        iteration on."""
        self.cfg, self.env, self.eval_env, self.dist = cfg, env, eval_env, dist
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.device = torch.device(device)
        g = torch.Generator().manual_seed(int(cfg.seed))  # identical initial params on every rank
        self.policy = GaussianPolicy(env.obs_dim, env.act_dim, cfg.policy_hidden_layer_specs, cfg.log_std_init,
                                     g).to(self.device)
        self.value = ValueNet(env.obs_dim, cfg.value_hidden_layer_specs, g).to(self.device)
        if dist is not None:
            for p in list(self.policy.parameters()) + list(self.value.parameters()):
                dist.broadcast(p.data, 0)
        self.opt_p = _adam(self.policy.parameters(), cfg.lr_policy)
        self.opt_v = _adam(self.value.parameters(), cfg.lr_value)
        self.updater = PPOUpdater(self.policy, self.value, self.opt_p, self.opt_v, cfg, dist, self.world,
                                  use_graph=use_graph and update_graph)
        self.rms = RunningMeanStd(env.obs_dim, self.device)
        self.gen = torch.Generator(device=self.device).manual_seed(int(cfg.seed) * 1000 + self.rank)
        # minibatch permutations drawn on the device they index (4 host randperms of T*B took ~30 ms)
        self.idx_gen = torch.Generator(device=self.device).manual_seed(int(cfg.seed) + 7919 * (self.rank + 1))
        self.jax_keys = bool(jax_keys) and self.device.type == "cuda" and hasattr(env, "set_reset_keys")
        if self.jax_keys:
            self._jax_init()
        self.obs = env.reset().clone()
        self.use_graph = bool(use_graph)
        self._buf, self._graph, self._rollouts = None, None, 0
        self.fused_policy = bool(fused_policy)
        self._pol_dims, self._pol_params = None, None
        self._pool_n = None  # device int: pooled resets per env for the next rollout
        if reset_pool > 0 and not self.jax_keys and self.device.type == "cuda" and hasattr(env, "enable_reset_pool"):
            env.enable_reset_pool(int(reset_pool))
            self._pool_n = torch.full((1,), min(4, int(reset_pool)), dtype=torch.int32, device=self.device)
        self.allreduce_events = None  # a list to time the per-minibatch all-reduce (bench.py, event_ms)
        self.phase_events = None  # a list: per iteration 4 CUDA events (rollout | between | update), bench.py
        self.total_env_steps = 0.0
        self.start = time.time()
        self.out_dir = out_dir if self.rank == 0 else None
        if self.out_dir:
            for sub in ("checkpoints", "logs"):
                os.makedirs(os.path.join(self.out_dir, sub), exist_ok=True)
            with open(os.path.join(self.out_dir, "config.json"), "w") as f:
                json.dump(_jsonable(cfg), f, indent=2)

    # ------------------------------------------------------------------ jax.random key chain
    def _jax_init(self):
        from . import jaxrng
        self._jr = jaxrng
        B = self.env.num_envs
        self._key_rows = (self.rank * B, (self.rank + 1) * B)  # this rank's rows of the global key array
        rng = jaxrng.prng_key(self.cfg.seed, self.device)                 # train_ppo.py:88
        rng = jaxrng.split(rng)[0]                                        # :96 init_rng_p
        rng = jaxrng.split(rng)[0]                                        # :103 init_rng_v
        sp = jaxrng.split(rng)                                            # :117
        self._jax_rng = sp[0].clone()
        self._roll_rng = torch.empty_like(self._jax_rng)
        self._env_keys = torch.empty((B, 2), dtype=torch.int32, device=self.device)
        self._env_keys.copy_(self._global_keys(sp[1]))                    # :118
        self.env.set_reset_keys(self._env_keys, jaxrng.PARTITIONABLE)

    def _global_keys(self, key):
        r0, r1 = self._key_rows
        return self._jr.split(key, self.env.num_envs * self.world)[r0:r1]

    def _jax_split_main(self) -> torch.Tensor:
        """rng, sub = random.split(rng) on the main chain; returns sub."""
        sp = self._jr.split(self._jax_rng)
        self._jax_rng.copy_(sp[0])
        return sp[1]

    def _jax_step_keys(self):
        """One rollout step's splits (train_ppo.py:132 for the sampling key, :150-151 for the reset keys)."""
        sp = self._jr.split(self._roll_rng)
        sp2 = self._jr.split(sp[0])
        self._roll_rng.copy_(sp2[0])
        self._env_keys.copy_(self._global_keys(sp2[1]))

    # train_ppo.py:128-169
    def _rollout_buffers(self):
        if self._buf is None:
            T, B, env, dev = self.cfg.rollout_length, self.env.num_envs, self.env, self.device
            self._buf = {
                "obs": torch.empty((T + 1, B, env.obs_dim), device=dev), "act": torch.empty((T, B, env.act_dim), device=dev),
                "logp": torch.empty((T, B), device=dev), "rew": torch.empty((T, B), device=dev),
                "term": torch.empty((T, B), device=dev), "trunc": torch.empty((T, B), device=dev),
                "eps": torch.empty((T, B, env.act_dim), device=dev), "xn": torch.empty((B, env.obs_dim), device=dev)}
        return self._buf

    def _rollout_body(self, graph: bool):
        """One rollout into the static buffers: obs[t] is the obs before step t, the env writes
        obs[t + 1], rew / term / trunc [t] in place (no copies). With graph=True the RNG counters are
        relative to the env's device counter base (the body is being captured)."""
        bf, env = self._buf, self.env
        if self._pool_n is not None:  # this rollout's auto-resets, in bulk (counter 0: see fill_reset_pool)
            env.fill_reset_pool(self._pool_n, counter=0 if graph else None)
        native = bf["obs"].is_cuda  # normalisation and the policy head as two native launches
        fused = native and self._pol_dims is not None  # ... or the whole policy as one (mjl_policy_fwd)
        for t in range(self.cfg.rollout_length):
            if self.jax_keys:
                self._jax_step_keys()
            if fused:
                policy_fwd_native(bf["obs"][t], self.rms.mean, self.rms.var, 10.0, self._pol_params, self._pol_dims,
                                  self.policy.log_std, bf["eps"][t], bf["act"][t], bf["logp"][t])
                act = bf["act"][t]
            elif native:
                obs_normalize_native(bf["obs"][t], self.rms.mean, self.rms.var, 10.0, bf["xn"])
                act = bf["act"][t]
                policy_head_native(self.policy.mlp(bf["xn"]), self.policy.log_std, bf["eps"][t], act, bf["logp"][t])
            else:
                mean, log_std = self.policy(self.rms.normalize(bf["obs"][t]))
                act = torch.addcmul(mean, torch.exp(log_std), bf["eps"][t], out=bf["act"][t])
                gaussian_logprob(mean, log_std, act, out=bf["logp"][t])
            # physics + reward + obs + merge_if_done, one launch
            out = (bf["obs"][t + 1], bf["rew"][t], bf["term"][t], bf["trunc"][t])
            if graph:
                env.step(act, out=out, counter=t + 1)
            elif hasattr(env, "ctr_base"):
                env.step(act, out=out)
            else:  # envs without output buffers (CPU stand-ins)
                for dst, src in zip(out, env.step(act)):
                    dst.copy_(src)

    @torch.no_grad()
    def collect_rollout(self):
        """Rollout of T steps. On the GPU the second and later rollouts replay one hipGraph of the
        whole T-step loop (policy GEMMs, sampling, log-prob, env step; ~20 launches per step
        otherwise): the sampling noise for all T steps is drawn before it, and the env RNG counters
        come from the env's device counter base, so a replay is bit-identical to the eager loop."""
        bf, env, T = self._rollout_buffers(), self.env, self.cfg.rollout_length
        if self._pol_dims is None and self.fused_policy and bf["obs"].is_cuda:
            self._pol_dims = policy_fused_dims(self.policy)
        if self._pol_dims is not None:  # the policy changed in the update: repack into the static buffer
            if self._pol_params is None:
                self._pol_params = pack_policy_params(self.policy)
            else:
                pack_policy_params(self.policy, out=self._pol_params)
        bf["eps"].normal_(generator=self.gen)
        bf["obs"][0].copy_(self.obs)
        if self.jax_keys:
            self._roll_rng.copy_(self._jax_split_main())  # train_ppo.py:325 key_roll
        use_graph = self.use_graph and self.device.type == "cuda" and hasattr(env, "ctr_base")
        if use_graph and self._graph is None and self._rollouts > 0:
            self._graph = torch.cuda.CUDAGraph()
            with graph_capture(self._graph):
                self._rollout_body(graph=True)
        if use_graph and self._graph is not None:
            env.ctr_base.fill_(env.counter)
            self._graph.replay()
            env.counter += T
            env.ctr_base.zero_()
        else:
            self._rollout_body(graph=False)
        self._rollouts += 1
        if self._pool_n is not None:  # next rollout's pool: the busiest env's auto-resets + 1 (no host sync)
            busiest = (torch.maximum(bf["term"], bf["trunc"]) > 0.5).sum(0).max()
            self._pool_n.copy_(torch.clamp(busiest + 1, max=self.env.pool_slots))
        self.obs = bf["obs"][T]
        return bf["obs"][:T], bf["act"], bf["logp"], bf["rew"], bf["term"], bf["trunc"]

    def _mark(self, evs, i):
        if evs is not None:
            evs[i].record()

    def iteration(self, it: int) -> dict:
        cfg, dev = self.cfg, self.device
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        evs = None
        if self.phase_events is not None and dev.type == "cuda":
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            self.phase_events.append(evs)
        t0 = time.time()
        self._mark(evs, 0)
        obs_t, act_t, logp_t, r_t, te_t, tr_t = self.collect_rollout()
        self._mark(evs, 1)
        T, B = r_t.shape
        if self.jax_keys:
            self._jax_split_main()  # train_ppo.py:359 rng_idx (the minibatch permutation is torch's)
        self.rms.update(obs_t, self.dist)
        with torch.no_grad():
            obs_n = self.rms.normalize(obs_t)
            last_n = self.rms.normalize(self.obs)
            v = self.value(torch.cat([obs_n, last_n[None]], 0).reshape((T + 1) * B, -1)).reshape(T + 1, B)
            adv, ret = compute_gae(r_t, v, te_t, tr_t, cfg.gamma, cfg.lam)
        mb = cfg.minibatch_size // self.world
        idx = make_index_batches(T * B, mb, cfg.epochs, self.idx_gen, dev)
        self._mark(evs, 2)
        self.updater.run(obs_n.reshape(T * B, -1), act_t.reshape(T * B, -1), logp_t.reshape(-1), ret.reshape(-1),
                         adv.reshape(-1), idx, self.allreduce_events)
        self._mark(evs, 3)
        self.last_update_rows = int(idx.numel())
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = max(time.time() - t0, 1e-9)
        ep_ret = r_t.sum(0)
        stats = torch.stack([ep_ret.sum(), torch.maximum(te_t, tr_t).sum(), torch.tensor(float(B), device=dev)])
        mx = ep_ret.max().reshape(1)
        if self.dist is not None:
            self.dist.all_reduce(stats)
            self.dist.all_reduce(mx, op=self.dist.ReduceOp.MAX)
        env_steps = float(T) * float(stats[2])
        self.total_env_steps += env_steps
        dones = float(stats[1])
        return {"train_return_avg": float(stats[0] / stats[2]), "train_return_max": float(mx[0]),
                "train_eplen_avg": env_steps / dones if dones > 0 else float(T),
                "env_steps_per_sec": env_steps / dt}

    @torch.no_grad()
    def evaluate(self, it: int = 0, steps: int = 500) -> float:
        """train_ppo.py:261-313: deterministic mean action, auto-reset, mean summed reward; the eval
        envs are reseeded with seed + 10000 + iteration each time (train_ppo.py:268-270)."""
        env = self.eval_env
        if hasattr(env, "seed"):
            env.seed, env.counter = int(self.cfg.seed) + 10000 + it, 0
        keyed = self.jax_keys and hasattr(env, "set_reset_keys")
        if keyed:  # train_ppo.py:268-272, 292-293
            jr = self._jr
            sp = jr.split(jr.prng_key(int(self.cfg.seed) + 10000 + it, self.device))
            rng, keys = sp[0].clone(), jr.split(sp[1], env.num_envs).contiguous()
            env.set_reset_keys(keys, jr.PARTITIONABLE)
        obs = env.reset().clone()
        acc = torch.zeros(env.num_envs, device=self.device)
        for _ in range(steps):
            if keyed:
                sp = jr.split(rng)
                rng.copy_(sp[0])
                keys.copy_(jr.split(sp[1], env.num_envs))
            mean, _ = self.policy(self.rms.normalize(obs))
            obs, r, _, _ = env.step(mean)
            acc += r
        if keyed:
            env.set_reset_keys(None)
        return float(acc.mean())

    def dump_qpos_history(self, it: int) -> Optional[str]:
        """train_ppo.py:433-456 render_video (save_video): one env, deterministic mean action of the
        normalised obs for render_duration seconds, reset to its initial state when done; the qpos
        history goes to <training_dir>/videos/iter_<it+1:06d>.npz (mjx_amd/rendering.py)."""
        if not self.out_dir or self.eval_env is None or not hasattr(self.eval_env, "get_state"):
            return None
        from . import rendering
        from .envs import HumanoidEnv
        if getattr(self, "_render_env", None) is None:
            ev = self.eval_env
            self._render_env = HumanoidEnv(ev.sys, ev.cfg, 1, device=self.device.index or 0,
                                           seed=int(self.cfg.seed) + 20000)
        pol = lambda o: self.policy(self.rms.normalize(o))[0]  # noqa: E731
        qpos, act = rendering.rollout_qpos_history(self._render_env, pol, float(self.cfg.render_duration))
        path = os.path.join(self.out_dir, "videos", f"iter_{it + 1:06d}.npz")
        return rendering.save_qpos_history(path, qpos[:, 0], act[:, 0], float(self._render_env.sys.m.timestep),
                                           int(self.cfg.render_fps), os.path.basename(str(self.cfg.xml_path)),
                                           str(self.cfg.camera_name))

    def save_checkpoint(self, it: int, metrics: dict):
        """checkpoint_utils.py:38-61 layout (results/<ts>_ppo/checkpoints/), torch state dicts."""
        if not self.out_dir:
            return None
        path = os.path.join(self.out_dir, "checkpoints", f"checkpoint_{it:06d}.pt")
        torch.save({"step": it, "policy": self.policy.state_dict(), "value": self.value.state_dict(),
                    "rms": self.rms.state_dict(), "opt_policy": self.opt_p.state_dict(),
                    "opt_value": self.opt_v.state_dict(), "metrics": metrics}, path)
        return path

    def load_checkpoint(self, path: str):
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.policy.load_state_dict(ck["policy"])
        self.value.load_state_dict(ck["value"])
        self.rms.load_state_dict(ck["rms"])
        self.opt_p.load_state_dict(ck["opt_policy"])
        self.opt_v.load_state_dict(ck["opt_value"])
        return ck["step"]

    def log(self, it: int, metrics: dict):
        """checkpoint_utils.py:93-100 + training_utils.py:146-152: metrics.jsonl lines."""
        metrics["total_env_steps"] = self.total_env_steps
        metrics["elapsed_time"] = time.time() - self.start
        if self.out_dir:
            with open(os.path.join(self.out_dir, "logs", "metrics.jsonl"), "a") as f:
                f.write(json.dumps({"step": it, **metrics}) + "\n")

    def train(self, iterations: Optional[int] = None, verbose: bool = True) -> List[dict]:
        cfg = self.cfg
        n = cfg.total_iterations if iterations is None else iterations
        hist = []
        for it in range(n):
            m = self.iteration(it)
            should_eval = (it % cfg.eval_interval == 0) and self.eval_env is not None
            should_ckpt = it % cfg.checkpoint_every == 0
            if self.jax_keys and it % cfg.eval_interval == 0:
                self._jax_split_main()  # train_ppo.py:419 key_eval (evaluate reseeds from cfg.seed)
            if should_eval and self.rank == 0:
                m["eval_return"] = self.evaluate(it)
            if (it % cfg.log_interval == 0) or should_eval or should_ckpt or it == n - 1:
                self.log(it, m)
                if verbose and self.rank == 0:
                    s = (f"Iter {it:4d} | S/s: {m['env_steps_per_sec']:10.0f} | Train_Ret(Avg): "
                         f"{m['train_return_avg']:8.2f} | Train_Len(Avg): {m['train_eplen_avg']:6.0f}")
                    if "eval_return" in m:
                        s += f" | Eval_Ret(Avg): {m['eval_return']:8.2f}"
                    print(s, flush=True)
            if should_ckpt:
                self.save_checkpoint(it, m)
            if cfg.save_video and it % cfg.eval_interval == 0 and self.rank == 0:
                self.dump_qpos_history(it)
            hist.append(m)
        return hist

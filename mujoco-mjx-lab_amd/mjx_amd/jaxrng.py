"""jax.random keys on the device (threefry2x32), for resets drawn exactly as the reference draws them.

The reference resets envs with per-env keys: `keys = random.split(key_reset, num_envs)` then
`single_reset(key)` splits each key in four (src/envs.py:116-147, train_ppo.py:150-152). With
`HumanoidEnv.set_reset_keys(keys)` the native resets consume such keys and produce the reset state
MJX produces for them; `split` is `jax.random.split` over a batch of keys. Keys are uint32 pairs
held in int32 tensors (same bits). Mode: PARTITIONABLE (jax >= 0.5 default; the reference pins
jax==0.7.2) or ORIGINAL (the pre-0.5 layout).
"""
from __future__ import annotations

import torch

from ._lib import check, lib

PARTITIONABLE, ORIGINAL = 1, 2


def prng_key(seed: int, device="cuda") -> torch.Tensor:
    """jax.random.PRNGKey(seed) for a 32-bit seed: [0, seed]."""
    return torch.tensor([0, int(seed) & 0xFFFFFFFF], dtype=torch.int64).to(torch.int32).to(device)


def split(keys: torch.Tensor, num: int = 2, mode: int = PARTITIONABLE) -> torch.Tensor:
    """jax.random.split for each of n keys: [n, 2] (or [2]) -> [n, num, 2] (or [num, 2])."""
    single = keys.dim() == 1
    k = keys.reshape(-1, 2).to(torch.int32).contiguous()
    if not k.is_cuda:
        raise ValueError("keys must be a CUDA tensor")
    out = torch.empty((k.shape[0], num, 2), dtype=torch.int32, device=k.device)
    check(lib().mjl_prng_split(k.data_ptr(), k.shape[0], int(num), int(mode), out.data_ptr(),
                               torch.cuda.current_stream(k.device).cuda_stream))
    return out[0] if single else out

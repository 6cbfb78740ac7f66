"""Loader for the native library libmjx355.so (C ABI declared in include/mjx355.h).

The library is built in-tree (`mujoco-mjx-lab_amd/csrc/Makefile`, or `__graft_entry__.build()`).
There is no fallback: every entry point of the product path goes through this library, and a
missing library or GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

from . import _srchash, abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MJX355_LIB", os.path.join(_HERE, "libmjx355.so"))  # override: A/B builds
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

# every symbol include/mjx355.h declares
EXPORTS = [
    "mjl_last_error", "mjl_version", "mjl_model_create", "mjl_model_destroy", "mjl_model_nefc_max",
    "mjl_batch_create", "mjl_batch_destroy", "mjl_batch_nenv", "mjl_batch_set_option", "mjl_get", "mjl_set",
    "mjl_forward", "mjl_step", "mjl_speedtest_step", "mjl_env_config", "mjl_env_step", "mjl_env_reset",
    "mjl_step_vjp", "mjl_env_step_vjp", "mjl_gae", "mjl_batch_set_counter_base",
    "mjl_env_set_reset_keys", "mjl_prng_split", "mjl_env_step_vjp_guarded", "mjl_state_size", "mjl_get_state",
    "mjl_set_state", "mjl_obs_normalize", "mjl_policy_head", "mjl_colsum_scratch", "mjl_colsum", "mjl_tanh_bwd_colsum", "mjl_slice_sum", "mjl_tanh_inplace", "mjl_small_mlp_fwd",
    "mjl_small_mlp_bwd_input", "mjl_apg_obs_policy_fwd", "mjl_apg_policy_bwd_obs_vjp",
    "mjl_policy_param_floats", "mjl_policy_fwd",
    "mjl_step_vjp_full", "mjl_env_step_vjp_full", "mjl_env_fill_reset_pool",
    "mjl_apg_obs", "mjl_apg_post", "mjl_apg_obs_vjp", "mjl_env_step_record", "mjl_env_step_record_apg",
    "mjl_env_step_record_apg_next", "mjl_env_record_fused", "mjl_env_step_vjp_replay", "mjl_env_step_vjp_replay_apg",
    "mjl_ppo_loss_scratch", "mjl_ppo_surrogate", "mjl_mse", "mjl_gather_rows", "mjl_adam",
    "mjl_adam_dev",
    "mjl_colsum_batched_scratch", "mjl_colsum_batched", "mjl_tanh_bwd_colsum_batched", "mjl_slice_sum_batched",
    "mjl_mse_strided", "mjl_ppo_surrogate_clipped", "mjl_bias_act", "mjl_adam_multi",
    "mjl_gather_rows_indexed", "mjl_slice_sum_multi", "mjl_tanh_bwd_colsum_partials", "mjl_twin_loss_head_blocks", "mjl_twin_loss_head",
    "mjl_twin_fused_shapes", "mjl_twin_gather_in", "mjl_twin_head_bwd", "mjl_twin_head_blocks", "mjl_twin_head",
]

_lib = None


class MjlError(RuntimeError):
    pass


def source_hash() -> str:
    """sha256 prefix over the native sources (kernel + C ABI) of this tree (_srchash.py): the stamp a
    library built from them carries, and the key of recorded profiles."""
    return _srchash.source_hash(CSRC)


def stamped_hash(version: str) -> str:
    """The source hash a library stamped into its mjl_version() string ("... src=<hash>"), or ""."""
    return version.rsplit("src=", 1)[1].strip() if "src=" in version else ""


def build(force: bool = False):
    args = ["make", "-s", "-C", CSRC]
    if force:
        args.append("-B")
    subprocess.run(args, check=True)


def build_info() -> dict:
    """Which library this process runs and what it was built from (bench line, smoke)."""
    L = lib()
    v = L.mjl_version().decode()
    return {"lib": os.path.relpath(LIB_PATH, os.path.dirname(os.path.dirname(_HERE))), "version": v,
            "lib_src_hash": stamped_hash(v), "tree_src_hash": source_hash(),
            "override": "MJX355_LIB" in os.environ}


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MjlError(f"native library missing: {LIB_PATH} (run `make -C {CSRC}` or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    L.mjl_version.restype = C.c_char_p
    # provenance: the product library must have been built from this tree's sources. An explicit
    # MJX355_LIB (A/B and diagnostic builds) opts out of the check.
    if "MJX355_LIB" not in os.environ:
        built, tree = stamped_hash(L.mjl_version().decode()), source_hash()
        if built != tree:
            raise MjlError(f"stale native library {LIB_PATH}: built from sources {built or '(unstamped)'}, "
                           f"the tree's sources are {tree} (rebuild: make -C {CSRC})")
    P, vp, f32p, i32 = C.POINTER, C.c_void_p, C.c_void_p, C.c_int
    u64 = C.c_uint64
    L.mjl_last_error.restype = C.c_char_p
    L.mjl_version.restype = C.c_char_p
    L.mjl_model_create.argtypes = [P(abi.ModelDesc), P(vp)]
    L.mjl_model_destroy.argtypes = [vp]
    L.mjl_model_destroy.restype = None
    L.mjl_model_nefc_max.argtypes = [vp]
    L.mjl_batch_create.argtypes = [vp, i32, i32, P(vp)]
    L.mjl_batch_destroy.argtypes = [vp]
    L.mjl_batch_destroy.restype = None
    L.mjl_batch_nenv.argtypes = [vp]
    L.mjl_batch_set_option.argtypes = [vp, i32, i32]
    L.mjl_get.argtypes = [vp, i32, f32p, vp]
    L.mjl_set.argtypes = [vp, i32, f32p, f32p, vp]
    L.mjl_forward.argtypes = [vp, f32p, vp]
    L.mjl_step.argtypes = [vp, f32p, vp]
    L.mjl_speedtest_step.argtypes = [vp, f32p, f32p, vp]
    L.mjl_env_config.argtypes = [vp, P(abi.EnvConfigC)]
    L.mjl_env_step.argtypes = [vp, f32p, f32p, f32p, f32p, f32p, i32, u64, u64, vp]
    L.mjl_env_reset.argtypes = [vp, f32p, u64, u64, f32p, f32p, vp]
    L.mjl_env_fill_reset_pool.argtypes = [vp, vp, u64, u64, vp]
    L.mjl_ppo_loss_scratch.restype = C.c_longlong
    L.mjl_ppo_loss_scratch.argtypes = [i32, i32]
    L.mjl_ppo_surrogate.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, vp, vp, vp, vp, vp]
    L.mjl_mse.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    L.mjl_gather_rows.argtypes = [vp, i32, C.c_longlong, i32, vp, vp, vp, vp]
    L.mjl_adam.argtypes = [i32, vp, vp, vp, vp, vp, C.c_float, C.c_float, C.c_float, C.c_float, i32, vp]
    L.mjl_adam_dev.argtypes = [i32, vp, vp, vp, vp, vp, C.c_float, C.c_float, C.c_float, C.c_float, vp, vp]
    L.mjl_env_step_record.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
    L.mjl_env_step_record_apg.argtypes = [vp, i32, vp, vp, vp, vp, vp, C.c_float, C.c_float] + [vp] * 7
    L.mjl_env_record_fused.argtypes = [vp]
    L.mjl_env_step_vjp_replay_apg.argtypes = [vp, i32] + [vp] * 12 + [i32, vp, vp, vp, vp, vp, vp, vp, i32, vp]
    L.mjl_env_step_record_apg_next.argtypes = ([vp, i32, vp, vp, vp, vp, vp, C.c_float, C.c_float] + [vp] * 8 +
                                               [i32, vp, vp, vp, i32, vp, vp, vp, vp, vp])
    L.mjl_env_step_vjp_replay.argtypes = [vp, i32] + [vp] * 12 + [vp]
    L.mjl_apg_obs.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp]
    L.mjl_apg_post.argtypes = [vp, vp, vp, vp, C.c_float, C.c_float, vp, vp, vp, vp, vp, vp, vp]
    L.mjl_apg_obs_vjp.argtypes = [i32, i32, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp]
    L.mjl_batch_set_counter_base.argtypes = [vp, vp]
    L.mjl_env_set_reset_keys.argtypes = [vp, vp, i32]
    L.mjl_env_step_vjp_guarded.argtypes = [vp] + [vp] * 10 + [vp]
    L.mjl_state_size.argtypes = [vp]
    L.mjl_get_state.argtypes = [vp, vp, vp]
    L.mjl_set_state.argtypes = [vp, vp, vp, vp]
    L.mjl_prng_split.argtypes = [vp, i32, i32, i32, vp, vp]
    L.mjl_gae.argtypes = [f32p, f32p, f32p, f32p, i32, i32, C.c_double, C.c_double, f32p, f32p, vp]
    L.mjl_obs_normalize.argtypes = [f32p, f32p, f32p, i32, i32, C.c_float, f32p, vp]
    L.mjl_policy_head.argtypes = [f32p, f32p, f32p, i32, i32, f32p, f32p, vp]
    L.mjl_policy_param_floats.argtypes = [i32, C.POINTER(i32)]
    L.mjl_policy_param_floats.restype = C.c_longlong
    L.mjl_policy_fwd.argtypes = [f32p, f32p, f32p, C.c_float, f32p, i32, C.POINTER(i32), f32p, f32p, i32, f32p, f32p, vp]
    L.mjl_colsum_scratch.argtypes = [i32, i32]
    L.mjl_colsum_scratch.restype = C.c_longlong
    L.mjl_colsum.argtypes = [f32p, i32, i32, f32p, f32p, vp]
    L.mjl_tanh_bwd_colsum.argtypes = [f32p, f32p, i32, i32, f32p, f32p, f32p, vp]
    L.mjl_slice_sum.argtypes = [f32p, i32, C.c_longlong, f32p, vp]
    L.mjl_tanh_inplace.argtypes = [f32p, C.c_longlong, vp]
    L.mjl_colsum_batched_scratch.argtypes = [i32, i32, i32]
    L.mjl_colsum_batched_scratch.restype = C.c_longlong
    L.mjl_colsum_batched.argtypes = [f32p, i32, i32, i32, f32p, f32p, vp]
    L.mjl_tanh_bwd_colsum_batched.argtypes = [f32p, f32p, i32, i32, i32, f32p, f32p, f32p, vp]
    L.mjl_slice_sum_batched.argtypes = [f32p, i32, i32, C.c_longlong, f32p, vp]
    L.mjl_mse_strided.argtypes = [vp, i32, vp, i32, vp, vp, vp, vp]
    L.mjl_bias_act.argtypes = [vp, vp, i32, C.c_longlong, i32, C.c_uint, vp]
    L.mjl_adam_multi.argtypes = [i32, vp, vp, vp, vp, vp, vp, i32, vp, C.c_float, C.c_float, C.c_float, C.c_float,
                                 vp, vp, i32, vp]
    L.mjl_ppo_surrogate_clipped.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, C.c_float,
                                            C.c_float, vp, vp, vp, vp, vp]
    L.mjl_gather_rows_indexed.argtypes = [vp, vp, i32, C.c_longlong, i32, vp, vp, vp, vp]
    L.mjl_slice_sum_multi.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mjl_twin_loss_head_blocks.argtypes = [i32]
    L.mjl_twin_loss_head_blocks.restype = C.c_longlong
    L.mjl_twin_loss_head.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, C.c_float,
                                     C.c_float, vp, vp, vp, vp, vp, vp, vp]
    L.mjl_twin_fused_shapes.argtypes = [i32, i32, i32]
    L.mjl_twin_gather_in.argtypes = [vp, vp, i32, C.c_longlong, i32, i32, i32] + [vp] * 13 + [vp]
    L.mjl_twin_head_bwd.argtypes = [vp, vp, vp, i32, i32, i32, vp, vp, vp, vp]
    L.mjl_twin_head_blocks.argtypes = [i32]
    L.mjl_twin_head_blocks.restype = C.c_longlong
    L.mjl_twin_head.argtypes = ([vp] * 11 + [i32, i32, i32] + [C.c_float] * 4 + [vp] * 7 + [vp])
    L.mjl_tanh_bwd_colsum_partials.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, vp]
    L.mjl_small_mlp_fwd.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, vp]
    L.mjl_small_mlp_bwd_input.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, vp]
    L.mjl_apg_obs_policy_fwd.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp]
    L.mjl_apg_policy_bwd_obs_vjp.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp]
    L.mjl_step_vjp.argtypes = [vp, f32p, f32p, f32p, f32p, f32p, vp]
    L.mjl_env_step_vjp.argtypes = [vp, f32p, f32p, f32p, f32p, f32p, f32p, f32p, f32p, f32p, vp]
    L.mjl_step_vjp_full.argtypes = [vp] + [f32p] * 7 + [vp]
    L.mjl_env_step_vjp_full.argtypes = [vp] + [f32p] * 12 + [vp]
    _lib = L
    return L


def check(rc: int):
    if rc != 0:
        raise MjlError(f"mjx355 error {rc}: {lib().mjl_last_error().decode()}")

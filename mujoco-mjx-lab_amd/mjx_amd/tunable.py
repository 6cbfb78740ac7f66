"""Tuned GEMM choices for the trainers' dense layers (PyTorch TunableOp, results-file mode).

The PPO update's GEMMs (65,536-row minibatch: 256-wide layers, the split-K weight gradients; the
8,192-row per-rank shard of C5) and the APG policy's run on hipBLASLt / rocBLAS through torch. By
default torch takes the library heuristic's first solution; `tuning/gfx950_tunableop.csv` holds the
fastest solution per GEMM shape measured on MI355X by `tools/tune_gemms.sh` (every candidate timed,
TunableOp's own numerical check against the default solution). Loading it switches TunableOp on in
lookup-only mode: shapes in the file run their tuned solution, others the default, nothing is tuned
at run time. Measured: PPO update at 2048 envs 51.6 -> 47.5 ms (tools/ppo_update_probe.py graph).

The file's validators (torch, HIP, hipBLASLt, rocBLAS versions and the gfx arch) must match the
running stack or TunableOp ignores it (then: the default solutions, as without this module).
MJL_TUNED_GEMMS=0 disables; a user's own PYTORCH_TUNABLEOP_* configuration takes precedence."""
import os
import tempfile

import torch

TUNED_CSV = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "gfx950_tunableop.csv")
_state = {"done": False, "loaded": False}


def use_tuned_gemms(device) -> bool:
    """Enable the tuned GEMM table for `device` (once per process). Returns whether it is active."""
    if _state["done"]:
        return _state["loaded"]
    dev = torch.device(device)
    if dev.type != "cuda" or os.environ.get("MJL_TUNED_GEMMS", "1") != "1" or not os.path.exists(TUNED_CSV):
        return False
    if any(k.startswith("PYTORCH_TUNABLEOP_") for k in os.environ):
        _state["done"] = True  # the user's TunableOp configuration (e.g. tools/tune_gemms.sh) wins
        return False
    import torch.cuda.tunable as tn
    _state["done"] = True
    tn.enable(True)
    tn.tuning_enable(False)
    tn.record_untuned_enable(False)
    # results are written back only when tuning is on; point the file name away from the cwd anyway
    tn.set_filename(os.path.join(tempfile.gettempdir(), f"mjl_tunableop_{os.getpid()}_%d.csv"))
    _state["loaded"] = bool(tn.read_file(TUNED_CSV))
    if not _state["loaded"]:
        tn.enable(False)
    return _state["loaded"]

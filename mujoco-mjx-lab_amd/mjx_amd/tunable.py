"""Tuned GEMM choices for the trainers' dense layers (PyTorch TunableOp, results-file mode).

The PPO update's GEMMs (65,536-row minibatch: 256-wide layers, the split-K weight gradients; the
8,192-row per-rank shard of C5) and the APG policy's run on hipBLASLt / rocBLAS through torch. By
default torch takes the library heuristic's first solution; `tuning/gfx950_tunableop.csv` holds the
fastest solution per GEMM shape measured on MI355X by `tools/tune_gemms.sh` (every candidate timed,
TunableOp's own numerical check against the default solution). Loading it switches TunableOp on in
lookup-only mode: shapes in the file run their tuned solution, others the default, nothing is tuned
at run time. Measured: PPO update at 2048 envs 51.6 -> 47.5 ms (tools/ppo_update_probe.py graph).

Scope: the table is loaded once per process, but TunableOp is switched on only inside `tuned_gemms()`
(the PPO update's minibatch steps, the APG policy's parameter-gradient pass) and restored to its
previous state on exit, so GEMMs elsewhere in the user's process (evaluation, user code) keep the
library's default choices. A hipGraph captured inside the scope keeps the tuned kernels it captured.

The file's validators (torch, HIP, hipBLASLt, rocBLAS versions and the gfx arch) must match the
running stack or TunableOp ignores it (then: the default solutions, as without this module).
MJL_TUNED_GEMMS=0 disables; a user's own PYTORCH_TUNABLEOP_* configuration takes precedence."""
import contextlib
import os
import tempfile

import torch

TUNED_CSV = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "gfx950_tunableop.csv")
_state = {"done": False, "loaded": False}


def use_tuned_gemms(device) -> bool:
    """Load the tuned GEMM table for `device` (once per process; TunableOp stays off outside
    tuned_gemms()). Returns whether the table is loaded."""
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
    tn.enable(False)  # on only inside tuned_gemms()
    return _state["loaded"]


def table_loaded() -> bool:
    """Whether the tuned table is loaded in this process (recorded in the bench line)."""
    return bool(_state["loaded"])


@contextlib.contextmanager
def tuned_gemms(device=None):
    """TunableOp on (lookup only, the loaded table) for the GEMMs issued inside; its previous state
    restored on exit. A no-op when the table is not loaded or `device` is not a GPU."""
    if device is not None and torch.device(device).type == "cuda":
        use_tuned_gemms(device)
    if not _state["loaded"]:
        yield False
        return
    import torch.cuda.tunable as tn
    prev = tn.is_enabled()
    tn.enable(True)
    try:
        yield True
    finally:
        tn.enable(prev)

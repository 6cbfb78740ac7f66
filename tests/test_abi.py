"""C ABI: struct layouts agree across Python/ctypes, the oracle build and the product library;
the product library loads without a GPU and exports every symbol include/mjx355.h declares."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import mjx_amd
from mjx_amd import _lib, abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "mjx355.h")).read()
    declared = set(re.findall(r"^\s*(?:const char\*|long long|int|void)\s+(mjl_\w+)\(", hdr, re.M))
    assert declared == set(_lib.EXPORTS)
    L = _lib.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert b"gfx950" in L.mjl_version()


def test_struct_layouts_match_oracle_build():
    import oracle as orc
    L = orc.lib()  # asserts sizeof(OrcState/ModelDesc/EnvConfig) against the C compiler
    assert L.orc_desc_size() == C.sizeof(abi.ModelDesc)
    assert L.orc_envcfg_size() == C.sizeof(abi.EnvConfigC)


def test_model_create_validates_without_gpu():
    L = _lib.lib()
    m = mjx_amd.load_model("humanoid_mjx")
    d = abi.model_desc(m)
    h = C.c_void_p()
    assert L.mjl_model_create(C.byref(d), C.byref(h)) == 0
    assert L.mjl_model_nefc_max(h) == 16 * 4 + 100 + 21 + 2  # nefc <= 187
    L.mjl_model_destroy(h)
    bad = abi.model_desc(m)
    bad.integrator = 1  # RK4
    assert L.mjl_model_create(C.byref(bad), C.byref(h)) == 2
    assert b"integrator" in L.mjl_last_error()


def test_no_silent_cpu_fallback():
    """Without a GPU the product path fails loudly instead of falling back to the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mjx_amd import mjx
    sys_ = mjx.put_model(mjx_amd.load_model("humanoid_mjx"))
    with pytest.raises(_lib.MjlError):
        mjx.make_data(sys_, 4)


def test_batch_create_rejects_empty_and_null_without_gpu():
    """An empty or negative batch and a null model are argument errors, reported before any device
    call (so also on a host without a GPU)."""
    L = _lib.lib()
    m = mjx_amd.load_model("humanoid_mjx")
    d = abi.model_desc(m)
    h, b = C.c_void_p(), C.c_void_p()
    assert L.mjl_model_create(C.byref(d), C.byref(h)) == 0
    for n in (0, -1):
        assert L.mjl_batch_create(h, n, 0, C.byref(b)) == 1  # MJL_ERR_ARG
        assert b"bad argument" in L.mjl_last_error()
    assert L.mjl_batch_create(None, 4, 0, C.byref(b)) == 1
    L.mjl_model_destroy(h)


def test_fused_apg_entries_reject_null_without_gpu():
    """The fused APG entry points (record + bookkeeping + next policy, replay + policy backward) report a
    null batch or a null buffer as an argument error before any device call; the eligibility query says
    0 for a null batch."""
    L = _lib.lib()
    assert L.mjl_env_record_fused(None) == 0
    z = [None] * 7
    assert L.mjl_env_step_record_apg(None, 0, None, None, None, None, None, 0.99, 0.0, *z) == 1
    assert b"bad argument" in L.mjl_last_error()
    assert L.mjl_env_step_record_apg_next(None, 0, None, None, None, None, None, 0.99, 0.0, *([None] * 8), 0, None,
                                          None, None, 1, None, None, None, None, None) == 1
    assert L.mjl_env_step_vjp_replay_apg(None, 0, *([None] * 12), 1, None, None, None, None, None, None, None, 0,
                                         None) == 1

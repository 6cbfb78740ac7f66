"""The kernarg-pointer fault class (round 5): `__builtin_amdgcn_kernarg_segment_ptr()`
inside a called (non-kernel) function is not the kernel's segment — the compiler materialises it as
a zeroed SGPR pair (`s_mov_b64 s[4:5], 0`) and the loads through it fault (hipErrorIllegalAddress in
test_env_reset_parity, gpurun_out/r5a). Reference path that faulted: single_reset
(/root/reference/src/envs.py:115-202) -> env_reset in csrc/step_kernels.hip.

Guard: the SHIPPED code object (gfx950, unbundled from libmjx355.so's .hip_fatbin) is disassembled and
every non-kernel function is scanned for a scalar load whose base pair was zeroed by `s_mov_b64` and
not written since. No GPU needed. The debug build (make debug) adds a __builtin_trap() on a null
pointer in kparams_late()."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mujoco-mjx-lab_amd", "mjx_amd", "libmjx355.so")
LLVM = "/opt/rocm/lib/llvm/bin"

_FUNC = re.compile(r"^[0-9a-f]+ <(?P<name>[^>]+)>:")
_ZERO = re.compile(r"^\s*s_mov_b64\s+s\[(\d+):(\d+)\],\s*0\s*(//.*)?$")
_LOAD = re.compile(r"^\s*s_(?:buffer_)?load_\w+\s+[^,]+,\s*s\[(\d+):(\d+)\]")
_DST = re.compile(r"^\s*[sv]_\w+\s+(s\[(\d+):(\d+)\]|s(\d+))(?=[,\s]|$)")


def zeroed_base_loads(asm_lines, kernels):
    """(function, line) of every scalar load in a non-kernel function through an SGPR pair set to 0 by
    s_mov_b64 and not overwritten since (straight-line tracking within a function, reset at labels is
    not needed: a zeroed pair that reaches a load on any path is what faulted)."""
    hits, fn, zero = [], None, set()
    for ln in asm_lines:
        m = _FUNC.match(ln)
        if m:
            fn, zero = m.group("name"), set()
            continue
        if fn is None or fn in kernels:
            continue
        m = _ZERO.match(ln)
        if m:
            zero.add((int(m.group(1)), int(m.group(2))))
            continue
        m = _LOAD.match(ln)
        if m and (int(m.group(1)), int(m.group(2))) in zero:
            hits.append((fn, ln.split("//")[0].strip()))
        m = _DST.match(ln)
        if m and zero:  # an instruction writing any register of a tracked pair ends its tracking
            lo, hi = (int(m.group(2)), int(m.group(3))) if m.group(2) else (int(m.group(4)), int(m.group(4)))
            zero = {p for p in zero if p[1] < lo or p[0] > hi}
    return hits


def test_scanner_flags_the_round5_pattern():
    asm = ["0000000000001000 <_ZN3mjl9env_resetI...>:",
           "\ts_mov_b64 s[4:5], 0",
           "\ts_load_dwordx2 s[8:9], s[4:5], 0x10",
           "0000000000002000 <_ZN3mjl11step_kernel...>:",
           "\ts_mov_b64 s[4:5], 0",
           "\ts_load_dwordx2 s[8:9], s[4:5], 0x10",
           "0000000000003000 <_ZN3mjl7callee...>:",
           "\ts_mov_b64 s[4:5], 0",
           "\ts_mov_b64 s[4:5], s[0:1]",
           "\ts_load_dword s8, s[4:5], 0x10"]
    hits = zeroed_base_loads(asm, kernels={"_ZN3mjl11step_kernel..."})
    assert hits == [("_ZN3mjl9env_resetI...", "s_load_dwordx2 s[8:9], s[4:5], 0x10")]


def _code_object(tmp_path):
    for tool in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump", "llvm-readelf"):
        if not os.path.exists(os.path.join(LLVM, tool)):
            pytest.skip(f"{tool} not in {LLVM}")
    if not os.path.exists(LIB):
        pytest.skip("libmjx355.so not built")
    fat, co = tmp_path / "fat.bin", tmp_path / "co.elf"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, str(tmp_path / "host.so")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def _scan_elf(co):
    """(kernels, non-kernel functions, hits) of a gfx950 code object."""
    syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "-W", str(co)], check=True, capture_output=True,
                          text=True).stdout
    kernels = {s[:-3] for s in re.findall(r"\s(\S+\.kd)\s*$", syms, re.M)}
    funcs = set(re.findall(r"\sFUNC\s+\S+\s+\S+\s+\S+\s+(\S+)\s*$", syms, re.M))
    asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", str(co)], check=True,
                         capture_output=True, text=True).stdout.splitlines()
    return kernels, funcs - kernels, zeroed_base_loads(asm, kernels)


# the round-5 bug in miniature: the segment pointer taken inside an out-of-line callee
_BAD_CALLEE = r"""
#include <hip/hip_runtime.h>
struct P { float* out; int n; int pad[30]; float* out2; };
__device__ __noinline__ void callee(int i) {
  const __attribute__((address_space(4))) P* p =
      (const __attribute__((address_space(4))) P*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  if (i < p->n) p->out2[i] = 1.f;
}
__global__ void kern(P a) { callee(threadIdx.x); a.out[threadIdx.x] = 2.f; }
"""


def test_scanner_catches_a_compiled_null_kernarg_callee(tmp_path):
    """Positive control on real compiler output: hipcc lowers the intrinsic in the callee to
    `s_mov_b64 s[2:3], 0` + `s_load_dword s0, s[2:3], 0x8`, and the scanner flags exactly that callee."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    src, obj = tmp_path / "k.hip", tmp_path / "k.o"
    src.write_text(_BAD_CALLEE)
    subprocess.run([hipcc, "-O2", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output", "-c",
                    "-o", str(obj), str(src)], check=True)
    kernels, callees, hits = _scan_elf(obj)
    assert callees == {"_Z6calleei"}
    assert hits and {f for f, _ in hits} == {"_Z6calleei"}


def test_shipped_code_object_has_no_zeroed_kernarg_loads(tmp_path):
    kernels, callees, hits = _scan_elf(_code_object(tmp_path))
    assert kernels and callees, "expected both kernels and called functions in the code object"
    assert any("env_reset" in f for f in callees)  # the function that faulted is out of line
    assert not hits, f"scalar loads through a zeroed SGPR pair in non-kernel functions: {hits[:5]}"


def test_debug_build_traps_on_null_kernarg_pointer():
    src = open(os.path.join(ROOT, "mujoco-mjx-lab_amd", "csrc", "step_kernels.hip")).read()
    body = src[src.index("INL const CSTA KParams* kparams_late()"):]
    body = body[:body.index("\n}\n")]
    assert "#ifdef MJL_DEBUG" in body and "__builtin_trap()" in body
    mk = subprocess.run(["make", "-n", "-C", os.path.join(ROOT, "mujoco-mjx-lab_amd", "csrc"), "debug"],
                        check=True, capture_output=True, text=True).stdout
    assert "-DMJL_DEBUG" in mk

"""Diagnostic: per-launch time of the twin update's dense kernels (mjl_twin_dense_fwd /
mjl_twin_dense_dx_tanh, tile shape from MJL_DENSE_CFG) against the library path they replace
(torch.bmm + mjl_bias_act, torch.bmm + mjl_tanh_bwd_colsum_partials), at the per-rank 8,192-row
minibatch of C5 and the 65,536-row one of C3. Prints one JSON line per (M, layer). Not product code."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

from mjx_amd._lib import check, lib  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


def main():
    L = lib()
    st = torch.cuda.current_stream().cuda_stream
    cfg = int(os.environ.get("MJL_DENSE_CFG", "0"))
    for M in (8192, 65536):
        for name, N, K, shared in (("fwd_l0", 256, 54, True), ("fwd_hidden", 256, 256, False), ("fwd_head", 21, 256, False)):
            x = torch.randn((1 if shared else 2, M, K), device="cuda")
            w = torch.randn((2, N, K), device="cuda") / K ** 0.5
            b = torch.randn((2, N), device="cuda")
            y = torch.empty((2, M, N), device="cuda")
            xe = x.expand(2, M, K)
            nat = timed(lambda: check(L.mjl_twin_dense_fwd(x.data_ptr(), 0 if shared else M * K, w.data_ptr(), b.data_ptr(),
                                                           2, M, N, K, 3, y.data_ptr(), st)))

            def lib_path():
                h = torch.bmm(xe, w.transpose(1, 2))
                check(L.mjl_bias_act(h.data_ptr(), b.data_ptr(), 2, M, N, 3, st))
            ref = timed(lib_path)
            fl = 2 * 2 * M * N * K
            print(json.dumps({"cfg": cfg, "M": M, "layer": name, "native_us": round(nat, 2), "bmm_plus_pass_us": round(ref, 2),
                              "native_tflops": round(fl / nat / 1e6, 1)}), flush=True)
        for name, N, K in (("dx_hidden", 256, 256), ("dx_head", 21, 256)):
            g = torch.randn((2, M, N), device="cuda")
            w = torch.randn((2, N, K), device="cuda") / N ** 0.5
            h = torch.tanh(torch.randn((2, M, K), device="cuda"))
            dz = torch.empty((2, M, K), device="cuda")
            R = int(L.mjl_twin_dense_partial_rows(M))
            part = torch.empty((2, R, K), device="cuda")
            nat = timed(lambda: check(L.mjl_twin_dense_dx_tanh(g.data_ptr(), w.data_ptr(), h.data_ptr(), 2, M, N, K,
                                                               dz.data_ptr(), part.data_ptr(), st)))
            part2 = torch.empty((2, M // 32, K), device="cuda")

            def lib_path():
                gg = torch.bmm(g, w)
                check(L.mjl_tanh_bwd_colsum_partials(gg.data_ptr(), h.data_ptr(), 2, M, K, 32, dz.data_ptr(),
                                                     part2.data_ptr(), st))
            ref = timed(lib_path)
            fl = 2 * 2 * M * N * K
            print(json.dumps({"cfg": cfg, "M": M, "layer": name, "native_us": round(nat, 2), "bmm_plus_pass_us": round(ref, 2),
                              "native_tflops": round(fl / nat / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

"""A/B of the two implicit record kernels (LDS rows vs global rows): which envs' states differ per step.
python tools/record_ab_probe.py [solver cg44|model] [pose overflow|none]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from mjx_amd import abi  # noqa: E402
from test_vjp_tape import _pair  # noqa: E402

solver = sys.argv[1] if len(sys.argv) > 1 else "cg44"
pose = sys.argv[2] if len(sys.argv) > 2 else "overflow"
m, (lds, glb) = _pair(solver, "implicit", B=32)
glb.env.data.set_option(abi.OPT_FORCE_GLOBAL_ROWS, 1)
B, H = 32, 8
for e in (lds, glb):
    e.enable_vjp_tape(H)
    e.reset()
st = lds.get_state()
if pose == "overflow":
    q = m.key_qpos[m.names["key"].index("supine")].copy()
    for j in range(1, m.njnt):
        q[m.jnt_qposadr[j]] = m.jnt_range[j][1] + 0.05
    st[0, :m.nq] = torch.tensor(q, dtype=torch.float32, device="cuda")
    st[0, m.nq:m.nq + 2 * m.nv] = 0.0
for e in (lds, glb):
    e.env.set_state(st)
g = torch.Generator(device="cuda").manual_seed(3)
for t in range(H):
    a = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
    lds.step_record(t, a)
    glb.step_record(t, a)
    for f in ("qpos", "qvel", "qacc_warmstart", "aux"):
        x, y = lds.env.data.get(f), glb.env.data.get(f)
        bad = (x != y).any(dim=1).nonzero().flatten().tolist()
        if bad:
            print(t, f, bad, float((x - y).abs().max()))
print("done")

"""Exploratory parity probe: HIP kernel vs oracle (fp64 and fp32) on a set of states."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mujoco-mjx-lab_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import mjx_amd
from mjx_amd import mjx
from oracle import Oracle, state_arrays

name = sys.argv[1] if len(sys.argv) > 1 else "humanoid_mjx"
m = mjx_amd.load_model(name)
rng = np.random.default_rng(0)
states = []
for k in range(m.nkey):
    states.append((m.key_qpos[k].copy(), np.zeros(m.nv), np.zeros(m.nu)))
od = Oracle(m)
for i in range(24):
    q = m.qpos0.copy(); q[7:] += rng.uniform(-0.3, 0.3, m.nq - 7)
    q[2] += rng.uniform(-0.25, 0.05)
    v = rng.uniform(-1, 1, m.nv); c = rng.uniform(-1, 1, m.nu)
    s = od.new_state(q, v, ctrl=c)
    nst = int(rng.integers(0, 60))
    if nst: od.rollout(s, rng.uniform(-1, 1, (nst, m.nu)))
    a = state_arrays(m, s)
    states.append((a["qpos"], a["qvel"], rng.uniform(-1, 1, m.nu)))
B = len(states)
sys_ = mjx.put_model(m)
d = mjx.make_data(sys_, B)
Q = torch.tensor(np.array([s[0] for s in states]), dtype=torch.float32)
V = torch.tensor(np.array([s[1] for s in states]), dtype=torch.float32)
U = torch.tensor(np.array([s[2] for s in states]), dtype=torch.float32)
d.set("qpos", Q.cuda()); d.set("qvel", V.cuda()); d.set("ctrl", U.cuda())
mjx.forward(sys_, d)
torch.cuda.synchronize()
fields = ["qacc", "qacc_smooth", "qfrc_bias", "qfrc_passive", "qfrc_actuator", "qfrc_constraint", "xpos", "sensordata", "stats"]
G = {f: d.get(f).cpu().numpy() for f in fields}
of = Oracle(m, use_float=True)
for tag, orc in (("f64", od), ("f32", of)):
    errs = {f: [] for f in fields[:-1]}
    for i, (q, v, c) in enumerate(states):
        s = orc.new_state(np.float32(q), np.float32(v), ctrl=np.float32(c))
        orc.forward(s); a = state_arrays(m, s)
        for f in fields[:-1]:
            ref = a[f].reshape(-1); got = G[f][i].reshape(-1)[: ref.size]
            errs[f].append(np.abs(ref - got).max() / (1 + np.abs(ref).max()))
        if tag == "f64" and i < 8:
            print(i, "ncon/nefc/iter gpu", G["stats"][i], "orc", a["ncon"], a["nefc"], a["niter"])
    print(tag, {f: "%.2e" % np.max(e) for f, e in errs.items()})
# step parity (1 step)
d2 = mjx.make_data(sys_, B)
d2.set("qpos", Q.cuda()); d2.set("qvel", V.cuda())
mjx.step(sys_, d2, U.cuda()); torch.cuda.synchronize()
q1 = d2.get("qpos").cpu().numpy(); v1 = d2.get("qvel").cpu().numpy()
eq, ev = [], []
for i, (q, v, c) in enumerate(states):
    s = od.new_state(np.float32(q), np.float32(v), ctrl=np.float32(c)); od.step(s); a = state_arrays(m, s)
    eq.append(np.abs(a["qpos"] - q1[i]).max()); ev.append(np.abs(a["qvel"] - v1[i]).max() / (1 + np.abs(a["qvel"]).max()))
print("step qpos err max %.2e  qvel rel err max %.2e" % (max(eq), max(ev)))
# speedtest
vel = torch.linspace(0, 1, 64).cuda()
out = mjx.speedtest_step(sys_, mjx.make_data(sys_, 64), vel); torch.cuda.synchronize()
ref = od.speedtest(vel.cpu().numpy().astype(np.float64))
print("speedtest max err %.2e" % np.abs(out.cpu().numpy() - ref).max())
# timing
for B in (2048, 4096):
    dd = mjx.make_data(sys_, B); vel = torch.linspace(0, 1, B).cuda(); out = torch.empty_like(vel)
    for _ in range(3): mjx.speedtest_step(sys_, dd, vel, out)
    torch.cuda.synchronize(); t = time.time(); n = 20
    for _ in range(n): mjx.speedtest_step(sys_, dd, vel, out)
    torch.cuda.synchronize(); dt = time.time() - t
    print(f"speedtest B={B}: {B*n/dt:,.0f} steps/s ({dt/n*1e3:.3f} ms/step)")

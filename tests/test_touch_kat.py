"""Touch-sensor known answers from MuJoCo's documented semantics, on the oracle and on the HIP kernel
(the touch sensor's site-box test was pinned only by oracle-vs-kernel agreement).

MuJoCo's touch sensor (XML reference, `sensor/touch`; engine_sensor.c mjSENS_TOUCH; MJX sensor.py):
the sum of the normal forces of the contacts of the site's body whose point lies in the site's box, or
whose normal ray — pointing out of the site's body — enters the box. The humanoid's foot sensors
(models/humanoid_mjx.xml:145,163,261-262) feed envs.py:89-106's stance terms.

A capsule lying on the floor (two plane-capsule contacts at its end caps, each carrying half the
weight by symmetry) with four box sites on its body:
  all    the whole capsule                               -> m g
  half   the x > 0 half (one contact point inside)        -> m g / 2
  above  a box above the capsule (no point, ray goes down) -> 0
  below  a box under the floor (the ray from each contact, pointing out of the capsule, enters it) -> m g
"""
import numpy as np
import pytest
import torch

from mjx_amd import mjcf

XML = """<mujoco><option timestep="0.005"/><worldbody><geom type="plane" size="0 0 1"/>
  <body pos="0 0 0.05"><freejoint/><geom type="capsule" fromto="-0.2 0 0 0.2 0 0" size="0.05"/>
    <site name="all" type="box" pos="0 0 0" size="0.3 0.1 0.1"/>
    <site name="half" type="box" pos="0.15 0 0" size="0.15 0.1 0.1"/>
    <site name="above" type="box" pos="0 0 0.2" size="0.3 0.1 0.05"/>
    <site name="below" type="box" pos="0 0 -0.25" size="0.3 0.1 0.05"/>
  </body></worldbody>
  <sensor><touch site="all"/><touch site="half"/><touch site="above"/><touch site="below"/></sensor></mujoco>"""


def _expected(m):
    w = m.body_mass[1] * 9.81
    return np.array([w, 0.5 * w, 0.0, w])


def test_touch_kat_oracle():
    from oracle import Oracle, state_arrays
    m = mjcf.compile_xml_string(XML)
    o = Oracle(m)
    s = o.new_state()
    o.step(s, 400)
    o.forward(s)
    a = state_arrays(m, s)
    assert a["ncon"] == 2 and np.abs(a["qvel"]).max() < 1e-6
    np.testing.assert_allclose(a["sensordata"], _expected(m), rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_touch_kat_on_gpu():
    """The same on the fp32 kernel (rtol 2e-3: the steady-state soft-contact forces in fp32)."""
    from mjx_amd import mjx
    m = mjcf.compile_xml_string(XML)
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, 3)
    q = np.tile(m.qpos0, (3, 1))
    q[:, 0] = [0.0, 1.0, -2.0]  # translated copies read the same
    d.set("qpos", torch.tensor(q, dtype=torch.float32))
    for _ in range(400):
        mjx.step(sys_, d)
    mjx.forward(sys_, d)
    sd = d.get("sensordata").cpu().numpy().astype(np.float64)
    st = d.get("stats").cpu().numpy()
    assert np.all(st[:, 0] == 2)
    for i in range(3):
        np.testing.assert_allclose(sd[i], _expected(m), rtol=2e-3, atol=1e-6)

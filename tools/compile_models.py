"""Compile the reference's MJCF models into the package's pre-compiled JSON assets.

Run in the build container (where /root/reference exists):
    python tools/compile_models.py /root/reference/models
The JSON holds only compiled numeric constants (masses, inertias, frames, pair tables ...)
produced by mjx_amd/mjcf.py, plus the source file's sha256.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mujoco-mjx-lab_amd"))
from mjx_amd import ASSETS, mjcf  # noqa: E402


def main(src_dir):
    os.makedirs(ASSETS, exist_ok=True)
    for name in ("humanoid_mjx", "humanoid"):
        m = mjcf.compile_xml(os.path.join(src_dir, name + ".xml"))
        out = os.path.join(ASSETS, name + ".json")
        with open(out, "w") as f:
            json.dump(m.to_json_dict(), f)
        print(f"{out}: nq={m.nq} nv={m.nv} npair={m.npair} mass={m.body_mass.sum():.4f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/models")

"""mjx_amd — MI355X-native batched humanoid physics step + on-policy trainers.

Host-side mirror of the reference's interface (son-engr-kr/mujoco-mjx-lab): model compile
(`mjcf`), the mjx-shaped device API (`mjx`), the batched walker env (`envs`), networks and the
PPO/APG trainers. Every physics call goes to the native library libmjx355.so (HIP, gfx950).
"""
import os

from .config import APGConfig, EnvConfig, PPOConfig, reference_ppo_config
from .mjcf import CompiledModel, MJCFError, compile_xml, compile_xml_string

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")
BUILTIN_MODELS = ("humanoid_mjx", "humanoid")


def load_model(name_or_path: str) -> CompiledModel:
    """`mujoco.MjModel.from_xml_path` analog. Accepts an MJCF path, a compiled `.json`, or one
    of the built-in names ("humanoid_mjx", "humanoid", also "models/humanoid_mjx.xml" as the
    reference writes it) which resolve to the pre-compiled assets shipped with the package."""
    from . import mjcf
    base = os.path.splitext(os.path.basename(name_or_path))[0]
    if not os.path.exists(name_or_path) and base in BUILTIN_MODELS:
        return mjcf.load_model(os.path.join(ASSETS, base + ".json"))
    return mjcf.load_model(name_or_path)

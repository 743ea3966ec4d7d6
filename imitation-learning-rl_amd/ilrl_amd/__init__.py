"""ilrl_amd - MI355X-native vectorised humanoid imitation environment.

Hot path of AdityaPutraS/Imitation-Learning-RL (`LowLevelHumanoidEnv.step()/reset()` + imitation
reward) as hand-written HIP kernels for gfx950 behind the C-ABI in include/humanoid_env.h.
"""
from .clips import CLIP_NAMES, Clip, load_clip  # noqa: F401

__all__ = ["CLIP_NAMES", "Clip", "load_clip", "HumanoidVecEnv", "LowLevelHumanoidEnv", "HumanoidVectorEnv"]


def __getattr__(name):   # lazy: torch/HIP are only needed when an env is created
    if name == "HumanoidVecEnv":
        from .vec_env import HumanoidVecEnv
        return HumanoidVecEnv
    if name in ("LowLevelHumanoidEnv", "HumanoidVectorEnv"):
        from . import low_level_env
        return getattr(low_level_env, name)
    raise AttributeError(name)

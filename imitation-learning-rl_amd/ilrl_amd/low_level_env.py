"""Drop-in Python surface for the reference hot path, backed by the HIP kernel (no CPU fallback).

* `LowLevelHumanoidEnv`  - gym.Env-shaped single env with the reference's constructor, methods and
  attribute names (low_level_env.py:36-526): reset(resetYaw), resetFromFrame(...), step(action, debug),
  frame, cur_timestep, target, robot_pos, starting_robot_pos, usePredefinedTarget, predefinedTarget, ...
* `HumanoidVectorEnv`    - RLlib-1.2 VectorEnv protocol (vector_reset / reset_at / vector_step /
  get_unwrapped) over N lanes of ONE kernel launch per step; get_unwrapped() returns lane views with the
  attributes RewardLogCallback reads (custom_callback.py:43-80).
* `make_env_low`, `register_envs` - the registration contract of train_config.py:13-15,29,320-321.

gym and ray are optional imports (absent in this image); the spaces fall back to a minimal Box.
"""
import numpy as np

from . import _native as N
from .vec_env import HumanoidVecEnv

ENV_LOW = "HumanoidBulletEnv-v0-Low"


def _box(low, high, shape):
    try:
        from gym.spaces import Box
        return Box(low=low, high=high, shape=shape, dtype=np.float32)
    except Exception:  # gym absent: minimal stand-in with the attributes RLlib reads
        class _Box:
            def __init__(self):
                self.low = np.full(shape, low, dtype=np.float32)
                self.high = np.full(shape, high, dtype=np.float32)
                self.shape = tuple(shape)
                self.dtype = np.dtype(np.float32)

            def sample(self):
                return np.random.uniform(max(low, -1), min(high, 1), self.shape).astype(np.float32)
        return _Box()


OBS_SPACE = lambda: _box(-np.inf, np.inf, (8 + 17 * 2 + 14 * 2,))   # low_level_env.py:53-55
ACT_SPACE = lambda: _box(-1.0, 1.0, (17,))                          # flat_env.action_space


class _BookView:
    """Attribute view of one lane's bookkeeping (refreshed lazily after each step)."""

    _SCALARS = {"frame": int, "cur_timestep": int, "predefinedTargetIndex": int, "highLevelDegTarget": float,
                "lowTargetScore": float, "deltaJoints": float, "deltaVelJoints": float, "bodyPostureScore": float,
                "electricityScore": float, "jointLimitScore": float, "aliveReward": float,
                "delta_lowTargetScore": float}
    _VECS = {"target": 3, "starting_robot_pos": 3, "robot_pos": 3, "starting_ep_pos": 3, "walk_target": 2}
    # reference attributes that are constant 0 in the low-level env (custom_callback.py reads them)
    _ZERO = ("deltaEndPoints", "baseReward", "highTargetScore", "driftScore", "cumulative_driftScore")

    def _book(self):
        raise NotImplementedError

    def __getattr__(self, name):
        if name in _BookView._SCALARS:
            return _BookView._SCALARS[name](self._book()[N.BK[name]])
        if name in _BookView._VECS:
            k = N.BK[name]
            return self._book()[k:k + _BookView._VECS[name]].copy()
        if name in _BookView._ZERO:
            return 0
        raise AttributeError(name)


class LowLevelHumanoidEnv(_BookView):
    """Single-env view (n = 1 lane) with the reference signature (low_level_env.py:39)."""

    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 60}

    def __init__(self, reference_name="motion08_03", useCustomEnv=False, customRobot=None, seed=0, device=0,
                 precision="fp32", **physics):
        if useCustomEnv:
            raise NotImplementedError("useCustomEnv (heightfield terrain, humanoid.py:68-188) is out of scope")
        self.__dict__["_v"] = HumanoidVecEnv(1, clips=(reference_name,), seed=seed, device=device,
                                             precision=precision, **physics)
        self.__dict__["_cache"] = None
        self.__dict__["_debug"] = False
        self.__dict__["_pred_on"] = False
        self.__dict__["_pred"] = np.array([[]])
        self.observation_space = OBS_SPACE()
        self.action_space = ACT_SPACE()
        self.max_timestep = 3000
        self.skipFrame = 2
        self.targetLen = 5
        self.max_frame = self._v.clips[0].max_frame

    def __setattr__(self, name, value):
        if name == "usePredefinedTarget":
            self.__dict__["_pred_on"] = bool(value)
            self._sync_modes()
        elif name == "predefinedTarget":
            arr = np.asarray(value, dtype=np.float64)
            self.__dict__["_pred"] = arr
            if arr.size:
                self._v.set_predefined_targets(arr.reshape(-1, 3))
        else:
            self.__dict__[name] = value

    @property
    def usePredefinedTarget(self):
        return self._pred_on

    @property
    def predefinedTarget(self):
        return self._pred

    def _sync_modes(self):
        self._v.set_modes(debug=self._debug, predefined=self._pred_on)

    def _book(self):
        if self._cache is None:
            self.__dict__["_cache"] = self._v.get_state()[1][0]
        return self._cache

    def _obs(self, t):
        self.__dict__["_cache"] = None
        return t[0].double().cpu().numpy()

    def reset(self, resetYaw=0):                                        # low_level_env.py:224-232
        return self._obs(self._v.reset(reset_yaw=float(resetYaw)))

    def resetFromFrame(self, startFrame=0, resetYaw=0, startFromRef=True, initVel=True):   # :247-305
        if not (startFromRef and initVel):
            raise NotImplementedError("resetFromFrame supports startFromRef=True, initVel=True (all reference callers)")
        return self._obs(self._v.reset(start_frame=int(startFrame), reset_yaw=float(resetYaw)))

    def step(self, action, debug=False):                                # :322-323, :475-526
        a = np.asarray(action, dtype=np.float32).reshape(1, 17)
        assert np.isfinite(a).all()                                     # humanoid.py:55
        if bool(debug) != self._debug:
            self.__dict__["_debug"] = bool(debug)
            self._sync_modes()
        obs, rew, done, _ = self._v.step(a)
        o = self._obs(obs)
        return o, float(rew[0].item()), bool(done[0].item()), {}

    def close(self):
        self._v.close()

    def render(self, mode="human"):
        raise NotImplementedError("rendering is out of scope (env_vis_low.py)")


class LaneView(_BookView):
    """get_unwrapped()[i] of HumanoidVectorEnv: reference attribute names for lane i."""

    def __init__(self, venv, i):
        self.__dict__["_venv"] = venv
        self.__dict__["_i"] = i

    def _book(self):
        return self._venv._books()[self._i]


class HumanoidVectorEnv:
    """RLlib 1.2 `VectorEnv` protocol over N lanes (one kernel launch per vector_step).

    vector_step returns the terminal observation for done lanes (gym semantics); the sampler then calls
    reset_at(i), which is served from the auto-reset buffer the same launch already filled.
    """

    def __init__(self, num_envs, reference_name="motion09_03", seed=0, device=0, precision="fp32",
                 clips=None, **physics):
        clips = clips or (reference_name,)
        self.venv = HumanoidVecEnv(num_envs, clips=clips, seed=seed, device=device, precision=precision, **physics)
        self.num_envs = num_envs
        self.observation_space = OBS_SPACE()
        self.action_space = ACT_SPACE()
        self._book_cache = None
        self._reset_obs = None
        self._views = [LaneView(self, i) for i in range(num_envs)]

    def _books(self):
        if self._book_cache is None:
            self._book_cache = self.venv.get_state()[1]
        return self._book_cache

    def vector_reset(self):
        obs = self.venv.reset().cpu().numpy()
        self._book_cache = None
        return [o for o in obs]

    def reset_at(self, index):
        if self._reset_obs is not None and self._reset_pending[index]:
            self._reset_pending[index] = False
            return self._reset_obs[index]
        mask = np.zeros(self.num_envs, dtype=np.uint8)
        mask[index] = 1
        obs = self.venv.reset(mask=mask)[index].cpu().numpy()
        self._book_cache = None
        return obs

    def vector_step(self, actions):
        a = np.asarray(actions, dtype=np.float32).reshape(self.num_envs, 17)
        obs, rew, done, _ = self.venv.step(a, autoreset=True)
        o, r, d = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        if self.venv.error_flags() & N.HUM_EFLAG_NONFINITE_ACTION:
            raise AssertionError("non-finite action (humanoid.py:55)")
        self._reset_obs = self.venv.obs_reset.cpu().numpy()
        self._reset_pending = d.copy()
        self._book_cache = None
        return [x for x in o], [float(x) for x in r], [bool(x) for x in d], [{} for _ in range(self.num_envs)]

    def get_unwrapped(self):
        return self._views

    def try_render_at(self, index=None):
        return None


def make_env_low(env_config=None):
    """train_config.py:13-15 (clip motion09_03; env_config ignored like the reference)."""
    return LowLevelHumanoidEnv(reference_name="motion09_03")


def register_envs():
    """register_env(ENV_LOW, make_env_low) (train_config.py:321) when Ray is importable."""
    from ray.tune.registry import register_env
    register_env(ENV_LOW, make_env_low)
    return ENV_LOW

"""Drop-in Python surface for the reference hot path, backed by the HIP kernel (no CPU fallback).

* `LowLevelHumanoidEnv`  - gym.Env-shaped single env with the reference's constructor, methods and
  attribute names (low_level_env.py:36-526): reset(resetYaw), resetFromFrame(...), step(action, debug),
  frame, cur_timestep, target, robot_pos, starting_robot_pos, usePredefinedTarget, predefinedTarget, ...
* `HumanoidVectorEnv`    - RLlib-1.2 VectorEnv protocol (vector_reset / reset_at / vector_step /
  get_unwrapped) over N lanes of ONE kernel launch per step; get_unwrapped() returns lane views with the
  attributes RewardLogCallback reads (custom_callback.py:43-80).
* `make_env_low`, `make_env_low_vec`, `register_envs` - the registration contract of train_config.py:13-15,29,
  320-321: `make_env_low` returns the single-env gym view (one lane per env, the reference's shape);
  `make_env_low_vec` returns ONE N-lane `HumanoidVectorEnv` per RLlib worker, which RLlib uses as the worker's
  vector env directly (BaseEnv.to_base_env recognises VectorEnv subclasses), so a sampler step is one launch.

gym and ray are optional imports (absent in this image): `LowLevelHumanoidEnv` subclasses gym.Env and
`HumanoidVectorEnv` subclasses ray.rllib.env.vector_env.VectorEnv when those import; the spaces fall back to
a minimal Box.
"""
import gc
import secrets

import numpy as np

from . import _native as N
from .vec_env import HostStaging, HumanoidVecEnv

ENV_LOW = "HumanoidBulletEnv-v0-Low"


def _optional_base(module, name):
    try:
        mod = __import__(module, fromlist=[name])
        return getattr(mod, name)
    except Exception:
        return object


def env_seed(env_config=None, n_lanes=1):
    """(seed, lane_offset) for an env built by a registration creator.  The reference draws from an unseeded
    np.random.default_rng() per env (low_level_env.py:84), so copies never share a stream: an explicit
    env_config["seed"] is honoured, RLlib's worker_index / vector_index give each copy its own global lanes,
    and without a seed the job seed comes from OS entropy."""
    cfg = env_config if env_config is not None else {}
    seed = cfg.get("seed") if hasattr(cfg, "get") else None
    if seed is None:
        seed = secrets.randbits(63)
    worker = int(getattr(cfg, "worker_index", 0) or 0)
    vector = int(getattr(cfg, "vector_index", 0) or 0)
    return int(seed), (worker * 4096 + vector) * int(n_lanes)


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


class LowLevelHumanoidEnv(_BookView, _optional_base("gym", "Env")):
    """Single-env view (n = 1 lane) with the reference signature (low_level_env.py:39)."""

    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 60}

    def __init__(self, reference_name="motion08_03", useCustomEnv=False, customRobot=None, seed=None, device=0,
                 precision="fp32", lane_offset=0, **physics):
        if seed is None:   # the reference's unseeded default_rng() (:84): a fresh stream per env
            seed = secrets.randbits(63)
        self.__dict__["_v"] = HumanoidVecEnv(1, clips=(reference_name,), seed=seed, device=device,
                                             lane_offset=lane_offset, precision=precision, **physics)
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
        self.__dict__["_n_vel"] = int(self._v.clips[0].vel.shape[0])
        self.useCustomEnv = bool(useCustomEnv)
        if self.useCustomEnv:   # :41-42 CustomHumanoid: CustomScene's random heightfield instead of the plane
            self._v.set_terrain(N.HUM_TERRAIN_RANDOM_BLOCKS)
            self.__dict__["flat_env"] = _CustomEnvView(self._v)

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

    def _scene_restart(self):
        # flat_env.reset() -> CustomScene.episode_restart: a fresh random terrain, whatever replaceHeightfieldData
        # installed during the previous episode (humanoid.py:89-113)
        if self.useCustomEnv and self._v.terrain != N.HUM_TERRAIN_RANDOM_BLOCKS:
            self._v.set_terrain(N.HUM_TERRAIN_RANDOM_BLOCKS)

    def _vel_row_check(self, when):
        """The reference reads JointSpeedRadSec.iloc[frame] (low_level_env.py:208, :310, :345): motion13_13 has 120
        velocity rows for 220 pose rows, so once the frame reaches the table's end pandas raises IndexError there.
        (Vector / benchmark handles keep stepping on the clamped last row and flag HUM_EFLAG_VEL_ROW instead.)"""
        if self.frame >= self._n_vel:
            raise IndexError("single positional indexer is out-of-bounds (%s: frame %d, %d velocity rows)"
                             % (when, self.frame, self._n_vel))

    def reset(self, resetYaw=0):                                        # low_level_env.py:224-232
        self._scene_restart()
        o = self._obs(self._v.reset(reset_yaw=float(resetYaw)))
        self._vel_row_check("reset")
        return o

    def resetFromFrame(self, startFrame=0, resetYaw=0, startFromRef=True, initVel=True):   # :247-305
        if startFromRef and not 0 <= int(startFrame) < self.max_frame + 1:   # DataFrame.iloc (:208) raises
            raise IndexError("single positional indexer is out-of-bounds (startFrame=%d)" % int(startFrame))
        self._scene_restart()
        o = self._obs(self._v.reset(start_frame=int(startFrame), reset_yaw=float(resetYaw),
                                    start_from_ref=startFromRef, init_vel=initVel))
        self._vel_row_check("resetFromFrame")
        return o

    def step(self, action, debug=False):                                # :322-323, :475-526
        a = np.asarray(action, dtype=np.float32).reshape(1, 17)
        assert np.isfinite(a).all()                                     # humanoid.py:55
        self._vel_row_check("step")                                     # :345 calcJointVelScore
        if bool(debug) != self._debug:
            self.__dict__["_debug"] = bool(debug)
            self._sync_modes()
        obs, rew, done, _ = self._v.step(a)
        o = self._obs(obs)
        self._vel_row_check("step")                                     # :310 getLowLevelObs after incFrame
        return o, float(rew[0].item()), bool(done[0].item()), {}

    def close(self):
        self._v.close()

    def render(self, mode="human"):
        raise NotImplementedError("rendering is out of scope (env_vis_low.py)")


class _CustomSceneView:
    """flat_env.stadium_scene of a useCustomEnv env (humanoid.py:68-86 CustomScene): replaceHeightfieldData(d)
    installs a 256 x 256 heightfield (d[i + j*256], i along x) at z 0.25 until the next reset, as in
    env_vis_low.py:155-171."""
    numHeightfieldRows = 256
    numHeightfieldColumns = 256

    def __init__(self, venv):
        self._venv = venv
        self.heightfieldData = [0] * (self.numHeightfieldRows * self.numHeightfieldColumns)

    # btHeightfieldTerrainShape's vertical centre from the CustomScene creation terrain (random blocks in [0, 0.5)
    # with a zero centre patch: (min + max) / 2 ~ 0.25); pybullet's replaceHeightfieldIndex path keeps it
    CREATION_CENTRE = 0.25

    def replaceHeightfieldData(self, newData):
        self.heightfieldData = list(newData)
        self._venv.set_terrain(N.HUM_TERRAIN_HEIGHTFIELD, heights=np.asarray(self.heightfieldData, dtype=np.float32),
                               w=self.numHeightfieldRows, l=self.numHeightfieldColumns, scale=(1.0, 1.0, 1.0),
                               origin=(0.0, 0.0, 0.25), centre=self.CREATION_CENTRE)


class _CustomEnvView:
    """flat_env of a useCustomEnv env: the CustomHumanoid scene handle (stadium_scene)."""

    def __init__(self, venv):
        self.stadium_scene = _CustomSceneView(venv)


# RewardLogCallback attributes (custom_callback.py:43-80) served from the device aux row of ONE lane
_AUX_ATTR = {"deltaJoints": "deltaJoints", "deltaEndPoints": "deltaEndPoints", "lowTargetScore": "lowTargetScore",
             "deltaVelJoints": "deltaVelJoints", "bodyPostureScore": "bodyPostureScore",
             "highTargetScore": "highTargetScore", "driftScore": "driftScore", "baseReward": "baseReward",
             "aliveReward": "aliveReward", "electricityScore": "electricityScore",
             "jointLimitScore": "jointLimitScore"}


class LaneView(_BookView):
    """get_unwrapped()[i] of HumanoidVectorEnv: reference attribute names for lane i.  The callback terms and
    robot_pos come from lane i's row of hum_get_aux (one small device->host copy per step, cached); the other
    bookkeeping attributes (frame, target, ...) from a full state read."""

    def __init__(self, venv, i):
        self.__dict__["_venv"] = venv
        self.__dict__["_i"] = i

    def _book(self):
        return self._venv._books()[self._i]

    def __getattr__(self, name):
        if name in _AUX_ATTR:
            return float(self._venv._aux_row(self._i)[N.AUX.index(_AUX_ATTR[name])])
        if name == "robot_pos":
            k = N.AUX.index("robot_pos_x")
            return self._venv._aux_row(self._i)[k:k + 3].astype(np.float64)
        return _BookView.__getattr__(self, name)


class HumanoidVectorEnv(_optional_base("ray.rllib.env.vector_env", "VectorEnv")):
    """RLlib 1.2 `VectorEnv` over N lanes (one kernel launch per vector_step); a subclass of RLlib's VectorEnv
    when ray imports, so `BaseEnv.to_base_env` drives it directly.

    vector_step returns the terminal observation for done lanes (gym semantics); the sampler then calls
    reset_at(i), which is served from the auto-reset buffer the same launch already filled.
    """

    def __init__(self, num_envs, reference_name="motion09_03", seed=None, device=0, precision="fp32",
                 clips=None, lane_offset=0, **physics):
        clips = clips or (reference_name,)
        if seed is None:
            seed = secrets.randbits(63)
        self.venv = HumanoidVecEnv(num_envs, clips=clips, seed=seed, device=device, lane_offset=lane_offset,
                                   precision=precision, **physics)
        self.num_envs = num_envs
        self.observation_space = OBS_SPACE()
        self.action_space = ACT_SPACE()
        if type(self).__mro__[1] is not object:   # ray's VectorEnv.__init__(observation_space, action_space, n)
            super().__init__(self.observation_space, self.action_space, num_envs)
        self._book_cache = None
        self._aux_rows = {}
        self._reset_rows = {}
        self._act_dev = None
        self._io = None
        self._views = [LaneView(self, i) for i in range(num_envs)]

    def _books(self):
        if self._book_cache is None:
            self._book_cache = self.venv.get_state()[1]
        return self._book_cache

    def _aux_row(self, i):
        if i not in self._aux_rows:
            if not self._aux_rows:
                self.venv.get_aux()
            self._aux_rows[i] = self.venv.aux[i].cpu().numpy()
        return self._aux_rows[i]

    def _invalidate(self):
        self._book_cache = None
        self._aux_rows = {}

    def vector_reset(self):
        obs = self.venv.reset().cpu().numpy()
        self._invalidate()
        self._reset_rows = {}
        return list(obs)

    def reset_at(self, index):
        row = self._reset_rows.pop(index, None)
        if row is not None:   # the auto-reset observation the step launch already produced for this lane
            return row
        mask = np.zeros(self.num_envs, dtype=np.uint8)
        mask[index] = 1
        obs = self.venv.reset(mask=mask)[index].cpu().numpy()
        self._invalidate()
        return obs

    def vector_step(self, actions):
        """One launch for every lane.  Host work is kept to what the VectorEnv API needs: the actions (RLlib hands a
        list of per-env rows) are stacked once and uploaded through a pinned buffer; obs / reward / done come back
        through pinned buffers with one stream synchronize; only the done lanes' auto-reset rows are fetched
        (reset_at serves them); rewards and dones become Python lists in one call each."""
        a = actions if isinstance(actions, np.ndarray) else np.concatenate(actions)
        a = np.asarray(a, dtype=np.float32).reshape(self.num_envs, 17)
        if not np.isfinite(a).all():   # humanoid.py:55, checked on the host copy RLlib hands over (no device sync)
            raise AssertionError("non-finite action (humanoid.py:55)")
        v = self.venv
        if self._act_dev is None:
            self._act_dev = v.torch.empty(self.num_envs, 17, dtype=v.torch.float32, device=v.device)
            self._io = HostStaging(v.torch, v.device)
        obs, rew, done, _ = v.step(self._io.upload("act", a, self._act_dev), autoreset=True)
        h = self._io.fetch(obs=obs, rew=rew, done=done)
        o = h["obs"].copy()   # the rows handed out outlive the pinned buffer
        d = h["done"].astype(bool)
        self._reset_rows = {}
        idx = np.flatnonzero(d)
        if idx.size:   # the done lanes' auto-reset observations only (reset_at serves them)
            rows = self._io.fetch_rows("reset", v.obs_reset.index_select(0, v.torch.from_numpy(idx).to(v.device)),
                                       self.num_envs).copy()
            self._reset_rows = dict(zip(idx.tolist(), rows))
        self._invalidate()
        gc_on = gc.isenabled()   # ~2 n acyclic objects follow: keep the cyclic collector from rescanning them
        gc.disable()
        try:
            return list(o), h["rew"].tolist(), d.tolist(), [{} for _ in range(self.num_envs)]
        finally:
            if gc_on:
                gc.enable()

    def get_unwrapped(self):
        return self._views

    def try_render_at(self, index=None):
        return None


def make_env_low(env_config=None):
    """train_config.py:13-15: one single-lane env per call (clip motion09_03), each with its own RNG stream
    (env_seed: env_config["seed"] / RLlib worker and vector index, else OS entropy)."""
    seed, off = env_seed(env_config, 1)
    return LowLevelHumanoidEnv(reference_name="motion09_03", seed=seed, lane_offset=off)


def make_env_low_vec(env_config=None):
    """One N-lane VectorEnv per RLlib worker (env_config["num_lanes"], default 1024; clip motion09_03): RLlib
    uses a VectorEnv as the worker's vector env as-is, so every sampler step is one kernel launch."""
    cfg = env_config if env_config is not None else {}
    n = int(cfg.get("num_lanes", 1024)) if hasattr(cfg, "get") else 1024
    seed, off = env_seed(env_config, n)
    return HumanoidVectorEnv(n, reference_name="motion09_03", seed=seed, lane_offset=off)


def register_envs(vectorised=True):
    """register_env(ENV_LOW, ...) (train_config.py:321) when Ray is importable: the N-lane vector env per worker
    (default), or the reference's one-env-per-call creator."""
    from ray.tune.registry import register_env
    register_env(ENV_LOW, make_env_low_vec if vectorised else make_env_low)
    return ENV_LOW

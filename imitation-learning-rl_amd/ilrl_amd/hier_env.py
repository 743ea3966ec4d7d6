"""Drop-in Python surface for the reference's two-level env, backed by the same HIP kernel (no CPU fallback).

* `HierVecEnv` - N device-resident lanes of `HierarchicalHumanoidEnv` (hier_env.py:38-641) on one GPU; one
  `hum_hier_step` launch advances every lane by one agent transition: lanes whose acting agent is the high level
  run high_level_step (heading -> walk target, no physics), the others low_level_step (4 physics substeps +
  imitation reward + level hand-back every 5 steps).
* `HierarchicalHumanoidEnv` - the reference's single-env MultiAgentEnv view (reset() / resetFromFrame() /
  step(action_dict, debug)) returning the same {"high_level_agent": ..., "low_level_agent": ...} dicts, with
  the reference's attribute names (target, robot_pos, highTargetScore, driftScore, steps_remaining_at_level, ...).
* `HierarchicalVectorEnv` - RLlib 1.2 has no vectorised MultiAgentEnv, so the drop-in for N lanes is a
  `BaseEnv` (poll / send_actions / try_reset / get_unwrapped) over one HierVecEnv.
* `make_env_hier`, `register_envs` - train_config.py:18-20,320.

ray is optional (absent in this image): BaseEnv is subclassed only when importable.
"""
import gc
import secrets

import numpy as np

from . import _native as N
from .low_level_env import _box, _BookView, _optional_base, env_seed
from .vec_env import HostStaging, HumanoidVecEnv, _ptr

ENV_HIER = "HumanoidBulletEnv-v0-Hier"
HIGH, LOW = "high_level_agent", "low_level_agent"
HIER_CLIP = "motion09_03"   # motion_list[selected_motion] (hier_env.py:50,170)

HIGH_OBS_SPACE = lambda: _box(-np.inf, np.inf, (8 + 17 * 2 + 2,))      # hier_env.py:52
HIGH_ACT_SPACE = lambda: _box(-1.0, 1.0, (2,))                          # :53-55
LOW_OBS_SPACE = lambda: _box(-np.inf, np.inf, (8 + 17 * 2 + 14 * 2,))   # :57
LOW_ACT_SPACE = lambda: _box(-1.0, 1.0, (17,))                          # :58


class HierVecEnv(HumanoidVecEnv):
    """N lanes of HierarchicalHumanoidEnv behind hum_hier_reset / hum_hier_step (include/humanoid_env.h)."""

    def __init__(self, n, clip=HIER_CLIP, seed=0, device=0, lane_offset=0, precision="fp32", **physics):
        super().__init__(n, clips=(clip,), seed=seed, device=device, lane_offset=lane_offset, precision=precision,
                         hier=1, **physics)
        t, f32 = self.torch, self.torch.float32
        self.obs_high = t.zeros(self.n, N.HUM_NOBS_HIGH, dtype=f32, device=self.device)
        self.obs_high_reset = t.zeros(self.n, N.HUM_NOBS_HIGH, dtype=f32, device=self.device)
        self.reward_high = t.zeros(self.n, dtype=f32, device=self.device)
        self.agents = t.zeros(self.n, dtype=t.uint8, device=self.device)
        self._zero_high = t.zeros(self.n, N.HUM_NACT_HIGH, dtype=f32, device=self.device)
        self._zero_low = t.zeros(self.n, N.HUM_NACT, dtype=f32, device=self.device)

    def reset(self, mask=None, start_frame=None, reset_yaw=None, start_from_ref=True, init_vel=True):
        """reset() (start_frame None: startFrame and resetYaw drawn per lane) or resetFromFrame(); -> [n,44]."""
        m, sf, ry, flags = self._reset_args(mask, start_frame, reset_yaw, start_from_ref, init_vel)
        N.check(N.lib().hum_hier_reset_ex(self.h, _ptr(m), _ptr(sf), _ptr(ry), flags, _ptr(self.obs_high),
                                          self._stream()), "hum_hier_reset")
        self._clear_done(m)
        return self.obs_high

    def _act(self, a, width, zero):
        if a is None:
            return zero
        t = self.torch
        a = t.as_tensor(a, dtype=t.float32, device=self.device).contiguous()
        if a.shape != (self.n, width):
            raise ValueError("actions must be [%d, %d], got %s" % (self.n, width, tuple(a.shape)))
        return a

    def step(self, high_actions=None, low_actions=None, agent=None, autoreset=False, skip_physics=False):
        """One agent transition per lane.  Returns (agents, obs_high, obs_low, rew_high, rew_low, done, frame)."""
        t = self.torch
        ah = self._act(high_actions, N.HUM_NACT_HIGH, self._zero_high)
        al = self._act(low_actions, N.HUM_NACT, self._zero_low)
        ag = None if agent is None else t.as_tensor(agent, dtype=t.uint8, device=self.device).expand(self.n).contiguous()
        flags = (N.HUM_STEP_AUTORESET if autoreset else 0) | (N.HUM_STEP_SKIP_PHYSICS if skip_physics else 0)
        N.check(N.lib().hum_hier_step(self.h, _ptr(ah), _ptr(al), _ptr(ag), _ptr(self.agents), _ptr(self.obs_high),
                                      _ptr(self.obs), _ptr(self.reward_high), _ptr(self.reward), _ptr(self.done),
                                      _ptr(self.frame), flags, _ptr(self.obs_high_reset), self._stream()),
                "hum_hier_step")
        return self.agents, self.obs_high, self.obs, self.reward_high, self.reward, self.done, self.frame

    def step_k(self, high_actions, low_actions, agent=None, autoreset=False, skip_physics=False, out=None):
        """k agent transitions per lane in one launch (hum_hier_step_k).  high_actions [k,n,2], low_actions
        [k,n,17], agent [k,n] u8 or None (each lane's expected agent).  Returns device tensors (agents [k,n],
        obs_high [k,n,44], obs_low [k,n,70], rew_high [k,n], rew_low [k,n], done [k,n], frame [k,n],
        obs_high_reset [k,n,44]): row t is the t-th of k step() calls."""
        t = self.torch
        ah = t.as_tensor(high_actions, dtype=t.float32, device=self.device).contiguous()
        al = t.as_tensor(low_actions, dtype=t.float32, device=self.device).contiguous()
        k = ah.shape[0]
        if ah.shape != (k, self.n, N.HUM_NACT_HIGH) or al.shape != (k, self.n, N.HUM_NACT):
            raise ValueError("actions must be [k, %d, 2] and [k, %d, 17]" % (self.n, self.n))
        ag = None if agent is None else t.as_tensor(agent, dtype=t.uint8, device=self.device).expand(k, self.n).contiguous()
        if out is None or out[0].shape[0] != k:
            out = self.step_k_out(k)
        agents, oh, ol, rh, rl, done, frame, ohr = out
        flags = (N.HUM_STEP_AUTORESET if autoreset else 0) | (N.HUM_STEP_SKIP_PHYSICS if skip_physics else 0)
        N.check(N.lib().hum_hier_step_k(self.h, _ptr(ah), _ptr(al), _ptr(ag), _ptr(agents), _ptr(oh), _ptr(ol),
                                        _ptr(rh), _ptr(rl), _ptr(done), _ptr(frame), flags, _ptr(ohr), k,
                                        self._stream()), "hum_hier_step_k")
        return out

    def step_k_out(self, k):
        """A zeroed output tuple for step_k(..., out=) of k transitions (allocate it ahead of a timed loop)."""
        t, f32 = self.torch, self.torch.float32
        z = lambda *s, d=f32: t.zeros(*s, dtype=d, device=self.device)
        return (z(k, self.n, d=t.uint8), z(k, self.n, N.HUM_NOBS_HIGH), z(k, self.n, N.HUM_NOBS), z(k, self.n),
                z(k, self.n), z(k, self.n, d=t.uint8), z(k, self.n, d=t.int32), z(k, self.n, N.HUM_NOBS_HIGH))


class _HierBookView(_BookView):
    _HIER_SCALARS = {"selected_motion_frame": ("frame", int), "steps_remaining_at_level": (None, int),
                     "num_high_level_steps": (None, int), "highTargetScore": (None, float),
                     "driftScore": (None, float), "cumulative_driftScore": (None, float),
                     "delta_highTargetScore": (None, float), "cumulative_aliveReward": (None, float)}

    def __getattr__(self, name):
        if name in _HierBookView._HIER_SCALARS:
            key, typ = _HierBookView._HIER_SCALARS[name]
            return typ(self._book()[N.BK[key or name]])
        return _BookView.__getattr__(self, name)


class HierarchicalHumanoidEnv(_HierBookView):
    """Single-env MultiAgentEnv view (1 lane) with the reference signature (hier_env.py:43)."""

    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 60}

    def __init__(self, customRobot=None, seed=None, device=0, precision="fp32", lane_offset=0, **physics):
        if seed is None:   # the reference's unseeded default_rng() (hier_env.py:89)
            seed = secrets.randbits(63)
        self.__dict__["_v"] = HierVecEnv(1, seed=seed, device=device, lane_offset=lane_offset, precision=precision,
                                         **physics)
        self.__dict__["_cache"] = None
        self.__dict__["_debug"] = False
        self.__dict__["_pred_on"] = False
        self.__dict__["_pred"] = np.array([[]])
        self.high_level_obs_space = HIGH_OBS_SPACE()
        self.high_level_act_space = HIGH_ACT_SPACE()
        self.low_level_obs_space = LOW_OBS_SPACE()
        self.low_level_act_space = LOW_ACT_SPACE()
        self.motion_list = ["motion08_03", "motion09_03"]
        self.selected_motion = 1
        self.step_per_level = 5
        self.max_timestep = 3000
        self.skipFrame = 2
        self.targetLen = 5
        self.low_level_agent_id = LOW

    def __setattr__(self, name, value):
        if name == "usePredefinedTarget":
            self.__dict__["_pred_on"] = bool(value)
            self._v.set_modes(debug=self._debug, predefined=self._pred_on)
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

    def _book(self):
        if self._cache is None:
            self.__dict__["_cache"] = self._v.get_state()[1][0]
        return self._cache

    def reset(self):                                                    # hier_env.py:235-243
        self.__dict__["_cache"] = None
        return {HIGH: self._v.reset()[0].double().cpu().numpy()}

    def resetFromFrame(self, startFrame=0, resetYaw=0, startFromRef=True, initVel=True):   # :259-319
        if startFromRef and not 0 <= int(startFrame) < self._v.clips[0].pos.shape[0] - 1:   # iloc (:293-304)
            raise IndexError("single positional indexer is out-of-bounds (startFrame=%d)" % int(startFrame))
        self.__dict__["_cache"] = None
        return {HIGH: self._v.reset(start_frame=int(startFrame), reset_yaw=float(resetYaw), start_from_ref=startFromRef,
                                    init_vel=initVel)[0].double().cpu().numpy()}

    def step(self, action_dict, debug=False):                           # :355-366
        assert len(action_dict) == 1, action_dict
        if bool(debug) != self._debug:
            self.__dict__["_debug"] = bool(debug)
            self._v.set_modes(debug=self._debug, predefined=self._pred_on)
        if HIGH in action_dict:
            ah = np.asarray(action_dict[HIGH], dtype=np.float32).reshape(1, 2)
            out = self._v.step(high_actions=ah, agent=1)
        else:
            al = np.asarray(list(action_dict.values())[0], dtype=np.float32).reshape(1, 17)
            assert np.isfinite(al).all()                                # humanoid.py:55
            out = self._v.step(low_actions=al, agent=0)
        agents, oh, ol, rh, rl, done, _ = [x.cpu().numpy() for x in out]
        self.__dict__["_cache"] = None
        obs, rew = {}, {}
        if agents[0] & N.HUM_AGENT_HIGH:
            obs[HIGH] = oh[0].astype(np.float64)
            rew[HIGH] = float(rh[0])
        if agents[0] & N.HUM_AGENT_LOW:
            obs[LOW] = ol[0].astype(np.float64)
            rew[LOW] = float(rl[0])
        return obs, rew, {"__all__": bool(done[0])}, {}

    def close(self):
        self._v.close()

    def render(self, mode="human"):
        raise NotImplementedError("rendering is out of scope (env_vis_hier.py)")


class HierLaneView(_HierBookView):
    def __init__(self, venv, i):
        self.__dict__["_venv"] = venv
        self.__dict__["_i"] = i

    def _book(self):
        return self._venv._books()[self._i]


class HierarchicalVectorEnv(_optional_base("ray.rllib.env.base_env", "BaseEnv")):
    """RLlib 1.2 BaseEnv over N hierarchical lanes (one hum_hier_step launch per send_actions/poll round).

    poll() -> (obs, rewards, dones, infos, off_policy_actions) as {env_id: {agent_id: ...}} with
    dones[env_id]["__all__"]; send_actions({env_id: {agent_id: action}}); done lanes are reset inside the step
    launch and try_reset(env_id) serves the reset observation {"high_level_agent": obs}.
    """

    def __init__(self, num_envs, seed=None, device=0, precision="fp32", lane_offset=0, **physics):
        if seed is None:
            seed = secrets.randbits(63)
        self.venv = HierVecEnv(num_envs, seed=seed, device=device, lane_offset=lane_offset, precision=precision,
                               **physics)
        self.num_envs = num_envs
        self._views = [HierLaneView(self, i) for i in range(num_envs)]
        self._book_cache = None
        self._pending = None
        self._reset_rows = {}
        self._io = HostStaging(self.venv.torch, self.venv.device)
        t = self.venv.torch
        self._ah = np.zeros((num_envs, 2), np.float32)   # host staging of the per-env actions (rows of skipped
        self._al = np.zeros((num_envs, 17), np.float32)  # lanes / the other agent are never read by the kernel)
        self._dev = {"ah": t.empty(num_envs, 2, dtype=t.float32, device=self.venv.device),
                     "al": t.empty(num_envs, 17, dtype=t.float32, device=self.venv.device),
                     "ag": t.empty(num_envs, dtype=t.uint8, device=self.venv.device)}

    def _books(self):
        if self._book_cache is None:
            self._book_cache = self.venv.get_state()[1]
        return self._book_cache

    def _first_poll(self):
        oh = self.venv.reset().cpu().numpy().astype(np.float64)
        self._book_cache = None
        obs = {i: {HIGH: oh[i]} for i in range(self.num_envs)}
        return obs, {i: {HIGH: 0.0} for i in range(self.num_envs)}, \
            {i: {"__all__": False} for i in range(self.num_envs)}, {i: {HIGH: {}} for i in range(self.num_envs)}

    def poll(self):
        if self._pending is None:
            obs, rew, dones, infos = self._first_poll()
        else:
            obs, rew, dones, infos = self._pending
        self._pending = ({}, {}, {}, {})
        return obs, rew, dones, infos, {}

    def send_actions(self, action_dict):
        """Lanes absent from action_dict (RLlib did not act on them) are left unstepped (HUM_AGENT_SEL_SKIP).
        One pass over the per-env dicts sorts the actions by agent; they go up through pinned buffers, one launch
        runs, and every output comes back in one synchronize (the done lanes' reset rows in a second, only when a
        lane is done); the per-env result dicts are built from whole-array conversions."""
        n = self.num_envs
        items = action_dict.items()
        hi = [(i, ad[HIGH]) for i, ad in items if HIGH in ad]
        lo = [(i, ad[LOW]) for i, ad in items if LOW in ad]
        if len(hi) + len(lo) != len(action_dict):   # an env with both agents' actions, or neither's
            raise AssertionError("one action per env and transition (hier_env.py:355-366)")
        agent = np.full(n, N.HUM_AGENT_SEL_SKIP, np.uint8)
        if hi:
            ids, rows = zip(*hi)
            ids = np.fromiter(ids, np.int64, len(ids))
            self._ah[ids] = np.concatenate(rows).reshape(len(ids), 2)
            agent[ids] = 1
        if lo:
            ids, rows = zip(*lo)
            ids = np.fromiter(ids, np.int64, len(ids))
            la = np.concatenate(rows).reshape(len(ids), 17)
            if not np.isfinite(la).all():
                raise AssertionError("non-finite action (humanoid.py:55)")
            self._al[ids] = la
            agent[ids] = 0
        io, d, v = self._io, self._dev, self.venv
        out = v.step(io.upload("ah", self._ah, d["ah"]), io.upload("al", self._al, d["al"]),
                     agent=io.upload("ag", agent, d["ag"]), autoreset=True)
        agents, oh, ol, rh, rl, done, _ = out
        h = io.fetch(agents=agents, oh=oh, ol=ol, rh=rh, rl=rl, done=done)
        self._reset_rows = {}
        idx = np.flatnonzero(h["done"])
        if idx.size:   # the done lanes' auto-reset high-level observations only (try_reset serves them)
            rows = io.fetch_rows("reset", v.obs_high_reset.index_select(0, v.torch.from_numpy(idx).to(v.device)),
                                 n).astype(np.float64)
            self._reset_rows = dict(zip(idx.tolist(), rows))
        self._book_cache = None
        # the per-env result dicts, from whole-array conversions (the reference's float64 obs); the cyclic garbage
        # collector is paused while ~5 n acyclic containers are built (it would otherwise rescan them repeatedly)
        AH, AL = N.HUM_AGENT_HIGH, N.HUM_AGENT_LOW
        acted = list(action_dict)
        gc_on = gc.isenabled()
        gc.disable()
        try:
            ohr, olr = list(h["oh"].astype(np.float64)), list(h["ol"].astype(np.float64))
            rhl, rll, agl = h["rh"].tolist(), h["rl"].tolist(), h["agents"].tolist()
            dnl = h["done"].astype(bool).tolist()
            if len(acted) != n:
                agl = [agl[i] for i in acted]
                dnl = [dnl[i] for i in acted]
            obs = {i: ({HIGH: ohr[i]} if a == AH else {LOW: olr[i]} if a == AL else
                       {HIGH: ohr[i], LOW: olr[i]} if a == AH | AL else {}) for i, a in zip(acted, agl)}
            rew = {i: ({HIGH: rhl[i]} if a == AH else {LOW: rll[i]} if a == AL else
                       {HIGH: rhl[i], LOW: rll[i]} if a == AH | AL else {}) for i, a in zip(acted, agl)}
            infos = {i: ({HIGH: {}} if a == AH else {LOW: {}} if a == AL else
                         {HIGH: {}, LOW: {}} if a == AH | AL else {}) for i, a in zip(acted, agl)}
            dones = {i: {"__all__": x} for i, x in zip(acted, dnl)}
        finally:
            if gc_on:
                gc.enable()
        self._pending = (obs, rew, dones, infos)

    def try_reset(self, env_id):
        row = self._reset_rows.pop(env_id, None)
        if row is not None:
            return {HIGH: row}
        mask = np.zeros(self.num_envs, dtype=np.uint8)
        mask[env_id] = 1
        self._book_cache = None
        return {HIGH: self.venv.reset(mask=mask)[env_id].cpu().numpy().astype(np.float64)}

    def get_unwrapped(self):
        return self._views

    def stop(self):
        self.venv.close()


def make_env_hier(env_config=None):
    """train_config.py:18-20; each env gets its own RNG stream (low_level_env.env_seed)."""
    seed, off = env_seed(env_config, 1)
    return HierarchicalHumanoidEnv(seed=seed, lane_offset=off)


def make_env_hier_vec(env_config=None):
    """One N-lane BaseEnv per RLlib worker (env_config["num_lanes"], default 1024)."""
    cfg = env_config if env_config is not None else {}
    n = int(cfg.get("num_lanes", 1024)) if hasattr(cfg, "get") else 1024
    seed, off = env_seed(env_config, n)
    return HierarchicalVectorEnv(n, seed=seed, lane_offset=off)


def register_envs(vectorised=True):
    """register_env(ENV_HIER, ...) (train_config.py:320) when Ray is importable: the N-lane BaseEnv per worker
    (default, make_env_hier_vec: one launch per sampler step for all of the worker's envs), or the reference's
    one-env-per-call creator (make_env_hier: one handle and one launch per env)."""
    from ray.tune.registry import register_env
    register_env(ENV_HIER, make_env_hier_vec if vectorised else make_env_hier)
    return ENV_HIER

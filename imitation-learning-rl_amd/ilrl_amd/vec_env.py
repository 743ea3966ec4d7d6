"""HumanoidVecEnv: N device-resident env lanes on one GPU behind the C-ABI (include/humanoid_env.h).

Hot-path buffers are torch.cuda tensors (zero-copy device pointers); every launch goes on torch's
current HIP stream so it orders with the caller's tensor ops.  State get/set are host float64 arrays
(parity tests inject identical (state, action, reference-frame) inputs through them).
"""
import ctypes

import numpy as np

from . import _native as N
from .clips import CLIP_NAMES, load_clip


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class HostStaging:
    """Pinned host buffers for the drop-in adapters (one per slot name): device tensors are copied into them with
    non_blocking copies on the launch stream and ONE stream synchronize waits for all of them (a pageable .cpu() per
    tensor is one blocking round trip each).  The numpy views returned stay valid until that slot's next fetch;
    callers copy what they hand out.  `upload` stages a host array into a device tensor the same way (the next
    fetch's synchronize also retires the upload before the pinned buffer is reused)."""

    def __init__(self, torch, device):
        self.torch, self.device, self.buf = torch, device, {}

    def _pinned(self, name, shape, dtype):
        b = self.buf.get(name)
        if b is None or tuple(b.shape) != tuple(shape) or b.dtype != dtype:
            b = self.torch.empty(tuple(shape), dtype=dtype, pin_memory=True)
            self.buf[name] = b
        return b

    def fetch(self, **xs):
        out = {}
        for name, x in xs.items():
            b = self._pinned(name, x.shape, x.dtype)
            b.copy_(x, non_blocking=True)
            out[name] = b
        self.torch.cuda.current_stream(self.device).synchronize()
        return {k: v.numpy() for k, v in out.items()}

    def fetch_rows(self, name, x, cap):
        """x [m, ...] with m <= cap rows into a pinned buffer of cap rows (allocated once): one synchronize."""
        m = int(x.shape[0])
        b = self._pinned(name, (cap,) + tuple(x.shape[1:]), x.dtype)
        if m:
            b[:m].copy_(x, non_blocking=True)
            self.torch.cuda.current_stream(self.device).synchronize()
        return b.numpy()[:m]

    def upload(self, name, host, dev_out):
        b = self._pinned(name, host.shape, dev_out.dtype)
        b.numpy()[...] = host
        dev_out.copy_(b, non_blocking=True)
        return dev_out


class HumanoidVecEnv:
    """Batched LowLevelHumanoidEnv (low_level_env.py:36-526) - one lane per env instance."""

    def __init__(self, n, clips=("motion02_04",), clip_of_lane=None, seed=0, device=0, lane_offset=0,
                 precision="fp32", block_size=64, **physics):
        self.terrain = N.HUM_TERRAIN_PLANE
        import torch
        if not torch.cuda.is_available():
            raise N.NativeError("HumanoidVecEnv needs a HIP device (no CPU fallback by design)")
        self.torch = torch
        self.n = int(n)
        self.device = torch.device("cuda", device)
        cfg = N.default_config(n_lanes=self.n, device=device, seed=seed, lane_offset=lane_offset,
                               precision={"fp32": 0, "fp64": 1}[precision], block_size=block_size, **physics)
        self.cfg = cfg
        h = ctypes.c_void_p()
        N.check(N.lib().hum_create(ctypes.byref(cfg), ctypes.byref(h)), "hum_create")
        self.h = h
        self.clips = []
        for cid, c in enumerate(clips):
            clip = load_clip(c) if isinstance(c, str) else c
            self.clips.append(clip)
            N.check(N.lib().hum_set_clip(h, cid, _dp(clip.pos), clip.pos.shape[0], _dp(clip.vel), clip.vel.shape[0],
                                         _dp(clip.rel), clip.rel.shape[0], _dp(clip.ep), clip.ep.shape[0]),
                    "hum_set_clip")
        if clip_of_lane is None:
            clip_of_lane = np.arange(self.n) % len(self.clips)
        self.clip_of_lane = np.ascontiguousarray(clip_of_lane, dtype=np.int32)
        N.check(N.lib().hum_set_lane_clips(h, self.clip_of_lane.ctypes.data_as(ctypes.c_void_p)), "hum_set_lane_clips")
        f32 = torch.float32
        self.obs = torch.zeros(self.n, N.HUM_NOBS, dtype=f32, device=self.device)
        self.obs_reset = torch.zeros(self.n, N.HUM_NOBS, dtype=f32, device=self.device)
        self.reward = torch.zeros(self.n, dtype=f32, device=self.device)
        self.done = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
        self.frame = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self.aux = torch.zeros(self.n, N.HUM_NAUX, dtype=f32, device=self.device)

    # -------------------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "h", None):
            N.lib().hum_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_modes(self, debug=None, predefined=None):
        m = np.zeros(self.n, dtype=np.uint32)
        if debug is not None:
            m |= np.where(np.broadcast_to(debug, self.n), N.HUM_MODE_DEBUG, 0).astype(np.uint32)
        if predefined is not None:
            m |= np.where(np.broadcast_to(predefined, self.n), N.HUM_MODE_PREDEFINED, 0).astype(np.uint32)
        N.check(N.lib().hum_set_lane_modes(self.h, m.ctypes.data_as(ctypes.c_void_p)), "hum_set_lane_modes")

    def set_terrain(self, mode, heights=None, w=256, l=256, scale=(1.0, 1.0, 1.0), origin=(0.0, 0.0, 0.25),
                    centre=None):
        """Ground of every lane (hum_set_terrain_ex): N.HUM_TERRAIN_PLANE, N.HUM_TERRAIN_HEIGHTFIELD (heights [w*l],
        vertex (i, j) = heights[i + j*w], CustomScene.replaceHeightfieldData's layout; centre = the vertical centre
        Bullet keeps from the shape's creation, None = (min + max) / 2 of these heights) or
        N.HUM_TERRAIN_RANDOM_BLOCKS (LowLevelHumanoidEnv(useCustomEnv=True): a new CustomScene terrain per lane at
        every reset)."""
        h = None
        if mode == N.HUM_TERRAIN_HEIGHTFIELD:
            h = np.ascontiguousarray(heights, dtype=np.float32).reshape(-1)
            if h.size != w * l:
                raise ValueError("heights: %d values for a %d x %d heightfield" % (h.size, w, l))
        sc = np.ascontiguousarray(scale, dtype=np.float64)
        org = np.ascontiguousarray(origin, dtype=np.float64)
        ctr = None if centre is None else np.array([float(centre)], dtype=np.float64)
        N.check(N.lib().hum_set_terrain_ex(self.h, int(mode), h.ctypes.data if h is not None else None, int(w), int(l),
                                           _dp(sc), _dp(org), _dp(ctr) if ctr is not None else None), "hum_set_terrain")
        self.terrain = int(mode)

    def set_predefined_targets(self, xyz):
        xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 3)
        N.check(N.lib().hum_set_predefined_targets(self.h, _dp(xyz), xyz.shape[0]), "hum_set_predefined_targets")

    def _reset_args(self, mask, start_frame, reset_yaw, start_from_ref, init_vel):
        t = self.torch
        m = None if mask is None else t.as_tensor(mask, dtype=t.uint8, device=self.device).contiguous()
        sf = None if start_frame is None else t.as_tensor(start_frame, dtype=t.int32, device=self.device).expand(self.n).contiguous()
        ry = None if reset_yaw is None else t.as_tensor(reset_yaw, dtype=t.float64, device=self.device).expand(self.n).contiguous()
        flags = (0 if start_from_ref else N.HUM_RESET_NO_REF_POSE) | (0 if init_vel else N.HUM_RESET_NO_INIT_VEL)
        return m, sf, ry, flags

    def reset(self, mask=None, start_frame=None, reset_yaw=None, start_from_ref=True, init_vel=True):
        """reset()/resetFromFrame(startFrame, resetYaw, startFromRef, initVel) for masked lanes; returns the obs
        tensor [n,70] (device).  The reset lanes' done flags are cleared: `done` then means "the last step ended
        the episode" for the policy / rollout loops that read it (hum_rollout, DevicePolicy.act)."""
        m, sf, ry, flags = self._reset_args(mask, start_frame, reset_yaw, start_from_ref, init_vel)
        N.check(N.lib().hum_reset_ex(self.h, _ptr(m), _ptr(sf), _ptr(ry), flags, _ptr(self.obs), self._stream()),
                "hum_reset")
        self._clear_done(m)
        return self.obs

    def _clear_done(self, m):
        if m is None:
            self.done.zero_()
        else:
            self.done.masked_fill_(m.bool(), 0)

    def step(self, actions, autoreset=False, skip_physics=False):
        """One env step for all lanes. actions: float32 [n,17] (device tensor or array)."""
        t = self.torch
        a = t.as_tensor(actions, dtype=t.float32, device=self.device).contiguous()
        if a.shape != (self.n, N.HUM_NACT):
            raise ValueError("actions must be [%d, %d], got %s" % (self.n, N.HUM_NACT, tuple(a.shape)))
        flags = (N.HUM_STEP_AUTORESET if autoreset else 0) | (N.HUM_STEP_SKIP_PHYSICS if skip_physics else 0)
        N.check(N.lib().hum_step(self.h, _ptr(a), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                                 _ptr(self.frame), flags, _ptr(self.obs_reset), self._stream()), "hum_step")
        return self.obs, self.reward, self.done, self.frame

    def step_k(self, actions, autoreset=False, skip_physics=False, out=None):
        """k env steps for all lanes in one launch (hum_step_k).  actions: float32 [k,n,17]; returns device tensors
        (obs [k,n,70], reward [k,n], done [k,n], frame [k,n], obs_reset [k,n,70]) - row t is what the t-th of k
        step() calls returns.  `out` reuses a previous call's tuple of the same k."""
        t = self.torch
        a = t.as_tensor(actions, dtype=t.float32, device=self.device).contiguous()
        if a.dim() != 3 or a.shape[1:] != (self.n, N.HUM_NACT):
            raise ValueError("actions must be [k, %d, %d], got %s" % (self.n, N.HUM_NACT, tuple(a.shape)))
        k = a.shape[0]
        if out is None or out[0].shape[0] != k:
            out = self.step_k_out(k)
        obs, rew, done, frame, obs_reset = out
        flags = (N.HUM_STEP_AUTORESET if autoreset else 0) | (N.HUM_STEP_SKIP_PHYSICS if skip_physics else 0)
        N.check(N.lib().hum_step_k(self.h, _ptr(a), _ptr(obs), _ptr(rew), _ptr(done), _ptr(frame), flags,
                                   _ptr(obs_reset), k, self._stream()), "hum_step_k")
        return out

    def step_k_out(self, k):
        """A zeroed output tuple for step_k(..., out=) of k steps (allocate it ahead of a timed loop)."""
        t, f32 = self.torch, self.torch.float32
        return (t.zeros(k, self.n, N.HUM_NOBS, dtype=f32, device=self.device),
                t.zeros(k, self.n, dtype=f32, device=self.device),
                t.zeros(k, self.n, dtype=t.uint8, device=self.device),
                t.zeros(k, self.n, dtype=t.int32, device=self.device),
                t.zeros(k, self.n, N.HUM_NOBS, dtype=f32, device=self.device))

    def get_aux(self):
        N.check(N.lib().hum_get_aux(self.h, _ptr(self.aux), self._stream()), "hum_get_aux")
        return self.aux

    def sync(self):
        self.torch.cuda.current_stream(self.device).synchronize()
        N.check(N.lib().hum_sync(self.h), "hum_sync")

    def get_state(self):
        self.sync()
        phys = np.zeros((self.n, N.HUM_NSTATE))
        book = np.zeros((self.n, N.HUM_NBOOK))
        N.check(N.lib().hum_get_state(self.h, _dp(phys), _dp(book)), "hum_get_state")
        return phys, book

    def set_state(self, phys=None, book=None):
        self.sync()
        p = None if phys is None else np.ascontiguousarray(phys, dtype=np.float64).reshape(self.n, N.HUM_NSTATE)
        b = None if book is None else np.ascontiguousarray(book, dtype=np.float64).reshape(self.n, N.HUM_NBOOK)
        N.check(N.lib().hum_set_state(self.h, _dp(p) if p is not None else None, _dp(b) if b is not None else None),
                "hum_set_state")

    def get_parts(self):
        self.sync()
        out = np.zeros((self.n, 33, 3))
        N.check(N.lib().hum_get_parts(self.h, _dp(out)), "hum_get_parts")
        return out

    def error_flags(self):
        self.sync()
        f = ctypes.c_uint32(0)
        N.check(N.lib().hum_get_error_flags(self.h, ctypes.byref(f)), "hum_get_error_flags")
        return f.value


__all__ = ["HumanoidVecEnv", "CLIP_NAMES"]

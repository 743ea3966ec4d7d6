"""ORACLE - test infrastructure only (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg).

ctypes binding of `oracle/env_oracle.c`, the plain-C restatement of `oracle.py::OracleLowLevelEnv` (reset/step of
LowLevelHumanoidEnv, /root/reference/low_level_env.py:224-526) over the fp64 physics restatement.  Used as the
OpenMP CPU baseline (`bench`) and cross-checked against the Python oracle (tests/test_env_oracle_c.py).
"""
import ctypes

import numpy as np

import oracle as O

NREF = 14


class OeModel(ctypes.Structure):
    _fields_ = [("jm_dof", ctypes.c_int * NREF), ("jm_col", ctypes.c_int * NREF),
                ("jm_w", ctypes.c_double * NREF), ("jm_wv", ctypes.c_double * NREF),
                ("motor_dof", ctypes.c_int * 17), ("motor_power", ctypes.c_double * 17),
                ("ep_right_leg", ctypes.c_int), ("ep_right_foot", ctypes.c_int), ("part_right_foot", ctypes.c_int),
                ("numpy_semantics", ctypes.c_int)]


class OeClip(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_void_p), ("vel", ctypes.c_void_p), ("rel", ctypes.c_void_p), ("ep", ctypes.c_void_p),
                ("n_pos", ctypes.c_int), ("n_vel", ctypes.c_int), ("n_rel", ctypes.c_int), ("n_ep", ctypes.c_int)]


class OeEnv(ctypes.Structure):   # layout of env_oracle.c's oe_env (size checked against oe_env_size)
    _fields_ = [("st", ctypes.c_double * 47), ("frame", ctypes.c_int), ("cur_timestep", ctypes.c_int),
                ("max_frame", ctypes.c_int), ("key", ctypes.c_uint64), ("ctr", ctypes.c_uint64),
                ("target", ctypes.c_double * 3), ("srp", ctypes.c_double * 3), ("robot_pos", ctypes.c_double * 3),
                ("sep", ctypes.c_double * 3), ("wt", ctypes.c_double * 2), ("hldt", ctypes.c_double),
                ("lts", ctypes.c_double), ("dj", ctypes.c_double), ("dvj", ctypes.c_double), ("bps", ctypes.c_double),
                ("es", ctypes.c_double), ("jls", ctypes.c_double), ("alive", ctypes.c_double),
                ("dlts", ctypes.c_double), ("cur_obs", ctypes.c_float * 42), ("joint_speeds", ctypes.c_float * 17),
                ("jal", ctypes.c_int), ("bx", ctypes.c_double), ("by", ctypes.c_double)]


_bound = False


def lib():
    global _bound
    L = O.lib()
    if not _bound:
        P, M, C, E = (ctypes.POINTER(t) for t in (O.OmParams, OeModel, OeClip, OeEnv))
        dp = ctypes.POINTER(ctypes.c_double)
        L.oe_init.argtypes = [E, C, ctypes.c_uint64]
        L.oe_reset.argtypes = [M, C, E, ctypes.c_int, ctypes.c_double, dp]
        L.oe_step.argtypes = [M, C, P, E, ctypes.POINTER(ctypes.c_float), dp, dp]
        L.oe_step.restype = ctypes.c_int
        L.oe_bench.argtypes = [M, C, P, ctypes.c_int, ctypes.c_double, ctypes.c_uint64, dp]
        L.oe_bench.restype = ctypes.c_long
        assert L.oe_env_size() == ctypes.sizeof(OeEnv), "oe_env layout"
        _bound = True
    return L


def model(numpy_semantics=O.DEFAULT_NUMPY, ep_cols=None):
    m = OeModel()
    for j, (jm, col) in enumerate(O.JOINT_MAP):
        m.jm_dof[j] = O.DOF_NAMES.index(jm)
        m.jm_col[j] = -1   # the clip's column index: CClip
        m.jm_w[j] = O.JOINT_WEIGHT[jm]
        m.jm_wv[j] = O.JOINT_VEL_WEIGHT[jm]
    for i in range(17):
        m.motor_dof[i] = O.MOTOR_DOF[i]
        m.motor_power[i] = O.MOTOR_POWER[i]
    m.part_right_foot = [p["name"] for p in O.LINKS["parts"]].index("right_foot")
    m.numpy_semantics = numpy_semantics
    return m


class CClip:
    """A clip (ilrl_amd.clips.Clip-like: pos/vel/rel/ep arrays + jcol/ecol) packed for the C env; keeps the arrays
    alive."""

    def __init__(self, clip, numpy_semantics=O.DEFAULT_NUMPY):
        self.arrs = [np.ascontiguousarray(getattr(clip, k), dtype=np.float64) for k in ("pos", "vel", "rel", "ep")]
        self.c = OeClip(*[a.ctypes.data for a in self.arrs], *[a.shape[0] for a in self.arrs])
        self.m = model(numpy_semantics)
        for j, (_, col) in enumerate(O.JOINT_MAP):
            self.m.jm_col[j] = clip.jcol(col)
        self.m.ep_right_leg = clip.ecol("RightLeg_Xposition")
        self.m.ep_right_foot = clip.ecol("RightFoot_Xposition")


class CEnv:
    """One C oracle env lane with the same RNG stream as oracle.LaneRNG(seed, lane)."""

    def __init__(self, clip, seed=0, lane=0, params=None, numpy_semantics=O.DEFAULT_NUMPY):
        self.cc = CClip(clip, numpy_semantics)
        self.P = params or O.default_params()
        self.e = OeEnv()
        lib().oe_init(ctypes.byref(self.e), ctypes.byref(self.cc.c), O.lane_key(seed, lane))

    def reset(self, start_frame=-1, reset_yaw=0.0):
        obs = np.zeros(70)
        lib().oe_reset(ctypes.byref(self.cc.m), ctypes.byref(self.cc.c), ctypes.byref(self.e), start_frame,
                       reset_yaw, O._p(obs))
        return obs

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.float32)
        obs, rew = np.zeros(70), np.zeros(1)
        d = lib().oe_step(ctypes.byref(self.cc.m), ctypes.byref(self.cc.c), ctypes.byref(self.P), ctypes.byref(self.e),
                          a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), O._p(obs), O._p(rew))
        return obs, float(rew[0]), bool(d)


def bench(clip, threads, seconds, seed=1000, params=None):
    """CPU baseline: `threads` OpenMP lanes stepping uniform random actions (reset on done) for `seconds`.
    Returns (env steps, wall seconds of the slowest thread)."""
    cc = CClip(clip)
    P = params or O.default_params()
    wall = ctypes.c_double(0)
    n = lib().oe_bench(ctypes.byref(cc.m), ctypes.byref(cc.c), ctypes.byref(P), int(threads), float(seconds), seed,
                       ctypes.byref(wall))
    return int(n), wall.value

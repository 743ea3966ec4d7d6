"""ctypes binding of the C-ABI in include/humanoid_env.h (libhumenv.so, built for gfx950).

The product path has NO CPU fallback: if the HIP library is missing this module raises on use.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB_PATH = os.path.join(HERE, "_lib", "libhumenv.so")
LIB_PATH = os.environ.get("ILRL_AMD_LIB", DEFAULT_LIB_PATH)
# ILRL_AMD_AB=1 (same-box A/B runs against an older build named by ILRL_AMD_LIB): entry points the older library
# lacks stay unbound placeholders, and its ABI may be any of AB_COMPATIBLE_ABIS (ABIs whose structs and existing
# signatures are unchanged - later ones only added entry points).  Without it every library, override or not,
# must match HUM_ABI_VERSION and export every symbol.
AB_MODE = os.environ.get("ILRL_AMD_AB") == "1"
AB_COMPATIBLE_ABIS = (8, 9, 10, 11, 12, 13)   # ABI 10 added hum_policy_create_ex, hum_hier_rollout; 11 hum_pack_rows;
# 12 hum_hier_rollout_fused; 13 hum_rollout_fused_ex, hum_hier_rollout_fused_ex (the policy mean traces); 14 the
# heightfield ridge contacts (HUM_MAX_CONTACTS 95 -> 119) and the IPC fragment transport

HUM_ABI_VERSION = 14   # include/humanoid_env.h
HUM_NSTATE, HUM_NOBS, HUM_NACT, HUM_NBOOK, HUM_NAUX = 47, 70, 17, 48, 17
HUM_NOBS_HIGH, HUM_NACT_HIGH = 44, 2
HUM_AGENT_HIGH, HUM_AGENT_LOW, HUM_AGENT_SEL_SKIP = 1, 2, 255
HUM_STEP_AUTORESET, HUM_STEP_SKIP_PHYSICS, HUM_STEP_HOST_IO, HUM_STEP_CHECK_FINITE = 1, 2, 4, 8
HUM_MODE_DEBUG, HUM_MODE_PREDEFINED = 1, 2
HUM_EFLAG_NONFINITE_ACTION, HUM_EFLAG_VEL_ROW, HUM_EFLAG_CONTACT_OVERFLOW, HUM_EFLAG_BAD_START_FRAME = 1, 2, 4, 8
HUM_EFLAG_DIAG_BOUNDS = 0x80000000   # bounds-checked diagnostic builds only (-DHUM_BOUNDS_CHECK)
HUM_NUMPY_1, HUM_NUMPY_2 = 1, 2
HUM_RESET_NO_REF_POSE, HUM_RESET_NO_INIT_VEL = 1, 2
HUM_MAX_CONTACTS = 119
HUM_TERRAIN_PLANE, HUM_TERRAIN_HEIGHTFIELD, HUM_TERRAIN_RANDOM_BLOCKS = 0, 1, 2
HUM_OK, HUM_ERR_ARG, HUM_ERR_HIP, HUM_ERR_NOCLIP, HUM_ERR_STATE = 0, -1, -2, -3, -4

# bookkeeping layout (HUM_BK_*)
BK = dict(frame=0, cur_timestep=1, rng_counter=2, predefinedTargetIndex=3, target=4, starting_robot_pos=7,
          robot_pos=10, starting_ep_pos=13, highLevelDegTarget=16, walk_target=17, lowTargetScore=19,
          deltaJoints=20, deltaVelJoints=21, bodyPostureScore=22, electricityScore=23, jointLimitScore=24,
          aliveReward=25, delta_lowTargetScore=26, clip=27, mode=28, rng_key_lo=29, rng_key_hi=30,
          # hierarchical env (hier_env.py)
          steps_remaining_at_level=31, num_high_level_steps=32, expect_high=33, highTargetScore=34,
          cumulative_driftScore=35, driftScore=36, delta_highTargetScore=37, cumulative_aliveReward=38, body_xy=39,
          # HUM_TERRAIN_RANDOM_BLOCKS: the lane's current terrain key
          terrain_key_lo=41, terrain_key_hi=42)
AUX = ["deltaJoints", "deltaEndPoints", "lowTargetScore", "deltaVelJoints", "bodyPostureScore", "highTargetScore",
       "driftScore", "baseReward", "aliveReward", "electricityScore", "jointLimitScore", "dist_from_origin",
       "endPointScore", "endPointScoreExp", "robot_pos_x", "robot_pos_y", "robot_pos_z"]

# every symbol include/humanoid_env.h declares
EXPORTS = ["hum_abi_version", "hum_last_error", "hum_default_config", "hum_create", "hum_destroy", "hum_set_clip",
           "hum_set_lane_clips", "hum_set_lane_modes", "hum_set_predefined_targets", "hum_reset", "hum_step",
           "hum_step_graph", "hum_get_aux", "hum_get_state", "hum_set_state", "hum_get_parts",
           "hum_get_error_flags", "hum_sync", "hum_num_lanes", "hum_stream", "hum_hier_reset", "hum_hier_step",
           "hum_reset_ex", "hum_hier_reset_ex", "hum_clip_csv_sizes", "hum_clip_csv_parse", "hum_load_clip_csv",
           "hum_policy_create", "hum_policy_destroy", "hum_policy_act", "hum_rollout", "hum_rollout_fused", "hum_set_terrain",
           "hum_step_k", "hum_hier_step_k", "hum_set_terrain_ex", "hum_policy_act_ex", "hum_policy_create_ex",
           "hum_hier_rollout", "hum_pack_rows", "hum_hier_rollout_fused", "hum_rollout_fused_ex",
           "hum_hier_rollout_fused_ex", "hum_ipc_export", "hum_ipc_open", "hum_ipc_close", "hum_dma_copy",
           "hum_dma_wait"]


class HumConfig(ctypes.Structure):
    _fields_ = [("n_lanes", ctypes.c_int32), ("device", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("lane_offset", ctypes.c_int64), ("precision", ctypes.c_int32), ("block_size", ctypes.c_int32),
                ("dt_env", ctypes.c_double), ("substeps", ctypes.c_int32), ("gravity", ctypes.c_double),
                ("solver_iters", ctypes.c_int32), ("erp_contact", ctypes.c_double), ("erp_limit", ctypes.c_double),
                ("mu_ground", ctypes.c_double), ("mu_self", ctypes.c_double), ("contact_thresh", ctypes.c_double),
                ("lin_damp", ctypes.c_double), ("ang_damp", ctypes.c_double),
                ("limit_max_impulse", ctypes.c_double), ("max_coord_vel", ctypes.c_double),
                ("max_contacts", ctypes.c_int32), ("self_collision", ctypes.c_int32),
                ("joint_damping", ctypes.c_int32), ("kernel", ctypes.c_int32),
                ("hier", ctypes.c_int32), ("envs_per_block", ctypes.c_int32), ("lds_rows", ctypes.c_int32),
                ("numpy_semantics", ctypes.c_int32), ("split_penetration", ctypes.c_double)]


class HumHierIO(ctypes.Structure):   # hum_hier_io
    _fields_ = [(k, ctypes.c_void_p) for k in ("obs_high", "obs_high_reset", "obs_low", "done", "agents", "rew_high",
                                               "rew_low", "act_high", "act_low")]


class HumHierTraj(ctypes.Structure):   # hum_hier_traj
    _fields_ = [(k, ctypes.c_void_p) for k in ("acted", "obs_high", "act_high", "obs_low", "act_low", "agents",
                                               "rew_high", "rew_low", "done")]


HUM_PACK_MAX_FIELDS = 6


class HumDmaTicket(ctypes.Structure):   # hum_dma_ticket
    _fields_ = [("signal", ctypes.c_uint64), ("bytes", ctypes.c_uint64)]


HUM_IPC_HANDLE_BYTES = 64


class HumPackField(ctypes.Structure):   # hum_pack_field
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("src_step", ctypes.c_int64),
                ("src_lane", ctypes.c_int64), ("dst_step", ctypes.c_int64), ("dst_lane", ctypes.c_int64),
                ("row_bytes", ctypes.c_int32)]


class NativeError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libhumenv.so (raises if the HIP extension was not built - there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError("HIP library %s not found: build it with `make -C imitation-learning-rl_amd/csrc` "
                          "or __graft_entry__.build()" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    if AB_MODE:
        # an older build in a same-box A/B may predate later entry points; they stay unbound placeholders there
        # (tests/test_cpu_abi_model.py checks the shipped library has them all)
        L.hum_abi_version.restype = ctypes.c_int
        if L.hum_abi_version() not in AB_COMPATIBLE_ABIS + (HUM_ABI_VERSION,):
            raise NativeError("ILRL_AMD_AB: %s has ABI %d, not one of %s" % (LIB_PATH, L.hum_abi_version(),
                                                                           AB_COMPATIBLE_ABIS + (HUM_ABI_VERSION,)))
        import types
        for name in EXPORTS:
            if not hasattr(L, name):
                setattr(L, name, types.SimpleNamespace())
    vp, i32, u32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
    dp = ctypes.POINTER(ctypes.c_double)
    L.hum_abi_version.restype = ctypes.c_int
    L.hum_last_error.restype = ctypes.c_char_p
    L.hum_default_config.argtypes = [ctypes.POINTER(HumConfig)]
    L.hum_default_config.restype = None
    L.hum_create.argtypes = [ctypes.POINTER(HumConfig), ctypes.POINTER(vp)]
    L.hum_destroy.argtypes = [vp]
    L.hum_set_clip.argtypes = [vp, i32, dp, i32, dp, i32, dp, i32, dp, i32]
    L.hum_set_lane_clips.argtypes = [vp, vp]
    L.hum_set_lane_modes.argtypes = [vp, vp]
    L.hum_set_predefined_targets.argtypes = [vp, dp, i32]
    L.hum_set_terrain.argtypes = [vp, i32, vp, i32, i32, dp, dp]
    L.hum_set_terrain_ex.argtypes = [vp, i32, vp, i32, i32, dp, dp, dp]
    L.hum_reset.argtypes = [vp, vp, vp, vp, vp, vp]
    L.hum_reset_ex.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    L.hum_clip_csv_sizes.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(i32)]
    L.hum_clip_csv_parse.argtypes = [ctypes.c_char_p, ctypes.c_char_p, dp, dp, dp, dp]
    L.hum_load_clip_csv.argtypes = [vp, i32, ctypes.c_char_p, ctypes.c_char_p]
    L.hum_policy_create.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, u64, ctypes.POINTER(vp)]
    L.hum_policy_create_ex.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, u64, ctypes.POINTER(vp)]
    L.hum_hier_rollout.argtypes = [vp, vp, vp, i32, i32, u64, ctypes.POINTER(HumHierIO), ctypes.POINTER(HumHierTraj), vp]
    L.hum_hier_rollout_fused.argtypes = L.hum_hier_rollout.argtypes
    L.hum_hier_rollout_fused_ex.argtypes = L.hum_hier_rollout.argtypes[:-1] + [vp, vp, vp]
    L.hum_policy_destroy.argtypes = [vp]
    L.hum_pack_rows.argtypes = [ctypes.POINTER(HumPackField), i32, i32, i32, i32, vp]
    L.hum_ipc_export.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(u64)]
    L.hum_ipc_open.argtypes = [ctypes.c_char_p, u64, ctypes.POINTER(vp)]
    L.hum_ipc_close.argtypes = [vp]
    L.hum_dma_copy.argtypes = [vp, vp, u64, i32, ctypes.POINTER(HumDmaTicket)]
    L.hum_dma_wait.argtypes = [ctypes.POINTER(HumDmaTicket)]
    L.hum_policy_act.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, i32, u64, vp]
    L.hum_policy_act_ex.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp, i32, u64, vp]
    L.hum_rollout.argtypes = [vp, vp, i32, i32, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.hum_rollout_fused.argtypes = [vp, vp, i32, i32, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.hum_rollout_fused_ex.argtypes = [vp, vp, i32, i32, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.hum_hier_reset_ex.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    L.hum_step.argtypes = [vp, vp, vp, vp, vp, vp, u32, vp, vp]
    L.hum_step_k.argtypes = [vp, vp, vp, vp, vp, vp, u32, vp, i32, vp]
    L.hum_hier_reset.argtypes = [vp, vp, vp, vp, vp, vp]
    L.hum_hier_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp, vp]
    L.hum_hier_step_k.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp, i32, vp]
    L.hum_step_graph.argtypes = [vp, vp, vp, vp, vp, vp, u32, vp, i32]
    L.hum_get_aux.argtypes = [vp, vp, vp]
    L.hum_get_state.argtypes = [vp, dp, dp]
    L.hum_set_state.argtypes = [vp, dp, dp]
    L.hum_get_parts.argtypes = [vp, dp]
    L.hum_get_error_flags.argtypes = [vp, ctypes.POINTER(u32)]
    L.hum_sync.argtypes = [vp]
    L.hum_num_lanes.argtypes = [vp]
    L.hum_num_lanes.restype = i32
    L.hum_stream.argtypes = [vp]
    L.hum_stream.restype = vp
    for name in EXPORTS:
        getattr(L, name)  # AttributeError if the library lacks a declared symbol
    if L.hum_abi_version() != HUM_ABI_VERSION and not AB_MODE:
        raise NativeError("%s: ABI %d != binding ABI %d: rebuild the library"
                          % (LIB_PATH, L.hum_abi_version(), HUM_ABI_VERSION))
    if hasattr(L, "hum_debug_phase_cycles"):   # diagnostic builds only
        L.hum_debug_phase_cycles.argtypes = [vp, ctypes.c_int]
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        raise NativeError("%s failed (%d): %s" % (what, rc, lib().hum_last_error().decode()))


def default_config(**kw):
    c = HumConfig()
    lib().hum_default_config(ctypes.byref(c))
    for k, v in kw.items():
        if not hasattr(c, k):
            raise TypeError("unknown hum_config field %r" % k)
        setattr(c, k, v)
    return c

/* humanoid_env.h - C-ABI of the MI355X-native vectorised humanoid imitation environment.
 *
 * Drop-in boundary for the reference hot path `LowLevelHumanoidEnv.reset()/step()`
 * (/root/reference/low_level_env.py:36-526, registered as "HumanoidBulletEnv-v0-Low" by
 * train_config.py:29,321) and its two-level counterpart `HierarchicalHumanoidEnv.reset()/step()`
 * (/root/reference/hier_env.py:38-641, "HumanoidBulletEnv-v0-Hier", train_config.py:18-20,320), selected
 * per handle by hum_config.hier.  One handle = N independent env lanes resident on ONE GPU, advanced by one
 * HIP kernel launch per env step.  The Python mirror (`ilrl_amd.low_level_env`) binds this header with
 * ctypes; INTEGRATION.md shows the binding a maintainer adds on the reference side.
 *
 * Conventions
 *   - extern "C", plain pointers + sizes, int status (0 = ok, < 0 = error, hum_last_error() for text);
 *     no exceptions cross the ABI.
 *   - Hot-path I/O (actions, obs, reward, done, frame) are DEVICE pointers on the handle's GPU (e.g.
 *     torch.cuda tensors) - zero-copy - or, with HUM_STEP_HOST_IO, host pointers (staged through the device and
 *     synchronised before the call returns).  State get/set use HOST pointers (bulk copies for parity tests).
 *   - `stream` is a hipStream_t (NULL = the HIP null stream; hum_stream() returns the handle's own
 *     stream).  Launches are asynchronous on that stream; state get/set, error flags and hum_sync
 *     synchronise the device.  A handle is bound to one device and is not thread-safe.
 *   - Lane physics state (47 doubles, HUM_NSTATE): base pos[3] (COM, world), base quat[4] (x,y,z,w),
 *     base lin vel[3] (world), base ang vel[3] (world), q[17], qd[17]; dofs in MJCF order
 *     abdomen_z, abdomen_y, abdomen_x, right_hip_x, right_hip_z, right_hip_y, right_knee, left_hip_x,
 *     left_hip_z, left_hip_y, left_knee, right_shoulder_y, right_shoulder_x, right_elbow,
 *     left_shoulder_y, left_shoulder_x, left_elbow  (== WalkerBase.ordered_joints, obs order).
 *   - Actions: float32 [n,17] in CustomHumanoidRobot motor order (humanoid.py:28-37).
 *   - Observation: float32 [n,70] = calc_state (42) ++ 14 x (relative target, target velocity)
 *     (low_level_env.py:307-320).
 */
#ifndef HUMANOID_ENV_H
#define HUMANOID_ENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HUM_ABI_VERSION 14
#define HUM_NSTATE 47   /* physics state per lane */
#define HUM_NOBS 70     /* observation_space shape, low_level_env.py:53-55 */
#define HUM_NACT 17     /* action_space shape, low_level_env.py:56 */
#define HUM_NBOOK 48    /* bookkeeping doubles per lane, layout HUM_BK_* below */
#define HUM_NOBS_HIGH 44   /* high_level_obs_space shape, hier_env.py:52 */
#define HUM_NACT_HIGH 2    /* high_level_act_space shape (cos, sin of the heading), hier_env.py:53-55 */
#define HUM_NAUX 17     /* RewardLogCallback terms + calcEndPointScore + robot_pos per lane, HUM_AUX_* below */
#define HUM_MAX_CLIPS 8
#define HUM_MAX_CONTACTS 119  /* every contact candidate: 29 sphere / capsule-end ground points, 24 heightfield ridge
                                points (2 per capsule, ABI 14), 66 geom pairs */

/* status codes */
#define HUM_OK 0
#define HUM_ERR_ARG -1
#define HUM_ERR_HIP -2
#define HUM_ERR_NOCLIP -3
#define HUM_ERR_STATE -4

/* hum_step flags */
#define HUM_STEP_AUTORESET 1u     /* reset done lanes inside the same launch (obs_reset receives the new obs) */
#define HUM_STEP_SKIP_PHYSICS 2u  /* treat the current physics state as post-step (parity: injected physics) */
#define HUM_STEP_HOST_IO 4u       /* actions / outputs are HOST pointers: copied to and from the device around the
                                     launch on `stream`, which the call then synchronises (the gym view's path) */
#define HUM_STEP_CHECK_FINITE 8u  /* wait for the launch and return HUM_ERR_ARG if a lane's action was non-finite
                                     (humanoid.py:55 `assert np.isfinite(a).all()`; those lanes are not stepped and
                                     the sticky HUM_EFLAG_NONFINITE_ACTION bit is consumed).  Without it the launch
                                     stays asynchronous and only the sticky bit records the event.  A checked call
                                     clears that bit before its launch: a non-finite action of an EARLIER unchecked
                                     call that hum_get_error_flags has not yet reported is consumed with it (read
                                     the flags first to keep it); the other bits stay sticky. */

/* hum_reset_ex / hum_hier_reset_ex flags: resetFromFrame(startFromRef, initVel) (low_level_env.py:247-305,
 * hier_env.py:259-319); both False-able independently, default (0) = True, True as reset() uses */
#define HUM_RESET_NO_REF_POSE 1u  /* startFromRef=False: frame unchanged, joints at flat_env.reset()'s U(-0.1, 0.1) */
#define HUM_RESET_NO_INIT_VEL 2u  /* initVel=False: no starting base velocity from the reference */

/* per-lane mode bits (hum_set_lane_modes) */
#define HUM_MODE_DEBUG 1u         /* step(action, debug=True): done only on fall (low_level_env.py:470-471) */
#define HUM_MODE_PREDEFINED 2u    /* usePredefinedTarget (low_level_env.py:253-255, 419-421) */

/* error flag bits (hum_get_error_flags) */
#define HUM_EFLAG_NONFINITE_ACTION 1u   /* humanoid.py:55 assert np.isfinite(a).all(): lane not stepped */
#define HUM_EFLAG_VEL_ROW 2u            /* frame beyond the velocity table (motion13_13): clamped row used */
#define HUM_EFLAG_CONTACT_OVERFLOW 4u   /* more contacts than a lowered max_contacts (never with the default) */
#define HUM_EFLAG_BAD_START_FRAME 8u    /* resetFromFrame start frame past the clip (the reference's iloc raises
                                           IndexError): lane left unchanged */
#define HUM_EFLAG_DIAG_BOUNDS 0x80000000u  /* bounds-checked diagnostic builds only (-DHUM_BOUNDS_CHECK): an index left
                                         its slice at a former generic-pointer access site (clamped) */

/* bookkeeping layout (doubles; integers stored exactly) */
enum {
    HUM_BK_FRAME = 0, HUM_BK_TIMESTEP, HUM_BK_RNG_COUNTER, HUM_BK_PRED_INDEX,
    HUM_BK_TARGET /* 3 */ = 4, HUM_BK_START_ROBOT_POS = 7, HUM_BK_ROBOT_POS = 10, HUM_BK_START_EP_POS = 13,
    HUM_BK_HL_DEG_TARGET = 16, HUM_BK_WALK_TARGET /* 2 */ = 17, HUM_BK_LOW_TARGET_SCORE = 19,
    HUM_BK_DELTA_JOINTS = 20, HUM_BK_DELTA_VEL_JOINTS = 21, HUM_BK_BODY_POSTURE = 22, HUM_BK_ELECTRICITY = 23,
    HUM_BK_JOINT_LIMIT = 24, HUM_BK_ALIVE = 25, HUM_BK_DELTA_LOW_TARGET = 26, HUM_BK_CLIP = 27,
    HUM_BK_MODE = 28,
    /* 64-bit RNG stream key as two u32 halves; initialised to splitmix64(splitmix64(seed) ^ (lane_offset + lane)) */
    HUM_BK_RNG_KEY_LO = 29, HUM_BK_RNG_KEY_HI = 30,
    /* hierarchical env only (hier_env.py): steps_remaining_at_level, num_high_level_steps, the agent expected
       to act next (1 = high), highTargetScore, cumulative_driftScore, driftScore, delta_highTargetScore,
       cumulative_aliveReward, flat_env.robot.body_xyz[0:2] of the last calc_state */
    HUM_BK_LEVEL_REMAINING = 31, HUM_BK_NUM_HIGH_STEPS = 32, HUM_BK_EXPECT_HIGH = 33, HUM_BK_HIGH_TARGET_SCORE = 34,
    HUM_BK_CUM_DRIFT = 35, HUM_BK_DRIFT = 36, HUM_BK_DELTA_HIGH_TARGET = 37, HUM_BK_CUM_ALIVE = 38,
    HUM_BK_BODY_XY /* 2 */ = 39,
    /* HUM_TERRAIN_RANDOM_BLOCKS: the 64-bit key of the lane's current terrain (two u32 halves), redrawn at every
       reset as CustomScene.episode_restart regenerates the heightfield (humanoid.py:89-113) */
    HUM_BK_TERRAIN_KEY_LO = 41, HUM_BK_TERRAIN_KEY_HI = 42
};

/* hum_set_terrain modes: the ground the contacts are generated against */
#define HUM_TERRAIN_PLANE 0          /* HumanoidBulletEnv's StadiumScene plane z = 0 (default; every config) */
#define HUM_TERRAIN_HEIGHTFIELD 1    /* one heightfield shared by all lanes (CustomScene.replaceHeightfieldData) */
#define HUM_TERRAIN_RANDOM_BLOCKS 2  /* LowLevelHumanoidEnv(useCustomEnv=True): per-lane CustomScene terrain */

/* hum_hier_step per-lane agent mask (which entries of the reference's obs/rew dicts are present) */
#define HUM_AGENT_HIGH 1u   /* "high_level_agent" obs + reward */
#define HUM_AGENT_LOW 2u    /* "low_level_agent" obs + reward */
/* hum_hier_step `agent` selector values: 1 = high, 0 = low, HUM_AGENT_SEL_SKIP = the lane got no action this
 * round (absent from RLlib's action dict): nothing is stepped or written for it except agents[i] = 0 */
#define HUM_AGENT_SEL_SKIP 255u

/* aux (RewardLogCallback, custom_callback.py:43-80) layout, float32 */
enum {
    HUM_AUX_DELTA_JOINTS = 0, HUM_AUX_DELTA_END_POINTS, HUM_AUX_LOW_TARGET_SCORE, HUM_AUX_DELTA_VEL_JOINTS,
    HUM_AUX_BODY_POSTURE, HUM_AUX_HIGH_TARGET_SCORE, HUM_AUX_DRIFT_SCORE, HUM_AUX_BASE_REWARD, HUM_AUX_ALIVE,
    HUM_AUX_ELECTRICITY, HUM_AUX_JOINT_LIMIT, HUM_AUX_DIST_FROM_ORIGIN,
    /* calcEndPointScore (low_level_env.py:361-382) of the lane's current state, frame, starting_ep_pos and
       highLevelDegTarget, as the reference method returns it when called after step()/resetFromFrame()
       (param_check.py:43-60): useExp=False and useExp=True.  Off the reward path in the reference (:445), so
       HUM_AUX_DELTA_END_POINTS stays the reference attribute's constant 0. */
    HUM_AUX_END_POINT_SCORE, HUM_AUX_END_POINT_SCORE_EXP,
    HUM_AUX_ROBOT_POS /* 3: robot_pos (custom_callback.py:79 reads it) */
};

/* hum_config.numpy_semantics: the float32 scalar arithmetic of the reference under the NumPy it runs with.
 * Two expressions mix a float32 numpy scalar with a Python float: `cur_obs[0] + initial_z` (calcAliveReward,
 * low_level_env.py:386, hier_env.py:448) and `force_gain * power * self.power * np.clip(a[i], -1, 1)`
 * (CustomHumanoidRobot.apply_action, humanoid.py:57-59).  NumPy 1.x (the reference's era: Ray 1.2.0, 2021)
 * promotes them to float64; NumPy >= 2 (NEP 50) keeps float32. */
#define HUM_NUMPY_1 1   /* default */
#define HUM_NUMPY_2 2

typedef struct hum_env hum_env;

typedef struct hum_config {
    int32_t n_lanes;          /* env instances on this GPU */
    int32_t device;           /* HIP device ordinal */
    uint64_t seed;            /* counter-based RNG seed (replaces the unseeded default_rng, :84) */
    int64_t lane_offset;      /* global id of lane 0 (RNG stream key) -> results independent of sharding */
    int32_t precision;        /* 0 = fp32 physics (default), 1 = fp64 physics */
    int32_t block_size;       /* threads per block (multiple of 64) */
    /* physics (defaults = pybullet_envs HumanoidBulletEnv: World(gravity 9.8, timestep 0.0165/4, frame_skip 4),
       numSolverIterations 5, setDefaultContactERP 0.9; see DESIGN.md for each choice) */
    double dt_env;            /* 0.0165 */
    int32_t substeps;         /* 4 */
    double gravity;           /* 9.8 */
    int32_t solver_iters;     /* 5 */
    double erp_contact, erp_limit, mu_ground, mu_self, contact_thresh;
    double lin_damp, ang_damp, limit_max_impulse, max_coord_vel;
    int32_t max_contacts;     /* HUM_MAX_CONTACTS (default: every candidate, nothing dropped); lower = diagnostic cap */
    int32_t self_collision;   /* 1 */
    int32_t joint_damping;    /* 1 = implicit MJCF joint damping */
    int32_t kernel;           /* 1 = cooperative (16 lanes/env, LDS-resident; default), 0 = one env per lane */
    int32_t hier;             /* 0 = LowLevelHumanoidEnv semantics (hum_reset/hum_step), 1 = HierarchicalHumanoidEnv
                                 (hum_hier_reset/hum_hier_step; clip = the selected motion, motion09_03) */
    int32_t envs_per_block;   /* cooperative kernel: envs per wavefront-block (4 = 64 threads (default), 2 = 32,
                                 1 = 16).  Fewer envs per wave buys SIMD co-residency but multiplies the wave
                                 instruction stream per env: measured 0.39 / 0.64 / 0.98 ms at 4096 envs */
    int32_t lds_rows;         /* cooperative kernel: constraint rows per block kept in LDS; 0 (default) = the whole
                                 pool (envs_per_block * 30), k > 0 caps it at k rows so the rest take the global
                                 spill path (testing) */
    int32_t numpy_semantics;  /* HUM_NUMPY_1 (default) or HUM_NUMPY_2, see above */
    double split_penetration; /* -0.04: Bullet's split impulse (btContactSolverInfo m_splitImpulse on,
                                 m_splitImpulsePenetrationThreshold -0.04).  A joint-limit or contact row whose
                                 penetration is deeper than this carries no position bias, only the velocity
                                 term: its position part goes to m_rhsPenetration, which btMultiBodyConstraintSolver
                                 never applies to multibodies.  -1e30 = every violation corrected at ERP */
} hum_config;

/* Version / build info. */
int hum_abi_version(void);
const char* hum_last_error(void);

/* Fill `cfg` with the reference defaults (n_lanes = 1, device 0, seed 0). */
void hum_default_config(hum_config* cfg);

/* Replaces LowLevelHumanoidEnv.__init__ (low_level_env.py:39-172) for n lanes. */
int hum_create(const hum_config* cfg, hum_env** out);
int hum_destroy(hum_env* env);

/* Upload one clip's four reference tables (low_level_env.py:59-70), row-major float64, fixed column
 * order: joints = rightHipX, rightHipY, rightHipZ, rightKnee, leftHipX, leftHipY, leftHipZ, leftKnee,
 * rightShoulderX, rightShoulderY, rightElbow, leftShoulderX, leftShoulderY, leftElbow (14);
 * end points = {LeftLeg, LeftFoot, RightLeg, RightFoot, Head, LeftForeArm, LeftHand, RightForeArm,
 * RightHand} x {X,Y,Z} (27).  max_frame = n_pos - 1 (:80-82). */
int hum_set_clip(hum_env* env, int32_t clip_id, const double* pos, int32_t n_pos, const double* vel, int32_t n_vel,
                 const double* rel, int32_t n_rel, const double* ep, int32_t n_ep);
/* Runtime clip ingestion (host code): parse the reference's CSV quadruple <dir>/<name>{JointPosRad,
 * JointSpeedRadSec,JointPosRadRelative,JointVecFromHip}.csv (low_level_env.py:58-70) with pandas' default float
 * converter (bit-identical tables), columns by header name in hum_set_clip's order.
 *   hum_clip_csv_sizes: rows of the four tables -> sizes4[4] (no GPU needed)
 *   hum_clip_csv_parse: the tables into caller buffers sized from hum_clip_csv_sizes (no GPU needed)
 *   hum_load_clip_csv: parse + hum_set_clip(env, clip_id, ...)
 * Errors: HUM_ERR_ARG with the reason in hum_last_error(). */
int hum_clip_csv_sizes(const char* dir, const char* name, int32_t* sizes4);
int hum_clip_csv_parse(const char* dir, const char* name, double* pos, double* vel, double* rel, double* ep);
int hum_load_clip_csv(hum_env* env, int32_t clip_id, const char* dir, const char* name);

/* Ground of the handle's lanes (LowLevelHumanoidEnv(useCustomEnv=True) -> humanoid.py:68-144 CustomScene, a
 * pybullet GEOM_HEIGHTFIELD body instead of the plane).  Cooperative kernel (hum_config.kernel = 1), low-level
 * env (hier = 0) only.
 *   HUM_TERRAIN_PLANE: the plane z = 0 (default).
 *   HUM_TERRAIN_HEIGHTFIELD: heights[w * l] float32, vertex (i, j) = heights[i + j * w] (pybullet heightfieldData
 *     order: i along x), mesh scale scale3, body at origin3 (identity orientation); Bullet's btHeightfieldTerrainShape
 *     geometry: vertex (i, j) at origin + scale * (i - (w-1)/2, j - (l-1)/2, h - (min + max)/2), two triangles per
 *     cell split by diamond subdivision.  CustomScene.replaceHeightfieldData(d) = (d, 256, 256, {1,1,1}, {0,0,0.25}).
 *     Requires scale x, y >= 0.25 (a candidate then tests at most 2 x 2 cells per substep).
 *   HUM_TERRAIN_RANDOM_BLOCKS: CustomScene.episode_restart's terrain per lane, regenerated at every reset: 256 x 256
 *     vertices in 2 x 2 blocks of height random.uniform(0, 0.05) * 10, the four centre blocks 0, body at
 *     (0, 0, 0.25); block heights are counter-based draws from the lane's terrain key (HUM_BK_TERRAIN_KEY_*),
 *     and the vertical centring uses the distribution's range (0 + 0.5) / 2.  heights / w / l /
 *     scale3 / origin3 are ignored (may be NULL).
 * Contacts: every sphere / capsule-end ground candidate against the closest point of the terrain surface (the
 * cells within reach).  A captured step graph is recaptured. */
int hum_set_terrain(hum_env* env, int32_t mode, const float* heights, int32_t w, int32_t l, const double* scale3,
                    const double* origin3);
/* hum_set_terrain with the heightfield's vertical centre given: Bullet's btHeightfieldTerrainShape centres the data
 * on (min + max) / 2 of the heights it was CREATED with, and pybullet's createCollisionShape(replaceHeightfieldIndex=
 * ...) - CustomScene.replaceHeightfieldData, humanoid.py:75-85 - replaces the heights but keeps that centre (the
 * CustomScene creation terrain's, 0.25).  centre NULL = (min + max) / 2 of `heights` (a newly created shape). */
int hum_set_terrain_ex(hum_env* env, int32_t mode, const float* heights, int32_t w, int32_t l, const double* scale3,
                       const double* origin3, const double* centre);

/* clip id per lane (host array of n_lanes); default all 0 */
int hum_set_lane_clips(hum_env* env, const int32_t* clip_of_lane);
/* per-lane HUM_MODE_* bits (host array of n_lanes) */
int hum_set_lane_modes(hum_env* env, const uint32_t* modes);
/* shared predefined target course (env_check.py:104-116): n x 3 float64 */
int hum_set_predefined_targets(hum_env* env, const double* xyz, int32_t n);

/* reset()/resetFromFrame() (low_level_env.py:224-305) for lanes with lane_mask[i] != 0 (device u8, NULL = all).
 * start_frame (device i32, NULL or < 0 = draw from the lane RNG as reset() does; >= the clip's pose rows =
 * HUM_EFLAG_BAD_START_FRAME, lane unchanged), reset_yaw_deg (device f64, NULL = 0).
 * obs_out: device float32 [n,70] (rows of unmasked lanes untouched). */
int hum_reset(hum_env* env, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
              float* obs_out, void* stream);

/* hum_reset with resetFromFrame's startFromRef / initVel switches (HUM_RESET_* flags). */
int hum_reset_ex(hum_env* env, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
                 uint32_t flags, float* obs_out, void* stream);

/* step(action) (low_level_env.py:475-526) for all lanes: device float32 actions [n,17] ->
 * obs [n,70] f32, reward [n] f32, done [n] u8, frame [n] i32 (frame may be NULL).
 * With HUM_STEP_AUTORESET, done lanes are reset in the same launch; their post-reset observation is
 * written to obs_reset (device [n,70], may be NULL) while `obs` keeps the terminal observation. */
int hum_step(hum_env* env, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
             uint32_t flags, float* obs_reset, void* stream);

/* k env steps for all lanes in ONE launch (the loop RLlib's sampler runs over a rollout fragment,
 * low_level_env.py:475-526 per step): actions [k,n,17] f32 -> obs [k,n,70], reward [k,n], done [k,n],
 * frame [k,n] (may be NULL); step t reads actions[t] and writes row t of every output, and with
 * HUM_STEP_AUTORESET a lane done at step t is reset before step t + 1 (obs_reset [k,n,70], rows of the lanes
 * reset at step t written, may be NULL).  Results are identical to k hum_step calls on the same buffers' rows;
 * each env's working set stays on chip between its steps, and a fast wavefront runs ahead instead of waiting
 * for the slowest one of every launch.  k = 1 is hum_step. */
int hum_step_k(hum_env* env, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
               uint32_t flags, float* obs_reset, int32_t k, void* stream);

/* Capture `k` consecutive steps (same buffers, same flags) in a hipGraph and replay it on the handle's
 * own stream (hum_stream()); inputs must be ready (synchronise the producing stream first). */
int hum_step_graph(hum_env* env, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
                   uint32_t flags, float* obs_reset, int32_t k);

/* HierarchicalHumanoidEnv.reset()/resetFromFrame() (hier_env.py:235-319) for masked lanes (hier handles only):
 * start_frame NULL = reset(): draw startFrame then resetYaw from the lane RNG (:239-240); given = resetFromFrame
 * with reset_yaw_deg (NULL = 0).  high_obs_out: device float32 [n,44] = {"high_level_agent": obs}. */
int hum_hier_reset(hum_env* env, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
                   float* high_obs_out, void* stream);

/* hum_hier_reset with resetFromFrame's startFromRef / initVel switches (HUM_RESET_* flags). */
int hum_hier_reset_ex(hum_env* env, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
                      uint32_t flags, float* high_obs_out, void* stream);

/* HierarchicalHumanoidEnv.step(action_dict) (hier_env.py:355-366, 538-641) for all lanes: each lane applies the
 * action of the agent it expects (the one that received an observation; `agent` (device u8 [n], 1 = high, 0 = low,
 * HUM_AGENT_SEL_SKIP = not stepped) overrides it, NULL = expected): high_act [n,2] f32 -> high_level_step (no physics), low_act [n,17] f32 ->
 * low_level_step.  Outputs: agents [n] u8 (HUM_AGENT_* bits present in the reference's returned dicts),
 * high_obs [n,44] / low_obs [n,70] (rows written only where present), high_rew / low_rew [n] (0 where absent),
 * done [n] u8 (done["__all__"]), frame [n] i32 (may be NULL).  HUM_STEP_AUTORESET resets done lanes in the
 * same launch and writes their new high-level obs to high_obs_reset ([n,44], may be NULL). */
int hum_hier_step(hum_env* env, const float* high_act, const float* low_act, const uint8_t* agent, uint8_t* agents,
                  float* high_obs, float* low_obs, float* high_rew, float* low_rew, uint8_t* done, int32_t* frame,
                  uint32_t flags, float* high_obs_reset, void* stream);

/* k agent transitions per lane in ONE launch (hum_hier_step's semantics per transition): every per-transition
 * array gains a leading [k] axis (high_act [k,n,2], low_act [k,n,17], agent [k,n] or NULL, agents [k,n],
 * high_obs [k,n,44], low_obs [k,n,70], high_rew / low_rew / done / frame [k,n], high_obs_reset [k,n,44]).
 * With agent == NULL every lane applies the action of the agent it expects at that transition. */
int hum_hier_step_k(hum_env* env, const float* high_act, const float* low_act, const uint8_t* agent, uint8_t* agents,
                    float* high_obs, float* low_obs, float* high_rew, float* low_rew, uint8_t* done, int32_t* frame,
                    uint32_t flags, float* high_obs_reset, int32_t k, void* stream);

/* ---- Trajectory packing for the learner feed (reference: RLlib rollout workers ship SampleBatches of
 * obs / actions / rewards / dones to the learner, train_config.py:33-34).  One launch copies k steps x n lanes of up to
 * HUM_PACK_MAX_FIELDS row fields from their time-major step outputs (row (t, i) at src + t * src_step + i * src_lane
 * bytes, e.g. hum_step_k's [k,n,70] obs) into a lane-major record buffer (row (t, i) at dst + i * dst_lane +
 * (t0 + t) * dst_step bytes): each lane's record then holds its steps contiguously, and a rank's whole fragment is one
 * message for the gather.  Rows are copied as raw bytes (row_bytes a multiple of 4, or 1 for u8 fields of width 1). */
#define HUM_PACK_MAX_FIELDS 6
typedef struct {
    const void* src;
    void* dst;
    int64_t src_step, src_lane, dst_step, dst_lane;   /* byte strides */
    int32_t row_bytes;
} hum_pack_field;
int hum_pack_rows(const hum_pack_field* fields, int32_t nfields, int32_t k, int32_t n, int32_t t0, void* stream);

/* ---- The fragment transport without compute units (ABI 14; reference: the rollout workers' sample
 * batches travel to the learner, train_config.py:33-34).  The env kernel occupies every CU for a launch's whole
 * duration (a SIMD's register file per wave, a CU's LDS per four blocks), so a collective's kernels cannot run beside
 * it; the SDMA copy engines can.  Each rank exports its packed send buffers once (hum_ipc_export: a device pointer,
 * possibly inside a larger allocation, -> handle + offset), the learner rank maps them (hum_ipc_open) and pulls each
 * fragment with hum_dma_copy (an SDMA engine, forced; over xGMI between GPUs), completing with hum_dma_wait.  Host
 * calls only: ordering against the streams that produce / consume the buffers is the caller's
 * (ilrl_amd/parallel.py DmaGather: events and a host control channel). */
#define HUM_IPC_HANDLE_BYTES 64
int hum_ipc_export(const void* dev_ptr, uint8_t* handle /* [HUM_IPC_HANDLE_BYTES] */, uint64_t* offset);
int hum_ipc_open(const uint8_t* handle, uint64_t offset, void** dev_ptr);
int hum_ipc_close(void* dev_ptr);   /* the pointer hum_ipc_open returned minus its offset (the mapping's base) */
typedef struct {
    uint64_t signal;   /* the copy's completion signal (0: none in flight) */
    uint64_t bytes;
} hum_dma_ticket;
/* engine: an index into the SDMA engines the runtime reports for this (dst, src) pair, taken modulo their count, so
 * concurrent pulls from several peers can spread over engines */
int hum_dma_copy(void* dst, const void* src, uint64_t bytes, int32_t engine, hum_dma_ticket* ticket);
int hum_dma_wait(hum_dma_ticket* ticket);

/* ---- On-GPU policy inference: the reference's PPO policy network (train_config.py:107-111,
 * RLlib FullyConnectedNetwork, fcnet_hiddens [256, 256], tanh, free_log_std) evaluated on the env's device
 * buffers, so a sampler loop needs no host round trip.  Weights: host float32, TF kernel layout [in][out]:
 * w1 [70,256], b1 [256], w2 [256,256], b2 [256], w3 [256,17], b3 [17], log_std [17] (NULL = zeros). */
typedef struct hum_policy hum_policy;
int hum_policy_create(int32_t device, const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* w3, const float* b3, const float* log_std, uint64_t seed, hum_policy** out);
/* The same network for any input / output width n_in <= 72, n_out <= 32: w1 [n_in,256], w3 [256,n_out], b3 and
 * log_std [n_out]; the observation and action rows of hum_policy_act are then n_in / n_out wide.  The hierarchical
 * env's high-level policy is 44 -> 2 (train_config.py:23-27, 262-298: "high_level_policy" on the 44-dim high
 * observation, 2-dim heading action, same FCNet config); hum_policy_create is (70, 17).  hum_rollout and
 * hum_rollout_fused need a (70, 17) policy. */
int hum_policy_create_ex(int32_t device, int32_t n_in, int32_t n_out, const float* w1, const float* b1, const float* w2,
                         const float* b2, const float* w3, const float* b3, const float* log_std, uint64_t seed,
                         hum_policy** out);
int hum_policy_destroy(hum_policy* policy);
/* actions [n,17] (device) = clip(mean + explore * exp(log_std) * N(0,1), -1, 1) (RLlib clip_actions) for the
 * observations obs [n,70]; lanes with done[i] != 0 read obs_reset[i] instead (the auto-reset observation; both
 * NULL = obs only).  mean_out [n,17] and obs_in_out [n,70] (the observation rows used) are optional.  Noise is
 * counter-based: (seed, lane, step, action index). */
int hum_policy_act(hum_policy* policy, const float* obs, const float* obs_reset, const uint8_t* done, int32_t n,
                   float* actions, float* mean_out, float* obs_in_out, int32_t explore, uint64_t step, void* stream);
/* hum_policy_act that also returns raw_out [n,17] (device, may be NULL): the sample before clip_actions, i.e. the
 * action RLlib's SampleBatch records and PPO evaluates its likelihood ratio on. */
int hum_policy_act_ex(hum_policy* policy, const float* obs, const float* obs_reset, const uint8_t* done, int32_t n,
                      float* actions, float* mean_out, float* obs_in_out, float* raw_out, int32_t explore, uint64_t step,
                      void* stream);
/* k sampler steps (policy -> hum_step with HUM_STEP_AUTORESET) on `stream` with no host round trip.  obs,
 * obs_reset, done, reward: the env-step buffers (device [n,70], [n,70], [n], [n]); on entry obs holds the current
 * observation and done the previous step's flags (zeros after a reset); act_buf [n,17] scratch.  Optional device
 * trajectory outputs: obs_traj [k,n,70] (the policy inputs), act_traj [k,n,17] (the samples before clip_actions, as
 * RLlib records them; the env steps on their clip), rew_traj [k,n], done_traj [k,n].  The env handle and the policy
 * must be on the same device (HUM_ERR_ARG otherwise). */
int hum_rollout(hum_env* env, hum_policy* policy, int32_t k, int32_t explore, uint64_t step0, float* obs,
                float* obs_reset, uint8_t* done, float* reward, float* act_buf, float* obs_traj, float* act_traj,
                float* rew_traj, uint8_t* done_traj, void* stream);
/* hum_rollout in ONE launch: the policy network is evaluated inside the multi-step env kernel (per wave, before
 * each step's physics), so the k steps keep their state in LDS and the launch's slowest-wave tail is paid once per k
 * steps instead of once per step.  Same arguments and outputs as hum_rollout (act_buf receives the last step's
 * clipped actions; obs / done / reward end as the last step left them) with one difference: obs_reset receives
 * the reset observation of the lanes done at the LAST step only (hum_rollout writes it at every step's resets;
 * inside the launch a reset lane's new observation goes straight to the next step's policy and into obs_traj).
 * Without rew_traj / done_traj the per-step rows go to scratch kept on the handle (grown on demand, no sync; the
 * scratch is ordered on the call's stream only, so every call on one handle must use one stream, or the caller
 * orders its streams with events).  The policy arithmetic is the
 * same k-ordered fp32 fma chains; the physics is the benchmarked kernel's.  Needs a handle with the cooperative fp32
 * kernel, 4 envs per block, plane ground and the low-level env (HUM_ERR_STATE otherwise: use hum_rollout).
 * Replaces: the RLlib sampler's compute_actions -> env.step loop (train_config.py:107-111, low_level_env.py:475). */
int hum_rollout_fused(hum_env* env, hum_policy* policy, int32_t k, int32_t explore, uint64_t step0, float* obs,
                      float* obs_reset, uint8_t* done, float* reward, float* act_buf, float* obs_traj, float* act_traj,
                      float* rew_traj, uint8_t* done_traj, void* stream);
/* hum_rollout_fused with one more optional trace (ABI 13): mean_traj [k,n,17], the policy's mean per step and lane
 * (the DiagGaussian's loc, the first half of RLlib's action_dist_inputs) as the in-kernel network forms it before the
 * sample - bitwise what hum_policy_act_ex's mean_out gives for the same observation row.  With it a SampleBatch's
 * action_dist_inputs / action_logp need no second network evaluation. */
int hum_rollout_fused_ex(hum_env* env, hum_policy* policy, int32_t k, int32_t explore, uint64_t step0, float* obs,
                         float* obs_reset, uint8_t* done, float* reward, float* act_buf, float* obs_traj,
                         float* act_traj, float* rew_traj, uint8_t* done_traj, float* mean_traj, void* stream);

/* ---- Two-level sampler loop (BASELINE config 5; hier_env.py:355-366, 538-642 driven by the reference's two PPO
 * policies, train_config.py:262-298 policy_mapping_fn: "high_level_agent" -> high_level_policy (44 -> 2),
 * "low_level_agent" -> low_level_policy (70 -> 17)).  Per transition, on `stream`: the high-level policy acts on
 * every lane's latest high observation (lanes done at the previous transition: their auto-reset high observation),
 * the low-level policy on every lane's latest low observation, then one hum_hier_step with HUM_STEP_AUTORESET
 * steps each lane with the action of the agent it expects (its own level counter, hier_env.py:363-366).  The env
 * buffers (device, all required) persist across calls: */
typedef struct {
    float* obs_high;        /* [n,44] in/out: each lane's latest high-level observation (after hum_hier_reset: its obs) */
    float* obs_high_reset;  /* [n,44] in/out: the high observation of lanes auto-reset at the last transition */
    float* obs_low;         /* [n,70] in/out: each lane's latest low-level observation */
    uint8_t* done;          /* [n] in/out: the last transition's done flags (zeros after hum_hier_reset) */
    uint8_t* agents;        /* [n] out: agents in the last transition's returned dicts (HUM_AGENT_*) */
    float* rew_high;        /* [n] out */
    float* rew_low;         /* [n] out */
    float* act_high;        /* [n,2] out: the last transition's clipped high-level actions */
    float* act_low;         /* [n,17] out: the last transition's clipped low-level actions */
} hum_hier_io;
/* Per-transition trajectory rows [k,n,...] (device; the struct pointer or any field may be NULL): */
typedef struct {
    uint8_t* acted;         /* [k,n] the agent that acted (HUM_AGENT_HIGH / HUM_AGENT_LOW) */
    float* obs_high;        /* [k,n,44] the high policy's inputs */
    float* act_high;        /* [k,n,2] its samples before clip_actions (what RLlib's SampleBatch records) */
    float* obs_low;         /* [k,n,70] the low policy's inputs */
    float* act_low;         /* [k,n,17] its samples before clip_actions */
    uint8_t* agents;        /* [k,n] agents in the returned dicts */
    float* rew_high;        /* [k,n] */
    float* rew_low;         /* [k,n] */
    uint8_t* done;          /* [k,n] */
} hum_hier_traj;
/* Equal, bitwise, to the loop hum_policy_act_ex(high) ; hum_policy_act_ex(low) ; hum_hier_step(agent = NULL,
 * HUM_STEP_AUTORESET) driven step by step (noise step index step0 + t for both policies, each with its own seed).
 * Needs a hierarchical handle, a (44, 2) and a (70, 17) policy on its device (HUM_ERR_ARG / _STATE otherwise).
 * Replaces: RLlib's multi-agent sampler loop over HierarchicalHumanoidEnv (Train Ray RLLib Hierarchical.py:48-88). */
int hum_hier_rollout(hum_env* env, hum_policy* high, hum_policy* low, int32_t k, int32_t explore, uint64_t step0,
                     const hum_hier_io* io, const hum_hier_traj* traj, void* stream);
/* hum_hier_rollout in ONE launch: both networks run inside the cooperative kernel's step loop, each only for the
 * lanes whose expected agent it is.  Equal, bitwise, to hum_hier_rollout on everything the acting agent produces:
 * the acting agent's trajectory rows (obs / act of the high or the low policy, per `acted`), agents, both rewards,
 * done, acted, the env buffers' observations and the final state.  Differences: trajectory rows of the agent that
 * did NOT act on a lane are left unwritten (hum_hier_rollout evaluates both networks on every lane and records
 * both), and io->act_high / io->act_low receive the last transition's clipped action of the acting agent only (the
 * other agent's row keeps its previous content).  Needs the cooperative fp32 kernel (hum_config.kernel = 1,
 * precision fp32, envs_per_block 4) and plane ground (HUM_ERR_STATE otherwise: use hum_hier_rollout).  Missing
 * agents / reward / done trajectory rows go to the handle's scratch, which is stream-ordered: every call on one
 * handle must use one stream (or order its streams with events). */
int hum_hier_rollout_fused(hum_env* env, hum_policy* high, hum_policy* low, int32_t k, int32_t explore,
                           uint64_t step0, const hum_hier_io* io, const hum_hier_traj* traj, void* stream);
/* hum_hier_rollout_fused with the two policies' mean traces (ABI 13, each optional): mean_high [k,n,2], mean_low
 * [k,n,17], written for the acting agent's rows only (the other agent's rows are left unwritten), bitwise what
 * hum_policy_act_ex's mean_out gives for the recorded observation row. */
int hum_hier_rollout_fused_ex(hum_env* env, hum_policy* high, hum_policy* low, int32_t k, int32_t explore,
                              uint64_t step0, const hum_hier_io* io, const hum_hier_traj* traj, float* mean_high,
                              float* mean_low, void* stream);

/* RewardLogCallback terms (custom_callback.py:43-80) per lane: device float32 [n, HUM_NAUX]. */
int hum_get_aux(hum_env* env, float* aux_out, void* stream);

/* Synchronous state access (host float64): phys [n,47], book [n,HUM_NBOOK]; either may be NULL. */
int hum_get_state(hum_env* env, double* phys, double* book);
int hum_set_state(hum_env* env, const double* phys, const double* book);

/* Parts positions (33 x 3, pybullet parts dict order incl. 'floor') per lane, host float64 [n,33,3]. */
int hum_get_parts(hum_env* env, double* parts);

/* Sticky error bits (HUM_EFLAG_*) accumulated by kernels since the last call; synchronises. */
int hum_get_error_flags(hum_env* env, uint32_t* flags);

int hum_sync(hum_env* env);
int32_t hum_num_lanes(const hum_env* env);
/* hipStream_t of the handle (as void*) */
void* hum_stream(hum_env* env);

#ifdef __cplusplus
}
#endif
#endif /* HUMANOID_ENV_H */

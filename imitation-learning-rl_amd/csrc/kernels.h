// kernels.h - device side of the vectorised humanoid env: SoA lane I/O, LowLevelHumanoidEnv and
// HierarchicalHumanoidEnv logic (reset / post-physics step), and the step / reset / aux kernels.
//
// Shared by two translation units: humanoid_env.hip (C-ABI host code + every kernel variant except the
// benchmarked one) and group_f32.hip, which instantiates ONLY step_group_kernel<float, 4>.  Compiling the
// hot kernel alone keeps its code generation independent of its sibling variants (co-compiled template
// variants share inlining and register-allocation decisions: measured 0.294 vs 0.250 ms per step).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/humanoid_env.h"
#include "physics.h"
#include "envlogic.h"
#include "physics_group.h"

namespace hkk {
using namespace hk;

constexpr int NBOOK_I = 13;   // frame, timestep, pred_idx, clip, rng_ctr, mode, rng key lo, rng key hi
                              // | hier: level_rem, n_high, expect_high | terrain key lo, hi (terrain 2)
constexpr int NBOOK_D = 30;   // target3 srp3 robot_pos3 sep3 hldt wt2 lts dj dvj bps es jls alive dlts
                              // | hier: hts cum_drift drift dhts cum_alive bxy2

struct DevState {
    void* phys;        // Real [47][n]
    int* bi;           // [6][n]
    double* bd;        // [23][n]
    void* scratch;     // Real [SCRATCH_PER_LANE][n]
    float* aux_tmp;
};

struct KArgs {
    int n;
    unsigned long long seed;
    long long lane_offset;
    PhysParams P;
    const ClipDev* clips;   // device array [HUM_MAX_CLIPS] (a by-value array here is dynamically indexed -> scratch copy)
    const double* pred;
    int npred;
    void* phys;
    int* bi;
    double* bd;
    void* scratch;
    unsigned* eflags;
    // step
    const float* act;
    float* obs;
    float* rew;
    unsigned char* done;
    int* frame_out;
    float* obs_reset;
    unsigned flags;
    // reset
    const unsigned char* mask;
    const int* start_frame;
    const double* reset_yaw;
    unsigned reset_flags;           // HUM_RESET_* (resetFromFrame startFromRef / initVel = False)
    float* aux;
    // hierarchical env (hum_hier_step / hum_hier_reset)
    int hier;
    int np1;                        // hum_config.numpy_semantics == HUM_NUMPY_1: float64 scalar promotion
    const float* act_high;          // [n,2]
    const unsigned char* agent_sel; // [n] 1 = high, 0 = low (NULL = the lane's expected agent)
    unsigned char* agents;          // [n] HUM_AGENT_* present in the returned dicts
    float* obs_high;                // [n,44]
    float* rew_high;                // [n]
    float* obs_high_reset;          // [n,44]
    // multi-step launch (hum_step_k / hum_hier_step_k): env steps per launch; the per-step inputs and outputs
    // above are then [ksteps, n, ...] arrays, step-major: lane i's row of step t is io = t * n + i
    int ksteps;
    // fused rollout (hum_rollout_fused, POLICY kernels): the policy network acts inside the step loop.  pw = the
    // hum_policy weight block (w1 [72][256] with rows 70, 71 zero, b1 [256], w2 [256][256], b2 [256], w3 [256][17],
    // b3 [17], log_std [17]); done_in = the previous step's done flags (step 0 input); per-step traces [k, n, ...]
    const float* pw;
    const unsigned char* done_in;
    float* obs_traj;
    float* act_traj;
    float* act_last;                // [n,17] the last step's clipped actions (hum_rollout's act_buf)
    unsigned long long pseed, pstep0;
    int pexplore;
    // hierarchical env, optional [ksteps, n]: the agent that acted in each transition (HUM_AGENT_HIGH / _LOW; 0 = the
    // lane was not stepped: no action for it, or a non-finite low-level action) - hum_hier_rollout's trajectory
    unsigned char* acted;
    // fused two-level rollout (hum_hier_rollout_fused, the POLICY == 2 kernel): the high-level network (the same
    // block layout at 44 -> 2) and its seed / trace rows; the low level uses pw / pseed / obs_traj / act_traj /
    // act_last above.  The [n, ...] observation buffers (obs, obs_high, obs_high_reset) are then updated in place
    // (row i) rather than per step, exactly as the step-by-step loop's env buffers are.
    const float* pw_high;
    unsigned long long pseed_high;
    float* obs_traj_high;
    float* act_traj_high;
    float* act_last_high;
    // optional [ksteps, n, 17] / [ksteps, n, 2]: the policy means (RLlib's action_dist_inputs mean half) of the acting
    // envs, as the networks form them before the DiagGaussian sample (hum_rollout_fused_ex / hum_hier_rollout_fused_ex)
    float* mean_traj;
    float* mean_traj_high;
};

// CustomHumanoidRobot.apply_action torque of motor k (humanoid.py:54-60): float(force_gain * power * 0.41 *
// np.clip(a, -1, 1)) - a float32 product under NumPy >= 2 (NEP 50), float64 under NumPy 1.x
__device__ inline double motor_torque(bool np1, float gain_f, double gain_d, float act) {
    const float c = fminf(fmaxf(act, -1.f), 1.f);
    return np1 ? gain_d * (double)c : (double)(gain_f * c);
}
// calcAliveReward (low_level_env.py:384-387): cur_obs[0] (float32) + initial_z 0.8 > 0.75, same promotion rule
__device__ inline double alive_reward(bool np1, float obs0) {
    return (np1 ? ((double)obs0 + 0.8) > 0.75 : (obs0 + 0.8f) > 0.75f) ? 2.0 : -1.0;
}

// ----------------------------------------------------------------------------------- SoA lane I/O
// full = false: the cooperative kernel's low-level step, which overwrites robot_pos and the reward terms (dj, dvj,
// bps, es, jls, alive, dlts) before it reads them (low_level_env.py:481-511): those 80 B are not fetched
__device__ inline void load_book(const KArgs& a, int i, Book& b, bool full = true) {
    const int* bi = a.bi;
    b.frame = bi[0 * a.n + i]; b.timestep = bi[1 * a.n + i]; b.pred_idx = bi[2 * a.n + i];
    b.clip = bi[3 * a.n + i]; b.rng_ctr = (unsigned)bi[4 * a.n + i]; b.mode = (unsigned)bi[5 * a.n + i];
    b.rng_key = (unsigned long long)(unsigned)bi[6 * a.n + i] | ((unsigned long long)(unsigned)bi[7 * a.n + i] << 32);
    b.terrain_key = a.P.terrain == HUM_TERRAIN_RANDOM_BLOCKS
        ? ((unsigned long long)(unsigned)bi[11 * a.n + i] | ((unsigned long long)(unsigned)bi[12 * a.n + i] << 32)) : 0ull;
    const double* d = a.bd;
    auto D = [&](int e) { return d[(long)e * a.n + i]; };
    for (int k = 0; k < 3; k++) { b.target[k] = D(k); b.srp[k] = D(3 + k); b.sep[k] = D(9 + k); }
    b.hldt = D(12); b.wt[0] = D(13); b.wt[1] = D(14); b.lts = D(15);
    if (full) {
        for (int k = 0; k < 3; k++) b.robot_pos[k] = D(6 + k);
        b.dj = D(16); b.dvj = D(17); b.bps = D(18); b.es = D(19); b.jls = D(20); b.alive = D(21); b.dlts = D(22);
    }
    if (a.hier) {
        b.level_rem = bi[8 * a.n + i]; b.n_high = bi[9 * a.n + i]; b.expect_high = bi[10 * a.n + i];
        b.hts = D(23); b.cum_drift = D(24); b.drift = D(25); b.dhts = D(26); b.cum_alive = D(27);
        b.bxy[0] = D(28); b.bxy[1] = D(29);
    }
}
template <typename T>
__device__ inline void load_lane(const KArgs& a, int i, T* st, Book& b) {
    const T* ph = (const T*)a.phys;
#pragma unroll
    for (int e = 0; e < HUM_NSTATE; e++) st[e] = ph[(long)e * a.n + i];
    load_book(a, i, b);
}
__device__ inline void store_book(const KArgs& a, int i, const Book& b) {
    int* bi = a.bi;
    bi[0 * a.n + i] = b.frame; bi[1 * a.n + i] = b.timestep; bi[2 * a.n + i] = b.pred_idx;
    bi[3 * a.n + i] = b.clip; bi[4 * a.n + i] = (int)b.rng_ctr; bi[5 * a.n + i] = (int)b.mode;
    if (a.P.terrain == HUM_TERRAIN_RANDOM_BLOCKS) {
        bi[11 * a.n + i] = (int)(unsigned)(b.terrain_key & 0xffffffffull);
        bi[12 * a.n + i] = (int)(unsigned)(b.terrain_key >> 32);
    }
    double* d = a.bd;
    auto D = [&](int e) -> double& { return d[(long)e * a.n + i]; };
    for (int k = 0; k < 3; k++) { D(k) = b.target[k]; D(3 + k) = b.srp[k]; D(6 + k) = b.robot_pos[k]; D(9 + k) = b.sep[k]; }
    D(12) = b.hldt; D(13) = b.wt[0]; D(14) = b.wt[1]; D(15) = b.lts;
    D(16) = b.dj; D(17) = b.dvj; D(18) = b.bps; D(19) = b.es; D(20) = b.jls; D(21) = b.alive; D(22) = b.dlts;
    if (a.hier) {
        bi[8 * a.n + i] = b.level_rem; bi[9 * a.n + i] = b.n_high; bi[10 * a.n + i] = b.expect_high;
        D(23) = b.hts; D(24) = b.cum_drift; D(25) = b.drift; D(26) = b.dhts; D(27) = b.cum_alive;
        D(28) = b.bxy[0]; D(29) = b.bxy[1];
    }
}
template <typename T>
__device__ inline void store_lane(const KArgs& a, int i, const T* st, const Book& b) {
    T* ph = (T*)a.phys;
#pragma unroll
    for (int e = 0; e < HUM_NSTATE; e++) ph[(long)e * a.n + i] = st[e];
    store_book(a, i, b);
}

__device__ inline int draw(const KArgs& a, int i, Book& b, int lo, int hi) {
    return lane_draw_key(b.rng_key, b.rng_ctr++, lo, hi);
}

// flat_env.reset()'s WalkerBase.robot_specific_reset: every joint at U(-0.1, 0.1), velocity 0, drawn from the
// robot's own np_random (a stream apart from the env's rng): key' = splitmix64(key ^ salt), 32 counters per
// reset taken at the env stream's current counter (oracle/oracle.py::LaneRNG.joint_noise)
template <typename T>
__device__ inline void joint_noise(const Book& b, T* st) {
    const unsigned long long k2 = splitmix64(b.rng_key ^ 0xD1B54A32D192ED03ull);
#pragma unroll
    for (int d = 0; d < NDOF; d++) {
        const unsigned long long x = splitmix64(k2 + (((unsigned long long)b.rng_ctr << 5) | (unsigned)d));
        const double u = (double)(x >> 11) * 0x1.0p-53;
        st[13 + d] = (T)(-0.1 + (0.1 - -0.1) * u);
        st[30 + d] = T(0);
    }
}

// ----------------------------------------------------------------------------------- reset
// LowLevelHumanoidEnv.reset() / resetFromFrame() (low_level_env.py:224-305)
template <typename T>
__device__ __attribute__((always_inline)) void reset_lane(const KArgs& a, int i, T* st, Book& b, int start_frame, double reset_yaw, float* obs,
                           unsigned& ef, const T* scs = nullptr) {   // scs: the reset pose's hinge sin / cos
    const ClipDev& c = a.clips[b.clip];
    // flat_env.reset() -> CustomScene.episode_restart: a new random terrain (humanoid.py:89-113)
    if (a.P.terrain == HUM_TERRAIN_RANDOM_BLOCKS) b.terrain_key = next_terrain_key(b.terrain_key, b.rng_key);
    const bool ref = !(a.reset_flags & HUM_RESET_NO_REF_POSE);                // startFromRef
    const bool init_vel = ref && !(a.reset_flags & HUM_RESET_NO_INIT_VEL);   // startFromRef and initVel (:291)
    if (ref && start_frame < 0) start_frame = draw(a, i, b, 0, c.max_frame - 5);   // :228
    // flat_env.reset(): restoreState -> zero velocities, joints re-randomised (all 17 overwritten below when
    // starting from the reference)
#pragma unroll
    for (int e = 0; e < HUM_NSTATE; e++) st[e] = 0;
    st[6] = 1;
    if (!ref) joint_noise(b, st);
    b.timestep = 0;
    if ((b.mode & HUM_MODE_PREDEFINED) && a.npred > 0) {                   // :253-255
        b.pred_idx = 0;
        for (int k = 0; k < 3; k++) b.target[k] = a.pred[k];
    } else {                                                                // :257, getRandomVec :240-245
        const double r = 0 + (double)draw(a, i, b, -180, 180) * DEG2RAD;
        b.target[0] = cos(r) * 5;
        b.target[1] = sin(r) * 5;
        b.target[2] = 0;
    }
    if (ref) {                                                              // :259-261 setJointsOrientation
        b.frame = start_frame;
        int vrow = start_frame;
        if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
        for (int j = 0; j < NREF; j++) {
            st[13 + JM_DOF[j]] = (T)c.gpos()[start_frame * 14 + JM_COL[j]];
            st[30 + JM_DOF[j]] = (T)c.gvel()[vrow * 14 + JM_COL[j]];
        }
    }
    for (int k = 0; k < 3; k++) { b.robot_pos[k] = 0; b.srp[k] = 0; }      // :264-268
    st[0] = 0; st[1] = 0; st[2] = (T)1.17;
    const double degToTarget = atan2(b.target[1], b.target[0]) * RAD2DEG;  // :270
    b.wt[0] = cos(degToTarget) * 1000;                                      // :271 (degrees into cos: quirk)
    b.wt[1] = sin(degToTarget) * 1000;
    const double th = (degToTarget + reset_yaw) * DEG2RAD;                  // :272-273 scipy from_euler
    st[3] = 0; st[4] = 0; st[5] = (T)sin(th / 2); st[6] = (T)cos(th / 2);
    b.hldt = degToTarget * DEG2RAD;                                         // :275
    // starting_ep_pos (:277-289) and the initial base velocity (:291-295); the right foot's position comes from
    // the reset pose's calc_state (:304-305, computed once: the pose is final once the velocity is set)
    const int f0 = b.frame, f1 = (b.frame + 2) % c.max_frame;
    const double phi = degToTarget * DEG2RAD;
    const double qz = sin(phi / 2), qw = cos(phi / 2);
    const double r00 = -(qz * qz) + qw * qw, r01 = 2 * (0.0 - qz * qw), r10 = 2 * (0.0 + qz * qw), r11 = -(qz * qz) + qw * qw;
    const HUM_GLOBAL double* e0 = c.gep() + f0 * 27;
    const HUM_GLOBAL double* e1 = c.gep() + f1 * 27;
    {
        const double l0x = r00 * e0[EP_RIGHT_LEG] + r01 * e0[EP_RIGHT_LEG + 1], l0y = r10 * e0[EP_RIGHT_LEG] + r11 * e0[EP_RIGHT_LEG + 1];
        const double l1x = r00 * e1[EP_RIGHT_LEG] + r01 * e1[EP_RIGHT_LEG + 1], l1y = r10 * e1[EP_RIGHT_LEG] + r11 * e1[EP_RIGHT_LEG + 1];
        if (init_vel) {
            st[7] = (T)(((l1x - l0x) / 0.0165) / 1.2);
            st[8] = (T)(((l1y - l0y) / 0.0165) / 1.2);
            st[9] = (T)(((e1[EP_RIGHT_LEG + 2] - e0[EP_RIGHT_LEG + 2]) / 0.0165) / 1.2);
        }
    }
    float js[NDOF];
    int jal;
    PostPhys<T> pp;
    calc_state(st, b.wt, obs, js, jal, pp, ref ? scs : nullptr);            // :304-305
    {
        const double refx = r00 * e0[EP_RIGHT_FOOT] + r01 * e0[EP_RIGHT_FOOT + 1];
        const double refy = r10 * e0[EP_RIGHT_FOOT] + r11 * e0[EP_RIGHT_FOOT + 1];
        b.sep[0] = pp.rfoot[0] - refx; b.sep[1] = pp.rfoot[1] - refy; b.sep[2] = 0;
    }
    b.lts = 0; b.dj = 0; b.dvj = 0; b.bps = 0; b.es = 0; b.jls = 0; b.alive = 0; b.dlts = 0;   // initReward
    inc_frame(b, c, 2);                                                     // :302
    ref_obs(c, b.frame, obs + 42, ef);
}

// Post-physics part of step (low_level_env.py:481-526) + optional auto-reset; stores state, book, outputs.
template <typename T>
__device__ __attribute__((always_inline)) void post_step(const KArgs& a, int i, long io, T* st, Book& b, const float* act,
                                                          unsigned& ef, const T* scs = nullptr,
                                                          bool* defer_reset = nullptr,   // the caller runs the
                                                                                         // auto-reset and the store
                                                          float* obs_dst = nullptr,      // obs row (default: a.obs)
                                                          const float* js_pre = nullptr,  // the joint block done by
                                                          int jal_pre = 0) {              // the env's lanes (obs_dst)
    // i: the lane (state, bookkeeping); io: its output row of this step (t * n + i, hum_step_k)
    const ClipDev& c = a.clips[b.clip];
    float obs[HUM_NOBS];
    // calc_state (:481) and robot_pos (:483-486)
    float js[NDOF];
    int jal = jal_pre;
    PostPhys<T> pp;
    calc_state(st, b.wt, obs, js, jal, pp, scs, js_pre == nullptr);
    if (js_pre) {
#pragma unroll
        for (int k = 0; k < NDOF; k++) js[k] = js_pre[k];
    }
    POST_SUBPHASE(19);
    b.robot_pos[0] = pp.bx; b.robot_pos[1] = pp.by; b.robot_pos[2] = 0;
    // updateReward (:441-465)
    double dJ = 0, dV = 0;
#pragma unroll
    for (int j = 0; j < NREF; j++) {
        dJ = dJ + fabs(pp.q[JM_DOF[j]] - c.gpos()[b.frame * 14 + JM_COL[j]]) * JM_W[j];
    }
    int vrow = b.frame;
    if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
    for (int j = 0; j < NREF; j++) {
        dV = dV + fabs(pp.qd[JM_DOF[j]] - c.gvel()[vrow * 14 + JM_COL[j]]) * JM_WV[j];
    }
    const double jointScore = exp(4 * (-dJ / JOINT_WEIGHT_SUM));
    const double jointVelScore = exp((-dV / JOINT_VEL_WEIGHT_SUM) / 2);
    const double lowTarget = -norm3_blas(b.target[0] - b.robot_pos[0], b.target[1] - b.robot_pos[1], b.target[2] - b.robot_pos[2]);
    const double posture = exp(-((fabs(pp.yaw - b.hldt) + fabs(pp.roll)) + fabs(pp.pitch)));
    b.dlts = (lowTarget - b.lts) / 0.0165 * 0.1;
    b.dj = jointScore;
    b.dvj = jointVelScore;
    b.lts = lowTarget;
    {
        const float run = pairwise_sum_f<HUM_NACT>([&](int k) { return fabsf(act[k] * js[k]); }) / 17.0f;
        const float stall = pairwise_sum_f<HUM_NACT>([&](int k) { return act[k] * act[k]; }) / 17.0f;
        b.es = -1.0 * (double)run + -0.1 * (double)stall;
    }
    b.jls = -0.1 * jal;
    b.alive = alive_reward(a.np1, obs[0]);
    b.bps = posture;
    double total = 0;
    total = total + b.dj * REWARD_W[0];
    total = total + b.dvj * REWARD_W[1];
    total = total + b.dlts * REWARD_W[2];
    total = total + b.es * REWARD_W[3];
    total = total + b.jls * REWARD_W[4];
    total = total + b.alive * REWARD_W[5];
    total = total + b.bps * REWARD_W[6];
    inc_frame(b, c, 2);                                                      // :513
    POST_SUBPHASE(20);
    // checkTarget (:412-434)
    {
        const double dist = norm3_blas(b.robot_pos[0] - b.target[0], b.robot_pos[1] - b.target[1], b.robot_pos[2] - b.target[2]);
        if (dist <= 0.5) {
            const double rr = pp.yaw + (double)draw(a, i, b, -180, 180) * DEG2RAD;
            double nt[3] = {b.robot_pos[0] + cos(rr) * 5, b.robot_pos[1] + sin(rr) * 5, b.robot_pos[2] + 0.0};
            if ((b.mode & HUM_MODE_PREDEFINED) && a.npred > 0) {
                b.pred_idx = (b.pred_idx + 1) % a.npred;
                for (int k = 0; k < 3; k++) nt[k] = a.pred[3 * b.pred_idx + k];
            }
            for (int k = 0; k < 3; k++) { b.srp[k] = b.target[k]; b.target[k] = nt[k]; }
            b.lts = -norm3_blas(b.target[0] - b.srp[0], b.target[1] - b.srp[1], b.target[2] - b.srp[2]);
        }
        set_walk_target_hl(b);
    }
    POST_SUBPHASE(21);
    ref_obs(c, b.frame, obs + 42, ef);                                        // :519
    bool done;                                                                // :521-524
    {
        const bool alive = b.alive > 0;
        const bool near = norm3_blas(b.target[0] - b.robot_pos[0], b.target[1] - b.robot_pos[1], b.target[2] - b.robot_pos[2]) <=
                          norm3_blas(b.target[0] - b.srp[0], b.target[1] - b.srp[1], b.target[2] - b.srp[2]) + 3;
        done = (b.mode & HUM_MODE_DEBUG) ? !alive : !(alive && near);
        b.timestep += 1;
        if (b.timestep >= 3000) done = true;
    }
    POST_SUBPHASE(22);
    float* orow = obs_dst ? obs_dst : a.obs + io * HUM_NOBS;
#pragma unroll
    for (int k = 0; k < HUM_NOBS; k++)
        if (!js_pre || k < 8 || k >= 42) orow[k] = obs[k];
    POST_SUBPHASE(16);
    a.rew[io] = (float)total;
    a.done[io] = done ? 1 : 0;
    if (a.frame_out) a.frame_out[io] = b.frame;
    POST_SUBPHASE(23);
    if (defer_reset) {
        *defer_reset = done && (a.flags & HUM_STEP_AUTORESET);
        return;
    }
    if (done && (a.flags & HUM_STEP_AUTORESET)) {
        float o2[HUM_NOBS];
        reset_lane(a, i, st, b, -1, 0.0, o2, ef);
        if (a.obs_reset) {
#pragma unroll
            for (int k = 0; k < HUM_NOBS; k++) a.obs_reset[io * HUM_NOBS + k] = o2[k];
        }
    }
    store_lane(a, i, st, b);
    if (ef) atomicOr(a.eflags, ef);
}


// ----------------------------------------------------------------------------------- hierarchical env
// HierarchicalHumanoidEnv (/root/reference/hier_env.py) on the same lanes/physics.  float64 in the reference's
// operation order; contraction off (numpy never fuses a*b+c); 3-vector norms/dots in OpenBLAS ddot order.
#pragma clang fp contract(off)

// getHighLevelObs (hier_env.py:336-353): [obs0, cos/sin(angle to target), cos/sin(angle to start), obs3..41]
__device__ inline void hier_high_obs(const float* obs42, const Book& b, double yaw, float* o44) {
    const double targetTheta = atan2(b.target[1] - b.robot_pos[1], b.target[0] - b.robot_pos[0]);
    const double angleToTarget = targetTheta - yaw;
    const double startPosTheta = atan2(b.srp[1] - b.robot_pos[1], b.srp[0] - b.robot_pos[0]);
    const double angleToStart = startPosTheta - yaw;
    o44[0] = obs42[0];
    o44[1] = (float)cos(angleToTarget);
    o44[2] = (float)sin(angleToTarget);
    o44[3] = (float)cos(angleToStart);
    o44[4] = (float)sin(angleToStart);
#pragma unroll
    for (int k = 3; k < 42; k++) o44[k + 2] = obs42[k];
}

// reset() / resetFromFrame() (hier_env.py:235-319)
template <typename T>
__device__ __attribute__((always_inline)) void hier_reset_lane(const KArgs& a, int i, T* st, Book& b, int start_frame, double reset_yaw, float* o44,
                                unsigned& ef) {
    const ClipDev& c = a.clips[b.clip];
    const bool ref = !(a.reset_flags & HUM_RESET_NO_REF_POSE);
    const bool init_vel = ref && !(a.reset_flags & HUM_RESET_NO_INIT_VEL);
    if (start_frame < 0) {                                                  // :238-241 (argument order)
        start_frame = draw(a, i, b, 0, c.max_frame - 5);
        reset_yaw = (double)draw(a, i, b, -180, 180);
    }
#pragma unroll
    for (int e = 0; e < HUM_NSTATE; e++) st[e] = 0;                         // flat_env.reset()
    st[6] = 1;
    if (!ref) joint_noise(b, st);
    b.timestep = 0;
    if ((b.mode & HUM_MODE_PREDEFINED) && a.npred > 0) {                   // :264-266
        b.pred_idx = 0;
        for (int k = 0; k < 3; k++) b.target[k] = a.pred[k];
    } else {                                                                // :268, getRandomVec :251-257
        const double r = 0 + (double)draw(a, i, b, -180, 180) * DEG2RAD;
        b.target[0] = cos(r) * 5;
        b.target[1] = sin(r) * 5;
        b.target[2] = 0;
    }
    if (ref) {                                                              // :272-274 setJointsOrientation
        b.frame = start_frame;
        int vrow = start_frame;
        if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
        for (int j = 0; j < NREF; j++) {
            st[13 + JM_DOF[j]] = (T)c.gpos()[start_frame * 14 + JM_COL[j]];
            st[30 + JM_DOF[j]] = (T)c.gvel()[vrow * 14 + JM_COL[j]];
        }
    }
    for (int k = 0; k < 3; k++) { b.robot_pos[k] = 0; b.srp[k] = 0; }      // :277-281
    st[0] = 0; st[1] = 0; st[2] = (T)1.17;
    const double degToTarget = atan2(b.target[1], b.target[0]) * RAD2DEG + reset_yaw;   // :284
    b.wt[0] = cos(degToTarget) * 1000;                                      // :285 (degrees into cos: quirk)
    b.wt[1] = sin(degToTarget) * 1000;
    const double th = degToTarget * DEG2RAD;                                // :286-287 scipy from_euler
    st[3] = 0; st[4] = 0; st[5] = (T)sin(th / 2); st[6] = (T)cos(th / 2);
    b.hldt = degToTarget * DEG2RAD;                                         // :289
    {                                                                       // :291-304 starting velocity
        const int f0 = b.frame, f1 = b.frame + 1;
        const double qz = sin(th / 2), qw = cos(th / 2);
        const double r00 = -(qz * qz) + qw * qw, r01 = 2 * (0.0 - qz * qw), r10 = 2 * (0.0 + qz * qw), r11 = -(qz * qz) + qw * qw;
        const HUM_GLOBAL double* e0 = c.gep() + f0 * 27;
        const HUM_GLOBAL double* e1 = c.gep() + f1 * 27;
        const double l0x = r00 * e0[EP_RIGHT_LEG] + r01 * e0[EP_RIGHT_LEG + 1], l0y = r10 * e0[EP_RIGHT_LEG] + r11 * e0[EP_RIGHT_LEG + 1];
        const double l1x = r00 * e1[EP_RIGHT_LEG] + r01 * e1[EP_RIGHT_LEG + 1], l1y = r10 * e1[EP_RIGHT_LEG] + r11 * e1[EP_RIGHT_LEG + 1];
        if (init_vel) {
            st[7] = (T)((l1x - l0x) / 0.0165);
            st[8] = (T)((l1y - l0y) / 0.0165);
            st[9] = (T)((e1[EP_RIGHT_LEG + 2] - e0[EP_RIGHT_LEG + 2]) / 0.0165);
        }
    }
    // initReward (:183-206); starting_ep_pos is NOT reset by the hierarchical env
    b.lts = 0; b.dj = 0; b.dvj = 0; b.bps = 0; b.es = 0; b.jls = 0; b.alive = 0; b.dlts = 0;
    b.hts = -5.0; b.drift = 0; b.cum_drift = 0; b.dhts = 0; b.cum_alive = 0;
    b.level_rem = 5; b.n_high = 0; b.expect_high = 1;                       // :308-309
    inc_frame(b, c, 2);                                                     // :312
    float obs[42], js[NDOF];
    int jal;
    PostPhys<T> pp;
    calc_state(st, b.wt, obs, js, jal, pp);                                 // :317
    b.bxy[0] = pp.bx; b.bxy[1] = pp.by;
    hier_high_obs(obs, b, pp.yaw, o44);                                     // :318
}

// updateRewardHigh (hier_env.py:524-536); returns the high-level reward (:627, :633)
__device__ inline float hier_update_reward_high(Book& b) {
    const double hts = -norm3_blas(b.target[0] - b.robot_pos[0], b.target[1] - b.robot_pos[1], b.target[2] - b.robot_pos[2]);
    const double k = (double)(5 - b.level_rem + 1);
    b.dhts = (hts - b.hts) / 0.0165;
    b.dhts = b.dhts / k;
    b.hts = hts;
    b.drift = b.cum_drift / k;
    b.cum_drift = 0;
    return (float)(b.dhts * 0.3 + b.drift * 0.7);
}

// step(action_dict) (hier_env.py:355-366) -> high_level_step (:538-571) or low_level_step (:583-641), after the
// physics of a low step; stores state/book and writes the dict-shaped outputs.
template <typename T>
__device__ __attribute__((always_inline)) void hier_post(const KArgs& a, int i, long io, T* st, Book& b, bool high, unsigned& ef,
                                                          const T* scs = nullptr, bool store_state = true, long ro = -1,
                                                          const float* lact = nullptr, const float* hact = nullptr) {
    // ro: the row of the [.., n, 44/70] observation outputs (default the step's row io; the fused rollout's
    // in-place [n, ...] buffers: i); lact / hact: the step's low / high actions in registers (default a.act / a.act_high)
    if (ro < 0) ro = io;
    const ClipDev& c = a.clips[b.clip];
    b.robot_pos[0] = b.bxy[0]; b.robot_pos[1] = b.bxy[1]; b.robot_pos[2] = 0;   // step(): :358-361
    float obs[HUM_NOBS], js[NDOF], o44[HUM_NOBS_HIGH];
    int jal;
    PostPhys<T> pp;
    unsigned agents = 0;
    bool done = false;
    float rew_low = 0.f, rew_high = 0.f;
    if (high) {
        // cur_obs is the last calc_state (same physics state, walk target before this call); scs: the cooperative
        // kernel's hinge sin / cos of this (unchanged) state, the same hinge_sincos values forward_kinematics forms
        calc_state(st, b.wt, obs, js, jal, pp, scs);
        const float a0 = hact ? hact[0] : a.act_high[2 * io], a1 = hact ? hact[1] : a.act_high[2 * io + 1];
        const float actionDegree = (float)atan2((double)a1, (double)a0) * (float)RAD2DEG;   // :540 (float32)
        const double newDegree = (double)actionDegree + pp.yaw * RAD2DEG;                   // :543
        b.hldt = newDegree * DEG2RAD;
        const double ct = cos(b.hldt), sn = sin(b.hldt);
        const double nw0 = b.robot_pos[0] + ct * 5, nw1 = b.robot_pos[1] + sn * 5, nw2 = b.robot_pos[2] + 0.0 * 5;
        b.wt[0] = nw0; b.wt[1] = nw1;                                                       // :553
        const double v0 = nw0 - b.robot_pos[0], v1 = nw1 - b.robot_pos[1], v2 = nw2 - b.robot_pos[2];
        const double lenSEP = norm3_blas(b.sep[0] - b.robot_pos[0], b.sep[1] - b.robot_pos[1], b.sep[2] - b.robot_pos[2]);
        const double nv = norm3_blas(v0, v1, v2);
        b.sep[0] = (-v0 / nv) * lenSEP + b.robot_pos[0];                                    // :556-561
        b.sep[1] = (-v1 / nv) * lenSEP + b.robot_pos[1];
        b.sep[2] = (-v2 / nv) * lenSEP + b.robot_pos[2];
        b.level_rem = 5;
        b.n_high += 1;
        b.expect_high = 0;
        ref_obs(c, b.frame, obs + 42, ef);                                                  // :567 getLowLevelObs
        agents = HUM_AGENT_LOW;
    } else {
        b.level_rem -= 1;                                                                   // :584
        calc_state(st, b.wt, obs, js, jal, pp, scs);                                        // :591
        const float* act = lact ? lact : a.act + io * HUM_NACT;
        // updateReward (:494-522)
        double dJ = 0, dV = 0;
#pragma unroll
        for (int j = 0; j < NREF; j++) dJ = dJ + fabs(pp.q[JM_DOF[j]] - c.gpos()[b.frame * 14 + JM_COL[j]]) * JM_W[j];
        int vrow = b.frame;
        if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
        for (int j = 0; j < NREF; j++) dV = dV + fabs(pp.qd[JM_DOF[j]] - c.gvel()[vrow * 14 + JM_COL[j]]) * JM_WV[j];
        const double jointScore = exp(4 * (-dJ / JOINT_WEIGHT_SUM));
        const double jointVelScore = exp((-dV / JOINT_VEL_WEIGHT_SUM) / 2);
        const double posture = exp(-((fabs(pp.yaw - b.hldt) + fabs(pp.roll)) + fabs(pp.pitch)));
        b.dlts = (0.0 - b.lts) / 0.0165 * 0.1;                                              // lowTargetScore == 0
        b.dj = jointScore;
        b.dvj = jointVelScore;
        b.lts = 0;
        {
            const float run = pairwise_sum_f<HUM_NACT>([&](int k) { return fabsf(act[k] * js[k]); }) / 17.0f;
            const float stall = pairwise_sum_f<HUM_NACT>([&](int k) { return act[k] * act[k]; }) / 17.0f;
            b.es = -1.0 * (double)run + -0.1 * (double)stall;
        }
        b.jls = -0.1 * jal;
        b.alive = alive_reward(a.np1, obs[0]);
        b.cum_alive = b.cum_alive + b.alive;
        b.bps = posture;
        {                                                                                   // calcDriftScore :461-467
            const double l0 = b.target[0] - b.srp[0], l1 = b.target[1] - b.srp[1], l2 = b.target[2] - b.srp[2];
            const double lineLen = norm3_blas(l0, l1, l2);
            double t = dot3_blas(b.robot_pos[0] - b.srp[0], b.robot_pos[1] - b.srp[1], b.robot_pos[2] - b.srp[2],
                                 l0, l1, l2) / (lineLen * lineLen);
            t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);   // np.clip keeps NaN
            const double p0 = b.srp[0] + t * l0, p1 = b.srp[1] + t * l1, p2 = b.srp[2] + t * l2;
            const double score = norm3_blas(p0 - b.robot_pos[0], p1 - b.robot_pos[1], p2 - b.robot_pos[2]);
            b.cum_drift = b.cum_drift + exp(-6 * score);
        }
        double total = 0;                                                                   // :598-611
        total = total + b.dj * REWARD_W[0];
        total = total + b.dvj * REWARD_W[1];
        total = total + b.dlts * REWARD_W[2];
        total = total + b.es * REWARD_W[3];
        total = total + b.jls * REWARD_W[4];
        total = total + b.alive * REWARD_W[5];
        total = total + b.bps * REWARD_W[6];
        rew_low = (float)total;
        inc_frame(b, c, 2);                                                                 // :613
        {                                                                                   // checkTarget :469-487
            const double dist = norm3_blas(b.robot_pos[0] - b.target[0], b.robot_pos[1] - b.target[1], b.robot_pos[2] - b.target[2]);
            if (dist <= 0.5) {
                const double rr = pp.yaw + (double)draw(a, i, b, -180, 180) * DEG2RAD;
                double nt[3] = {b.robot_pos[0] + cos(rr) * 5, b.robot_pos[1] + sin(rr) * 5, b.robot_pos[2] + 0.0};
                if ((b.mode & HUM_MODE_PREDEFINED) && a.npred > 0) {
                    b.pred_idx = (b.pred_idx + 1) % a.npred;
                    for (int k = 0; k < 3; k++) nt[k] = a.pred[3 * b.pred_idx + k];
                }
                for (int k = 0; k < 3; k++) { b.srp[k] = b.target[k]; b.target[k] = nt[k]; }
                b.hts = -norm3_blas(b.target[0] - b.srp[0], b.target[1] - b.srp[1], b.target[2] - b.srp[2]);
            }
        }
        const bool alive = b.alive > 0;                                                     // checkIfDone :573-581
        const bool near = norm3_blas(b.target[0] - b.robot_pos[0], b.target[1] - b.robot_pos[1], b.target[2] - b.robot_pos[2]) <=
                          norm3_blas(b.target[0] - b.srp[0], b.target[1] - b.srp[1], b.target[2] - b.srp[2]) + 1;
        done = (b.mode & HUM_MODE_DEBUG) ? !alive : !(alive && near);
        b.timestep += 1;
        ref_obs(c, b.frame, obs + 42, ef);
        if (done || b.timestep >= 3000) {                                                   // :624-630
            done = true;
            rew_high = hier_update_reward_high(b);
            hier_high_obs(obs, b, pp.yaw, o44);
            agents = HUM_AGENT_HIGH | HUM_AGENT_LOW;
            b.cum_alive = 0;
        } else if (b.level_rem <= 0) {                                                      // :631-636
            rew_high = hier_update_reward_high(b);
            hier_high_obs(obs, b, pp.yaw, o44);
            agents = HUM_AGENT_HIGH;
            b.cum_alive = 0;
            b.expect_high = 1;
        } else {
            agents = HUM_AGENT_LOW;
        }
        b.bxy[0] = pp.bx; b.bxy[1] = pp.by;                                                 // flat_env.robot.body_xyz
    }
    if (agents & HUM_AGENT_LOW) {
#pragma unroll
        for (int k = 0; k < HUM_NOBS; k++) a.obs[ro * HUM_NOBS + k] = obs[k];
    }
    if (agents & HUM_AGENT_HIGH) {
#pragma unroll
        for (int k = 0; k < HUM_NOBS_HIGH; k++) a.obs_high[ro * HUM_NOBS_HIGH + k] = o44[k];
    }
    a.rew[io] = (agents & HUM_AGENT_LOW) ? rew_low : 0.f;   // the level hand-back drops the low reward (:631-636)
    a.rew_high[io] = rew_high;
    a.agents[io] = (unsigned char)agents;
    a.done[io] = done ? 1 : 0;
    if (a.frame_out) a.frame_out[io] = b.frame;
    if (done && (a.flags & HUM_STEP_AUTORESET)) {
        float r44[HUM_NOBS_HIGH];
        hier_reset_lane(a, i, st, b, -1, 0.0, r44, ef);
        if (a.obs_high_reset) {
#pragma unroll
            for (int k = 0; k < HUM_NOBS_HIGH; k++) a.obs_high_reset[ro * HUM_NOBS_HIGH + k] = r44[k];
        }
    }
    if (store_state) store_lane(a, i, st, b);
    else store_book(a, i, b);
    if (ef) atomicOr(a.eflags, ef);
}

// non-finite action on a lane (humanoid.py:55 assert): lane not stepped, flagged, outputs neutral
__device__ inline void nonfinite_outputs(const KArgs& a, long io, int frame, float* obs_dst = nullptr) {
    if (!a.hier) {   // the LDS staging row or the global row, each through its own address space (no flat stores)
        if (obs_dst) {
            HUM_LDS float* orow = (HUM_LDS float*)obs_dst;
            for (int k = 0; k < HUM_NOBS; k++) orow[k] = 0.f;
        } else {
            long ro = io;
#ifdef HUM_BOUNDS_CHECK
            unsigned bf = 0;
            HUM_BOUNDS(bf, ro >= 0 && ro < (long)a.ksteps * a.n, ro = 0);
            if (bf) atomicOr(a.eflags, bf);
#endif
            HUM_GLOBAL float* orow = (HUM_GLOBAL float*)(a.obs + ro * HUM_NOBS);
            for (int k = 0; k < HUM_NOBS; k++) orow[k] = 0.f;
        }
    } else {
        a.rew_high[io] = 0.f;
        a.agents[io] = 0;
    }
    a.rew[io] = 0.f;
    a.done[io] = 1;
    if (a.frame_out) a.frame_out[io] = frame;
}

#pragma clang fp contract(on)


// ----------------------------------------------------------------------------------- step
template <typename T>
__global__ void __launch_bounds__(256) step_kernel(KArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    T st[HUM_NSTATE];
    Book b;
    load_lane(a, i, st, b);
    unsigned ef = 0;
#pragma unroll 1
    for (int t = 0; t < a.ksteps; t++) {   // env steps of this launch (state and book stay in registers)
        const long io = (long)t * a.n + i;
        // hierarchical env: the lane's acting agent (step(action_dict) dispatch, hier_env.py:363-366); a lane with
        // no action this round (HUM_AGENT_SEL_SKIP) is left untouched and reports no agent
        if (a.hier && a.agent_sel && a.agent_sel[io] == HUM_AGENT_SEL_SKIP) {
            a.agents[io] = 0;
            if (a.acted) a.acted[io] = 0;
            continue;
        }
        const bool high = a.hier && (a.agent_sel ? a.agent_sel[io] != 0 : b.expect_high != 0);
        float act[HUM_NACT];
        bool finite = true;
#pragma unroll
        for (int k = 0; k < HUM_NACT; k++) {
            act[k] = a.act[io * HUM_NACT + k];
            finite &= isfinite(act[k]);
        }
        if (a.hier && a.acted) a.acted[io] = !finite && !high ? 0 : (high ? HUM_AGENT_HIGH : HUM_AGENT_LOW);
        if (!finite && !high) {   // humanoid.py:55 assert: lane not stepped, flagged for the host
            ef |= HUM_EFLAG_NONFINITE_ACTION;
            nonfinite_outputs(a, io, b.frame);
            continue;
        }
        if (!(a.flags & HUM_STEP_SKIP_PHYSICS) && !high) {
            T tau[NDOF];
#pragma unroll
            for (int k = 0; k < HUM_NACT; k++)   // apply_action
                tau[act_dof[k]] = (T)motor_torque(a.np1, (float)act_gain[k], act_gain[k], act[k]);
            Lane<T> rows{(T*)a.scratch + i, (long)a.n};
#pragma unroll 1
            for (int s = 0; s < a.P.nsub; s++) {
                if (substep(a.P, st, tau, rows)) ef |= HUM_EFLAG_CONTACT_OVERFLOW;
            }
        }
        unsigned ef1 = 0;   // hier_post / post_step publish their own flags
        if (a.hier) hier_post(a, i, io, st, b, high, ef1);
        else post_step(a, i, io, st, b, act, ef1);
    }
    if (ef) atomicOr(a.eflags, ef);
}

// ----------------------------------------------------------------------------------- fused policy
// The policy network of policy.hip (RLlib FCNet 70-256-256-17 tanh + DiagGaussian sample + clip_actions) for the
// EPB_ envs of a wave, evaluated by all 64 lanes before the step's physics: lane l owns hidden units 4 l + m
// (m < 4) of every env (one 16-byte weight load per k, two v_pk_fma_f32 per env), each a k-ordered fma chain
// from 0 (the order policy.hip's v_mfma_f32_16x16x4_f32 tiles accumulate in), then tanhf(acc + bias); the output layer's 16 x EPB_ (env, column)
// chains go one to a lane, the 17th column's EPB_ chains ride along in lanes < EPB_ (one pass).  One wave per SIMD
// cannot hide the L2 latency of the weight loads, so the k loops are unrolled deep enough to keep 10-16 loads in
// flight.  Scratch (float units past the env's ABA transients, dead before the physics): input row, h1, h2, actions.
constexpr int PX_OFF = 0, PH1_OFF = 72, PH2_OFF = 328, PACT_OFF = 584, PSCR = 608;
template <typename T>
__device__ __attribute__((always_inline)) inline float* policy_scratch(GroupLDS<T>& S) {
    static_assert(sizeof(S.x) >= sizeof(S.x.aba) + PSCR * sizeof(float), "policy scratch");
    return reinterpret_cast<float*>(reinterpret_cast<char*>(&S.x) + sizeof(S.x.aba));
}
__device__ inline unsigned long long pmix64(unsigned long long z) {   // policy.hip's mix64
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
typedef float pf4 __attribute__((ext_vector_type(4)));
// one hidden layer: F[e][dst + 4 lane + m] = tanh(sum_k F[e][src + k] W[k][4 lane + m] + B[4 lane + m])
template <int EPB_, int K, int UNROLL>
__device__ __attribute__((always_inline)) inline void policy_hidden(HUM_LDS float* const (&F)[EPB_], const HUM_GLOBAL float* W,
                                                                    const HUM_GLOBAL float* B, int src, int dst,
                                                                    int lane) {
    float acc[EPB_][4];
#pragma unroll
    for (int e = 0; e < EPB_; e++)
#pragma unroll
        for (int m = 0; m < 4; m++) acc[e][m] = 0.f;
    // packed: v_pk_fma_f32 does units (4 lane, 4 lane + 1) and (4 lane + 2, 4 lane + 3) of an env in one op each
    typedef float pf2 __attribute__((ext_vector_type(2)));
    pf2 pacc[EPB_][2];
#pragma unroll
    for (int e = 0; e < EPB_; e++) pacc[e][0] = pacc[e][1] = pf2{0.f, 0.f};
#pragma unroll UNROLL
    for (int k = 0; k < K; k++) {
        const pf4 w = *reinterpret_cast<const HUM_GLOBAL pf4*>(W + k * 256 + 4 * lane);
        const pf2 w01 = {w[0], w[1]}, w23 = {w[2], w[3]};
#pragma unroll
        for (int e = 0; e < EPB_; e++) {
            const float x = F[e][src + k];
            const pf2 xx = {x, x};
            pacc[e][0] = __builtin_elementwise_fma(xx, w01, pacc[e][0]);
            pacc[e][1] = __builtin_elementwise_fma(xx, w23, pacc[e][1]);
        }
    }
#pragma unroll
    for (int e = 0; e < EPB_; e++) {
        acc[e][0] = pacc[e][0][0];
        acc[e][1] = pacc[e][0][1];
        acc[e][2] = pacc[e][1][0];
        acc[e][3] = pacc[e][1][1];
    }
    const pf4 bias = *reinterpret_cast<const HUM_GLOBAL pf4*>(B + 4 * lane);
#pragma unroll
    for (int e = 0; e < EPB_; e++)
#pragma unroll
        for (int m = 0; m < 4; m++) F[e][dst + 4 * lane + m] = tanhf(acc[e][m] + bias[m]);
}
// NIN -> 256 -> 256 -> NOUT: the low-level network (70 -> 17, weights pw, seed pseed) or the hierarchical env's
// high-level one (44 -> 2); emask: bit GL e set = env e of the wave acts with this network (the others' results are
// dropped: a wave whose envs expect different agents runs both networks, each keeping its own envs' actions)
#ifndef HUM_PH2_UNROLL
#define HUM_PH2_UNROLL 16   // the 256 x 256 layer's unroll (weight loads in flight)
#endif
// COMPACT (the two-level kernel, whose emask varies per wave): the hidden layers run for the acting envs only - each
// env's chains are separate instructions (policy_hidden's per-env accumulators), so a network needed by one env of
// the wave costs a quarter of the full one; every chain keeps its k order (bitwise the same values)
template <typename T, int EPB_, int NIN = HUM_NOBS, int NOUT = HUM_NACT, bool COMPACT = false>
__device__ __attribute__((always_inline)) void policy_wave(const KArgs& a, GroupLDS<T>* sh, int blk, int t, const float* pw,
                                                           unsigned long long pseed, unsigned long long emask,
                                                           float* act_traj, float* act_last, float* mean_traj) {
    static_assert(EPB_ * 16 == 64, "policy_wave: one (env, column) chain per lane");
    static_assert(NOUT == 17 || NOUT * EPB_ <= 64, "policy_wave: output chains");
    const int lane = threadIdx.x & 63;
    const HUM_GLOBAL float* W1 = (const HUM_GLOBAL float*)pw;
    const HUM_GLOBAL float* B1 = W1 + 72 * 256;
    const HUM_GLOBAL float* W2 = B1 + 256;
    const HUM_GLOBAL float* B2 = W2 + 256 * 256;
    const HUM_GLOBAL float* W3 = B2 + 256;
    const HUM_GLOBAL float* B3 = W3 + 256 * NOUT;
    const HUM_GLOBAL float* LSTD = B3 + NOUT;
    HUM_LDS float* F[EPB_];   // LDS-typed: no generic (flat) access
#pragma unroll
    for (int e = 0; e < EPB_; e++) F[e] = (HUM_LDS float*)policy_scratch(sh[e]);
    // hidden layer 1 (K = NIN: policy.hip's zero rows NIN .. 71 add exact zeros), hidden layer 2
    auto hidden = [&](auto ne_c, HUM_LDS float* const (&Fa)[decltype(ne_c)::value]) {
        constexpr int NE = decltype(ne_c)::value;
        policy_hidden<NE, NIN, (NIN % 10 == 0 ? 10 : 11)>(Fa, W1, B1, PX_OFF, PH1_OFF, lane);
        wave_sync();
        policy_hidden<NE, 256, HUM_PH2_UNROLL>(Fa, W2, B2, PH1_OFF, PH2_OFF, lane);
        wave_sync();
    };
    if constexpr (COMPACT && EPB_ == 4) {
        // the acting envs in ascending order (emask is wave-uniform: scalar bit arithmetic)
        unsigned m = 0;
#pragma unroll
        for (int e = 0; e < EPB_; e++) m |= (unsigned)((emask >> (GL * e)) & 1ull) << e;
        const int i0 = __builtin_ctz(m | 16u), m1 = m & (m - 1), i1 = __builtin_ctz(m1 | 16u);
        const int m2 = m1 & (m1 - 1), i2 = __builtin_ctz(m2 | 16u);
        auto Fi = [&](int e) { return (HUM_LDS float*)policy_scratch(sh[e < EPB_ ? e : 0]); };
        switch (__builtin_popcount(m)) {
            case 1: { HUM_LDS float* const Fa[1] = {Fi(i0)}; hidden(std::integral_constant<int, 1>{}, Fa); break; }
            case 2: { HUM_LDS float* const Fa[2] = {Fi(i0), Fi(i1)}; hidden(std::integral_constant<int, 2>{}, Fa); break; }
            case 3: { HUM_LDS float* const Fa[3] = {Fi(i0), Fi(i1), Fi(i2)}; hidden(std::integral_constant<int, 3>{}, Fa); break; }
            default: hidden(std::integral_constant<int, EPB_>{}, F); break;
        }
    } else {
        hidden(std::integral_constant<int, EPB_>{}, F);
    }
    // output layer: 17 wide: chain A = (env lane / 16, column lane % 16), chain B = (env lane, column 16) in lanes
    // < EPB_; narrower: chain A = (env lane / NOUT, column lane % NOUT) in lanes < EPB_ NOUT
    constexpr bool WIDE = NOUT == 17;
    const int eA = WIDE ? lane >> 4 : (lane < EPB_ * NOUT ? lane / NOUT : 0);
    const int cA = WIDE ? lane & 15 : (lane < EPB_ * NOUT ? lane % NOUT : 0);
    const bool onA = WIDE || lane < EPB_ * NOUT;
    const int eB = lane < EPB_ ? lane : 0;
    const HUM_LDS float* hA = F[0] + PH2_OFF;
    const HUM_LDS float* hB = F[0] + PH2_OFF;
#pragma unroll
    for (int q = 1; q < EPB_; q++) {
        hA = eA == q ? F[q] + PH2_OFF : hA;
        hB = eB == q ? F[q] + PH2_OFF : hB;
    }
    float accA = 0.f, accB = 0.f;
#pragma unroll 16
    for (int k = 0; k < 256; k++) {
        const HUM_GLOBAL float* wr = W3 + k * NOUT;
        accA = fmaf(hA[k], wr[cA], accA);
        if constexpr (WIDE) accB = fmaf(hB[k], wr[16], accB);
    }
    // + DiagGaussian sample + clip_actions
    auto finish = [&](int e, int c, float acc) {
        if (!((emask >> (GL * e)) & 1ull)) return;
        const float mean = acc + B3[c];
        float v = mean;
        const int i = blk * EPB_ + e;
        if (a.pexplore) {   // policy.hip: (seed, lane, step, column) through separate mixing rounds, Box-Muller
            const unsigned long long x = pmix64(pmix64(pmix64(pseed ^ (unsigned long long)i) ^ (a.pstep0 + t)) ^
                                                (unsigned long long)c);
            const float u1 = ((float)(x >> 40) + 1.f) * 0x1.0p-24f;
            const float u2 = (float)((x >> 16) & 0xFFFFFFull) * 0x1.0p-24f;
            v = mean + expf(LSTD[c]) * sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
        }
        HUM_LDS float* pa = F[0] + PACT_OFF;
#pragma unroll
        for (int q = 1; q < EPB_; q++) pa = e == q ? F[q] + PACT_OFF : pa;
        pa[c] = fminf(fmaxf(v, -1.f), 1.f);
        if (i < a.n) {
            const long io = (long)t * a.n + i;
            if (act_traj) act_traj[io * NOUT + c] = v;   // the sample before clip_actions (SampleBatch)
            if (mean_traj) mean_traj[io * NOUT + c] = mean;   // the distribution's mean (action_dist_inputs)
            if (act_last && t == a.ksteps - 1) act_last[(long)i * NOUT + c] = pa[c];
        }
    };
    if (onA) finish(eA, cA, accA);
    if (WIDE && lane < EPB_) finish(eB, 16, accB);
    wave_sync();
}

// Cooperative step: 16 lanes per env, EPB_ envs per block of EPB_*16 threads (one wavefront), env working
// set in LDS.  EPB_ = 4 fills the wave; EPB_ = 2 leaves half of it idle but lets a SIMD hold two waves
// (19.3 KB LDS per block), so one wave's LDS/memory waits overlap the other's VALU issue.
#ifndef HUM_GROUP_MIN_WAVES
#define HUM_GROUP_MIN_WAVES 1
#endif
// POLICY: 0 = actions from a.act, either env (hum_step_k / hum_hier_step_k: fp64, envs_per_block 1 / 2, terrain),
// 1 = the low-level network inside the step loop (hum_rollout_fused), 2 = both networks of the hierarchical env
// (hum_hier_rollout_fused), 3 = actions from a.act, the low-level env only (hum_step_k's benchmarked fp32 kernel),
// 4 = actions from a.act, the hierarchical env only (hum_hier_step_k's fp32 kernel)
template <typename T, int EPB_, bool TERRAIN = false, int POLICY = 0>
__global__ void __launch_bounds__(EPB_ * GL, HUM_GROUP_MIN_WAVES) step_group_kernel(KArgs a0) {
    __shared__ GroupLDS<T> sh[EPB_];
    const int ksteps = a0.ksteps;
    // XCD-aware env mapping: the dispatcher deals blocks round-robin over the 8 XCDs (block b -> XCD b % 8),
    // so consecutive blocks would put the 4-env (16/32-byte) slices of one SoA cache line into 8 different L2s,
    // each fetching the whole line.  Give XCD x one contiguous run of blocks instead (a bijection for any grid).
    const int nb = gridDim.x, xq = nb >> 3, xr = nb & 7, xcd = blockIdx.x & 7;
    const int blk = xcd * xq + min(xcd, xr) + (blockIdx.x >> 3);
#ifdef HUM_WLOG_ON
    const unsigned long long t_wave0 = __builtin_amdgcn_s_memtime();
    const unsigned long long rt_wave0 = __builtin_amdgcn_s_memrealtime();
#ifdef HUM_WAVE_LOG
    if (threadIdx.x < 24) s_phase[threadIdx.x] = 0;
#endif
#endif
    load_tab_lds<T>();
    {   // the env's state stays in LDS over the steps of the launch; lane 0 carries the per-env integers the other
        // lanes read (the agent the hierarchical env expects, the random-terrain key) in the pad slots of tau
        const int l = threadIdx.x & (GL - 1), ge = threadIdx.x / GL, i = blk * EPB_ + ge;
        const bool valid = i < a0.n;
        GroupLDS<T>& S = sh[ge];
        for (int e = l; e < HUM_NSTATE; e += GL)
            S.st[e] = valid ? ((const T*)a0.phys)[(long)e * a0.n + i] : (e == 2 ? T(1.17) : (e == 6 ? T(1) : T(0)));
        static_assert(sizeof(T) * 3 >= 3 * sizeof(int), "carry slots");
        int* carry = reinterpret_cast<int*>(&S.tau[NDOF]);
        if (l == 0) {
            carry[0] = valid && a0.hier ? a0.bi[10 * a0.n + i] : 0;
            carry[1] = TERRAIN && a0.P.terrain == HUM_TERRAIN_RANDOM_BLOCKS && valid ? a0.bi[11 * a0.n + i] : 0;
            carry[2] = TERRAIN && a0.P.terrain == HUM_TERRAIN_RANDOM_BLOCKS && valid ? a0.bi[12 * a0.n + i] : 0;
        }
    }
    __syncthreads();
    unsigned ef = 0;
    bool prev_reset = false;   // POLICY: the env auto-reset at the previous step (its next input is the reset obs)
#pragma unroll 1
    for (int t = 0; t < ksteps; t++) {
    // Everything the step body derives from the launch arguments or the lane index is recomputed in every step:
    // the arguments are re-read from the kernarg segment and the lane index is laundered, so the compiler cannot
    // hoist those values out of the step loop (which would keep them live across the whole body and spill).
    const __attribute__((address_space(4))) KArgs* kp =
        (const __attribute__((address_space(4))) KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    const KArgs& a = *(const KArgs*)kp;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int l = tid & (GL - 1), ge = tid / GL;
    const int i = blk * EPB_ + ge;
    const bool valid = i < a.n;
    GroupLDS<T>& S = sh[ge];
    const ModelTab<T>& M = tab_fresh<T>();
    int* carry = reinterpret_cast<int*>(&S.tau[NDOF]);
    const int gbit = (tid & 63) & ~(GL - 1);
    const long io = (long)t * a.n + i;   // this step's input / output row of the env
    constexpr bool HP = POLICY == 2;
    constexpr bool NET = POLICY == 1 || POLICY == 2;       // a network acts inside the step loop
    // the env-specialised instantiations compile the other env's branches out (bitwise equal, faster: DESIGN.md
    // section 4); the generic one (POLICY 0) reads the env from the launch arguments
    constexpr bool LOWONLY = POLICY == 1 || POLICY == 3;   // the low-level env only (the launchers check a.hier)
    constexpr bool HIERONLY = POLICY == 2 || POLICY == 4;  // the hierarchical env only
    const bool hier = HIERONLY || (!LOWONLY && a.hier);
    if constexpr (HP) {
        // the two-level sampler's input (hum_hier_rollout's per-transition policy calls): an env expecting the high
        // agent reads its latest high observation (done at the previous transition: its auto-reset one), the others
        // their latest low observation - the handle's [n, ...] rows, updated in place by the previous step's lane 0
        float* X = policy_scratch(S) + PX_OFF;
        const bool hi = valid && carry[0] != 0;
        const bool dprev = valid && (t == 0 ? (a.done_in && a.done_in[i]) : a.done[io - a.n] != 0);
        const HUM_GLOBAL float* src = nullptr;
        if (valid)
            src = (const HUM_GLOBAL float*)(hi ? (dprev ? a.obs_high_reset : a.obs_high) + (long)i * HUM_NOBS_HIGH
                                               : a.obs + (long)i * HUM_NOBS);
        const int nin = hi ? HUM_NOBS_HIGH : HUM_NOBS;
        float xv[5];
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const int k = l + GL * j;
            xv[j] = (valid && k < nin) ? src[k] : 0.f;
        }
        HUM_GLOBAL float* trow = nullptr;
        if (valid) {
            if (hi && a.obs_traj_high) trow = (HUM_GLOBAL float*)(a.obs_traj_high + io * HUM_NOBS_HIGH);
            if (!hi && a.obs_traj) trow = (HUM_GLOBAL float*)(a.obs_traj + io * HUM_NOBS);
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const int k = l + GL * j;
            if (k < HUM_NOBS) X[k] = xv[j];
            if (trow && k < nin) trow[k] = xv[j];
        }
        wave_sync();
        // each network only for the envs that act with it; a network no env of the wave needs is skipped
        const unsigned long long hm = __ballot(l == 0 && hi), lm = __ballot(l == 0 && valid && !hi);
        if (hm) policy_wave<T, EPB_, HUM_NOBS_HIGH, HUM_NACT_HIGH, true>(a, sh, blk, t, a.pw_high, a.pseed_high, hm,
                                                                    a.act_traj_high, a.act_last_high, a.mean_traj_high);
        if (lm) policy_wave<T, EPB_, HUM_NOBS, HUM_NACT, true>(a, sh, blk, t, a.pw, a.pseed, lm, a.act_traj, a.act_last,
                                                             a.mean_traj);
    } else if constexpr (POLICY == 1) {
        // the sampler's input: step 0 the handle's current observation (a lane done at the previous step: its reset
        // observation), later steps the row the previous step staged (its reset row if it reset)
        float* X = policy_scratch(S) + PX_OFF;
        // step 0 from global memory, later steps from LDS: two address-space-typed loads (no flat access)
        float xv[5];
        if (t == 0) {
            const HUM_GLOBAL float* src = nullptr;
            if (valid) src = (const HUM_GLOBAL float*)(((a.done_in && a.done_in[i]) ? a.obs_reset : a.obs) + (long)i * HUM_NOBS);
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const int k = l + GL * j;
                xv[j] = (valid && k < HUM_NOBS) ? src[k] : 0.f;
            }
        } else {
            const HUM_LDS float* src = (const HUM_LDS float*)reinterpret_cast<const float*>(&S.x.aba.IA[0][0] + (prev_reset ? 144 : 72));
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const int k = l + GL * j;
                xv[j] = (valid && k < HUM_NOBS) ? src[k] : 0.f;
            }
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const int k = l + GL * j;
            if (k < HUM_NOBS) {
                X[k] = xv[j];
                if (valid && a.obs_traj) a.obs_traj[io * HUM_NOBS + k] = xv[j];
            }
        }
        wave_sync();
        policy_wave<T, EPB_>(a, sh, blk, t, a.pw, a.pseed, ~0ull, a.act_traj, a.act_last, a.mean_traj);
    }
    // POLICY: the env's clipped actions held in registers across the physics (which reuses the scratch), one per lane
    // (lane 0 also the 17th); post_step reads them back from LDS for the electricity cost
    float pact0 = 0.f, pact1 = 0.f;
    if constexpr (NET) {
        pact0 = policy_scratch(S)[PACT_OFF + l];
        pact1 = policy_scratch(S)[PACT_OFF + GL];
    }
    bool fin = true;
    for (int k = l; k < HUM_NACT; k += GL) {   // apply_action (humanoid.py:54-60)
        const float av = !valid ? 0.f : (NET ? policy_scratch(S)[PACT_OFF + k] : a.act[io * HUM_NACT + k]);
        fin = fin && isfinite(av);
        S.tau[M.act_dof[k]] = (T)motor_torque(a.np1, M.act_gain[k], M.act_gain_d[k], isfinite(av) ? av : 0.f);
    }
    // hierarchical env: envs whose acting agent is the high level take no physics step (hier_env.py:538-571)
    const unsigned char sel = hier && valid && a.agent_sel ? a.agent_sel[io] : (unsigned char)0;
    const bool skip = hier && valid && a.agent_sel && sel == HUM_AGENT_SEL_SKIP;   // no action: lane untouched
    const bool high = hier && valid && !skip && (a.agent_sel ? sel != 0 : carry[0] != 0);
    const bool env_ok = high || ((__ballot(!fin) >> gbit) & 0xFFFFull) == 0;
    // an env that takes no physics step this round rides along with the wave's physics and keeps its LDS state
    const bool frozen = !valid || skip || high || !env_ok;
    const bool any_phys = __ballot(!frozen) != 0;   // wave-uniform
    // the env's terrain (HUM_TERRAIN_RANDOM_BLOCKS: drawn at its last reset)
    const unsigned long long tkey = TERRAIN && a.P.terrain == HUM_TERRAIN_RANDOM_BLOCKS && valid
        ? ((unsigned long long)(unsigned)carry[1] | ((unsigned long long)(unsigned)carry[2] << 32)) : 0ull;
    __syncthreads();
    if (!(a.flags & HUM_STEP_SKIP_PHYSICS) && any_phys) {
#pragma unroll 1
        for (int s = 0; s < a.P.nsub; s++)
            group_substep<T, EPB_, TERRAIN>(a.P, sh, ge, (T*)a.scratch + (long)blockIdx.x * grow_block_size(EPB_, a.P.lds_rows),
                                   l, ef, tkey, frozen);
    }
#ifdef HUM_SKIP_POST   // lane-utilisation study (tools/lane_util.py): the physics alone, no env logic / outputs
    __syncthreads();
    continue;
#endif
    // hinge sin / cos of the final physics state, one dof per lane, for calc_state's kinematics on lane 0
    T* scs = &sh[ge].x.aba.IA[0][0];
    for (int d = l; d < NDOF; d += GL) {
        T sn, cs;
        hinge_sincos(S.st[13 + d], &sn, &cs);
        scs[2 * d] = sn;
        scs[2 * d + 1] = cs;
    }
    // LDS staging of the low-level env's output rows (the ABA scratch is dead after the physics): lane 0 writes
    // them, then every lane of the env stores its share, 16 consecutive words per store instruction
    // (IA words [0, 70): the hinge sin / cos below and the reset exchange; [72, 142): obs; [144, 214): reset obs)
    float* ostage = reinterpret_cast<float*>(scs + 72);    // this step's observation
    float* rstage = reinterpret_cast<float*>(scs + 144);   // the auto-reset observation
    static_assert(sizeof(sh[0].x.aba.IA) >= (144 + HUM_NOBS) * sizeof(T) && 2 * NDOF + 2 + 2 * NDOF <= 72,
                  "output row staging");
    if constexpr (NET) {   // the step's actions for post_step, in the reset-obs staging row (written after it)
        rstage[l] = pact0;
        if (l == 0) rstage[GL] = pact1;
    }
    // low-level env: calc_state's joint block (obs 8..41, the joint speeds, the at-limit count) one dof per lane, into
    // the staging row (clamped like the observation) and the joint speeds past the reset obs row
    float* jstage = reinterpret_cast<float*>(scs + 216);
    static_assert(sizeof(sh[0].x.aba.IA) >= (216 + NDOF) * sizeof(T), "joint speed staging");
    int jal_l = 0;
    if (!hier) {
        unsigned jmask = 0;
        for (int d = l; d < NDOF; d += GL) {
            float rp, rv;
            if (joint_obs(S.st, d, rp, rv)) jmask |= 1u << (d / GL);
            ostage[8 + 2 * d] = fminf(fmaxf(rp, -5.0f), 5.0f);
            ostage[9 + 2 * d] = fminf(fmaxf(rv, -5.0f), 5.0f);
            jstage[d] = rv;
        }
        const unsigned long long b0 = __ballot(jmask & 1u), b1 = __ballot((jmask >> 1) & 1u);
        jal_l = __popcll((b0 >> gbit) & 0xFFFFull) + __popcll((b1 >> gbit) & 0xFFFFull);
    }
    wave_sync();
    PHASE_INIT;
    Book b;
    T st[HUM_NSTATE];
    bool rst = false, booked = false;
    if (valid && l == 0 && a.acted) a.acted[io] = skip || !env_ok ? 0 : (high ? HUM_AGENT_HIGH : HUM_AGENT_LOW);
    if (valid && l == 0 && skip) {
        a.agents[io] = 0;
    } else if (valid && l == 0) {
        load_book(a, i, b, hier);
        POST_SUBPHASE(17);
        if (!env_ok) {   // humanoid.py:55 assert: env not stepped, flagged for the host
            ef |= HUM_EFLAG_NONFINITE_ACTION;
            nonfinite_outputs(a, io, b.frame, hier ? nullptr : ostage);
        } else {
            // the env's current state (a frozen env's: unchanged by the wave's physics)
#pragma unroll
            for (int e = 0; e < HUM_NSTATE; e++) st[e] = S.st[e];
            booked = true;
            if (HP) {   // the actions out of the staging row into registers; observation rows in place (row i)
                float lact[HUM_NACT];
#pragma unroll
                for (int k = 0; k < HUM_NACT; k++) lact[k] = rstage[k];
                hier_post(a, i, io, st, b, high, ef, scs, false, (long)i, lact, lact);
#pragma unroll
                for (int e = 0; e < HUM_NSTATE; e++) S.st[e] = st[e];   // an auto-reset replaced it
            } else if (a.hier) {
                hier_post(a, i, io, st, b, high, ef, scs, false);
#pragma unroll
                for (int e = 0; e < HUM_NSTATE; e++) S.st[e] = st[e];   // an auto-reset replaced it
            } else {
                float act[HUM_NACT];
#pragma unroll
                for (int k = 0; k < HUM_NACT; k++) act[k] = NET ? rstage[k] : a.act[io * HUM_NACT + k];
                post_step(a, i, io, st, b, act, ef, scs, &rst, ostage, jstage, jal_l);
            }
        }
    }
    POST_SUBPHASE(18);
    if (!hier) {
        // auto-reset (low-level env): lane 0 draws the start frame (reset_lane's first draw), the env's lanes
        // compute the reset pose's hinge sin / cos, lane 0 finishes reset_lane with them
        int* xch = reinterpret_cast<int*>(scs + 2 * NDOF);
        if (valid && l == 0) {
            int sf = -1;
            if (rst) sf = draw(a, i, b, 0, a.clips[b.clip].max_frame - 5);   // low_level_env.py:228
            xch[0] = sf;
            xch[1] = b.clip;
        }
        wave_sync();
        const int sf = valid ? xch[0] : -1;
        T* scs_r = scs + 2 * NDOF + 2;
        if (__ballot(sf >= 0) != 0) {
            if (sf >= 0) {
                const ClipDev& c = a.clips[xch[1]];
                for (int d = l; d < NDOF; d += GL) {
                    T q = T(0);
#pragma unroll
                    for (int j = 0; j < NREF; j++)
                        if (JM_DOF[j] == d) q = (T)c.gpos()[sf * 14 + JM_COL[j]];
                    T sn, cs;
                    hinge_sincos(q, &sn, &cs);
                    scs_r[2 * d] = sn;
                    scs_r[2 * d + 1] = cs;
                }
            }
            wave_sync();
        }
        if (valid && l == 0 && booked) {
            if (rst) {
                float o2[HUM_NOBS];
                reset_lane(a, i, st, b, sf, 0.0, o2, ef, scs_r);
#pragma unroll
                for (int k = 0; k < HUM_NOBS; k++) rstage[k] = o2[k];
#pragma unroll
                for (int e = 0; e < HUM_NSTATE; e++) S.st[e] = st[e];
            }
            store_book(a, i, b);
        }
        wave_sync();
        // the output rows, coalesced (POLICY: the next step's input stays in LDS; only the last step's rows go to
        // the handle's [n, 70] obs / obs_reset buffers)
        const long orow_i = NET ? (long)i : io;
        if (valid && (!NET || t == ksteps - 1)) {
            float* orow = a.obs + orow_i * HUM_NOBS;
            for (int k = l; k < HUM_NOBS; k += GL) orow[k] = ostage[k];
            if (sf >= 0 && a.obs_reset) {
                float* rrow = a.obs_reset + orow_i * HUM_NOBS;
                for (int k = l; k < HUM_NOBS; k += GL) rrow[k] = rstage[k];
            }
        }
        prev_reset = sf >= 0;
    }
    PHASE(10);
    if (valid && l == 0 && booked) {   // the per-env integers the next step's lanes read
        carry[0] = hier ? b.expect_high : 0;
        carry[1] = (int)(unsigned)(b.terrain_key & 0xffffffffull);
        carry[2] = (int)(unsigned)(b.terrain_key >> 32);
    }
    __syncthreads();
    }   // steps of the launch
    {   // the launch's final physics state (it stays in LDS between the steps): each lane of an env stores its share
        const int l = threadIdx.x & (GL - 1), ge = threadIdx.x / GL, i = blk * EPB_ + ge;
        if (i < a0.n) {
#pragma unroll
            for (int e = l; e < HUM_NSTATE; e += GL) ((T*)a0.phys)[(long)e * a0.n + i] = sh[ge].st[e];
        }
    }
#ifdef HUM_WLOG_ON
    if (threadIdx.x == 0) {   // wave duration: max (tail) and mean
        const unsigned long long dtw = __builtin_amdgcn_s_memtime() - t_wave0;
#ifdef HUM_PHASE_TIMING
        atomicMax(&g_phase_cycles[16], dtw);
        atomicAdd(&g_phase_cycles[17], dtw);
        atomicAdd(&g_phase_cycles[18], 1ull);
#endif
        if (blockIdx.x < 65536) {
            g_wave_log[blockIdx.x][0] = (unsigned)dtw;
            g_wave_log[blockIdx.x][5] = (unsigned)rt_wave0;   // 100 MHz, device-wide
            g_wave_log[blockIdx.x][4] = (unsigned)(__builtin_amdgcn_s_memrealtime() - rt_wave0);
            g_wave_log[blockIdx.x][6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
            g_wave_log[blockIdx.x][7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
#ifdef HUM_WAVE_LOG
            for (int k = 1; k <= 23; k++) g_wave_log[blockIdx.x][8 + k] = (unsigned)s_phase[k];
#endif
        }
    }
#endif
    if (ef) atomicOr(a0.eflags, ef);
}

template <typename T>
__global__ void __launch_bounds__(256) reset_kernel(KArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    if (a.mask && !a.mask[i]) return;
    T st[HUM_NSTATE];
    Book b;
    load_lane(a, i, st, b);
    unsigned ef = 0;
    float obs[HUM_NOBS];
    const int sf = a.start_frame ? a.start_frame[i] : -1;
    const double ry = a.reset_yaw ? a.reset_yaw[i] : 0.0;
    {   // resetFromFrame past the clip: the reference's DataFrame.iloc raises IndexError (low_level_env.py:208,
        // :282-291; hier_env.py:293-304 also reads end-point row startFrame + 1)
        const ClipDev& c = a.clips[b.clip];
        if (!(a.reset_flags & HUM_RESET_NO_REF_POSE) && sf >= (a.hier ? c.n_pos - 1 : c.n_pos)) {
            atomicOr(a.eflags, HUM_EFLAG_BAD_START_FRAME);
            return;
        }
    }
    if (a.hier) {
        hier_reset_lane(a, i, st, b, sf, ry, obs, ef);
        if (a.obs_high) {
#pragma unroll
            for (int k = 0; k < HUM_NOBS_HIGH; k++) a.obs_high[(long)i * HUM_NOBS_HIGH + k] = obs[k];
        }
    } else {
        reset_lane(a, i, st, b, sf, ry, obs, ef);
        if (a.obs) {
#pragma unroll
            for (int k = 0; k < HUM_NOBS; k++) a.obs[(long)i * HUM_NOBS + k] = obs[k];
        }
    }
    store_lane(a, i, st, b);
    if (ef) atomicOr(a.eflags, ef);
}

static __global__ void init_kernel(KArgs a) {   // fresh lanes: clip 0, no mode, RNG key from (seed, global lane)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    // non-additive key (oracle/oracle.py::lane_key): (seed s, lane i+1) and (seed s+1, lane i) differ
    const unsigned long long k = splitmix64(splitmix64(a.seed) ^ (unsigned long long)(a.lane_offset + i));
    a.bi[6 * a.n + i] = (int)(unsigned)(k & 0xffffffffull);
    a.bi[7 * a.n + i] = (int)(unsigned)(k >> 32);
}

// calcEndPointScore (low_level_env.py:361-382): sum over {link0_11: RightLeg 1, right_foot: RightFoot 3,
// link0_18: LeftLeg 1, left_foot: LeftFoot 3} of w * |starting_ep_pos + Rz(highLevelDegTarget) ref - part|,
// score = -sum / 8 (useExp: exp(3 score)); scipy's from_euler('z') matrix and apply() order, float64
#pragma clang fp contract(off)
template <typename T>
__device__ inline void end_point_score(const KArgs& a, const T* st, const Book& b, double& score, double& score_exp) {
    const ClipDev& c = a.clips[b.clip];
    Kin<T> K;
    forward_kinematics(st + 3, st + 13, K);
    T pp[NPART][3];
    part_positions(K, pp);
    const double qz = sin(b.hldt / 2), qw = cos(b.hldt / 2);
    const double r00 = -(qz * qz) + qw * qw, r01 = 2 * (0.0 - qz * qw), r10 = 2 * (0.0 + qz * qw);
    const double r11 = -(qz * qz) + qw * qw, r22 = qz * qz + qw * qw;
    constexpr int PART[4] = {10, 12, 17, 19}, EPC[4] = {6, 9, 0, 3};   // link0_11, right_foot, link0_18, left_foot
    constexpr double W[4] = {1, 3, 1, 3};
    const HUM_GLOBAL double* e = c.gep() + b.frame * 27;
    double d = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const double x = e[EPC[k]], y = e[EPC[k] + 1], z = e[EPC[k] + 2];
        const double v2x = b.sep[0] + ((r00 * x + r01 * y) + 0.0 * z);
        const double v2y = b.sep[1] + ((r10 * x + r11 * y) + 0.0 * z);
        const double v2z = b.sep[2] + ((0.0 * x + 0.0 * y) + r22 * z);
        const double v1x = (double)st[0] + (double)pp[PART[k]][0], v1y = (double)st[1] + (double)pp[PART[k]][1];
        const double v1z = (double)st[2] + (double)pp[PART[k]][2];
        d = d + norm3_blas(v2x - v1x, v2y - v1y, v2z - v1z) * W[k];
    }
    score = -d / 8;
    score_exp = exp(3 * score);
}
#pragma clang fp contract(on)

template <typename T>
__global__ void aux_kernel(KArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    T st[HUM_NSTATE];
    Book b;
    load_lane(a, i, st, b);
    float* o = a.aux + (long)i * HUM_NAUX;
    o[HUM_AUX_DELTA_JOINTS] = (float)b.dj;
    o[HUM_AUX_DELTA_END_POINTS] = 0.f;   // calcEndPointScore is not on the reward path (:445)
    o[HUM_AUX_LOW_TARGET_SCORE] = (float)b.lts;
    o[HUM_AUX_DELTA_VEL_JOINTS] = (float)b.dvj;
    o[HUM_AUX_BODY_POSTURE] = (float)b.bps;
    o[HUM_AUX_HIGH_TARGET_SCORE] = a.hier ? (float)b.hts : 0.f;
    o[HUM_AUX_DRIFT_SCORE] = a.hier ? (float)b.drift : 0.f;
    o[HUM_AUX_BASE_REWARD] = 0.f;
    o[HUM_AUX_ALIVE] = (float)b.alive;
    o[HUM_AUX_ELECTRICITY] = (float)b.es;
    o[HUM_AUX_JOINT_LIMIT] = (float)b.jls;
    o[HUM_AUX_DIST_FROM_ORIGIN] = (float)norm3_blas(b.robot_pos[0], b.robot_pos[1], b.robot_pos[2]);
    double sc, sce;
    end_point_score(a, st, b, sc, sce);
    o[HUM_AUX_END_POINT_SCORE] = (float)sc;
    o[HUM_AUX_END_POINT_SCORE_EXP] = (float)sce;
    for (int k = 0; k < 3; k++) o[HUM_AUX_ROBOT_POS + k] = (float)b.robot_pos[k];
}

template <typename T>
__global__ void parts_kernel(KArgs a, double* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    T st[HUM_NSTATE];
    Book b;
    load_lane(a, i, st, b);
    Kin<T> K;
    forward_kinematics(st + 3, st + 13, K);
    T pp[NPART][3];
    part_positions(K, pp);
    for (int k = 0; k < NPART; k++)
        for (int e = 0; e < 3; e++)
            out[((long)i * NPART + k) * 3 + e] = part_body[k] < 0 ? 0.0 : (double)st[e] + (double)pp[k][e];
}


// the benchmarked cooperative kernel lives in its own translation unit (group_f32.hip)
hipError_t launch_group_f32_4(const KArgs& a, int nblocks, hipStream_t s);
hipError_t launch_group_f32_4_low(const KArgs& a, int nblocks, hipStream_t s);
hipError_t launch_group_f32_4_policy(const KArgs& a, int nblocks, hipStream_t s);
hipError_t launch_group_f32_4_hier_policy(const KArgs& a, int nblocks, hipStream_t s);

}  // namespace hkk

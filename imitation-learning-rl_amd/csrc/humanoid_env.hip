// humanoid_env.hip - HIP kernels + C-ABI (include/humanoid_env.h) for the vectorised humanoid env.
//
// One launch = one env step for all lanes (4 physics substeps fused with the observation, imitation
// reward, frame/target bookkeeping and optional auto-reset).  One env per lane; lane state is SoA in
// HBM (element-major: value e of lane i at base[e * n + i]) so every load/store is coalesced.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/humanoid_env.h"
#include "physics.h"
#include "envlogic.h"
#include "physics_group.h"

using namespace hk;

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return fail(HUM_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

constexpr int NBOOK_I = 11;   // frame, timestep, pred_idx, clip, rng_ctr, mode, rng key lo, rng key hi
                              // | hier: level_rem, n_high, expect_high
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
    float* aux;
    // hierarchical env (hum_hier_step / hum_hier_reset)
    int hier;
    const float* act_high;          // [n,2]
    const unsigned char* agent_sel; // [n] 1 = high, 0 = low (NULL = the lane's expected agent)
    unsigned char* agents;          // [n] HUM_AGENT_* present in the returned dicts
    float* obs_high;                // [n,44]
    float* rew_high;                // [n]
    float* obs_high_reset;          // [n,44]
};

// ----------------------------------------------------------------------------------- SoA lane I/O
__device__ inline void load_book(const KArgs& a, int i, Book& b) {
    const int* bi = a.bi;
    b.frame = bi[0 * a.n + i]; b.timestep = bi[1 * a.n + i]; b.pred_idx = bi[2 * a.n + i];
    b.clip = bi[3 * a.n + i]; b.rng_ctr = (unsigned)bi[4 * a.n + i]; b.mode = (unsigned)bi[5 * a.n + i];
    b.rng_key = (unsigned long long)(unsigned)bi[6 * a.n + i] | ((unsigned long long)(unsigned)bi[7 * a.n + i] << 32);
    const double* d = a.bd;
    auto D = [&](int e) { return d[(long)e * a.n + i]; };
    for (int k = 0; k < 3; k++) { b.target[k] = D(k); b.srp[k] = D(3 + k); b.robot_pos[k] = D(6 + k); b.sep[k] = D(9 + k); }
    b.hldt = D(12); b.wt[0] = D(13); b.wt[1] = D(14); b.lts = D(15);
    b.dj = D(16); b.dvj = D(17); b.bps = D(18); b.es = D(19); b.jls = D(20); b.alive = D(21); b.dlts = D(22);
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

// ----------------------------------------------------------------------------------- reset
// LowLevelHumanoidEnv.reset() / resetFromFrame() (low_level_env.py:224-305)
template <typename T>
__device__ void reset_lane(const KArgs& a, int i, T* st, Book& b, int start_frame, double reset_yaw, float* obs,
                           unsigned& ef) {
    const ClipDev& c = a.clips[b.clip];
    if (start_frame < 0) start_frame = draw(a, i, b, 0, c.max_frame - 5);   // :228
    // flat_env.reset(): restoreState -> zero velocities (all 17 joints overwritten below)
#pragma unroll
    for (int e = 0; e < HUM_NSTATE; e++) st[e] = 0;
    st[6] = 1;
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
    b.frame = start_frame;                                                  // :259-261 setJointsOrientation
    int vrow = start_frame;
    if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
    for (int j = 0; j < NREF; j++) {
        st[13 + JM_DOF[j]] = (T)c.pos[start_frame * 14 + JM_COL[j]];
        st[30 + JM_DOF[j]] = (T)c.vel[vrow * 14 + JM_COL[j]];
    }
    for (int k = 0; k < 3; k++) { b.robot_pos[k] = 0; b.srp[k] = 0; }      // :264-268
    st[0] = 0; st[1] = 0; st[2] = (T)1.17;
    const double degToTarget = atan2(b.target[1], b.target[0]) * RAD2DEG;  // :270
    b.wt[0] = cos(degToTarget) * 1000;                                      // :271 (degrees into cos: quirk)
    b.wt[1] = sin(degToTarget) * 1000;
    const double th = (degToTarget + reset_yaw) * DEG2RAD;                  // :272-273 scipy from_euler
    st[3] = 0; st[4] = 0; st[5] = (T)sin(th / 2); st[6] = (T)cos(th / 2);
    b.hldt = degToTarget * DEG2RAD;                                         // :275
    // starting_ep_pos (:277-289) and the initial base velocity (:291-295)
    const int f0 = b.frame, f1 = (b.frame + 2) % c.max_frame;
    const double phi = degToTarget * DEG2RAD;
    const double qz = sin(phi / 2), qw = cos(phi / 2);
    const double r00 = -(qz * qz) + qw * qw, r01 = 2 * (0.0 - qz * qw), r10 = 2 * (0.0 + qz * qw), r11 = -(qz * qz) + qw * qw;
    {
        Kin<T> K;
        forward_kinematics(st + 3, st + 13, K);
        T pp[NPART][3];
        part_positions(K, pp);
        const double rfx = (double)st[0] + (double)pp[PART_RIGHT_FOOT][0];
        const double rfy = (double)st[1] + (double)pp[PART_RIGHT_FOOT][1];
        const double* e0 = c.ep + f0 * 27;
        const double* e1 = c.ep + f1 * 27;
        const double refx = r00 * e0[EP_RIGHT_FOOT] + r01 * e0[EP_RIGHT_FOOT + 1];
        const double refy = r10 * e0[EP_RIGHT_FOOT] + r11 * e0[EP_RIGHT_FOOT + 1];
        b.sep[0] = rfx - refx; b.sep[1] = rfy - refy; b.sep[2] = 0;
        const double l0x = r00 * e0[EP_RIGHT_LEG] + r01 * e0[EP_RIGHT_LEG + 1], l0y = r10 * e0[EP_RIGHT_LEG] + r11 * e0[EP_RIGHT_LEG + 1];
        const double l1x = r00 * e1[EP_RIGHT_LEG] + r01 * e1[EP_RIGHT_LEG + 1], l1y = r10 * e1[EP_RIGHT_LEG] + r11 * e1[EP_RIGHT_LEG + 1];
        st[7] = (T)(((l1x - l0x) / 0.0165) / 1.2);
        st[8] = (T)(((l1y - l0y) / 0.0165) / 1.2);
        st[9] = (T)(((e1[EP_RIGHT_LEG + 2] - e0[EP_RIGHT_LEG + 2]) / 0.0165) / 1.2);
    }
    b.lts = 0; b.dj = 0; b.dvj = 0; b.bps = 0; b.es = 0; b.jls = 0; b.alive = 0; b.dlts = 0;   // initReward
    inc_frame(b, c, 2);                                                     // :302
    float js[NDOF];
    int jal;
    PostPhys<T> pp;
    calc_state(st, b.wt, obs, js, jal, pp);                                 // :304-305
    ref_obs(c, b.frame, obs + 42, ef);
}

// Post-physics part of step (low_level_env.py:481-526) + optional auto-reset; stores state, book, outputs.
template <typename T>
__device__ void post_step(const KArgs& a, int i, T* st, Book& b, const float* act, unsigned& ef) {
    const ClipDev& c = a.clips[b.clip];
    float obs[HUM_NOBS];
    // calc_state (:481) and robot_pos (:483-486)
    float js[NDOF];
    int jal;
    PostPhys<T> pp;
    calc_state(st, b.wt, obs, js, jal, pp);
    b.robot_pos[0] = pp.bx; b.robot_pos[1] = pp.by; b.robot_pos[2] = 0;
    // updateReward (:441-465)
    double dJ = 0, dV = 0;
#pragma unroll
    for (int j = 0; j < NREF; j++) {
        dJ = dJ + fabs(pp.q[JM_DOF[j]] - c.pos[b.frame * 14 + JM_COL[j]]) * JM_W[j];
    }
    int vrow = b.frame;
    if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
    for (int j = 0; j < NREF; j++) {
        dV = dV + fabs(pp.qd[JM_DOF[j]] - c.vel[vrow * 14 + JM_COL[j]]) * JM_WV[j];
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
    b.alive = ((obs[0] + 0.8f) > 0.75f) ? 2.0 : -1.0;
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
#pragma unroll
    for (int k = 0; k < HUM_NOBS; k++) a.obs[(long)i * HUM_NOBS + k] = obs[k];
    a.rew[i] = (float)total;
    a.done[i] = done ? 1 : 0;
    if (a.frame_out) a.frame_out[i] = b.frame;
    if (done && (a.flags & HUM_STEP_AUTORESET)) {
        float o2[HUM_NOBS];
        reset_lane(a, i, st, b, -1, 0.0, o2, ef);
        if (a.obs_reset) {
#pragma unroll
            for (int k = 0; k < HUM_NOBS; k++) a.obs_reset[(long)i * HUM_NOBS + k] = o2[k];
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
__device__ void hier_reset_lane(const KArgs& a, int i, T* st, Book& b, int start_frame, double reset_yaw, float* o44,
                                unsigned& ef) {
    const ClipDev& c = a.clips[b.clip];
    if (start_frame < 0) {                                                  // :238-241 (argument order)
        start_frame = draw(a, i, b, 0, c.max_frame - 5);
        reset_yaw = (double)draw(a, i, b, -180, 180);
    }
#pragma unroll
    for (int e = 0; e < HUM_NSTATE; e++) st[e] = 0;                         // flat_env.reset()
    st[6] = 1;
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
    b.frame = start_frame;                                                  // :272-274 setJointsOrientation
    int vrow = start_frame;
    if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
    for (int j = 0; j < NREF; j++) {
        st[13 + JM_DOF[j]] = (T)c.pos[start_frame * 14 + JM_COL[j]];
        st[30 + JM_DOF[j]] = (T)c.vel[vrow * 14 + JM_COL[j]];
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
        const double* e0 = c.ep + f0 * 27;
        const double* e1 = c.ep + f1 * 27;
        const double l0x = r00 * e0[EP_RIGHT_LEG] + r01 * e0[EP_RIGHT_LEG + 1], l0y = r10 * e0[EP_RIGHT_LEG] + r11 * e0[EP_RIGHT_LEG + 1];
        const double l1x = r00 * e1[EP_RIGHT_LEG] + r01 * e1[EP_RIGHT_LEG + 1], l1y = r10 * e1[EP_RIGHT_LEG] + r11 * e1[EP_RIGHT_LEG + 1];
        st[7] = (T)((l1x - l0x) / 0.0165);
        st[8] = (T)((l1y - l0y) / 0.0165);
        st[9] = (T)((e1[EP_RIGHT_LEG + 2] - e0[EP_RIGHT_LEG + 2]) / 0.0165);
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
__device__ void hier_post(const KArgs& a, int i, T* st, Book& b, bool high, unsigned& ef) {
    const ClipDev& c = a.clips[b.clip];
    b.robot_pos[0] = b.bxy[0]; b.robot_pos[1] = b.bxy[1]; b.robot_pos[2] = 0;   // step(): :358-361
    float obs[HUM_NOBS], js[NDOF], o44[HUM_NOBS_HIGH];
    int jal;
    PostPhys<T> pp;
    unsigned agents = 0;
    bool done = false;
    float rew_low = 0.f, rew_high = 0.f;
    if (high) {
        // cur_obs is the last calc_state (same physics state, walk target before this call)
        calc_state(st, b.wt, obs, js, jal, pp);
        const float a0 = a.act_high[2 * (long)i], a1 = a.act_high[2 * (long)i + 1];
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
        calc_state(st, b.wt, obs, js, jal, pp);                                             // :591
        const float* act = a.act + (long)i * HUM_NACT;
        // updateReward (:494-522)
        double dJ = 0, dV = 0;
#pragma unroll
        for (int j = 0; j < NREF; j++) dJ = dJ + fabs(pp.q[JM_DOF[j]] - c.pos[b.frame * 14 + JM_COL[j]]) * JM_W[j];
        int vrow = b.frame;
        if (vrow >= c.n_vel) { vrow = c.n_vel - 1; ef |= HUM_EFLAG_VEL_ROW; }
#pragma unroll
        for (int j = 0; j < NREF; j++) dV = dV + fabs(pp.qd[JM_DOF[j]] - c.vel[vrow * 14 + JM_COL[j]]) * JM_WV[j];
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
        b.alive = ((obs[0] + 0.8f) > 0.75f) ? 2.0 : -1.0;
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
        for (int k = 0; k < HUM_NOBS; k++) a.obs[(long)i * HUM_NOBS + k] = obs[k];
    }
    if (agents & HUM_AGENT_HIGH) {
#pragma unroll
        for (int k = 0; k < HUM_NOBS_HIGH; k++) a.obs_high[(long)i * HUM_NOBS_HIGH + k] = o44[k];
    }
    a.rew[i] = (agents & HUM_AGENT_LOW) ? rew_low : 0.f;   // the level hand-back drops the low reward (:631-636)
    a.rew_high[i] = rew_high;
    a.agents[i] = (unsigned char)agents;
    a.done[i] = done ? 1 : 0;
    if (a.frame_out) a.frame_out[i] = b.frame;
    if (done && (a.flags & HUM_STEP_AUTORESET)) {
        float r44[HUM_NOBS_HIGH];
        hier_reset_lane(a, i, st, b, -1, 0.0, r44, ef);
        if (a.obs_high_reset) {
#pragma unroll
            for (int k = 0; k < HUM_NOBS_HIGH; k++) a.obs_high_reset[(long)i * HUM_NOBS_HIGH + k] = r44[k];
        }
    }
    store_lane(a, i, st, b);
    if (ef) atomicOr(a.eflags, ef);
}

// non-finite action on a lane (humanoid.py:55 assert): lane not stepped, flagged, outputs neutral
__device__ inline void nonfinite_outputs(const KArgs& a, int i, int frame) {
    if (!a.hier) {
        for (int k = 0; k < HUM_NOBS; k++) a.obs[(long)i * HUM_NOBS + k] = 0.f;
    } else {
        a.rew_high[i] = 0.f;
        a.agents[i] = 0;
    }
    a.rew[i] = 0.f;
    a.done[i] = 1;
    if (a.frame_out) a.frame_out[i] = frame;
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
    // hierarchical env: the lane's acting agent (step(action_dict) dispatch, hier_env.py:363-366)
    const bool high = a.hier && (a.agent_sel ? a.agent_sel[i] != 0 : b.expect_high != 0);
    float act[HUM_NACT];
    bool finite = true;
#pragma unroll
    for (int k = 0; k < HUM_NACT; k++) {
        act[k] = a.act[(long)i * HUM_NACT + k];
        finite &= isfinite(act[k]);
    }
    if (!finite && !high) {   // humanoid.py:55 assert: lane not stepped, flagged for the host
        ef |= HUM_EFLAG_NONFINITE_ACTION;
        nonfinite_outputs(a, i, b.frame);
        atomicOr(a.eflags, ef);
        return;
    }
    if (!(a.flags & HUM_STEP_SKIP_PHYSICS) && !high) {
        T tau[NDOF];
#pragma unroll
        for (int k = 0; k < HUM_NACT; k++) {   // apply_action: float(1 * power * 0.41 * clip(a)) in float32
            const float g = (float)act_gain[k];
            tau[act_dof[k]] = (T)(double)(g * fminf(fmaxf(act[k], -1.f), 1.f));
        }
        Lane<T> rows{(T*)a.scratch + i, (long)a.n};
#pragma unroll 1
        for (int s = 0; s < a.P.nsub; s++) {
            if (substep(a.P, st, tau, rows)) ef |= HUM_EFLAG_CONTACT_OVERFLOW;
        }
    }
    if (a.hier) hier_post(a, i, st, b, high, ef);
    else post_step(a, i, st, b, act, ef);
}

// Cooperative step: 16 lanes per env, EPB_ envs per block of EPB_*16 threads (one wavefront), env working
// set in LDS.  EPB_ = 4 fills the wave; EPB_ = 2 leaves half of it idle but lets a SIMD hold two waves
// (19.3 KB LDS per block), so one wave's LDS/memory waits overlap the other's VALU issue.
template <typename T, int EPB_>
__global__ void __launch_bounds__(EPB_ * GL) step_group_kernel(KArgs a) {
    __shared__ GroupLDS<T> sh[EPB_];
    const int l = threadIdx.x & (GL - 1), ge = threadIdx.x / GL;
    const int i = blockIdx.x * EPB_ + ge;
    const bool valid = i < a.n;
    GroupLDS<T>& S = sh[ge];
    const ModelTab<T>& M = tab<T>();
    for (int e = l; e < HUM_NSTATE; e += GL)
        S.st[e] = valid ? ((const T*)a.phys)[(long)e * a.n + i] : (e == 2 ? T(1.17) : (e == 6 ? T(1) : T(0)));
    bool fin = true;
    for (int k = l; k < HUM_NACT; k += GL) {   // apply_action (humanoid.py:54-60), float32 product
        const float av = valid ? a.act[(long)i * HUM_NACT + k] : 0.f;
        fin = fin && isfinite(av);
        S.tau[M.act_dof[k]] = (T)(double)(M.act_gain[k] * fminf(fmaxf(isfinite(av) ? av : 0.f, -1.f), 1.f));
    }
    const int gbit = (threadIdx.x & 63) & ~(GL - 1);
    // hierarchical env: envs whose acting agent is the high level take no physics step (hier_env.py:538-571)
    const bool high = a.hier && valid && (a.agent_sel ? a.agent_sel[i] != 0 : a.bi[10 * a.n + i] != 0);
    const bool env_ok = high || ((__ballot(!fin) >> gbit) & 0xFFFFull) == 0;
    const bool any_phys = __ballot(valid && !high) != 0;   // wave-uniform
    __syncthreads();
    unsigned ef = 0;
    if (!(a.flags & HUM_STEP_SKIP_PHYSICS) && any_phys) {
#pragma unroll 1
        for (int s = 0; s < a.P.nsub; s++)
            group_substep<T, EPB_>(a.P, sh, ge, (T*)a.scratch + (long)blockIdx.x * EPB_ * GROW_PER_ENV, l, ef);
    }
    PHASE_INIT;
    if (valid && l == 0) {
        Book b;
        load_book(a, i, b);
        if (!env_ok) {   // humanoid.py:55 assert: env not stepped, flagged for the host
            ef |= HUM_EFLAG_NONFINITE_ACTION;
            nonfinite_outputs(a, i, b.frame);
        } else {
            T st[HUM_NSTATE];
            if (high) {   // physics (if the wave ran it) is discarded: the HBM state is the current one
#pragma unroll
                for (int e = 0; e < HUM_NSTATE; e++) st[e] = ((const T*)a.phys)[(long)e * a.n + i];
            } else {
#pragma unroll
                for (int e = 0; e < HUM_NSTATE; e++) st[e] = S.st[e];
            }
            if (a.hier) {
                hier_post(a, i, st, b, high, ef);
            } else {
                float act[HUM_NACT];
#pragma unroll
                for (int k = 0; k < HUM_NACT; k++) act[k] = a.act[(long)i * HUM_NACT + k];
                post_step(a, i, st, b, act, ef);
            }
        }
    }
    PHASE(10);
    if (ef) atomicOr(a.eflags, ef);
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

__global__ void init_kernel(KArgs a) {   // fresh lanes: clip 0, no mode, RNG key from (seed, global lane)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const unsigned long long k = splitmix64(a.seed + (unsigned long long)(a.lane_offset + i));
    a.bi[6 * a.n + i] = (int)(unsigned)(k & 0xffffffffull);
    a.bi[7 * a.n + i] = (int)(unsigned)(k >> 32);
}

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

}  // namespace

// ======================================================================================= C-ABI
struct hum_env {
    hum_config cfg;
    int n;
    hipStream_t stream;
    DevState d;
    size_t real_size;
    double* clip_dev[HUM_MAX_CLIPS];
    ClipDev clips[HUM_MAX_CLIPS];
    ClipDev* clips_dev;   // device copy of clips[] read by the kernels
    bool clip_set[HUM_MAX_CLIPS];
    double* pred;
    int npred;
    unsigned* eflags;
    hipGraphExec_t graph;
    int graph_k;
    const void* graph_key[6];
    unsigned graph_flags;
};

namespace {
KArgs make_args(hum_env* e) {
    KArgs a;
    memset(&a, 0, sizeof a);
    a.n = e->n;
    a.seed = e->cfg.seed;
    a.lane_offset = e->cfg.lane_offset;
    const hum_config& c = e->cfg;
    a.P.dt = c.dt_env / c.substeps;
    a.P.nsub = c.substeps;
    a.P.gravity = c.gravity;
    a.P.iters = c.solver_iters;
    a.P.erp_contact = c.erp_contact;
    a.P.erp_limit = c.erp_limit;
    a.P.mu_ground = c.mu_ground;
    a.P.mu_self = c.mu_self;
    a.P.contact_thresh = c.contact_thresh;
    a.P.lin_damp = c.lin_damp;
    a.P.ang_damp = c.ang_damp;
    a.P.limit_max_impulse = c.limit_max_impulse;
    a.P.max_coord_vel = c.max_coord_vel;
    a.P.max_contacts = c.max_contacts;
    a.P.self_collision = c.self_collision;
    a.P.joint_damping = c.joint_damping;
    a.hier = c.hier;
    a.clips = e->clips_dev;
    a.pred = e->pred;
    a.npred = e->npred;
    a.phys = e->d.phys;
    a.bi = e->d.bi;
    a.bd = e->d.bd;
    a.scratch = e->d.scratch;
    a.eflags = e->eflags;
    return a;
}
dim3 grid_of(hum_env* e) { return dim3((e->n + e->cfg.block_size - 1) / e->cfg.block_size); }
hipStream_t stream_of(hum_env*, void* s) { return (hipStream_t)s; }   // NULL = HIP null stream
bool any_clip(hum_env* e) {
    for (int k = 0; k < HUM_MAX_CLIPS; k++)
        if (e->clip_set[k]) return true;
    return false;
}
}  // namespace

namespace { int launch_step(hum_env* e, const KArgs& a, hipStream_t s); }

extern "C" {

int hum_abi_version(void) { return HUM_ABI_VERSION; }
const char* hum_last_error(void) { return g_err.c_str(); }

void hum_default_config(hum_config* c) {
    memset(c, 0, sizeof *c);
    c->n_lanes = 1;
    c->device = 0;
    c->seed = 0;
    c->lane_offset = 0;
    c->precision = 0;
    c->block_size = 64;
    c->dt_env = 0.0165;
    c->substeps = 4;
    c->gravity = 9.8;
    c->solver_iters = 5;
    c->erp_contact = 0.9;
    c->erp_limit = 0.2;
    c->mu_ground = 2.0 * 0.8;
    c->mu_self = 2.0 * 2.0;
    c->contact_thresh = 0.02;
    c->lin_damp = 0.04;
    c->ang_damp = 0.04;
    c->limit_max_impulse = 100.0;
    c->max_coord_vel = 100.0;
    c->max_contacts = 16;
    c->self_collision = 1;
    c->joint_damping = 1;
    c->kernel = 1;
    c->hier = 0;
    c->envs_per_block = 4;
}

int hum_create(const hum_config* cfg, hum_env** out) {
    if (!cfg || !out) return fail(HUM_ERR_ARG, "hum_create: null argument");
    if (cfg->n_lanes <= 0) return fail(HUM_ERR_ARG, "hum_create: n_lanes must be > 0");
    if (cfg->block_size <= 0 || cfg->block_size > 256 || cfg->block_size % 16)
        return fail(HUM_ERR_ARG, "hum_create: block_size must be a multiple of 16 in [16, 256]");
    if (cfg->precision != 0 && cfg->precision != 1) return fail(HUM_ERR_ARG, "hum_create: precision must be 0 or 1");
    if (cfg->substeps <= 0 || cfg->solver_iters < 0) return fail(HUM_ERR_ARG, "hum_create: bad solver settings");
    if (cfg->kernel != 0 && cfg->kernel != 1) return fail(HUM_ERR_ARG, "hum_create: kernel must be 0 (per-lane) or 1 (cooperative)");
    if (cfg->hier != 0 && cfg->hier != 1) return fail(HUM_ERR_ARG, "hum_create: hier must be 0 or 1");
    if (cfg->envs_per_block != 1 && cfg->envs_per_block != 2 && cfg->envs_per_block != 4)
        return fail(HUM_ERR_ARG, "hum_create: envs_per_block must be 1, 2 or 4");
    if (cfg->max_contacts < 0 || cfg->max_contacts > (cfg->kernel == 1 ? MAXC_G : MAXC))
        return fail(HUM_ERR_ARG, "hum_create: max_contacts out of range for the selected kernel");
    HIPCHK(hipSetDevice(cfg->device));
    hum_env* e = new hum_env();
    e->cfg = *cfg;
    e->n = cfg->n_lanes;
    e->real_size = cfg->precision ? sizeof(double) : sizeof(float);
    const size_t n = (size_t)e->n;
    hipError_t st = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (st == hipSuccess) st = hipMalloc(&e->d.phys, HUM_NSTATE * n * e->real_size);
    if (st == hipSuccess) st = hipMalloc((void**)&e->d.bi, NBOOK_I * n * sizeof(int));
    if (st == hipSuccess) st = hipMalloc((void**)&e->d.bd, NBOOK_D * n * sizeof(double));
    if (st == hipSuccess)   // per-lane rows (kernel 0) or the per-env row spill region (kernel 1)
        // (cooperative kernel: per-block regions, so round the lane count up to a multiple of 4 envs)
        st = hipMalloc(&e->d.scratch, (size_t)(cfg->kernel == 1 ? GROW_PER_ENV * ((n + 3) / 4 * 4) : SCRATCH_PER_LANE * n) * e->real_size);
    if (st == hipSuccess) st = hipMalloc((void**)&e->eflags, sizeof(unsigned));
    if (st == hipSuccess) st = hipMalloc((void**)&e->clips_dev, HUM_MAX_CLIPS * sizeof(ClipDev));
    if (st == hipSuccess) st = hipMemset(e->clips_dev, 0, HUM_MAX_CLIPS * sizeof(ClipDev));
    if (st == hipSuccess) st = hipMemset(e->d.bi, 0, NBOOK_I * n * sizeof(int));
    if (st == hipSuccess) st = hipMemset(e->d.bd, 0, NBOOK_D * n * sizeof(double));
    if (st == hipSuccess) st = hipMemset(e->d.phys, 0, HUM_NSTATE * n * e->real_size);
    if (st == hipSuccess) st = hipMemset(e->eflags, 0, sizeof(unsigned));
    if (st == hipSuccess) {
        KArgs a = make_args(e);
        hipLaunchKernelGGL(init_kernel, grid_of(e), dim3(e->cfg.block_size), 0, e->stream, a);
        st = hipGetLastError();
        if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    }
    if (st != hipSuccess) {
        std::string m = std::string("hum_create: ") + hipGetErrorString(st);
        hum_destroy(e);
        return fail(HUM_ERR_HIP, m);
    }
    *out = e;
    return HUM_OK;
}

int hum_destroy(hum_env* e) {
    if (!e) return HUM_OK;
    (void)hipSetDevice(e->cfg.device);
    if (e->graph) (void)hipGraphExecDestroy(e->graph);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    (void)hipFree(e->d.phys);
    (void)hipFree(e->d.bi);
    (void)hipFree(e->d.bd);
    (void)hipFree(e->d.scratch);
    (void)hipFree(e->eflags);
    (void)hipFree(e->clips_dev);
    (void)hipFree(e->pred);
    for (int k = 0; k < HUM_MAX_CLIPS; k++) (void)hipFree(e->clip_dev[k]);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return HUM_OK;
}

int hum_set_clip(hum_env* e, int32_t id, const double* pos, int32_t n_pos, const double* vel, int32_t n_vel,
                 const double* rel, int32_t n_rel, const double* ep, int32_t n_ep) {
    if (!e || id < 0 || id >= HUM_MAX_CLIPS || !pos || !vel || !rel || !ep) return fail(HUM_ERR_ARG, "hum_set_clip: bad argument");
    if (n_pos < 8 || n_vel < 1 || n_rel < n_pos || n_ep < n_pos) return fail(HUM_ERR_ARG, "hum_set_clip: inconsistent table sizes");
    HIPCHK(hipSetDevice(e->cfg.device));
    if (e->clip_dev[id]) HIPCHK(hipFree(e->clip_dev[id]));
    const size_t np = (size_t)n_pos * 14, nv = (size_t)n_vel * 14, nr = (size_t)n_rel * 14, ne = (size_t)n_ep * 27;
    double* buf;
    HIPCHK(hipMalloc((void**)&buf, (np + nv + nr + ne) * sizeof(double)));
    HIPCHK(hipMemcpy(buf, pos, np * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(buf + np, vel, nv * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(buf + np + nv, rel, nr * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(buf + np + nv + nr, ep, ne * sizeof(double), hipMemcpyHostToDevice));
    e->clip_dev[id] = buf;
    e->clips[id] = ClipDev{buf, buf + np, buf + np + nv, buf + np + nv + nr, n_pos, n_vel, n_rel, n_ep, n_pos - 1};
    e->clip_set[id] = true;
    HIPCHK(hipMemcpy(e->clips_dev + id, &e->clips[id], sizeof(ClipDev), hipMemcpyHostToDevice));
    return HUM_OK;
}

int hum_set_lane_clips(hum_env* e, const int32_t* clip_of_lane) {
    if (!e || !clip_of_lane) return fail(HUM_ERR_ARG, "hum_set_lane_clips: null argument");
    for (int i = 0; i < e->n; i++)
        if (clip_of_lane[i] < 0 || clip_of_lane[i] >= HUM_MAX_CLIPS || !e->clip_set[clip_of_lane[i]])
            return fail(HUM_ERR_NOCLIP, "hum_set_lane_clips: lane refers to a clip that was not uploaded");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipMemcpy(e->d.bi + 3 * e->n, clip_of_lane, e->n * sizeof(int), hipMemcpyHostToDevice));
    return HUM_OK;
}

int hum_set_lane_modes(hum_env* e, const uint32_t* modes) {
    if (!e || !modes) return fail(HUM_ERR_ARG, "hum_set_lane_modes: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipMemcpy(e->d.bi + 5 * e->n, modes, e->n * sizeof(int), hipMemcpyHostToDevice));
    return HUM_OK;
}

int hum_set_predefined_targets(hum_env* e, const double* xyz, int32_t n) {
    if (!e || (n > 0 && !xyz) || n < 0) return fail(HUM_ERR_ARG, "hum_set_predefined_targets: bad argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    if (e->pred) HIPCHK(hipFree(e->pred));
    e->pred = nullptr;
    e->npred = n;
    if (n > 0) {
        HIPCHK(hipMalloc((void**)&e->pred, n * 3 * sizeof(double)));
        HIPCHK(hipMemcpy(e->pred, xyz, n * 3 * sizeof(double), hipMemcpyHostToDevice));
    }
    return HUM_OK;
}

int hum_reset(hum_env* e, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
              float* obs_out, void* stream) {
    if (!e) return fail(HUM_ERR_ARG, "hum_reset: null env");
    if (e->cfg.hier) return fail(HUM_ERR_STATE, "hum_reset: hierarchical handle (use hum_hier_reset)");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_reset: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.mask = lane_mask;
    a.start_frame = start_frame;
    a.reset_yaw = reset_yaw_deg;
    a.obs = obs_out;
    hipStream_t s = stream_of(e, stream);
    if (e->cfg.precision) hipLaunchKernelGGL(reset_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    else hipLaunchKernelGGL(reset_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    HIPCHK(hipGetLastError());
    return HUM_OK;
}

int hum_step(hum_env* e, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
             uint32_t flags, float* obs_reset, void* stream) {
    if (!e || !actions || !obs || !reward || !done) return fail(HUM_ERR_ARG, "hum_step: null argument");
    if (e->cfg.hier) return fail(HUM_ERR_STATE, "hum_step: hierarchical handle (use hum_hier_step)");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_step: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.act = actions;
    a.obs = obs;
    a.rew = reward;
    a.done = done;
    a.frame_out = frame;
    a.flags = flags;
    a.obs_reset = obs_reset;
    return launch_step(e, a, stream_of(e, stream));
}

int hum_hier_reset(hum_env* e, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
                   float* high_obs_out, void* stream) {
    if (!e) return fail(HUM_ERR_ARG, "hum_hier_reset: null env");
    if (!e->cfg.hier) return fail(HUM_ERR_STATE, "hum_hier_reset: handle was not created with hier = 1");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_hier_reset: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.mask = lane_mask;
    a.start_frame = start_frame;
    a.reset_yaw = reset_yaw_deg;
    a.obs_high = high_obs_out;
    hipStream_t s = stream_of(e, stream);
    if (e->cfg.precision) hipLaunchKernelGGL(reset_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    else hipLaunchKernelGGL(reset_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    HIPCHK(hipGetLastError());
    return HUM_OK;
}

int hum_hier_step(hum_env* e, const float* high_act, const float* low_act, const uint8_t* agent, uint8_t* agents,
                  float* high_obs, float* low_obs, float* high_rew, float* low_rew, uint8_t* done, int32_t* frame,
                  uint32_t flags, float* high_obs_reset, void* stream) {
    if (!e || !high_act || !low_act || !agents || !high_obs || !low_obs || !high_rew || !low_rew || !done)
        return fail(HUM_ERR_ARG, "hum_hier_step: null argument");
    if (!e->cfg.hier) return fail(HUM_ERR_STATE, "hum_hier_step: handle was not created with hier = 1");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_hier_step: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.act = low_act;
    a.act_high = high_act;
    a.agent_sel = agent;
    a.agents = agents;
    a.obs = low_obs;
    a.obs_high = high_obs;
    a.rew = low_rew;
    a.rew_high = high_rew;
    a.done = done;
    a.frame_out = frame;
    a.flags = flags;
    a.obs_high_reset = high_obs_reset;
    return launch_step(e, a, stream_of(e, stream));
}

}  // extern "C"

namespace {
int launch_step(hum_env* e, const KArgs& a, hipStream_t s) {
#ifdef HUM_DIAG_F32_ONLY   // diagnostic builds (phase timing): only the benchmarked kernel is instantiated
    if (e->cfg.kernel != 1 || e->cfg.precision || e->cfg.envs_per_block != 4)
        return fail(HUM_ERR_ARG, "diagnostic build: only kernel 1, fp32, envs_per_block 4");
    hipLaunchKernelGGL((step_group_kernel<float, 4>), dim3((e->n + 3) / 4), dim3(4 * GL), 0, s, a);
#else
    if (e->cfg.kernel == 1) {
        const int epb = e->cfg.envs_per_block;
        const dim3 g((e->n + epb - 1) / epb), blk(epb * GL);
        if (e->cfg.precision) {
            if (epb == 4) hipLaunchKernelGGL((step_group_kernel<double, 4>), g, blk, 0, s, a);
            else if (epb == 2) hipLaunchKernelGGL((step_group_kernel<double, 2>), g, blk, 0, s, a);
            else hipLaunchKernelGGL((step_group_kernel<double, 1>), g, blk, 0, s, a);
        } else {
            if (epb == 4) hipLaunchKernelGGL((step_group_kernel<float, 4>), g, blk, 0, s, a);
            else if (epb == 2) hipLaunchKernelGGL((step_group_kernel<float, 2>), g, blk, 0, s, a);
            else hipLaunchKernelGGL((step_group_kernel<float, 1>), g, blk, 0, s, a);
        }
    } else {
        if (e->cfg.precision) hipLaunchKernelGGL(step_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
        else hipLaunchKernelGGL(step_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    }
#endif
    HIPCHK(hipGetLastError());
    return HUM_OK;
}
}  // namespace

extern "C" {

int hum_step_graph(hum_env* e, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
                   uint32_t flags, float* obs_reset, int32_t k) {
    if (!e || k <= 0) return fail(HUM_ERR_ARG, "hum_step_graph: bad argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    const void* key[6] = {actions, obs, reward, done, frame, obs_reset};
    bool same = e->graph && e->graph_k == k && e->graph_flags == flags && memcmp(key, e->graph_key, sizeof key) == 0;
    if (!same) {
        if (e->graph) { (void)hipGraphExecDestroy(e->graph); e->graph = nullptr; }
        hipGraph_t g;
        HIPCHK(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
        for (int t = 0; t < k; t++) {
            int r = hum_step(e, actions, obs, reward, done, frame, flags, obs_reset, e->stream);
            if (r != HUM_OK) {
                (void)hipStreamEndCapture(e->stream, &g);
                return r;
            }
        }
        HIPCHK(hipStreamEndCapture(e->stream, &g));
        HIPCHK(hipGraphInstantiate(&e->graph, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
        e->graph_k = k;
        e->graph_flags = flags;
        memcpy(e->graph_key, key, sizeof key);
    }
    HIPCHK(hipGraphLaunch(e->graph, e->stream));
    return HUM_OK;
}

int hum_get_aux(hum_env* e, float* aux_out, void* stream) {
    if (!e || !aux_out) return fail(HUM_ERR_ARG, "hum_get_aux: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.aux = aux_out;
    hipStream_t s = stream_of(e, stream);
    if (e->cfg.precision) hipLaunchKernelGGL(aux_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    else hipLaunchKernelGGL(aux_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    HIPCHK(hipGetLastError());
    return HUM_OK;
}

int hum_get_state(hum_env* e, double* phys, double* book) {
    if (!e) return fail(HUM_ERR_ARG, "hum_get_state: null env");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    const size_t n = e->n;
    if (phys) {
        std::vector<unsigned char> tmp(HUM_NSTATE * n * e->real_size);
        HIPCHK(hipMemcpy(tmp.data(), e->d.phys, tmp.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++)
            for (int k = 0; k < HUM_NSTATE; k++)
                phys[i * HUM_NSTATE + k] = e->cfg.precision ? ((double*)tmp.data())[k * n + i] : (double)((float*)tmp.data())[k * n + i];
    }
    if (book) {
        std::vector<int> bi(NBOOK_I * n);
        std::vector<double> bd(NBOOK_D * n);
        HIPCHK(hipMemcpy(bi.data(), e->d.bi, bi.size() * sizeof(int), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(bd.data(), e->d.bd, bd.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++) {
            double* o = book + i * HUM_NBOOK;
            memset(o, 0, HUM_NBOOK * sizeof(double));
            o[HUM_BK_FRAME] = bi[0 * n + i];
            o[HUM_BK_TIMESTEP] = bi[1 * n + i];
            o[HUM_BK_PRED_INDEX] = bi[2 * n + i];
            o[HUM_BK_CLIP] = bi[3 * n + i];
            o[HUM_BK_RNG_COUNTER] = (double)(unsigned)bi[4 * n + i];
            o[HUM_BK_MODE] = (double)(unsigned)bi[5 * n + i];
            o[HUM_BK_RNG_KEY_LO] = (double)(unsigned)bi[6 * n + i];
            o[HUM_BK_RNG_KEY_HI] = (double)(unsigned)bi[7 * n + i];
            for (int k = 0; k < 3; k++) {
                o[HUM_BK_TARGET + k] = bd[(0 + k) * n + i];
                o[HUM_BK_START_ROBOT_POS + k] = bd[(3 + k) * n + i];
                o[HUM_BK_ROBOT_POS + k] = bd[(6 + k) * n + i];
                o[HUM_BK_START_EP_POS + k] = bd[(9 + k) * n + i];
            }
            o[HUM_BK_HL_DEG_TARGET] = bd[12 * n + i];
            o[HUM_BK_WALK_TARGET] = bd[13 * n + i];
            o[HUM_BK_WALK_TARGET + 1] = bd[14 * n + i];
            o[HUM_BK_LOW_TARGET_SCORE] = bd[15 * n + i];
            o[HUM_BK_DELTA_JOINTS] = bd[16 * n + i];
            o[HUM_BK_DELTA_VEL_JOINTS] = bd[17 * n + i];
            o[HUM_BK_BODY_POSTURE] = bd[18 * n + i];
            o[HUM_BK_ELECTRICITY] = bd[19 * n + i];
            o[HUM_BK_JOINT_LIMIT] = bd[20 * n + i];
            o[HUM_BK_ALIVE] = bd[21 * n + i];
            o[HUM_BK_DELTA_LOW_TARGET] = bd[22 * n + i];
            o[HUM_BK_LEVEL_REMAINING] = bi[8 * n + i];
            o[HUM_BK_NUM_HIGH_STEPS] = bi[9 * n + i];
            o[HUM_BK_EXPECT_HIGH] = bi[10 * n + i];
            o[HUM_BK_HIGH_TARGET_SCORE] = bd[23 * n + i];
            o[HUM_BK_CUM_DRIFT] = bd[24 * n + i];
            o[HUM_BK_DRIFT] = bd[25 * n + i];
            o[HUM_BK_DELTA_HIGH_TARGET] = bd[26 * n + i];
            o[HUM_BK_CUM_ALIVE] = bd[27 * n + i];
            o[HUM_BK_BODY_XY] = bd[28 * n + i];
            o[HUM_BK_BODY_XY + 1] = bd[29 * n + i];
        }
    }
    return HUM_OK;
}

int hum_set_state(hum_env* e, const double* phys, const double* book) {
    if (!e) return fail(HUM_ERR_ARG, "hum_set_state: null env");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    const size_t n = e->n;
    if (phys) {
        std::vector<unsigned char> tmp(HUM_NSTATE * n * e->real_size);
        for (size_t i = 0; i < n; i++)
            for (int k = 0; k < HUM_NSTATE; k++) {
                if (e->cfg.precision) ((double*)tmp.data())[k * n + i] = phys[i * HUM_NSTATE + k];
                else ((float*)tmp.data())[k * n + i] = (float)phys[i * HUM_NSTATE + k];
            }
        HIPCHK(hipMemcpy(e->d.phys, tmp.data(), tmp.size(), hipMemcpyHostToDevice));
    }
    if (book) {
        std::vector<int> bi(NBOOK_I * n);
        std::vector<double> bd(NBOOK_D * n);
        for (size_t i = 0; i < n; i++) {
            const double* o = book + i * HUM_NBOOK;
            const int clip = (int)o[HUM_BK_CLIP];
            if (clip < 0 || clip >= HUM_MAX_CLIPS || !e->clip_set[clip])
                return fail(HUM_ERR_NOCLIP, "hum_set_state: lane clip id not uploaded");
            bi[0 * n + i] = (int)o[HUM_BK_FRAME];
            bi[1 * n + i] = (int)o[HUM_BK_TIMESTEP];
            bi[2 * n + i] = (int)o[HUM_BK_PRED_INDEX];
            bi[3 * n + i] = clip;
            bi[4 * n + i] = (int)(unsigned)o[HUM_BK_RNG_COUNTER];
            bi[5 * n + i] = (int)(unsigned)o[HUM_BK_MODE];
            bi[6 * n + i] = (int)(unsigned)o[HUM_BK_RNG_KEY_LO];
            bi[7 * n + i] = (int)(unsigned)o[HUM_BK_RNG_KEY_HI];
            for (int k = 0; k < 3; k++) {
                bd[(0 + k) * n + i] = o[HUM_BK_TARGET + k];
                bd[(3 + k) * n + i] = o[HUM_BK_START_ROBOT_POS + k];
                bd[(6 + k) * n + i] = o[HUM_BK_ROBOT_POS + k];
                bd[(9 + k) * n + i] = o[HUM_BK_START_EP_POS + k];
            }
            bd[12 * n + i] = o[HUM_BK_HL_DEG_TARGET];
            bd[13 * n + i] = o[HUM_BK_WALK_TARGET];
            bd[14 * n + i] = o[HUM_BK_WALK_TARGET + 1];
            bd[15 * n + i] = o[HUM_BK_LOW_TARGET_SCORE];
            bd[16 * n + i] = o[HUM_BK_DELTA_JOINTS];
            bd[17 * n + i] = o[HUM_BK_DELTA_VEL_JOINTS];
            bd[18 * n + i] = o[HUM_BK_BODY_POSTURE];
            bd[19 * n + i] = o[HUM_BK_ELECTRICITY];
            bd[20 * n + i] = o[HUM_BK_JOINT_LIMIT];
            bd[21 * n + i] = o[HUM_BK_ALIVE];
            bd[22 * n + i] = o[HUM_BK_DELTA_LOW_TARGET];
            bi[8 * n + i] = (int)o[HUM_BK_LEVEL_REMAINING];
            bi[9 * n + i] = (int)o[HUM_BK_NUM_HIGH_STEPS];
            bi[10 * n + i] = (int)o[HUM_BK_EXPECT_HIGH];
            bd[23 * n + i] = o[HUM_BK_HIGH_TARGET_SCORE];
            bd[24 * n + i] = o[HUM_BK_CUM_DRIFT];
            bd[25 * n + i] = o[HUM_BK_DRIFT];
            bd[26 * n + i] = o[HUM_BK_DELTA_HIGH_TARGET];
            bd[27 * n + i] = o[HUM_BK_CUM_ALIVE];
            bd[28 * n + i] = o[HUM_BK_BODY_XY];
            bd[29 * n + i] = o[HUM_BK_BODY_XY + 1];
        }
        HIPCHK(hipMemcpy(e->d.bi, bi.data(), bi.size() * sizeof(int), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->d.bd, bd.data(), bd.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    return HUM_OK;
}

int hum_get_parts(hum_env* e, double* parts) {
    if (!e || !parts) return fail(HUM_ERR_ARG, "hum_get_parts: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    double* d;
    const size_t bytes = (size_t)e->n * NPART * 3 * sizeof(double);
    HIPCHK(hipMalloc((void**)&d, bytes));
    KArgs a = make_args(e);
    HIPCHK(hipDeviceSynchronize());
    if (e->cfg.precision) hipLaunchKernelGGL(parts_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, e->stream, a, d);
    else hipLaunchKernelGGL(parts_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, e->stream, a, d);
    hipError_t st = hipGetLastError();
    if (st == hipSuccess) st = hipDeviceSynchronize();
    if (st == hipSuccess) st = hipMemcpy(parts, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (st != hipSuccess) return fail(HUM_ERR_HIP, std::string("hum_get_parts: ") + hipGetErrorString(st));
    return HUM_OK;
}

int hum_get_error_flags(hum_env* e, uint32_t* flags) {
    if (!e || !flags) return fail(HUM_ERR_ARG, "hum_get_error_flags: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    unsigned v = 0;
    HIPCHK(hipMemcpy(&v, e->eflags, sizeof v, hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(e->eflags, 0, sizeof v));
    *flags = v;
    return HUM_OK;
}

int hum_sync(hum_env* e) {
    if (!e) return fail(HUM_ERR_ARG, "hum_sync: null env");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    return HUM_OK;
}

int32_t hum_num_lanes(const hum_env* e) { return e ? e->n : 0; }

#ifdef HUM_PHASE_TIMING
// diagnostic builds only: accumulated s_memtime cycles per cooperative-kernel phase (thread 0 of each block)
int hum_debug_phase_cycles(unsigned long long* out16, int reset) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_phase_cycles), 16 * sizeof(unsigned long long)));
    if (reset) {
        unsigned long long z[16] = {0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof z));
    }
    return HUM_OK;
}
#endif
void* hum_stream(hum_env* e) { return e ? (void*)e->stream : nullptr; }

}  // extern "C"

// envlogic.h - LowLevelHumanoidEnv reset/step bookkeeping, observation and imitation reward (device).
//
// Restates /root/reference/low_level_env.py (line numbers per function) and the pybullet_envs
// WalkerBase.calc_state transform, in float64 with the reference's operation order (numpy pairwise
// means, float32 observation block, OpenBLAS ddot for 3-vector norms), so that done / frame / target
// decisions are bit-identical to the reference given identical physics state.  fp-contraction is off
// in this file: numpy never fuses a*b+c.
#pragma once
#include "model_gen.h"
#include "physics.h"

#pragma clang fp contract(off)

namespace hk {

constexpr double DT_ENV = 0.0165;
constexpr double DEG2RAD = 0.017453292519943295;   // NPY_PI/180 (np.deg2rad)
constexpr double RAD2DEG = 57.29577951308232;      // 180/NPY_PI (np.rad2deg)
constexpr double JOINT_WEIGHT_SUM = 17.400000000000006;      // sum(joint_weight.values()), :119
constexpr double JOINT_VEL_WEIGHT_SUM = 8.599999999999998;   // sum(joint_vel_weight.values()), :137
constexpr int NREF = 14;

// joint_map (low_level_env.py:86-101) in dict order: (dof index, CSV column index, weight, vel weight)
// CSV columns: rightHipX 0, rightHipY 1, rightHipZ 2, rightKnee 3, leftHipX 4, leftHipY 5, leftHipZ 6,
// leftKnee 7, rightShoulderX 8, rightShoulderY 9, rightElbow 10, leftShoulderX 11, leftShoulderY 12, leftElbow 13
constexpr int JM_DOF[NREF] = {6, 3, 5, 4, 10, 7, 9, 8, 12, 11, 13, 15, 14, 16};
constexpr int JM_COL[NREF] = {3, 0, 1, 2, 7, 4, 5, 6, 8, 9, 10, 11, 12, 13};
constexpr double JM_W[NREF] = {3, 1, 3, 1, 3, 1, 3, 1, 0.1, 0.3, 0.3, 0.1, 0.3, 0.3};
constexpr double JM_WV[NREF] = {1, 1, 1, 1, 1, 1, 1, 1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1};
constexpr double REWARD_W[7] = {0.34, 0.1, 0.34, 0.034, 0.15, 0.034, 0.1};   // :507
// end-point table columns (X of each triple): LeftLeg 0, LeftFoot 3, RightLeg 6, RightFoot 9
constexpr int EP_RIGHT_LEG = 6, EP_RIGHT_FOOT = 9;
constexpr int PART_RIGHT_FOOT = 12;   // index of 'right_foot' in the pybullet parts order

#define HUM_GLOBAL __attribute__((address_space(1)))
// LDS, explicitly: a value read from either LDS or global memory goes through two address-space-typed loads, never
// one load through a generic pointer (a flat access; DESIGN.md section 4, the MachineLICM fault)
#define HUM_LDS __attribute__((address_space(3)))
struct ClipDev {
    const double* pos; const double* vel; const double* rel; const double* ep;
    int n_pos, n_vel, n_rel, n_ep, max_frame;
    // the tables as global-address-space pointers: loaded from a device struct, the plain pointers are generic, and
    // generic (flat) loads also count against the LDS counter, so every LDS wait nearby waited for the table fetches
    __device__ const HUM_GLOBAL double* gpos() const { return (const HUM_GLOBAL double*)pos; }
    __device__ const HUM_GLOBAL double* gvel() const { return (const HUM_GLOBAL double*)vel; }
    __device__ const HUM_GLOBAL double* grel() const { return (const HUM_GLOBAL double*)rel; }
    __device__ const HUM_GLOBAL double* gep() const { return (const HUM_GLOBAL double*)ep; }
};

struct Book {   // per-lane bookkeeping (mirrors HUM_BK_* in include/humanoid_env.h)
    int frame, timestep, pred_idx, clip;
    unsigned rng_ctr, mode;
    unsigned long long rng_key;
    unsigned long long terrain_key;   // HUM_TERRAIN_RANDOM_BLOCKS: the lane's current terrain
    double target[3], srp[3], robot_pos[3], sep[3];
    double hldt, wt[2], lts;
    double dj, dvj, bps, es, jls, alive, dlts;
    // hierarchical env (hier_env.py): level counter, agent expected next, high-level scores, body_xyz[0:2]
    int level_rem, n_high, expect_high;
    double hts, cum_drift, drift, dhts, cum_alive, bxy[2];
};

// --------------------------------------------------------------------------------------- helpers
__device__ inline double norm3_blas(double x0, double x1, double x2) {   // np.linalg.norm (OpenBLAS ddot)
    return sqrt(fma(x2, x2, fma(x1, x1, x0 * x0)));
}

// numpy pairwise summation (8 accumulators) for n in [8, 128]
template <int N, typename F>
__device__ inline double pairwise_sum(F at) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = at(j);
    int i = 8;
#pragma unroll
    for (; i < N - (N % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] = r[j] + at(i + j);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (; i < N; i++) res = res + at(i);
    return res;
}
template <int N, typename F>
__device__ inline float pairwise_sum_f(F at) {
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = at(j);
    int i = 8;
#pragma unroll
    for (; i < N - (N % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] = r[j] + at(i + j);
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (; i < N; i++) res = res + at(i);
    return res;
}

__device__ inline void euler_from_quat(const double* q, double& roll, double& pitch, double& yaw) {
    // pybullet getEulerFromQuaternion
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double squ = w * w, sqx = x * x, sqy = y * y, sqz = z * z;
    roll = atan2(2 * (y * z + w * x), squ - sqx - sqy + sqz);
    const double sarg = -2 * (x * z - w * y);
    pitch = sarg <= -1.0 ? -0.5 * 3.141592538 : (sarg >= 1.0 ? 0.5 * 3.141592538 : asin(sarg));
    yaw = atan2(2 * (x * y + w * z), squ + sqx - sqy - sqz);
}

__device__ inline unsigned long long splitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// counter-based lane draw in [lo, hi) (oracle/oracle.py::lane_draw); key = splitmix64(seed + lane)
__device__ inline int lane_draw_key(unsigned long long key, unsigned ctr, int lo, int hi) {
    unsigned long long x = splitmix64(key + ctr);
    return lo + (int)(((x >> 32) * (unsigned long long)(hi - lo)) >> 32);
}

template <typename T>
struct PostPhys {   // physics-derived quantities calc_state reads (pybullet getters)
    double q[NDOF], qd[NDOF];
    double bx, by, bz;          // body_xyz
    double roll, pitch, yaw;
    double lin[3];
    double rfoot[2];            // world x, y of the right foot part (resetFromFrame's starting_ep_pos)
};

// WalkerBase.calc_state (pybullet_envs/robot_locomotors.py) -> 42 float32 + side effects
// calc_state's joint block for one dof: obs 8 + 2d (relative position) and 9 + 2d (speed) before the observation clamp,
// and whether the joint counts as at its limit (the cooperative kernel computes the 17 dofs on 17 lanes)
template <typename T>
__device__ inline bool joint_obs(const T* st, int d, float& rp, float& rv) {
    const double q = (double)st[13 + d], qd = (double)st[30 + d];
    const double lo = dof_lo[d], hi = dof_hi[d];
    const double mid = 0.5 * (lo + hi);
    rp = (float)(2 * (q - mid) / (hi - lo));
    rv = (float)(qd * 0.1);
    return fabsf(rp) > 0.99f;
}

// joints = false: the joint block (obs 8..41, joint_speeds, joints_at_limit) is left to the caller (joint_obs per dof)
template <typename T>
__device__ inline void calc_state(const T* st, const double* wt, float* obs42, float* joint_speeds, int& joints_at_limit,
                                  PostPhys<T>& pp, const T* scs = nullptr, bool joints = true) {
    Kin<T> K;
    if (scs) forward_kinematics_pre(st + 3, scs, K);   // hinge sin / cos of this state precomputed across lanes
    else forward_kinematics(st + 3, st + 13, K);
    T parts[NPART][3];
    part_positions(K, parts);
    const double bpx = (double)st[0], bpy = (double)st[1];
    // world part positions in float64 (pybullet returns doubles); floor at the origin
    pp.bx = pairwise_sum<NPART>([&](int k) -> double { return part_body[k] < 0 ? 0.0 : bpx + (double)parts[k][0]; }) / NPART;
    pp.by = pairwise_sum<NPART>([&](int k) -> double { return part_body[k] < 0 ? 0.0 : bpy + (double)parts[k][1]; }) / NPART;
    pp.bz = (double)st[2];
    pp.rfoot[0] = bpx + (double)parts[PART_RIGHT_FOOT][0];
    pp.rfoot[1] = bpy + (double)parts[PART_RIGHT_FOOT][1];
    double qd4[4] = {(double)st[3], (double)st[4], (double)st[5], (double)st[6]};
    euler_from_quat(qd4, pp.roll, pp.pitch, pp.yaw);
    if (joints) joints_at_limit = 0;
#pragma unroll
    for (int i = 0; i < NDOF; i++) {
        pp.q[i] = (double)st[13 + i];
        pp.qd[i] = (double)st[30 + i];
        if (joints) {
            float rp, rv;
            if (joint_obs(st, i, rp, rv)) joints_at_limit++;
            obs42[8 + 2 * i] = rp;
            obs42[9 + 2 * i] = rv;
            joint_speeds[i] = rv;
        }
    }
#pragma unroll
    for (int i = 0; i < 3; i++) pp.lin[i] = (double)st[7 + i];
    const double theta = atan2(wt[1] - pp.by, wt[0] - pp.bx);
    const double angle = theta - pp.yaw;
    const double cy = cos(-pp.yaw), sy = sin(-pp.yaw);
    const double vx = cy * pp.lin[0] + (-sy) * pp.lin[1] + 0.0 * pp.lin[2];
    const double vy = sy * pp.lin[0] + cy * pp.lin[1] + 0.0 * pp.lin[2];
    const double vz = 0.0 * pp.lin[0] + 0.0 * pp.lin[1] + 1.0 * pp.lin[2];
    obs42[0] = (float)(pp.bz - 0.8);
    obs42[1] = (float)sin(angle);
    obs42[2] = (float)cos(angle);
    obs42[3] = (float)(0.3 * vx);
    obs42[4] = (float)(0.3 * vy);
    obs42[5] = (float)(0.3 * vz);
    obs42[6] = (float)pp.roll;
    obs42[7] = (float)pp.pitch;
#pragma unroll
    for (int i = 0; i < (joints ? 42 : 8); i++) obs42[i] = fminf(fmaxf(obs42[i], -5.0f), 5.0f);
}

// getLowLevelObs tail (low_level_env.py:307-320): 14 x (relative target, target velocity) at `frame`
__device__ inline void ref_obs(const ClipDev& c, int frame, float* out28, unsigned& eflags) {
    int vrow = frame;
    if (vrow >= c.n_vel) { vrow = c.n_vel - 1; eflags |= 2u; }   // HUM_EFLAG_VEL_ROW (motion13_13)
#pragma unroll
    for (int j = 0; j < NREF; j++) {
        out28[2 * j] = (float)c.grel()[frame * 14 + JM_COL[j]];
        out28[2 * j + 1] = (float)c.gvel()[vrow * 14 + JM_COL[j]];
    }
}

__device__ inline void inc_frame(Book& b, const ClipDev& c, int inc) {   // :218-222
    b.frame = (b.frame + inc) % (c.max_frame - 1);
    if (b.frame == 0) {
        b.sep[0] = b.robot_pos[0]; b.sep[1] = b.robot_pos[1]; b.sep[2] = b.robot_pos[2];
    }
}

__device__ inline double dot3_blas(double x0, double x1, double x2, double y0, double y1, double y2) {   // np.dot
    return fma(x2, y2, fma(x1, y1, x0 * y0));
}

__device__ inline void set_walk_target_hl(Book& b) {   // tail of checkTarget (:431-434)
    const double v0 = b.target[0] - b.robot_pos[0], v1 = b.target[1] - b.robot_pos[1];
    b.hldt = atan2(v1, v0);
    b.wt[0] = b.robot_pos[0] + cos(b.hldt) * 10;
    b.wt[1] = b.robot_pos[1] + sin(b.hldt) * 10;
}

}  // namespace hk

#pragma clang fp contract(on)

/* ORACLE - test infrastructure only.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it (as the checker / the CPU baseline), never the product path.
 *
 * Plain-C restatement of the single-lane oracle env `oracle/oracle.py::OracleLowLevelEnv` (which restates
 * LowLevelHumanoidEnv.reset()/step(), /root/reference/low_level_env.py:224-526) on top of the fp64 physics
 * restatement (physics_oracle.c).  Same operation order as the Python oracle: numpy pairwise sums for the
 * 33-part body_xyz means and the float32 electricity means, OpenBLAS-ddot style 3-vector norms, float32
 * observation block.  Its purpose is the CPU baseline SURVEY.md 8(d) plans ("the build's C++ CPU
 * restatement with OpenMP over all host cores"): oe_bench steps independent lanes on every host thread.
 * Parity against the Python oracle (and through it the reference's golden vectors) is tests/test_env_oracle_c.py.
 *
 * Clip tables come in the product's fixed column order (ilrl_amd.clips.JOINT_COLS / EP_COLS); the joint map and
 * motor gains come from oracle.py (the names live there), packed in oe_model.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "humanoid_links_gen.h"
#include "physics_oracle.h"

#define OE_NREF 14
#define OE_NOBS 70

typedef struct {
    int jm_dof[OE_NREF], jm_col[OE_NREF];   /* joint_map (low_level_env.py:86-101) in dict order */
    double jm_w[OE_NREF], jm_wv[OE_NREF];   /* joint_weight / joint_vel_weight */
    int motor_dof[17];                      /* CustomHumanoidRobot motor order -> dof (humanoid.py:28-37) */
    double motor_power[17];
    int ep_right_leg, ep_right_foot;        /* X column of RightLeg / RightFoot in the end-point table */
    int part_right_foot;                    /* index of 'right_foot' among the 33 parts */
    int numpy_semantics;                    /* 1: NumPy 1.x promotion (default), 2: NEP 50 */
} oe_model;

typedef struct {
    const double *pos, *vel, *rel, *ep;     /* [n][14] x3, [n_ep][27] */
    int n_pos, n_vel, n_rel, n_ep;
} oe_clip;

typedef struct {
    double st[47];
    int frame, cur_timestep, max_frame;
    uint64_t key;
    uint64_t ctr;
    double target[3], srp[3], robot_pos[3], sep[3], wt[2], hldt;
    double lts, dj, dvj, bps, es, jls, alive, dlts;
    float cur_obs[42], joint_speeds[17];
    int jal;
    double bx, by;
} oe_env;

/* ------------------------------------------------------------------------------------------ helpers */
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static int draw(oe_env* e, int lo, int hi) {   /* oracle.py::key_draw (Lemire map of the high 32 bits) */
    uint64_t x = splitmix64(e->key + e->ctr++);
    return lo + (int)(((x >> 32) * (uint64_t)(hi - lo)) >> 32);
}
static double norm3(double x0, double x1, double x2) { return sqrt(fma(x2, x2, fma(x1, x1, x0 * x0))); }
static double pairwise33(const double* v, int stride) {   /* numpy pairwise sum, n = 33 */
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = v[j * stride];
    int i = 8;
    for (; i < 32; i += 8)
        for (int j = 0; j < 8; j++) r[j] = r[j] + v[(i + j) * stride];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < 33; i++) res = res + v[i * stride];
    return res;
}
static float pairwise17f(const float* v) {   /* numpy float32 pairwise sum, n = 17 */
    float r[8];
    for (int j = 0; j < 8; j++) r[j] = v[j];
    for (int j = 0; j < 8; j++) r[j] = r[j] + v[8 + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    return res + v[16];
}
static const double DEG2RAD = 0.017453292519943295, RAD2DEG = 57.29577951308232;

static void euler(const double* q, double* roll, double* pitch, double* yaw) {   /* getEulerFromQuaternion */
    double x = q[0], y = q[1], z = q[2], w = q[3];
    double squ = w * w, sqx = x * x, sqy = y * y, sqz = z * z;
    *roll = atan2(2 * (y * z + w * x), squ - sqx - sqy + sqz);
    double sarg = -2 * (x * z - w * y);
    *pitch = sarg <= -1.0 ? -0.5 * 3.141592538 : (sarg >= 1.0 ? 0.5 * 3.141592538 : asin(sarg));
    *yaw = atan2(2 * (x * y + w * z), squ + sqx - sqy - sqz);
}

/* oracle.py::calc_state (WalkerBase.calc_state, foot_list = []) */
static void calc_state(const oe_model* m, oe_env* e, double* rfoot_xy) {
    double px[OM_NPART * 3];
    om_parts(e->st, px);
    e->bx = pairwise33(px, 3) / 33;
    e->by = pairwise33(px + 1, 3) / 33;
    if (rfoot_xy) { rfoot_xy[0] = px[3 * m->part_right_foot]; rfoot_xy[1] = px[3 * m->part_right_foot + 1]; }
    double r, p, yaw;
    euler(e->st + 3, &r, &p, &yaw);
    float* o = e->cur_obs;
    e->jal = 0;
    for (int i = 0; i < 17; i++) {
        double lo = om_lo[i], hi = om_hi[i], mid = 0.5 * (lo + hi);
        float rp = (float)(2 * (e->st[13 + i] - mid) / (hi - lo));
        float rv = (float)(e->st[30 + i] * 0.1);
        o[8 + 2 * i] = rp;
        o[9 + 2 * i] = rv;
        e->joint_speeds[i] = rv;
        if (fabsf(rp) > 0.99f) e->jal++;
    }
    double theta = atan2(e->wt[1] - e->by, e->wt[0] - e->bx);
    double angle = theta - yaw;
    double cy = cos(-yaw), sy = sin(-yaw);
    const double* v = e->st + 7;
    double vx = cy * v[0] + (-sy) * v[1] + 0.0 * v[2];
    double vy = sy * v[0] + cy * v[1] + 0.0 * v[2];
    double vz = 0.0 * v[0] + 0.0 * v[1] + 1.0 * v[2];
    o[0] = (float)(e->st[2] - 0.8);
    o[1] = (float)sin(angle);
    o[2] = (float)cos(angle);
    o[3] = (float)(0.3 * vx);
    o[4] = (float)(0.3 * vy);
    o[5] = (float)(0.3 * vz);
    o[6] = (float)r;
    o[7] = (float)p;
    for (int i = 0; i < 42; i++) o[i] = fminf(fmaxf(o[i], -5.0f), 5.0f);
}

static void low_level_obs(const oe_model* m, const oe_clip* c, const oe_env* e, double* obs) {   /* :307-320 */
    for (int i = 0; i < 42; i++) obs[i] = e->cur_obs[i];
    int vrow = e->frame < c->n_vel ? e->frame : c->n_vel - 1;   /* motion13_13: see DESIGN.md section 6 */
    for (int j = 0; j < OE_NREF; j++) {
        obs[42 + 2 * j] = c->rel[e->frame * 14 + m->jm_col[j]];
        obs[43 + 2 * j] = c->vel[vrow * 14 + m->jm_col[j]];
    }
}

static void inc_frame(oe_env* e, int inc) {   /* :218-222 */
    e->frame = (e->frame + inc) % (e->max_frame - 1);
    if (e->frame == 0) memcpy(e->sep, e->robot_pos, sizeof e->sep);
}

/* ------------------------------------------------------------------------------------------ entry points */
void oe_init(oe_env* e, const oe_clip* c, uint64_t key) {
    memset(e, 0, sizeof *e);
    e->st[6] = 1.0;
    e->max_frame = c->n_pos - 1;
    e->key = key;
    e->target[0] = 1;
    e->wt[0] = 10.0;
}

/* resetFromFrame(startFrame, resetYaw) with startFromRef = initVel = True; start_frame < 0 = reset() (:224-305) */
void oe_reset(const oe_model* m, const oe_clip* c, oe_env* e, int start_frame, double reset_yaw, double* obs) {
    if (start_frame < 0) start_frame = draw(e, 0, e->max_frame - 5);
    memset(e->st, 0, sizeof e->st);
    e->st[6] = 1.0;
    e->cur_timestep = 0;
    double rr = 0 + draw(e, -180, 180) * DEG2RAD;   /* getRandomVec(5, 0) */
    e->target[0] = cos(rr) * 5;
    e->target[1] = sin(rr) * 5;
    e->target[2] = 0;
    e->frame = start_frame;
    int vrow = start_frame < c->n_vel ? start_frame : c->n_vel - 1;
    for (int j = 0; j < OE_NREF; j++) {   /* setJointsOrientation (abdomen dofs stay 0) */
        e->st[13 + m->jm_dof[j]] = c->pos[start_frame * 14 + m->jm_col[j]];
        e->st[30 + m->jm_dof[j]] = c->vel[vrow * 14 + m->jm_col[j]];
    }
    for (int k = 0; k < 3; k++) { e->robot_pos[k] = 0; e->srp[k] = 0; }
    e->st[2] = 1.17;
    double deg = atan2(e->target[1], e->target[0]) * RAD2DEG;
    e->wt[0] = cos(deg) * 1000;
    e->wt[1] = sin(deg) * 1000;
    double th = (deg + reset_yaw) * DEG2RAD;
    e->st[5] = sin(th / 2);
    e->st[6] = cos(th / 2);
    e->hldt = deg * DEG2RAD;
    /* scipy Rotation.from_euler('z', deg).apply: matrix from the quaternion */
    double qz = sin(e->hldt / 2), qw = cos(e->hldt / 2);
    double r00 = -(qz * qz) + qw * qw, r01 = 2 * (0.0 - qz * qw), r10 = 2 * (0.0 + qz * qw), r11 = r00;
    int f0 = e->frame, f1 = (e->frame + 2) % e->max_frame;
    const double *e0 = c->ep + f0 * 27, *e1 = c->ep + f1 * 27;
    int L = m->ep_right_leg, F = m->ep_right_foot;
    double l0x = r00 * e0[L] + r01 * e0[L + 1], l0y = r10 * e0[L] + r11 * e0[L + 1];
    double l1x = r00 * e1[L] + r01 * e1[L + 1], l1y = r10 * e1[L] + r11 * e1[L + 1];
    e->st[7] = ((l1x - l0x) / 0.0165) / 1.2;
    e->st[8] = ((l1y - l0y) / 0.0165) / 1.2;
    e->st[9] = ((e1[L + 2] - e0[L + 2]) / 0.0165) / 1.2;
    double rf[2];
    calc_state(m, e, rf);
    e->sep[0] = rf[0] - (r00 * e0[F] + r01 * e0[F + 1]);
    e->sep[1] = rf[1] - (r10 * e0[F] + r11 * e0[F + 1]);
    e->sep[2] = 0;
    e->lts = e->dj = e->dvj = e->bps = e->es = e->jls = e->alive = e->dlts = 0;   /* initReward */
    inc_frame(e, 2);
    if (obs) low_level_obs(m, c, e, obs);
}

/* step(action) (:475-526): returns done; obs [70] f64, *reward */
int oe_step(const oe_model* m, const oe_clip* c, const om_params* P, oe_env* e, const float* action, double* obs,
            double* reward) {
    double tau[17] = {0};
    for (int i = 0; i < 17; i++) {   /* apply_action (humanoid.py:54-60) */
        float a = action[i] < -1.0f ? -1.0f : (action[i] > 1.0f ? 1.0f : action[i]);
        tau[m->motor_dof[i]] = m->numpy_semantics == 1 ? 1 * m->motor_power[i] * 0.41 * (double)a
                                                       : (double)((float)(1 * m->motor_power[i] * 0.41) * a);
    }
    om_step(P, e->st, tau, 0);
    calc_state(m, e, 0);
    e->robot_pos[0] = e->bx; e->robot_pos[1] = e->by; e->robot_pos[2] = 0;
    double dJ = 0, dV = 0;
    int vrow = e->frame < c->n_vel ? e->frame : c->n_vel - 1;
    for (int j = 0; j < OE_NREF; j++) dJ = dJ + fabs(e->st[13 + m->jm_dof[j]] - c->pos[e->frame * 14 + m->jm_col[j]]) * m->jm_w[j];
    for (int j = 0; j < OE_NREF; j++) dV = dV + fabs(e->st[30 + m->jm_dof[j]] - c->vel[vrow * 14 + m->jm_col[j]]) * m->jm_wv[j];
    double wsum = 0, wvsum = 0;
    for (int j = 0; j < OE_NREF; j++) { wsum = wsum + m->jm_w[j]; wvsum = wvsum + m->jm_wv[j]; }
    double js = exp(4 * (-dJ / wsum)), jvs = exp((-dV / wvsum) / 2);
    double lowt = -norm3(e->target[0] - e->robot_pos[0], e->target[1] - e->robot_pos[1], e->target[2] - e->robot_pos[2]);
    double r, p, yaw;
    euler(e->st + 3, &r, &p, &yaw);
    double post = exp(-((fabs(yaw - e->hldt) + fabs(r)) + fabs(p)));
    e->dlts = (lowt - e->lts) / 0.0165 * 0.1;
    e->dj = js;
    e->dvj = jvs;
    e->lts = lowt;
    float t1[17], t2[17];
    for (int k = 0; k < 17; k++) { t1[k] = fabsf(action[k] * e->joint_speeds[k]); t2[k] = action[k] * action[k]; }
    e->es = -1.0 * (double)(pairwise17f(t1) / 17.0f) + -0.1 * (double)(pairwise17f(t2) / 17.0f);
    e->jls = -0.1 * e->jal;
    double z = m->numpy_semantics == 1 ? (double)e->cur_obs[0] + 0.8 : (double)(e->cur_obs[0] + 0.8f);
    e->alive = z > 0.75 ? 2 : -1;
    e->bps = post;
    const double W[7] = {0.34, 0.1, 0.34, 0.034, 0.15, 0.034, 0.1};
    double terms[7] = {e->dj, e->dvj, e->dlts, e->es, e->jls, e->alive, e->bps}, total = 0;
    for (int k = 0; k < 7; k++) total = total + terms[k] * W[k];
    inc_frame(e, 2);
    if (norm3(e->robot_pos[0] - e->target[0], e->robot_pos[1] - e->target[1], e->robot_pos[2] - e->target[2]) <= 0.5) {
        double rr = yaw + draw(e, -180, 180) * DEG2RAD;   /* checkTarget (:412-434) */
        for (int k = 0; k < 3; k++) e->srp[k] = e->target[k];
        e->target[0] = e->robot_pos[0] + cos(rr) * 5;
        e->target[1] = e->robot_pos[1] + sin(rr) * 5;
        e->target[2] = e->robot_pos[2] + 0.0;
        e->lts = -norm3(e->target[0] - e->srp[0], e->target[1] - e->srp[1], e->target[2] - e->srp[2]);
    }
    e->hldt = atan2(e->target[1] - e->robot_pos[1], e->target[0] - e->robot_pos[0]);
    e->wt[0] = e->robot_pos[0] + cos(e->hldt) * 10;
    e->wt[1] = e->robot_pos[1] + sin(e->hldt) * 10;
    if (obs) low_level_obs(m, c, e, obs);
    int alive = e->alive > 0;
    int near = norm3(e->target[0] - e->robot_pos[0], e->target[1] - e->robot_pos[1], e->target[2] - e->robot_pos[2]) <=
               norm3(e->target[0] - e->srp[0], e->target[1] - e->srp[1], e->target[2] - e->srp[2]) + 3;
    int done = !(alive && near);
    e->cur_timestep += 1;
    if (e->cur_timestep >= 3000) done = 1;
    if (reward) *reward = total;
    return done;
}

/* CPU baseline: `threads` independent lanes (OpenMP, one lane per thread) stepping uniform random actions
 * (counter-based, per lane) with reset on done for `seconds` of wall time.  Returns total env steps; *wall =
 * the slowest thread's elapsed seconds. */
long oe_bench(const oe_model* m, const oe_clip* c, const om_params* P, int threads, double seconds, uint64_t seed,
              double* wall) {
    long total = 0;
    double wmax = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel reduction(+ : total) reduction(max : wmax)
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        oe_env e;
        oe_init(&e, c, splitmix64(splitmix64(seed) ^ (uint64_t)tid));
        oe_reset(m, c, &e, -1, 0.0, 0);
        uint64_t actr = splitmix64(seed + 0x5851F42D4C957F2Dull * (uint64_t)(tid + 1));
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        long n = 0;
        double el = 0;
        float a[17];
        double obs[OE_NOBS], rew;
        for (;;) {
            for (int k = 0; k < 17; k++) a[k] = (float)(-1.0 + 2.0 * (double)(splitmix64(actr++) >> 11) * 0x1.0p-53);
            if (oe_step(m, c, P, &e, a, obs, &rew)) oe_reset(m, c, &e, -1, 0.0, obs);
            n++;
            if ((n & 15) == 0) {
                clock_gettime(CLOCK_MONOTONIC, &t1);
                el = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
                if (el >= seconds) break;
            }
        }
        total += n;
        wmax = el;
    }
    if (wall) *wall = wmax;
    return total;
}

int oe_env_size(void) { return (int)sizeof(oe_env); }

/* ORACLE - test infrastructure only (imported by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the CHECKER; never linked into or called by the product path).
 *
 * CPU fp64 restatement of the rigid-multibody step that LowLevelHumanoidEnv.step() drives through
 * pybullet (reference: low_level_env.py:478-481 -> humanoid.py:54-60 apply_action -> pybullet
 * stepSimulation).  The physics lives in the third-party Bullet library (btMultiBody /
 * btMultiBodyConstraintSolver inside the `pybullet` wheel, version unknown, NOT present in
 * /root/reference or this image), so this file restates Bullet's published algorithm:
 *
 *   per env step: motor torques tau = 0.41*power*clip(a) (held over the substeps, as pybullet keeps
 *   TORQUE_CONTROL forces until stepSimulation returns); MJCF joint damping is integrated implicitly
 *   per substep (Bullet ignores MJCF armature, and explicit damping is unstable for this model)
 *   4 substeps of dt = 0.0165/4 (pybullet_envs World: fixedTimeStep 0.0165, numSubSteps 4), each:
 *     1. collision detection at the current pose (geom vs plane z=0, geom vs geom self-collision
 *        excluding ancestors; contact breaking threshold 0.02)
 *     2. Featherstone articulated-body algorithm in LOCAL link frames over pybullet's 32-link layout
 *        (zero-mass dummy links for every hinge, fixed links for bodies), gravity 9.8, Bullet's
 *        default link damping (linear/angular 0.04, velocity + velocity^2 terms), gyroscopic terms;
 *        velocities <- velocities + dt * accelerations (btMultiBody semi-implicit Euler)
 *     3. constraint rows built on those velocities, btMultiBodyConstraintSolver order:
 *        joint-limit rows (violated limits only, erp 0.2, impulse <= 100), contact normal rows
 *        (erp 0.9 = setDefaultContactERP, speculative -d/dt when separated; a limit or contact deeper than
 *        Bullet's split-impulse threshold -0.04 gets no position bias), two friction rows per
 *        contact (mu = 2.0*0.8 ground / 2.0*2.0 self, box bounds +-mu*lambda_n); PGS, 5 iterations;
 *        the constraint responses use the joint-space mass matrix H (built from link Jacobians) and
 *        its Cholesky factor - an independent route to the same M^-1 J^T the product kernel gets
 *        from its ABA factorisation
 *     4. positions <- positions + dt * velocities (base orientation by Bullet's exponential map)
 *
 * PARITY vs PyBullet: UNPINNED (pybullet absent; no reference test pins physics). See DESIGN.md.
 *
 * State vector (47 doubles, shared with the product C-ABI): base pos[3] (COM, world), base quat[4]
 * (x,y,z,w), base lin vel[3] (COM, world), base ang vel[3] (world), q[17], qd[17] (XML dof order).
 */
#include <string.h>
#include <tgmath.h>   /* sqrt / sin / cos / floor / fabs follow `real` */

#include "humanoid_links_gen.h"
#include "physics_oracle.h"

/* `real` is the arithmetic type of the whole restatement: double here; physics_oracle_f32.c re-includes this
 * file with OM_F32 (real = float, every literal single precision via -fsingle-precision-constant, the model
 * constants rounded to float once) - the same algorithm in float arithmetic, the yardstick for the fp32 kernel's
 * rounding error (tests/test_gpu_scale.py). */
#ifdef OM_F32
typedef float real;
#define OM_F32_TABLES(X) X(om_Rfix, 288) X(om_t, 96) X(om_axis, 96) X(om_mass, 32) X(om_com, 96) X(om_inertia, 288) \
    X(om_lo, 17) X(om_hi, 17) X(om_jdamp, 17) X(om_gr, 17) X(om_gp1, 51) X(om_gp2, 51) X(om_part_p, 99)
#define OM_F32_DECL(name, n) static float name##_f[n];
OM_F32_TABLES(OM_F32_DECL)
__attribute__((constructor)) static void om_f32_tables(void) {
#define OM_F32_COPY(name, n) for (int i = 0; i < n; i++) name##_f[i] = (float)name[i];
    OM_F32_TABLES(OM_F32_COPY)
}
#define om_Rfix om_Rfix_f
#define om_t om_t_f
#define om_axis om_axis_f
#define om_mass om_mass_f
#define om_com om_com_f
#define om_inertia om_inertia_f
#define om_lo om_lo_f
#define om_hi om_hi_f
#define om_jdamp om_jdamp_f
#define om_gr om_gr_f
#define om_gp1 om_gp1_f
#define om_gp2 om_gp2_f
#define om_part_p om_part_p_f
float om_block_height(unsigned long long key, int bi, int bj);   /* the terrain draw stays the double TU's */
#define block_height om_block_height
#else
typedef double real;
#endif

/* om_params in the arithmetic type */
typedef struct {
    real dt, gravity, erp_contact, erp_limit, mu_ground, mu_self, contact_thresh, lin_damp, ang_damp;
    real limit_max_impulse, max_coord_vel, hf_s[3], hf_o[3], hf_mid, split_pen;
    int nsub, iters, max_contacts, self_collision, joint_damping, terrain, hf_w, hf_l;
    const float* hf;
    unsigned long long terrain_key;
} rparams;

static void to_rparams(const om_params* P, rparams* Q) {
    Q->dt = (real)P->dt; Q->gravity = (real)P->gravity; Q->erp_contact = (real)P->erp_contact;
    Q->erp_limit = (real)P->erp_limit; Q->mu_ground = (real)P->mu_ground; Q->mu_self = (real)P->mu_self;
    Q->contact_thresh = (real)P->contact_thresh; Q->lin_damp = (real)P->lin_damp; Q->ang_damp = (real)P->ang_damp;
    Q->limit_max_impulse = (real)P->limit_max_impulse; Q->max_coord_vel = (real)P->max_coord_vel;
    for (int k = 0; k < 3; k++) { Q->hf_s[k] = (real)P->hf_s[k]; Q->hf_o[k] = (real)P->hf_o[k]; }
    Q->hf_mid = (real)P->hf_mid; Q->split_pen = (real)P->split_pen;
    Q->nsub = P->nsub; Q->iters = P->iters; Q->max_contacts = P->max_contacts; Q->self_collision = P->self_collision;
    Q->joint_damping = P->joint_damping; Q->terrain = P->terrain; Q->hf_w = P->hf_w; Q->hf_l = P->hf_l;
    Q->hf = P->hf; Q->terrain_key = P->terrain_key;
}

#define NV (6 + OM_ND)
/* contact list capacity: every candidate fits (29 sphere / capsule-end ground points + 2 terrain ridge points per
   capsule (12 capsules) + 66 geom pairs = 119), so the default max_contacts never truncates (Bullet has no global
   contact cap) */
#define MAXC 119
#define MAXROW (3 * MAXC + 2 * OM_ND)


/* ------------------------------------------------------------------------- small linear algebra */
static void mat3_mul(const real* A, const real* B, real* C) {
    real T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    memcpy(C, T, sizeof T);
}
static void mat3_vec(const real* A, const real* x, real* y) {
    real t[3];
    for (int i = 0; i < 3; i++) t[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
    memcpy(y, t, sizeof t);
}
static void mat3T_vec(const real* A, const real* x, real* y) {
    real t[3];
    for (int i = 0; i < 3; i++) t[i] = A[i] * x[0] + A[3 + i] * x[1] + A[6 + i] * x[2];
    memcpy(y, t, sizeof t);
}
static void cross(const real* a, const real* b, real* c) {
    real t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    memcpy(c, t, sizeof t);
}
static real dot3(const real* a, const real* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static real norm3(const real* a) { return sqrt(dot3(a, a)); }

static void axis_angle(const real* u, real q, real* R) {
    real c = cos(q), s = sin(q), C = 1 - c;
    real x = u[0], y = u[1], z = u[2];
    R[0] = c + x * x * C;     R[1] = x * y * C - z * s; R[2] = x * z * C + y * s;
    R[3] = y * x * C + z * s; R[4] = c + y * y * C;     R[5] = y * z * C - x * s;
    R[6] = z * x * C - y * s; R[7] = z * y * C + x * s; R[8] = c + z * z * C;
}
static void quat_to_mat(const real* q, real* R) { /* q = x,y,z,w */
    real x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z);     R[2] = 2 * (x * z + w * y);
    R[3] = 2 * (x * y + w * z);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
    R[6] = 2 * (x * z - w * y);     R[7] = 2 * (y * z + w * x);     R[8] = 1 - 2 * (x * x + y * y);
}

/* --------------------------------------------------------------------------- kinematics */
typedef struct {
    real R[OM_NL][9];   /* link frame -> world */
    real x[OM_NL][3];   /* link origin, world */
    real E[OM_NL][9];   /* parent coords -> link coords (rotation part of X) */
} om_kin;

static void fk(const real* st, om_kin* K) {
    quat_to_mat(st + 3, K->R[0]);
    memcpy(K->x[0], st, 3 * sizeof(real));
    for (int l = 1; l < OM_NL; l++) {
        int p = om_parent[l];
        real Rl[9];
        if (om_type[l] == 1) {
            real Ra[9];
            axis_angle(om_axis + 3 * l, st[13 + om_dof[l]], Ra);
            mat3_mul(om_Rfix + 9 * l, Ra, Rl);       /* parent <- link */
        } else {
            memcpy(Rl, om_Rfix + 9 * l, sizeof Rl);
        }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) K->E[l][3 * i + j] = Rl[3 * j + i];   /* transpose: link <- parent */
        mat3_mul(K->R[p], Rl, K->R[l]);
        real d[3];
        mat3_vec(K->R[p], om_t + 3 * l, d);
        for (int i = 0; i < 3; i++) K->x[l][i] = K->x[p][i] + d[i];
    }
}

#ifndef OM_F32
void om_parts(const double* st, double* out /* [OM_NPART][3] */) {
    om_kin K;
    fk(st, &K);
    for (int k = 0; k < OM_NPART; k++) {
        int l = om_part_link[k];
        if (l < 0) { out[3 * k] = out[3 * k + 1] = out[3 * k + 2] = 0.0; continue; }
        real d[3];
        mat3_vec(K.R[l], om_part_p + 3 * k, d);
        for (int i = 0; i < 3; i++) out[3 * k + i] = K.x[l][i] + d[i];
    }
}
#endif

/* world position of a point given in link coords */
static void link_point(const om_kin* K, int l, const real* p, real* w) {
    real d[3];
    mat3_vec(K->R[l], p, d);
    for (int i = 0; i < 3; i++) w[i] = K->x[l][i] + d[i];
}

/* --------------------------------------------------------------------------- Jacobians / mass matrix */
/* Generalised velocity nu = [w(3) world, v(3) base COM world, qd(ND)]. */
/* point Jacobian (3 x NV, row major) of a world point p rigidly attached to link l */
static void point_jacobian(const om_kin* K, int l, const real* p, real* J) {
    memset(J, 0, 3 * NV * sizeof(real));
    real d[3] = {p[0] - K->x[0][0], p[1] - K->x[0][1], p[2] - K->x[0][2]};
    /* w x d = -d x w  -> columns of -[d]x */
    J[0 * NV + 0] = 0;     J[0 * NV + 1] = d[2];  J[0 * NV + 2] = -d[1];
    J[1 * NV + 0] = -d[2]; J[1 * NV + 1] = 0;     J[1 * NV + 2] = d[0];
    J[2 * NV + 0] = d[1];  J[2 * NV + 1] = -d[0]; J[2 * NV + 2] = 0;
    J[0 * NV + 3] = 1; J[1 * NV + 4] = 1; J[2 * NV + 5] = 1;
    for (int k = l; k > 0; k = om_parent[k]) {
        if (om_type[k] != 1) continue;
        real u[3], r[3], c[3];
        mat3_vec(K->R[k], om_axis + 3 * k, u);
        for (int i = 0; i < 3; i++) r[i] = p[i] - K->x[k][i];
        cross(u, r, c);
        int col = 6 + om_dof[k];
        for (int i = 0; i < 3; i++) J[i * NV + col] = c[i];
    }
}
static void ang_jacobian(const om_kin* K, int l, real* J) {
    memset(J, 0, 3 * NV * sizeof(real));
    J[0 * NV + 0] = 1; J[1 * NV + 1] = 1; J[2 * NV + 2] = 1;
    for (int k = l; k > 0; k = om_parent[k]) {
        if (om_type[k] != 1) continue;
        real u[3];
        mat3_vec(K->R[k], om_axis + 3 * k, u);
        int col = 6 + om_dof[k];
        for (int i = 0; i < 3; i++) J[i * NV + col] = u[i];
    }
}

static void mass_matrix(const om_kin* K, real* H) {
    memset(H, 0, NV * NV * sizeof(real));
    real Jp[3 * NV], Jw[3 * NV];
    for (int l = 0; l < OM_NL; l++) {
        real m = om_mass[l];
        if (m <= 0) continue;
        real c[3], Iw[9], T[9], RT[9];
        link_point(K, l, om_com + 3 * l, c);
        point_jacobian(K, l, c, Jp);
        ang_jacobian(K, l, Jw);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) RT[3 * i + j] = K->R[l][3 * j + i];
        mat3_mul(K->R[l], om_inertia + 9 * l, T);
        mat3_mul(T, RT, Iw);
        for (int a = 0; a < NV; a++)
            for (int b = 0; b < NV; b++) {
                real s = 0;
                for (int i = 0; i < 3; i++) s += m * Jp[i * NV + a] * Jp[i * NV + b];
                for (int i = 0; i < 3; i++)
                    for (int j = 0; j < 3; j++) s += Jw[i * NV + a] * Iw[3 * i + j] * Jw[j * NV + b];
                H[a * NV + b] += s;
            }
    }
}

static int cholesky(real* A, int n) { /* in place, lower */
    for (int j = 0; j < n; j++) {
        real s = A[j * n + j];
        for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
        if (s <= 0) return -1;
        A[j * n + j] = sqrt(s);
        for (int i = j + 1; i < n; i++) {
            real t = A[i * n + j];
            for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = t / A[j * n + j];
        }
    }
    return 0;
}
static void chol_solve(const real* L, int n, real* b) {
    for (int i = 0; i < n; i++) {
        real s = b[i];
        for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k];
        b[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        real s = b[i];
        for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k];
        b[i] = s / L[i * n + i];
    }
}

/* --------------------------------------------------------------------------- spatial algebra (local frames) */
/* motion/force 6-vectors are [angular; linear]. */
static void crm(const real* v, const real* m, real* r) { /* v x m */
    real a[3], b[3], c[3];
    cross(v, m, a);
    cross(v, m + 3, b);
    cross(v + 3, m, c);
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
    r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
static void crf(const real* v, const real* f, real* r) { /* v x* f */
    real a[3], b[3], c[3];
    cross(v, f, a);
    cross(v + 3, f + 3, b);
    cross(v, f + 3, c);
    r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
    r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
/* spatial inertia at link origin, link coords, 6x6 row major */
static void spatial_inertia(int l, real* I6) {
    real m = om_mass[l];
    const real* c = om_com + 3 * l;
    const real* Ic = om_inertia + 9 * l;
    real cc = dot3(c, c);
    real cx[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
    memset(I6, 0, 36 * sizeof(real));
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            I6[6 * i + j] = Ic[3 * i + j] + m * ((i == j ? cc : 0) - c[i] * c[j]);
            I6[6 * i + 3 + j] = m * cx[3 * i + j];
            I6[6 * (3 + i) + j] = m * cx[3 * j + i];   /* (m c x)^T */
            I6[6 * (3 + i) + 3 + j] = (i == j) ? m : 0;
        }
}
static void mat6_vec(const real* A, const real* x, real* y) {
    real t[6];
    for (int i = 0; i < 6; i++) {
        real s = 0;
        for (int j = 0; j < 6; j++) s += A[6 * i + j] * x[j];
        t[i] = s;
    }
    memcpy(y, t, sizeof t);
}
/* X (parent->link) as a full 6x6: [[E,0],[-E rx, E]] */
static void build_X(const real* E, const real* r, real* X) {
    real rx[9] = {0, -r[2], r[1], r[2], 0, -r[0], -r[1], r[0], 0};
    real Erx[9];
    mat3_mul(E, rx, Erx);
    memset(X, 0, 36 * sizeof(real));
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            X[6 * i + j] = E[3 * i + j];
            X[6 * (3 + i) + 3 + j] = E[3 * i + j];
            X[6 * (3 + i) + j] = -Erx[3 * i + j];
        }
}

/* ABA: generalised accelerations (nu-dot, base classical accel in world) for state st, joint torques tau.
 * Returns acc[NV] = [w_dot world, v_com_dot world, qdd]. */
static void aba(const rparams* P, const real* st, const om_kin* K, const real* tau, real* acc) {
    real X[OM_NL][36], v[OM_NL][6], c[OM_NL][6], IA[OM_NL][36], pA[OM_NL][6];
    real U[OM_NL][6], D[OM_NL], u[OM_NL], a[OM_NL][6];
    const real g[3] = {0, 0, -P->gravity};
    /* base velocity in base coords */
    real wl[3], vl[3];
    mat3T_vec(K->R[0], st + 10, wl);
    mat3T_vec(K->R[0], st + 7, vl);
    for (int l = 0; l < OM_NL; l++) {
        if (l == 0) {
            v[0][0] = wl[0]; v[0][1] = wl[1]; v[0][2] = wl[2];
            v[0][3] = vl[0]; v[0][4] = vl[1]; v[0][5] = vl[2];
            memset(c[0], 0, sizeof c[0]);
        } else {
            int p = om_parent[l];
            build_X(K->E[l], om_t + 3 * l, X[l]);
            mat6_vec(X[l], v[p], v[l]);
            memset(c[l], 0, sizeof c[l]);
            if (om_type[l] == 1) {
                real qd = st[30 + om_dof[l]];
                real Sq[6] = {om_axis[3 * l] * qd, om_axis[3 * l + 1] * qd, om_axis[3 * l + 2] * qd, 0, 0, 0};
                for (int i = 0; i < 6; i++) v[l][i] += Sq[i];
                crm(v[l], Sq, c[l]);
            }
        }
        spatial_inertia(l, IA[l]);
        real Iv[6];
        mat6_vec(IA[l], v[l], Iv);
        crf(v[l], Iv, pA[l]);
        /* external: gravity + Bullet link damping, applied at the COM */
        real m = om_mass[l];
        if (m > 0) {
            const real* cm = om_com + 3 * l;
            real gl[3], vcom[3], wxc[3], F[3], n[3], Iw[3];
            mat3T_vec(K->R[l], g, gl);
            cross(v[l], cm, wxc);
            for (int i = 0; i < 3; i++) vcom[i] = v[l][3 + i] + wxc[i];
            real kv = P->lin_damp + P->lin_damp * norm3(vcom);
            real kw = P->ang_damp + P->ang_damp * norm3(v[l]);
            mat3_vec(om_inertia + 9 * l, v[l], Iw);
            for (int i = 0; i < 3; i++) {
                F[i] = m * gl[i] - m * vcom[i] * kv;
                n[i] = -Iw[i] * kw;
            }
            real cxF[3];
            cross(cm, F, cxF);
            for (int i = 0; i < 3; i++) {
                pA[l][i] -= n[i] + cxF[i];
                pA[l][3 + i] -= F[i];
            }
        }
    }
    for (int l = OM_NL - 1; l >= 1; l--) {
        int p = om_parent[l];
        real Ia[36], pa[6];
        memcpy(Ia, IA[l], sizeof Ia);
        memcpy(pa, pA[l], sizeof pa);
        if (om_type[l] == 1) {
            const real* ax = om_axis + 3 * l;
            real S[6] = {ax[0], ax[1], ax[2], 0, 0, 0};
            mat6_vec(IA[l], S, U[l]);
            D[l] = 0;
            for (int i = 0; i < 6; i++) D[l] += S[i] * U[l][i];
            real Sp = 0;
            for (int i = 0; i < 6; i++) Sp += S[i] * pA[l][i];
            u[l] = tau[om_dof[l]] - Sp;
            if (P->joint_damping) {   /* implicit Euler on -d*qd: (D + dt d) qdd = u - d qd */
                real dmp = om_jdamp[om_dof[l]];
                D[l] += P->dt * dmp;
                u[l] -= dmp * st[30 + om_dof[l]];
            }
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++) Ia[6 * i + j] -= U[l][i] * U[l][j] / D[l];
            real Iac[6];
            mat6_vec(Ia, c[l], Iac);
            for (int i = 0; i < 6; i++) pa[i] = pA[l][i] + Iac[i] + U[l][i] * u[l] / D[l];
        } else {
            real Iac[6];
            mat6_vec(Ia, c[l], Iac);
            for (int i = 0; i < 6; i++) pa[i] += Iac[i];
        }
        /* IA_p += X^T Ia X ; pA_p += X^T pa */
        real T[36];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                real s = 0;
                for (int k = 0; k < 6; k++) s += Ia[6 * i + k] * X[l][6 * k + j];
                T[6 * i + j] = s;
            }
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                real s = 0;
                for (int k = 0; k < 6; k++) s += X[l][6 * k + i] * T[6 * k + j];
                IA[p][6 * i + j] += s;
            }
        for (int i = 0; i < 6; i++) {
            real s = 0;
            for (int k = 0; k < 6; k++) s += X[l][6 * k + i] * pa[k];
            pA[p][i] += s;
        }
    }
    /* base: a0 = -IA0^{-1} pA0 */
    {
        real L[36], b[6];
        memcpy(L, IA[0], sizeof L);
        cholesky(L, 6);
        for (int i = 0; i < 6; i++) b[i] = -pA[0][i];
        chol_solve(L, 6, b);
        memcpy(a[0], b, sizeof b);
    }
    for (int l = 1; l < OM_NL; l++) {
        int p = om_parent[l];
        real ap[6];
        mat6_vec(X[l], a[p], ap);
        for (int i = 0; i < 6; i++) a[l][i] = ap[i] + c[l][i];
        if (om_type[l] == 1) {
            real Ua = 0;
            for (int i = 0; i < 6; i++) Ua += U[l][i] * a[l][i];
            real qdd = (u[l] - Ua) / D[l];
            acc[6 + om_dof[l]] = qdd;
            const real* ax = om_axis + 3 * l;
            a[l][0] += ax[0] * qdd; a[l][1] += ax[1] * qdd; a[l][2] += ax[2] * qdd;
        }
    }
    /* base: spatial -> classical, base coords -> world */
    real wd[3], lin[3], wxv[3];
    cross(wl, vl, wxv);
    for (int i = 0; i < 3; i++) lin[i] = a[0][3 + i] + wxv[i];
    mat3_vec(K->R[0], a[0], wd);
    real ld[3];
    mat3_vec(K->R[0], lin, ld);
    for (int i = 0; i < 3; i++) { acc[i] = wd[i]; acc[3 + i] = ld[i]; }
}

/* --------------------------------------------------------------------------- collision */
typedef struct {
    int la, lb;         /* links; lb = -1 for ground */
    real pa[3], pb[3]; /* contact points on A and B (world) */
    real n[3];        /* normal, from B to A */
    real d;           /* signed distance (<0 penetration) */
    real mu;
} om_contact;

static real clampd(real x, real lo, real hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* closest points between segments p1q1 and p2q2 (Ericson, Real-Time Collision Detection 5.1.9) */
static void seg_seg(const real* p1, const real* q1, const real* p2, const real* q2, real* c1, real* c2) {
    real d1[3], d2[3], r[3];
    for (int i = 0; i < 3; i++) { d1[i] = q1[i] - p1[i]; d2[i] = q2[i] - p2[i]; r[i] = p1[i] - p2[i]; }
    real a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    real s, t;
    const real EPS = 1e-12;
    if (a <= EPS && e <= EPS) { s = t = 0; }
    else if (a <= EPS) { s = 0; t = clampd(f / e, 0, 1); }
    else {
        real c = dot3(d1, r);
        if (e <= EPS) { t = 0; s = clampd(-c / a, 0, 1); }
        else {
            real b = dot3(d1, d2), den = a * e - b * b;
            s = (den > EPS) ? clampd((b * f - c * e) / den, 0, 1) : 0;
            t = (b * s + f) / e;
            if (t < 0) { t = 0; s = clampd(-c / a, 0, 1); }
            else if (t > 1) { t = 1; s = clampd((b - c) / a, 0, 1); }
        }
    }
    for (int i = 0; i < 3; i++) { c1[i] = p1[i] + d1[i] * s; c2[i] = p2[i] + d2[i] * t; }
}

/* --------------------------------------------------------------------------- heightfield ground
 * Bullet btHeightfieldTerrainShape (upAxis z, float data, diamond subdivision): vertex (i, j) at
 * origin + scale * (i - (w-1)/2, j - (l-1)/2, h - mid); cell (i, j) split along (i,j)-(i+1,j+1) when i + j is
 * even, along (i+1,j)-(i,j+1) otherwise.  A ground candidate sphere touches the closest point of the surface
 * over the triangles of the cells within reach; a centre below the plane of the triangle under it takes that
 * triangle's upward normal. */
#ifndef OM_F32
static unsigned long long sm64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
#endif
#ifndef OM_F32
float om_block_height(unsigned long long key, int bi, int bj);
float om_block_height(unsigned long long key, int bi, int bj) {   /* humanoid.py:94-111 */
    if ((bi == 63 || bi == 64) && (bj == 63 || bj == 64)) return 0.f;
    double u = (double)(sm64(key + (unsigned long long)(bi + 128 * bj)) >> 11) * (1.0 / 9007199254740992.0);
    return (float)((0.05 * u) * 10.0);
}
#define block_height om_block_height
#endif
static void hf_vertex(const rparams* P, int i, int j, real* v) {
    float h = P->terrain == 1 ? P->hf[i + j * P->hf_w] : block_height(P->terrain_key, i >> 1, j >> 1);
    v[0] = ((real)i - 0.5 * (P->hf_w - 1)) * P->hf_s[0] + P->hf_o[0];
    v[1] = ((real)j - 0.5 * (P->hf_l - 1)) * P->hf_s[1] + P->hf_o[1];
    v[2] = ((real)h - P->hf_mid) * P->hf_s[2] + P->hf_o[2];
}
static void tri_corners(int ci, int cj, int t, int* di, int* dj) {
    static const int A[2][2][6] = {{{0, 0, 1, 0, 1, 1}, {0, 1, 1, 0, 1, 0}}, {{0, 0, 1, 0, 1, 0}, {1, 0, 1, 0, 1, 1}}};
    const int* o = A[((ci + cj) & 1) ? 1 : 0][t];
    for (int k = 0; k < 3; k++) { di[k] = o[k]; dj[k] = o[3 + k]; }
}
/* closest point of triangle abc to p (Ericson 5.1.5) */
static void closest_tri(const real* p, const real* a, const real* b, const real* c, real* q) {
    real ab[3], ac[3], ap[3], bp[3], cp[3];
    for (int k = 0; k < 3; k++) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ap[k] = p[k] - a[k]; }
    real d1 = dot3(ab, ap), d2 = dot3(ac, ap);
    if (d1 <= 0 && d2 <= 0) { memcpy(q, a, 3 * sizeof(real)); return; }
    for (int k = 0; k < 3; k++) bp[k] = p[k] - b[k];
    real d3 = dot3(ab, bp), d4 = dot3(ac, bp);
    if (d3 >= 0 && d4 <= d3) { memcpy(q, b, 3 * sizeof(real)); return; }
    real vc = d1 * d4 - d3 * d2;
    if (vc <= 0 && d1 >= 0 && d3 <= 0) { real t = d1 / (d1 - d3); for (int k = 0; k < 3; k++) q[k] = a[k] + t * ab[k]; return; }
    for (int k = 0; k < 3; k++) cp[k] = p[k] - c[k];
    real d5 = dot3(ab, cp), d6 = dot3(ac, cp);
    if (d6 >= 0 && d5 <= d6) { memcpy(q, c, 3 * sizeof(real)); return; }
    real vb = d5 * d2 - d1 * d6;
    if (vb <= 0 && d2 >= 0 && d6 <= 0) { real t = d2 / (d2 - d6); for (int k = 0; k < 3; k++) q[k] = a[k] + t * ac[k]; return; }
    real va = d3 * d6 - d5 * d4;
    if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
        real t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        for (int k = 0; k < 3; k++) q[k] = b[k] + t * (c[k] - b[k]);
        return;
    }
    real den = 1.0 / (va + vb + vc), v = vb * den, w = vc * den;
    for (int k = 0; k < 3; k++) q[k] = a[k] + ab[k] * v + ac[k] * w;
}
static int terrain_contact(const rparams* P, const real* c, real r, real* n, real* d) {
    real u = (c[0] - P->hf_o[0]) / P->hf_s[0] + 0.5 * (P->hf_w - 1);
    real v = (c[1] - P->hf_o[1]) / P->hf_s[1] + 0.5 * (P->hf_l - 1);
    if (!(u > -2 && u < P->hf_w + 1 && v > -2 && v < P->hf_l + 1)) return 0;
    real reach = r + P->contact_thresh;
    int i0 = (int)floor(u - reach / P->hf_s[0]), i1 = (int)floor(u + reach / P->hf_s[0]);
    int j0 = (int)floor(v - reach / P->hf_s[1]), j1 = (int)floor(v + reach / P->hf_s[1]);
    if (i0 < 0) i0 = 0;
    if (j0 < 0) j0 = 0;
    if (i1 > P->hf_w - 2) i1 = P->hf_w - 2;
    if (j1 > P->hf_l - 2) j1 = P->hf_l - 2;
    if (i0 > i1 || j0 > j1) return 0;
    real best = -1, q[3] = {0, 0, 0};
    for (int cj = j0; cj <= j1; cj++)
        for (int ci = i0; ci <= i1; ci++)
            for (int t = 0; t < 2; t++) {
                int di[3], dj[3];
                real va[3], vb[3], vc[3], qq[3], dv[3];
                tri_corners(ci, cj, t, di, dj);
                hf_vertex(P, ci + di[0], cj + dj[0], va);
                hf_vertex(P, ci + di[1], cj + dj[1], vb);
                hf_vertex(P, ci + di[2], cj + dj[2], vc);
                closest_tri(c, va, vb, vc, qq);
                for (int k = 0; k < 3; k++) dv[k] = c[k] - qq[k];
                real d2 = dot3(dv, dv);
                if (best < 0 || d2 < best) { best = d2; memcpy(q, qq, sizeof q); }
            }
    real nf[3] = {0, 0, 1}, sd = 1;
    int fi = (int)floor(u), fj = (int)floor(v);
    if (fi >= 0 && fi <= P->hf_w - 2 && fj >= 0 && fj <= P->hf_l - 2) {
        real fa = u - fi, fb = v - fj;
        int t = !((fi + fj) & 1) ? (fb >= fa ? 0 : 1) : (fa + fb <= 1 ? 0 : 1);
        int di[3], dj[3];
        real va[3], vb[3], vc[3], e1[3], e2[3], ap[3];
        tri_corners(fi, fj, t, di, dj);
        hf_vertex(P, fi + di[0], fj + dj[0], va);
        hf_vertex(P, fi + di[1], fj + dj[1], vb);
        hf_vertex(P, fi + di[2], fj + dj[2], vc);
        for (int k = 0; k < 3; k++) { e1[k] = vb[k] - va[k]; e2[k] = vc[k] - va[k]; ap[k] = c[k] - va[k]; }
        cross(e1, e2, nf);
        real il = (nf[2] < 0 ? -1.0 : 1.0) / norm3(nf);
        for (int k = 0; k < 3; k++) nf[k] *= il;
        sd = dot3(ap, nf);
    }
    if (sd < 0) {
        memcpy(n, nf, 3 * sizeof(real));
        *d = sd - r;
    } else {
        real dist = sqrt(best);
        if (dist <= 1e-9) { memcpy(n, nf, 3 * sizeof(real)); *d = -r; }
        else { for (int k = 0; k < 3; k++) n[k] = (c[k] - q[k]) / dist; *d = dist - r; }
    }
    return *d < P->contact_thresh;
}

/* closest points between segments p1q1 and p2q2 with their parameters s (on p1q1) and t (on p2q2); the same
   clamping as seg_seg */
static void seg_seg_st(const real* p1, const real* q1, const real* p2, const real* q2, real* c1, real* c2, real* s_out,
                       real* t_out);

/* Capsule bodies against the heightfield: ridge contacts ("What's missing" 1).
 * Bullet collides a capsule with btHeightfieldTerrainShape through btConvexConcaveCollisionAlgorithm: every triangle
 * under the capsule's AABB gets a convex-triangle closest-point query, and the points go into one persistent manifold
 * (at most 4 points, breaking threshold 0.02).  Restated statelessly: the contacts of a capsule are the local minima of
 * the distance from its axis to the surface.  Along the axis over a planar facet that distance is linear, across a
 * concave edge it is the minimum of two linear functions (no interior minimum), so the minima are the two axis ends -
 * the end-cap candidates the plane also uses (terrain_contact) - and the points where the axis passes over a CONVEX
 * edge (a ridge: a block's top edge).  For every interior grid edge within reach of the capsule whose two triangles
 * meet convexly (the second triangle's far vertex more than RIDGE_FLAT = 1e-5 m below the first's plane):
 *   (s, e) = closest points of the axis [a, b] and the edge; kept when s is interior to the axis, more than the
 *   breaking threshold from both ends (nearer, the end cap is that contact), when the edge point is the surface's
 *   closest point to s (terrain_contact at s finds no face closer than |s - e| - 1e-5 m, or s lies inside the terrain)
 *   and when terrain_contact's signed distance at s is below contact_thresh; the contact is terrain_contact's at s.
 * Candidates within the breaking threshold of a kept one (the same convex vertex reached from two edges) are dropped;
 * at most RIDGE_MAX per capsule (with the two end caps, Bullet's 4-point manifold), a deeper candidate replacing the
 * shallowest kept.  Edge order: vertex rows j, then vertices i, then the horizontal, vertical and diagonal edge of
 * vertex (i, j).  The same walk in csrc/terrain.h (ridge_contacts).  PyBullet parity unpinned. */
#define RIDGE_MAX 2
#define RIDGE_BREAK 0.02
#define RIDGE_TOL 1e-5
#define RIDGE_FLAT 1e-5
typedef struct { real n[3], d, t; } ridge_hit;
static int ridge_contacts(const rparams* P, const real* a, const real* b, real r, ridge_hit* out) {
    real ua = (a[0] - P->hf_o[0]) / P->hf_s[0] + 0.5 * (P->hf_w - 1), ub = (b[0] - P->hf_o[0]) / P->hf_s[0] + 0.5 * (P->hf_w - 1);
    real va = (a[1] - P->hf_o[1]) / P->hf_s[1] + 0.5 * (P->hf_l - 1), vb = (b[1] - P->hf_o[1]) / P->hf_s[1] + 0.5 * (P->hf_l - 1);
    if (!(ua > -2 && ua < P->hf_w + 1 && va > -2 && va < P->hf_l + 1 && ub > -2 && ub < P->hf_w + 1 && vb > -2 &&
          vb < P->hf_l + 1)) return 0;
    real ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    real len = norm3(ab);
    if (len <= 2 * RIDGE_BREAK) return 0;   /* no interior point clear of both end caps */
    real reach = r + P->contact_thresh;
    int i0 = (int)floor((ua < ub ? ua : ub) - reach / P->hf_s[0]), i1 = (int)floor((ua > ub ? ua : ub) + reach / P->hf_s[0]);
    int j0 = (int)floor((va < vb ? va : vb) - reach / P->hf_s[1]), j1 = (int)floor((va > vb ? va : vb) + reach / P->hf_s[1]);
    if (i0 < 0) i0 = 0;
    if (j0 < 0) j0 = 0;
    if (i1 > P->hf_w - 2) i1 = P->hf_w - 2;
    if (j1 > P->hf_l - 2) j1 = P->hf_l - 2;
    int nk = 0;
    for (int j = j0; j <= j1 + 1; j++)
        for (int i = i0; i <= i1 + 1; i++)
            for (int kind = 0; kind < 3; kind++) {
                /* edge (e0, e1) and the far vertices c1, c2 of its two triangles (diamond subdivision) */
                int ev[4][2];
                const int even = !((i + j) & 1);
                if (kind == 0) {   /* horizontal (i, j)-(i+1, j): cells (i, j-1) and (i, j) */
                    if (i > i1 || j < 1 || j > P->hf_l - 2) continue;
                    int e[4][2] = {{i, j}, {i + 1, j}, {even ? i + 1 : i, j + 1}, {even ? i + 1 : i, j - 1}};
                    memcpy(ev, e, sizeof e);
                } else if (kind == 1) {   /* vertical (i, j)-(i, j+1): cells (i-1, j) and (i, j) */
                    if (j > j1 || i < 1 || i > P->hf_w - 2) continue;
                    int e[4][2] = {{i, j}, {i, j + 1}, {i + 1, even ? j + 1 : j}, {i - 1, even ? j + 1 : j}};
                    memcpy(ev, e, sizeof e);
                } else {   /* the diagonal of cell (i, j) */
                    if (i > i1 || j > j1) continue;
                    int e[4][2] = {{even ? i : i + 1, j}, {even ? i + 1 : i, j + 1}, {i, even ? j + 1 : j},
                                   {i + 1, even ? j : j + 1}};
                    memcpy(ev, e, sizeof e);
                }
                real A[3], B[3], C1[3], C2[3], e1[3], f1[3], n1[3], g2[3];
                hf_vertex(P, ev[0][0], ev[0][1], A);
                hf_vertex(P, ev[1][0], ev[1][1], B);
                hf_vertex(P, ev[2][0], ev[2][1], C1);
                hf_vertex(P, ev[3][0], ev[3][1], C2);
                for (int k = 0; k < 3; k++) { e1[k] = B[k] - A[k]; f1[k] = C1[k] - A[k]; g2[k] = C2[k] - A[k]; }
                cross(e1, f1, n1);
                real conv = dot3(g2, n1);
                if (n1[2] < 0) conv = -conv;
                /* flat (to RIDGE_FLAT: float32 height rounding of a planar field) or concave: no interior minimum */
                if (!(conv < -RIDGE_FLAT * norm3(n1))) continue;
                real sp[3], ep[3], t, u;
                seg_seg_st(a, b, A, B, sp, ep, &t, &u);
                if (!(t * len > RIDGE_BREAK && (1 - t) * len > RIDGE_BREAK)) continue;
                real dv[3] = {sp[0] - ep[0], sp[1] - ep[1], sp[2] - ep[2]};
                real dse = norm3(dv);
                if (!(dse - r < P->contact_thresh)) continue;
                real n[3], d;
                if (!terrain_contact(P, sp, r, n, &d)) continue;
                if (!(d + r < 0 || d + r >= dse - RIDGE_TOL)) continue;   /* a facet is closer: not a minimum */
                int dup = 0;
                for (int k = 0; k < nk; k++)
                    if (fabs(out[k].t - t) * len < RIDGE_BREAK) { dup = 1; break; }
                if (dup) continue;
                int slot = nk;
                if (nk == RIDGE_MAX) {   /* full: replace the shallowest kept if this one is deeper */
                    slot = out[0].d >= out[1].d ? 0 : 1;
                    if (!(d < out[slot].d)) continue;
                } else {
                    nk++;
                }
                for (int k = 0; k < 3; k++) out[slot].n[k] = n[k];
                out[slot].d = d;
                out[slot].t = t;
            }
    return nk;
}

static void seg_seg_st(const real* p1, const real* q1, const real* p2, const real* q2, real* c1, real* c2, real* s_out,
                       real* t_out) {
    real d1[3], d2[3], r[3];
    for (int i = 0; i < 3; i++) { d1[i] = q1[i] - p1[i]; d2[i] = q2[i] - p2[i]; r[i] = p1[i] - p2[i]; }
    real a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    real s, t;
    const real EPS = 1e-12;
    if (a <= EPS && e <= EPS) { s = t = 0; }
    else if (a <= EPS) { s = 0; t = clampd(f / e, 0, 1); }
    else {
        real c = dot3(d1, r);
        if (e <= EPS) { t = 0; s = clampd(-c / a, 0, 1); }
        else {
            real b = dot3(d1, d2), den = a * e - b * b;
            s = (den > EPS) ? clampd((b * f - c * e) / den, 0, 1) : 0;
            t = (b * s + f) / e;
            if (t < 0) { t = 0; s = clampd(-c / a, 0, 1); }
            else if (t > 1) { t = 1; s = clampd((b - c) / a, 0, 1); }
        }
    }
    for (int i = 0; i < 3; i++) { c1[i] = p1[i] + d1[i] * s; c2[i] = p2[i] + d2[i] * t; }
    *s_out = s;
    *t_out = t;
}

static int collide(const rparams* P, const om_kin* K, om_contact* C) {
    int nc = 0;
    real gp1[OM_NG][3], gp2[OM_NG][3];
    for (int g = 0; g < OM_NG; g++) {
        link_point(K, om_glink[g], om_gp1 + 3 * g, gp1[g]);
        link_point(K, om_glink[g], om_gp2 + 3 * g, gp2[g]);
    }
    for (int g = 0; g < OM_NG; g++) {
        int ne = om_gtype[g] == 0 ? 1 : 2;
        for (int e = 0; e < ne; e++) {
            const real* p = e == 0 ? gp1[g] : gp2[g];
            if (P->terrain) {   /* heightfield ground */
                real n[3], d;
                if (terrain_contact(P, p, om_gr[g], n, &d) && nc < P->max_contacts) {
                    om_contact* c = &C[nc++];
                    c->la = om_glink[g]; c->lb = -1;
                    for (int i = 0; i < 3; i++) {
                        c->n[i] = n[i];
                        c->pa[i] = p[i] - om_gr[g] * n[i];
                        c->pb[i] = c->pa[i] - d * n[i];
                    }
                    c->d = d; c->mu = P->mu_ground;
                }
                continue;
            }
            real d = p[2] - om_gr[g];
            if (d < P->contact_thresh && nc < P->max_contacts) {
                om_contact* c = &C[nc++];
                c->la = om_glink[g]; c->lb = -1;
                c->pa[0] = p[0]; c->pa[1] = p[1]; c->pa[2] = p[2] - om_gr[g];
                c->pb[0] = p[0]; c->pb[1] = p[1]; c->pb[2] = 0;
                c->n[0] = 0; c->n[1] = 0; c->n[2] = 1;
                c->d = d; c->mu = P->mu_ground;
            }
        }
    }
    if (P->terrain) {   /* capsule axes across convex terrain edges: slot 0 of every capsule, then slot 1 */
        ridge_hit rh[OM_NG][RIDGE_MAX];
        int nr[OM_NG];
        for (int g = 0; g < OM_NG; g++)
            nr[g] = om_gtype[g] == 0 ? 0 : ridge_contacts(P, gp1[g], gp2[g], om_gr[g], rh[g]);
        for (int slot = 0; slot < RIDGE_MAX; slot++)
            for (int g = 0; g < OM_NG; g++) {
                if (slot >= nr[g] || nc >= P->max_contacts) continue;
                const ridge_hit* h = &rh[g][slot];
                om_contact* c = &C[nc++];
                c->la = om_glink[g]; c->lb = -1;
                for (int i = 0; i < 3; i++) {
                    c->n[i] = h->n[i];
                    c->pa[i] = gp1[g][i] + h->t * (gp2[g][i] - gp1[g][i]) - om_gr[g] * h->n[i];
                    c->pb[i] = c->pa[i] - h->d * h->n[i];
                }
                c->d = h->d; c->mu = P->mu_ground;
            }
    }
    if (P->self_collision) {
        for (int k = 0; k < OM_NPAIR; k++) {
            int ga = om_pair_a[k], gb = om_pair_b[k];
            real ca[3], cb[3], dv[3];
            seg_seg(gp1[ga], gp2[ga], gp1[gb], gp2[gb], ca, cb);
            for (int i = 0; i < 3; i++) dv[i] = ca[i] - cb[i];
            real dist = norm3(dv);
            real d = dist - om_gr[ga] - om_gr[gb];
            if (d < P->contact_thresh && dist > 1e-9 && nc < P->max_contacts) {
                om_contact* c = &C[nc++];
                c->la = om_glink[ga]; c->lb = om_glink[gb];
                for (int i = 0; i < 3; i++) {
                    c->n[i] = dv[i] / dist;
                    c->pa[i] = ca[i] - om_gr[ga] * c->n[i];
                    c->pb[i] = cb[i] + om_gr[gb] * c->n[i];
                }
                c->d = d; c->mu = P->mu_self;
            }
        }
    }
    return nc;
}

#ifndef OM_F32
int om_contacts(const om_params* P, const double* st, double* out /* [MAXC][12] */) {
    om_kin K;
    om_contact C[MAXC];
    fk(st, &K);
    rparams Q;
    to_rparams(P, &Q);
    int nc = collide(&Q, &K, C);
    for (int i = 0; i < nc; i++) {
        double* o = out + 12 * i;
        o[0] = C[i].la; o[1] = C[i].lb; o[2] = C[i].d; o[3] = C[i].mu;
        for (int k = 0; k < 3; k++) { o[4 + k] = C[i].pa[k]; o[7 + k] = C[i].n[k]; }
        o[10] = 0; o[11] = 0;
    }
    return nc;
}
#endif

static void plane_space(const real* n, real* p, real* q) { /* btPlaneSpace1 */
    if (fabs(n[2]) > 0.7071067811865475244) {
        real a = n[1] * n[1] + n[2] * n[2], k = 1.0 / sqrt(a);
        p[0] = 0; p[1] = -n[2] * k; p[2] = n[1] * k;
        q[0] = a * k; q[1] = -n[0] * p[2]; q[2] = n[0] * p[1];
    } else {
        real a = n[0] * n[0] + n[1] * n[1], k = 1.0 / sqrt(a);
        p[0] = -n[1] * k; p[1] = n[0] * k; p[2] = 0;
        q[0] = -n[2] * p[1]; q[1] = n[2] * p[0]; q[2] = a * k;
    }
}

/* --------------------------------------------------------------------------- one substep */
typedef struct {
    real J[NV], MiJ[NV];
    real meff, b, lo, hi, lam;
    int kind;  /* 0 limit, 1 normal, 2 friction */
    int normal_row;
    real mu;
} om_row;

static void substep(const rparams* P, real* st, const real* tau, int* ncontact_out) {
    const real dt = P->dt;
    om_kin K;
    fk(st, &K);
    om_contact C[MAXC];
    int nc = collide(P, &K, C);
    if (ncontact_out) *ncontact_out = nc;

    /* 1. unconstrained dynamics -> nu* */
    real acc[NV], nu[NV];
    aba(P, st, &K, tau, acc);
    for (int i = 0; i < 3; i++) { nu[i] = st[10 + i] + dt * acc[i]; nu[3 + i] = st[7 + i] + dt * acc[3 + i]; }
    for (int j = 0; j < OM_ND; j++) nu[6 + j] = st[30 + j] + dt * acc[6 + j];
    for (int a = 0; a < NV; a++) nu[a] = clampd(nu[a], -P->max_coord_vel, P->max_coord_vel);

    /* 2. constraint rows */
    om_row rows[MAXROW];   /* on the stack: the OpenMP batch driver steps lanes concurrently */
    int nr = 0;
    real H[NV * NV];
    mass_matrix(&K, H);
    if (P->joint_damping)   /* constraint responses see the same implicit-damping inertia as the ABA */
        for (int j = 0; j < OM_ND; j++) H[(6 + j) * NV + 6 + j] += dt * om_jdamp[j];
    cholesky(H, NV);
    for (int j = 0; j < OM_ND; j++) {  /* joint limits: lower then upper */
        real q = st[13 + j];
        for (int side = 0; side < 2; side++) {
            real pen = side == 0 ? q - om_lo[j] : om_hi[j] - q;
            if (pen > 0) continue;
            om_row* r = &rows[nr++];
            memset(r->J, 0, sizeof r->J);
            r->J[6 + j] = side == 0 ? 1.0 : -1.0;
            r->kind = 0; r->lo = 0; r->hi = P->limit_max_impulse;
            r->b = pen > P->split_pen ? -pen * P->erp_limit / dt : 0.0;
        }
    }
    int first_normal = nr;
    real Jp[3 * NV], Jq[3 * NV];
    for (int k = 0; k < nc; k++) {
        om_contact* c = &C[k];
        point_jacobian(&K, c->la, c->pa, Jp);
        if (c->lb >= 0) {
            point_jacobian(&K, c->lb, c->pb, Jq);
            for (int i = 0; i < 3 * NV; i++) Jp[i] -= Jq[i];
        }
        om_row* r = &rows[nr++];
        for (int a = 0; a < NV; a++) r->J[a] = c->n[0] * Jp[a] + c->n[1] * Jp[NV + a] + c->n[2] * Jp[2 * NV + a];
        r->kind = 1; r->lo = 0; r->hi = 1e10;
        r->b = c->d > 0 ? -c->d / dt : (c->d > P->split_pen ? -c->d * P->erp_contact / dt : 0.0);
        r->mu = c->mu;
    }
    int first_fric = nr;
    for (int k = 0; k < nc; k++) {
        om_contact* c = &C[k];
        point_jacobian(&K, c->la, c->pa, Jp);
        if (c->lb >= 0) {
            point_jacobian(&K, c->lb, c->pb, Jq);
            for (int i = 0; i < 3 * NV; i++) Jp[i] -= Jq[i];
        }
        real vrel[3] = {0, 0, 0};
        for (int i = 0; i < 3; i++)
            for (int a = 0; a < NV; a++) vrel[i] += Jp[i * NV + a] * nu[a];
        real vn = dot3(vrel, c->n), lat[3], t1[3], t2[3];
        for (int i = 0; i < 3; i++) lat[i] = vrel[i] - c->n[i] * vn;
        real l2 = dot3(lat, lat);
        if (l2 > 1e-12) {
            real il = 1.0 / sqrt(l2);
            for (int i = 0; i < 3; i++) t1[i] = lat[i] * il;
            cross(t1, c->n, t2);
        } else {
            plane_space(c->n, t1, t2);
        }
        for (int f = 0; f < 2; f++) {
            const real* t = f == 0 ? t1 : t2;
            om_row* r = &rows[nr++];
            for (int a = 0; a < NV; a++) r->J[a] = t[0] * Jp[a] + t[1] * Jp[NV + a] + t[2] * Jp[2 * NV + a];
            r->kind = 2; r->b = 0; r->mu = c->mu; r->normal_row = first_normal + k;
            r->lo = 0; r->hi = 0;
        }
    }
    (void)first_fric;
    for (int i = 0; i < nr; i++) {
        memcpy(rows[i].MiJ, rows[i].J, sizeof rows[i].J);
        chol_solve(H, NV, rows[i].MiJ);
        real s = 0;
        for (int a = 0; a < NV; a++) s += rows[i].J[a] * rows[i].MiJ[a];
        rows[i].meff = 1.0 / s;
        rows[i].lam = 0;
    }
    /* 3. PGS */
    for (int it = 0; it < P->iters; it++) {
        for (int i = 0; i < nr; i++) {
            om_row* r = &rows[i];
            if (r->kind == 2) {
                real ln = rows[r->normal_row].lam;
                r->lo = -r->mu * ln;
                r->hi = r->mu * ln;
            }
            real Jv = 0;
            for (int a = 0; a < NV; a++) Jv += r->J[a] * nu[a];
            real lnew = clampd(r->lam + r->meff * (r->b - Jv), r->lo, r->hi);
            real dl = lnew - r->lam;
            r->lam = lnew;
            for (int a = 0; a < NV; a++) nu[a] += r->MiJ[a] * dl;
        }
    }
    /* 4. integrate */
    for (int i = 0; i < 3; i++) { st[10 + i] = nu[i]; st[7 + i] = nu[3 + i]; st[i] += dt * nu[3 + i]; }
    for (int j = 0; j < OM_ND; j++) { st[30 + j] = nu[6 + j]; st[13 + j] += dt * nu[6 + j]; }
    {
        const real* w = st + 10;
        real ang = norm3(w), ax[3];
        if (ang * dt > 0.25 * M_PI) ang = 0.25 * M_PI / dt;   /* ANGULAR_MOTION_THRESHOLD */
        if (ang < 0.001) {
            real s = 0.5 * dt - dt * dt * dt * 0.020833333333 * ang * ang;
            for (int i = 0; i < 3; i++) ax[i] = w[i] * s;
        } else {
            real s = sin(0.5 * ang * dt) / ang;
            for (int i = 0; i < 3; i++) ax[i] = w[i] * s;
        }
        real dw = cos(0.5 * ang * dt);
        real* q = st + 3; /* x y z w */
        real nq[4] = {dw * q[0] + ax[0] * q[3] + ax[1] * q[2] - ax[2] * q[1],
                        dw * q[1] + ax[1] * q[3] + ax[2] * q[0] - ax[0] * q[2],
                        dw * q[2] + ax[2] * q[3] + ax[0] * q[1] - ax[1] * q[0],
                        dw * q[3] - ax[0] * q[0] - ax[1] * q[1] - ax[2] * q[2]};
        real nn = sqrt(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
        for (int i = 0; i < 4; i++) q[i] = nq[i] / nn;
    }
}

/* ------------------------------------------------------------------------- public API */
#ifdef OM_F32
/* the float instantiation: one env step in float arithmetic from a double state (rounded to float on entry, the
   result widened back) */
void om_step_f32(const om_params* P, double* st, const double* tau_motor, int* ncontact_out);
void om_step_f32(const om_params* P, double* st, const double* tau_motor, int* ncontact_out) {
    rparams Q;
    to_rparams(P, &Q);
    real s[47], t[OM_ND];
    for (int i = 0; i < 47; i++) s[i] = (real)st[i];
    for (int i = 0; i < OM_ND; i++) t[i] = (real)tau_motor[i];
    for (int k = 0; k < Q.nsub; k++) substep(&Q, s, t, k == Q.nsub - 1 ? ncontact_out : 0);
    for (int i = 0; i < 47; i++) st[i] = (double)s[i];
}
#else
void om_default_params(om_params* P) {
    P->dt = 0.0165 / 4.0;
    P->nsub = 4;
    P->gravity = 9.8;
    P->iters = 5;
    P->erp_contact = 0.9;
    P->erp_limit = 0.2;
    P->mu_ground = 2.0 * 0.8;
    P->mu_self = 2.0 * 2.0;
    P->contact_thresh = 0.02;
    P->lin_damp = 0.04;
    P->ang_damp = 0.04;
    P->limit_max_impulse = 100.0;
    P->max_contacts = MAXC;
    P->self_collision = 1;
    P->joint_damping = 1;
    P->max_coord_vel = 100.0;
    P->terrain = 0;
    P->hf = 0;
    P->hf_w = P->hf_l = 256;
    for (int k = 0; k < 3; k++) { P->hf_s[k] = 1.0; P->hf_o[k] = 0.0; }
    P->hf_o[2] = 0.25;
    P->hf_mid = 0.25;
    P->terrain_key = 0;
    P->split_pen = -0.04;
}

/* one env step of physics: state (47) in place; tau_motor[17] in dof order (already 0.41*power*clip(a)). */
void om_step(const om_params* P, double* st, const double* tau_motor, int* ncontact_out) {
    rparams Q;
    to_rparams(P, &Q);
    for (int s = 0; s < Q.nsub; s++) substep(&Q, st, tau_motor, s == Q.nsub - 1 ? ncontact_out : 0);
}

/* diagnostics used by tests: unconstrained accelerations (ABA) and mass-matrix-based accelerations */
void om_aba(const om_params* P, const double* st, const double* tau, double* acc) {
    om_kin K;
    fk(st, &K);
    rparams Q;
    to_rparams(P, &Q);
    aba(&Q, st, &K, tau, acc);
}
void om_mass_matrix(const double* st, double* H) {
    om_kin K;
    fk(st, &K);
    mass_matrix(&K, H);
}
void om_link_frames(const double* st, double* R, double* x) {
    om_kin K;
    fk(st, &K);
    memcpy(R, K.R, sizeof K.R);
    memcpy(x, K.x, sizeof K.x);
}
int om_nv(void) { return NV; }

/* one ground candidate (sphere centre c, radius r) against the heightfield ground: 1 with normal n and signed
   distance d when in contact range (tests) */
int om_terrain_contact(const om_params* P, const double* c, double r, double* n, double* d) {
    rparams Q;
    to_rparams(P, &Q);
    return terrain_contact(&Q, c, r, n, d);
}
/* every geom's world segment: out[8 * g ...] = p1 (3), p2 (3), radius, type (0 sphere, 1 capsule) (tests) */
void om_geom_segments(const double* st, double* out) {
    om_kin K;
    fk(st, &K);
    for (int g = 0; g < OM_NG; g++) {
        link_point(&K, om_glink[g], om_gp1 + 3 * g, out + 8 * g);
        link_point(&K, om_glink[g], om_gp2 + 3 * g, out + 8 * g + 3);
        out[8 * g + 6] = om_gr[g];
        out[8 * g + 7] = om_gtype[g] == 0 ? 0 : 1;
    }
}
/* a capsule (axis a-b, radius r) against the heightfield's convex edges: the number of ridge contacts, each
   out[5 * k ...] = normal (3), signed distance, axis parameter t (tests) */
int om_ridge_contacts(const om_params* P, const double* a, const double* b, double r, double* out) {
    rparams Q;
    to_rparams(P, &Q);
    ridge_hit h[RIDGE_MAX];
    int n = ridge_contacts(&Q, a, b, r, h);
    for (int k = 0; k < n; k++) {
        for (int i = 0; i < 3; i++) out[5 * k + i] = h[k].n[i];
        out[5 * k + 3] = h[k].d;
        out[5 * k + 4] = h[k].t;
    }
    return n;
}
#endif

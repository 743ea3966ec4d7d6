// physics.h - per-lane rigid multibody step for the humanoid (device code, templated on Real).
//
// Replaces the Bullet btMultiBody step pybullet runs inside LowLevelHumanoidEnv.step()
// (reference: low_level_env.py:478-479 -> pybullet stepSimulation; algorithm restated in
// DESIGN.md "Physics model" and, independently, in oracle/physics_oracle.c).
//
// Formulation (MI355X-first, one env per lane):
//  * 11 bodies with multi-dof hinge groups (mechanically identical to pybullet's 31-link chain of
//    zero-mass dummy links), tree topology and all model constants compile-time (model_gen.h), so every
//    loop over bodies/dofs is unrolled and indices are immediates.
//  * All spatial quantities in ONE frame: world-aligned axes, origin at the base COM at the start of
//    the substep.  Articulated-inertia propagation then needs no 6x6 coordinate transforms
//    (IA_parent += IA_child - U D^-1 U^T), the dominant cost of local-frame ABA.
//  * Constraint responses M^-1 J^T from the ABA factorisation (test-impulse passes), PGS in Bullet's
//    row order (limits, contact normals, friction), rows staged in a per-lane SoA scratch in HBM.
#pragma once
#include "model_gen.h"

namespace hk {

using namespace hm;

// --------------------------------------------------------------------------------------- parameters
struct PhysParams {
    double dt;            // substep
    int nsub;
    double gravity;
    int iters;
    double erp_contact, erp_limit, mu_ground, mu_self, contact_thresh;
    double split_pen;     // split-impulse threshold: rows penetrating deeper get no position bias (hum_config)
    double lin_damp, ang_damp, limit_max_impulse, max_coord_vel;
    int max_contacts;
    int self_collision;
    int joint_damping;
    int lds_rows;         // cooperative kernel: constraint rows per block kept in LDS (block row pool capacity)
    // ground (hum_set_terrain, terrain.h): 0 = plane z = 0, 1 = shared heightfield hf, 2 = per-lane random blocks
    int terrain;
    const float* hf;      // terrain 1: heights [hf_w * hf_l], vertex (i, j) at hf[i + j * hf_w]
    int hf_w, hf_l;
    double hf_s[3], hf_o[3], hf_mid;   // mesh scale, body origin, vertical centre (min + max) / 2
};

constexpr int NV = 6 + NDOF;
// every contact candidate: one per sphere and two per capsule end against the ground plane, plus every
// non-ancestor geom pair (29 + 66 = 95), plus the heightfield's ridge points (24).  Bullet has no global contact
// cap, so neither do we: the list
// holds all of them (max_contacts may lower it for diagnostics; overflow is then flagged)
constexpr int NCAND_ALL = [] { int n = NPAIR; for (int g = 0; g < NGEOM; g++) n += geom_type[g] == 0 ? 1 : 2; return n; }();
// heightfield ground only (terrain.h ridge_contacts): up to 2 more ground contacts per capsule where its axis
// crosses a convex terrain edge
constexpr int NRIDGE_ALL = [] { int n = 0; for (int g = 0; g < NGEOM; g++) n += geom_type[g] == 0 ? 0 : 2; return n; }();
constexpr int MAXC = NCAND_ALL + NRIDGE_ALL;   // contact list capacity per substep (ground + ridge + self)
constexpr int ROW_STRIDE = 2 * NV + 6;   // J[NV], MiJ[NV], b, lo, hi, lam, meff, mu
constexpr int MAX_LIMIT_ROWS = NDOF;     // at most one side of a hinge can be violated
constexpr int MAXROWS = MAX_LIMIT_ROWS + 3 * MAXC;
constexpr int CON_STRIDE = 12;           // contact list entry: ba, bb, pa[3], pb[3], n[3], d  (+mu from bb)
constexpr int SCRATCH_PER_LANE = MAXROWS * ROW_STRIDE + MAXC * CON_STRIDE;

// symmetric 6x6 (upper triangle, row major)
__host__ __device__ constexpr int sidx(int i, int j) {
    return i <= j ? (i * 6 - i * (i - 1) / 2 + (j - i)) : (j * 6 - j * (j - 1) / 2 + (i - j));
}

template <typename T>
struct Lane {  // per-lane scratch view (SoA: element e of lane at base[e * stride])
    T* base;
    long stride;
    __device__ T& at(int e) const { return base[(long)e * stride]; }
};

template <typename T>
__device__ inline void cross3(const T* a, const T* b, T* c) {
    T x = a[1] * b[2] - a[2] * b[1];
    T y = a[2] * b[0] - a[0] * b[2];
    T z = a[0] * b[1] - a[1] * b[0];
    c[0] = x; c[1] = y; c[2] = z;
}
template <typename T>
__device__ inline T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

template <typename T>
__device__ inline void symmv(const T* S, const T* x, T* y) {  // y = S x, S sym6
#pragma unroll
    for (int i = 0; i < 6; i++) {
        T s = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) s += S[sidx(i, j)] * x[j];
        y[i] = s;
    }
}

// spatial cross products (motion / force), 6-vectors [angular; linear]
template <typename T>
__device__ inline void crm(const T* v, const T* m, T* r) {
    T a[3], b[3], c[3];
    cross3(v, m, a);
    cross3(v, m + 3, b);
    cross3(v + 3, m, c);
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
    r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
template <typename T>
__device__ inline void crf(const T* v, const T* f, T* r) {
    T a[3], b[3], c[3];
    cross3(v, f, a);
    cross3(v + 3, f + 3, b);
    cross3(v, f + 3, c);
    r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
    r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}

// post-multiply a 3x3 (row major) by an elementary rotation about axis `ax` with (c, s)
template <typename T>
__device__ inline void rot_post(T* M, int ax, T c, T s) {
#pragma clang fp contract(on)   // per-expression fusion only: the same frames in every inlining context
    const int i = (ax + 1) % 3, j = (ax + 2) % 3;  // columns mixed by a rotation about `ax`
#pragma unroll
    for (int r = 0; r < 3; r++) {
        T mi = M[3 * r + i], mj = M[3 * r + j];
        M[3 * r + i] = c * mi + s * mj;
        M[3 * r + j] = -s * mi + c * mj;
    }
}

// acc + x * c for a model constant c, as the fma that fp-contraction forms for `acc + x * c`: a term with c == 0 is
// skipped (fma(x, 0, acc) == acc up to the sign of a zero result) and c == 1 folds to an add, so the identity
// rotations and zero offsets of the model cost nothing while every other term rounds exactly as before.
template <typename T>
__device__ __attribute__((always_inline)) inline T fmak(T x, double c, T acc) {
    return c == 0.0 ? acc : fma(x, (T)c, acc);
}

template <typename T>
__device__ inline void quat_to_mat(const T* q, T* R) {
#pragma clang fp contract(on)   // per-expression fusion only: the same frames in every inlining context
    T x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z);     R[2] = 2 * (x * z + w * y);
    R[3] = 2 * (x * y + w * z);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
    R[6] = 2 * (x * z - w * y);     R[7] = 2 * (y * z + w * x);     R[8] = 1 - 2 * (x * x + y * y);
}

template <typename T>
__device__ inline T clampT(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }

// Physics-only fp32 reciprocal / square root / reciprocal square root on the hardware instructions (v_rcp_f32,
// v_sqrt_f32, v_rsq_f32: 1 ulp) instead of the ~10-instruction correctly rounded sequences, which sat on the
// dependent chains of the base Cholesky, the ABA pivots, the row scalings and the narrow phase (+1.5% measured).
// The physics is held to a tolerance against the fp64 oracle, not to bits; fp64 stays IEEE.  The env logic
// (rewards, observations) never uses these.
template <typename T>
__device__ inline T prcp(T x) {
#ifdef HUM_EXACT_MATH   // diagnostics: correctly rounded reciprocal / square roots (the fp32 accuracy study)
    if constexpr (sizeof(T) == 4) return 1.0f / x;
#endif
    if constexpr (sizeof(T) == 4) return __builtin_amdgcn_rcpf(x);
    else return T(1) / x;
}
template <typename T>
__device__ inline T psqrt(T x) {
#ifdef HUM_EXACT_MATH
    if constexpr (sizeof(T) == 4) return sqrtf(x);
#endif
    if constexpr (sizeof(T) == 4) return __builtin_amdgcn_sqrtf(x);
    else return sqrt(x);
}
template <typename T>
__device__ inline T prsqrt(T x) {
#ifdef HUM_EXACT_MATH
    if constexpr (sizeof(T) == 4) return 1.0f / sqrtf(x);
#endif
    if constexpr (sizeof(T) == 4) return __builtin_amdgcn_rsqf(x);
    else return T(1) / sqrt(x);
}

// the same by site class, for the fp32 accuracy study: the ABA / base pivots, the constraint
// rows' scalings, the narrow phase; -DHUM_EXACT_<class> makes that class correctly rounded
#define HUM_PREC_SITE(NAME, MACRO)                                                      \
    template <typename T>                                                              \
    __device__ inline T prcp_##NAME(T x) {                                             \
        if constexpr (sizeof(T) == 4 && MACRO) return 1.0f / x;                         \
        return prcp(x);                                                                \
    }                                                                                  \
    template <typename T>                                                              \
    __device__ inline T prsqrt_##NAME(T x) {                                           \
        if constexpr (sizeof(T) == 4 && MACRO) return 1.0f / sqrtf(x);                  \
        return prsqrt(x);                                                              \
    }
#ifdef HUM_EXACT_PIVOTS
#define HUM_EXACT_PIVOTS_ON 1
#else
#define HUM_EXACT_PIVOTS_ON 0
#endif
#ifdef HUM_EXACT_ROWS
#define HUM_EXACT_ROWS_ON 1
#else
#define HUM_EXACT_ROWS_ON 0
#endif
#ifdef HUM_EXACT_GEOM
#define HUM_EXACT_GEOM_ON 1
#else
#define HUM_EXACT_GEOM_ON 0
#endif
HUM_PREC_SITE(row, HUM_EXACT_ROWS_ON)
HUM_PREC_SITE(geo, HUM_EXACT_GEOM_ON)
// The ABA / base pivots (ldl_small's 1 / d, chol6_inv's 1 / sqrt).  Measured over 512 lanes from identical states
// (tools/diag_fp32_ab.py, two state samples): joint-speed error ratio to the fp32 yardstick p99 3.00 / 2.00 with the
// bare approximations, 2.53 / 2.26 correctly rounded, 2.09 (second sample) with one Newton step; correctly rounded row
// scalings or narrow phase: no change.  The differences are within the p99's sampling spread (an independent fp32
// oracle realisation against the envelope measures p99 1.9 - 2.3 over 512 lanes), so the kernel keeps the
// approximation (the Newton step cost 0.6 %, correctly rounded pivots 1.1 %).
HUM_PREC_SITE(piv, HUM_EXACT_PIVOTS_ON)

// ------------------------------------------------------------------------------------- kinematics
template <typename T>
struct Kin {
    T R[NB][9];      // body frame -> world
    T o[NB][3];      // body frame origin (pivot), relative to the base COM
    T u[NDOF][3];    // world hinge axes
};

template <typename T>
__device__ inline void forward_kinematics(const T* quat, const T* q, Kin<T>& K);   // below: via the _pre form

// the same with the hinge angles' sin / cos precomputed (scs[2d] = sin q_d, scs[2d+1] = cos q_d)
template <typename T>
__device__ inline void forward_kinematics_pre(const T* quat, const T* scs, Kin<T>& K) {
#pragma clang fp contract(on)   // per-expression fusion only: the same frames in every inlining context
    quat_to_mat(quat, K.R[0]);
    K.o[0][0] = K.o[0][1] = K.o[0][2] = 0;
#pragma unroll
    for (int b = 1; b < NB; b++) {
        const int p = body_parent[b];
        T M[9];
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) {   // R_p Roff: (R0 c0 + R1 c1) + R2 c2, fused as written
                const double c0 = body_Roff[9 * b + c];
                T m = c0 == 0.0 ? T(-0.0) : K.R[p][3 * r] * (T)c0;
                m = fmak(K.R[p][3 * r + 1], body_Roff[9 * b + 3 + c], m);
                M[3 * r + c] = fmak(K.R[p][3 * r + 2], body_Roff[9 * b + 6 + c], m);
            }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            T o = fmak(K.R[p][3 * i], body_toff[3 * b], K.o[p][i]);
            o = fmak(K.R[p][3 * i + 1], body_toff[3 * b + 1], o);
            K.o[b][i] = fmak(K.R[p][3 * i + 2], body_toff[3 * b + 2], o);
        }
#pragma unroll
        for (int k = 0; k < body_ndof[b]; k++) {
            const int d = body_dof0[b] + k, ax = dof_axis[d];
            const T sg = (T)dof_sign[d];
            K.u[d][0] = M[ax] * sg; K.u[d][1] = M[3 + ax] * sg; K.u[d][2] = M[6 + ax] * sg;
            rot_post(M, ax, scs[2 * d + 1], sg * scs[2 * d]);
        }
#pragma unroll
        for (int i = 0; i < 9; i++) K.R[b][i] = M[i];
    }
}

// every kinematics evaluation goes through forward_kinematics_pre, so a state's frames are bit-identical
// whether its hinge sin / cos were computed here or across lanes (cooperative kernel)
template <typename T>
__device__ inline void hinge_sincos(T q, T* sn, T* cs) {
    if constexpr (sizeof(T) == 4) sincosf(q, sn, cs);
    else sincos(q, sn, cs);
}
template <typename T>
__device__ inline void forward_kinematics(const T* quat, const T* q, Kin<T>& K) {
    T scs[2 * NDOF];
#pragma unroll
    for (int d = 0; d < NDOF; d++) hinge_sincos(q[d], &scs[2 * d], &scs[2 * d + 1]);
    forward_kinematics_pre(quat, scs, K);
}

// motion subspace column of dof d (body b) at the common origin: [u; o_b x u]
template <typename T>
__device__ inline void motion_col(const Kin<T>& K, int b, int d, T* S) {
    S[0] = K.u[d][0]; S[1] = K.u[d][1]; S[2] = K.u[d][2];
    cross3(K.o[b], K.u[d], S + 3);
}

// ------------------------------------------------------------------------------------- ABA
template <typename T>
struct Aba {
    T U[NDOF][6];        // IA S per dof
    T Dinv[NB][9];       // (S^T IA S + dt*damping)^-1 per body, k x k (row major in 3x3 slot)
    T L0[21];            // Cholesky factor of the base articulated inertia (lower, packed)
    T c[NB][6];          // bias accelerations
    T uu[NDOF];          // tau - S^T pA (- damping qd)
};

template <typename T, int K3>
__device__ inline void small_inverse(const T* D, T* Di) {  // symmetric k x k (k = K3), stored 3x3
    if constexpr (K3 == 1) {
        Di[0] = prcp(D[0]);
    } else if constexpr (K3 == 2) {
        T det = D[0] * D[4] - D[1] * D[3];
        T id = prcp(det);
        Di[0] = D[4] * id; Di[1] = -D[1] * id; Di[3] = -D[3] * id; Di[4] = D[0] * id;
    } else {
        T a = D[0], b = D[1], c = D[2], e = D[4], f = D[5], i = D[8];
        T A = e * i - f * f, B = c * f - b * i, C = b * f - c * e;
        T det = a * A + b * B + c * C;
        T id = prcp(det);
        Di[0] = A * id; Di[1] = B * id; Di[2] = C * id;
        Di[3] = B * id; Di[4] = (a * i - c * c) * id; Di[5] = (b * c - a * f) * id;
        Di[6] = C * id; Di[7] = (b * c - a * f) * id; Di[8] = (a * e - b * b) * id;
    }
}

// LDL^T factorisation of the symmetric positive definite k x k joint-space block D = S^T IA S (+ dt damping), k = K3,
// stored 3x3: unit lower L (strict part in Lf), the reciprocal pivots idd, and D^-1 = L^-T diag(idd) L^-1 in Di.
// Pass 2 downdates the articulated inertia through L and idd (Y = U L^-T; IA - sum_j Y_j Y_j^T idd_j: a sequence of
// symmetric rank-1 terms, the dof-by-dof elimination of a chain of single-dof links) instead of W U^T with the
// cofactor inverse: the cofactor determinant of a hip block cancels, and over 2048 lanes from identical states its
// fp32 error ratio was p99 3.1 against 2.1 here (tools/fp32lab).
template <typename T, int K3>
__device__ inline void ldl_small(const T* D, T* Lf, T* idd, T* Di) {
    T d[3];
#pragma unroll
    for (int j = 0; j < K3; j++) {
        T s = D[4 * j];
#pragma unroll
        for (int q = 0; q < j; q++) s -= Lf[3 * j + q] * Lf[3 * j + q] * d[q];
        d[j] = s;
        idd[j] = prcp_piv(s);
#pragma unroll
        for (int i = j + 1; i < K3; i++) {
            T t = D[3 * i + j];
#pragma unroll
            for (int q = 0; q < j; q++) t -= Lf[3 * i + q] * Lf[3 * j + q] * d[q];
            Lf[3 * i + j] = t * idd[j];
        }
    }
    // M = L^-1 (unit lower), Di = M^T diag(idd) M
    T Mi[9];
#pragma unroll
    for (int c = 0; c < K3; c++)
#pragma unroll
        for (int i = c; i < K3; i++) {
            T t = i == c ? T(1) : T(0);
#pragma unroll
            for (int q = c; q < i; q++) t -= Lf[3 * i + q] * Mi[3 * q + c];
            Mi[3 * i + c] = t;
        }
#pragma unroll
    for (int i = 0; i < K3; i++)
#pragma unroll
        for (int j = i; j < K3; j++) {
            T t = 0;
#pragma unroll
            for (int q = j; q < K3; q++) t += Mi[3 * q + i] * idd[q] * Mi[3 * q + j];
            Di[3 * i + j] = t;
            Di[3 * j + i] = t;
        }
}

// pivot shifts (axes stay world-aligned): a spatial force about o_b moved to o_b - r (n += r x f); a spatial inertia
// about o_b moved to o_b - r, I' = X^T I X with X = [[E, 0], [-[r]x, E]]:  B' = B + [r]x C, A' = A + [r]x B^T - B' [r]x
template <typename T>
__device__ inline void shift_force(const T* r, T* f) {
    T x[3];
    cross3(r, f + 3, x);
    f[0] += x[0]; f[1] += x[1]; f[2] += x[2];
}
template <typename T>
__device__ inline void shift_inertia(const T* r, T* I) {   // in place, sym6 packed (sidx)
    T B[3][3], Bp[3][3], rb[3][3], rbp[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) B[i][j] = I[sidx(i, 3 + j)];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const T cj[3] = {I[sidx(3, 3 + j)], I[sidx(4, 3 + j)], I[sidx(5, 3 + j)]};
        T x[3];
        cross3(r, cj, x);
#pragma unroll
        for (int i = 0; i < 3; i++) Bp[i][j] = B[i][j] + x[i];
    }
#pragma unroll
    for (int j = 0; j < 3; j++) { cross3(r, B[j], rb[j]); cross3(r, Bp[j], rbp[j]); }
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = i; j < 3; j++) I[sidx(i, j)] = I[sidx(i, j)] + rb[j][i] + rbp[i][j];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) I[sidx(i, 3 + j)] = Bp[i][j];
}

template <typename T>
__device__ inline void chol6(const T* A, T* L) {  // A sym6 packed (sidx) -> L lower packed row-wise
    // L index for (i, j), j <= i: i*(i+1)/2 + j
#pragma unroll
    for (int j = 0; j < 6; j++) {
        T s = A[sidx(j, j)];
#pragma unroll
        for (int k = 0; k < j; k++) s -= L[j * (j + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
        T djj = sqrt(s);
        L[j * (j + 1) / 2 + j] = djj;
        T inv = T(1) / djj;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            T t = A[sidx(i, j)];
#pragma unroll
            for (int k = 0; k < j; k++) t -= L[i * (i + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
            L[i * (i + 1) / 2 + j] = t * inv;
        }
    }
}
template <typename T>
__device__ inline void chol6_solve(const T* L, T* b) {
#pragma unroll
    for (int i = 0; i < 6; i++) {
        T s = b[i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= L[i * (i + 1) / 2 + k] * b[k];
        b[i] = s / L[i * (i + 1) / 2 + i];
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        T s = b[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) s -= L[k * (k + 1) / 2 + i] * b[k];
        b[i] = s / L[i * (i + 1) / 2 + i];
    }
}

// body spatial inertia at the common origin, packed sym6: mass m, COM c (rel origin), Icw (3x3 world)
template <typename T>
__device__ inline void spatial_inertia(T m, const T* c, const T* Icw, T* I) {
    T cc = dot3(c, c);
    I[sidx(0, 0)] = Icw[0] + m * (cc - c[0] * c[0]);
    I[sidx(0, 1)] = Icw[1] - m * c[0] * c[1];
    I[sidx(0, 2)] = Icw[2] - m * c[0] * c[2];
    I[sidx(1, 1)] = Icw[4] + m * (cc - c[1] * c[1]);
    I[sidx(1, 2)] = Icw[5] - m * c[1] * c[2];
    I[sidx(2, 2)] = Icw[8] + m * (cc - c[2] * c[2]);
    // B = m [c]x
    I[sidx(0, 3)] = 0;         I[sidx(0, 4)] = -m * c[2]; I[sidx(0, 5)] = m * c[1];
    I[sidx(1, 3)] = m * c[2];  I[sidx(1, 4)] = 0;         I[sidx(1, 5)] = -m * c[0];
    I[sidx(2, 3)] = -m * c[1]; I[sidx(2, 4)] = m * c[0];  I[sidx(2, 5)] = 0;
    I[sidx(3, 3)] = m; I[sidx(3, 4)] = 0; I[sidx(3, 5)] = 0;
    I[sidx(4, 4)] = m; I[sidx(4, 5)] = 0;
    I[sidx(5, 5)] = m;
}

// R I R^T for a constant local inertia (row-major 3x3 constexpr at offset)
template <typename T>
__device__ inline void rotate_inertia(const T* R, const double* Il, T* Iw) {
    T RI[9];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) RI[3 * r + c] = R[3 * r] * (T)Il[c] + R[3 * r + 1] * (T)Il[3 + c] + R[3 * r + 2] * (T)Il[6 + c];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) Iw[3 * r + c] = RI[3 * r] * R[3 * c] + RI[3 * r + 1] * R[3 * c + 1] + RI[3 * r + 2] * R[3 * c + 2];
}

// Unconstrained accelerations: acc[NV] = [w_dot, v_com_dot (classical, world), qdd]
// nu = [w(3), v_com(3), qd(17)];  tau = motor torques (dof order).
//
// Passes 1 and 2 run about each body's own pivot o_b (axes world-aligned): a body's spatial inertia carries its own
// m |c - o_b|^2 (~0.01-0.1 m^2) instead of m |c|^2 about the common origin (up to ~1.4 m^2 for a foot), and its hinge
// columns are [u; 0].  At the common origin the joint-space blocks S^T IA S were differences of m |c|^2-sized numbers,
// which cost fp32 kernel steps 2-3x the rounding error of the fp32 oracle (tools/fp32lab).  A
// child's articulated inertia and bias force are moved to its parent's pivot (shift_inertia / shift_force) before
// they are summed there.  The torso's pivot is the common origin, so the base solve is unchanged, and pass 3, the
// factorisation the constraint responses read (U, Dinv, L0) and c stay at the common origin.
template <typename T>
__device__ inline void aba(const PhysParams& P, const Kin<T>& K, const T* nu, const T* tau, Aba<T>& A, T* acc) {
    T V[NB][6], IA[NB][21], pA[NB][6], cl[NB][6];
    // ---- pass 1: velocities, bias accelerations, inertias, bias forces (about each pivot)
#pragma unroll
    for (int b = 0; b < NB; b++) {
        if (b == 0) {
#pragma unroll
            for (int i = 0; i < 6; i++) { V[0][i] = nu[i]; A.c[0][i] = 0; cl[0][i] = 0; }
        } else {
            const int p = body_parent[b];
#pragma unroll
            for (int i = 0; i < 6; i++) V[b][i] = V[p][i];
#pragma unroll
            for (int k = 0; k < body_ndof[b]; k++) {
                const int d = body_dof0[b] + k;
                T S[6];
                motion_col(K, b, d, S);
                const T qd = nu[6 + d];
#pragma unroll
                for (int i = 0; i < 6; i++) V[b][i] += S[i] * qd;
            }
        }
    }
    T Vl[NB][6];   // body velocities about their pivots: v_b = v_O + w x o_b
#pragma unroll
    for (int b = 0; b < NB; b++) {
        T x[3];
        cross3(V[b], K.o[b], x);
#pragma unroll
        for (int i = 0; i < 3; i++) { Vl[b][i] = V[b][i]; Vl[b][3 + i] = V[b][3 + i] + x[i]; }
    }
#pragma unroll
    for (int b = 0; b < NB; b++) {
        if (b > 0) {
            const int p = body_parent[b];
            // bias acceleration about the pivot: sum_k V^(k) x [u_k qd_k; 0], V^(0) the parent's velocity moved to o_b
            T Vk[6], x[3];
            cross3(V[p], K.o[b], x);
#pragma unroll
            for (int i = 0; i < 3; i++) { Vk[i] = V[p][i]; Vk[3 + i] = V[p][3 + i] + x[i]; cl[b][i] = 0; cl[b][3 + i] = 0; }
#pragma unroll
            for (int k = 0; k < body_ndof[b]; k++) {
                const int d = body_dof0[b] + k;
                const T qd = nu[6 + d];
                const T uq[3] = {K.u[d][0] * qd, K.u[d][1] * qd, K.u[d][2] * qd};
#pragma unroll
                for (int i = 0; i < 3; i++) Vk[i] += uq[i];
                T wx[3], vx[3];
                cross3(Vk, uq, wx);
                cross3(Vk + 3, uq, vx);
#pragma unroll
                for (int i = 0; i < 3; i++) { cl[b][i] += wx[i]; cl[b][3 + i] += vx[i]; }
            }
            // the same at the common origin (pass 3): v_O = v_b - w x o_b
            T y[3];
            cross3(cl[b], K.o[b], y);
#pragma unroll
            for (int i = 0; i < 3; i++) { A.c[b][i] = cl[b][i]; A.c[b][3 + i] = cl[b][3 + i] - y[i]; }
        }
        // inertia of the (merged) body about its pivot
        T Icw[9], c[3];
#pragma unroll
        for (int i = 0; i < 3; i++)
            c[i] = K.R[b][3 * i] * (T)body_com[3 * b] + K.R[b][3 * i + 1] * (T)body_com[3 * b + 1] +
                   K.R[b][3 * i + 2] * (T)body_com[3 * b + 2];
        rotate_inertia(K.R[b], body_inertia + 9 * b, Icw);
        spatial_inertia((T)body_mass[b], c, Icw, IA[b]);
        T h[6];
        symmv(IA[b], Vl[b], h);
        crf(Vl[b], h, pA[b]);
        // gravity on the body COM
        const T mg = -(T)body_mass[b] * (T)P.gravity;
        pA[b][0] -= c[1] * mg;   // (c x F)_x with F = (0,0,mg)
        pA[b][1] -= -c[0] * mg;
        pA[b][5] -= mg;
    }
    // Bullet per-link velocity damping (btMultiBody m_linearDamping / m_angularDamping), per pybullet link
#pragma unroll
    for (int l = 0; l < NLINK; l++) {
        const int b = link_body[l];
        T cp[3], vc[3], Iw[9], wI[3];
#pragma unroll
        for (int i = 0; i < 3; i++)
            cp[i] = K.R[b][3 * i] * (T)link_com[3 * l] + K.R[b][3 * i + 1] * (T)link_com[3 * l + 1] +
                    K.R[b][3 * i + 2] * (T)link_com[3 * l + 2];
        cross3(Vl[b], cp, vc);
#pragma unroll
        for (int i = 0; i < 3; i++) vc[i] += Vl[b][3 + i];
        const T kv = (T)P.lin_damp * (T(1) + sqrt(dot3(vc, vc)));
        const T kw = (T)P.ang_damp * (T(1) + sqrt(dot3(Vl[b], Vl[b])));
        rotate_inertia(K.R[b], link_inertia + 9 * l, Iw);
#pragma unroll
        for (int i = 0; i < 3; i++) wI[i] = Iw[3 * i] * Vl[b][0] + Iw[3 * i + 1] * Vl[b][1] + Iw[3 * i + 2] * Vl[b][2];
        const T m = (T)link_mass[l];
        T F[3], n[3], cxF[3];
#pragma unroll
        for (int i = 0; i < 3; i++) { F[i] = -m * vc[i] * kv; n[i] = -wI[i] * kw; }
        cross3(cp, F, cxF);
#pragma unroll
        for (int i = 0; i < 3; i++) { pA[b][i] -= n[i] + cxF[i]; pA[b][3 + i] -= F[i]; }
    }
    // ---- pass 2: articulated inertias (leaves -> root), about each pivot; hinge columns [u; 0]
#pragma unroll
    for (int b = NB - 1; b >= 1; b--) {
        const int p = body_parent[b], k = body_ndof[b], d0 = body_dof0[b];
        T Ul[3][6], D[9], Di[9], Lf[9], idd[3];
#pragma unroll
        for (int j = 0; j < k; j++) {
            const T* u = K.u[d0 + j];
#pragma unroll
            for (int e = 0; e < 6; e++) Ul[j][e] = IA[b][sidx(e, 0)] * u[0] + IA[b][sidx(e, 1)] * u[1] + IA[b][sidx(e, 2)] * u[2];
        }
#pragma unroll
        for (int i = 0; i < k; i++)
#pragma unroll
            for (int j = 0; j < k; j++) D[3 * i + j] = dot3(K.u[d0 + i], Ul[j]);
#pragma unroll
        for (int j = 0; j < k; j++) {
            T uj = tau[d0 + j] - dot3(K.u[d0 + j], pA[b]);
            if (P.joint_damping) {
                D[4 * j] += (T)P.dt * (T)dof_damping[d0 + j];
                uj -= (T)dof_damping[d0 + j] * nu[6 + d0 + j];
            }
            A.uu[d0 + j] = uj;
        }
        if (k == 1) ldl_small<T, 1>(D, Lf, idd, Di);
        else if (k == 2) ldl_small<T, 2>(D, Lf, idd, Di);
        else ldl_small<T, 3>(D, Lf, idd, Di);
#pragma unroll
        for (int i = 0; i < 9; i++) A.Dinv[b][i] = Di[i];
        // W = U Dinv (6 x k), Y = U L^-T
        T W[3][6], Y[3][6];
#pragma unroll
        for (int j = 0; j < k; j++)
#pragma unroll
            for (int e = 0; e < 6; e++) {
                T s = 0, y = Ul[j][e];
#pragma unroll
                for (int i = 0; i < k; i++) s += Ul[i][e] * Di[3 * i + j];
#pragma unroll
                for (int q = 0; q < j; q++) y -= Lf[3 * j + q] * Y[q][e];
                W[j][e] = s;
                Y[j][e] = y;
            }
        // Ia = IA - sum_j Y_j Y_j^T idd_j ; pa = pA + Ia c + W u
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int cc = r; cc < 6; cc++) {
                T s = IA[b][sidx(r, cc)];
#pragma unroll
                for (int j = 0; j < k; j++) s -= Y[j][r] * idd[j] * Y[j][cc];
                IA[b][sidx(r, cc)] = s;
            }
        T Iac[6], pa[6];
        symmv(IA[b], cl[b], Iac);
#pragma unroll
        for (int e = 0; e < 6; e++) {
            T s = pA[b][e] + Iac[e];
#pragma unroll
            for (int j = 0; j < k; j++) s += W[j][e] * A.uu[d0 + j];
            pa[e] = s;
        }
        // to the parent's pivot: r = o_b - o_p
        T r[3];
#pragma unroll
        for (int i = 0; i < 3; i++) r[i] = K.o[b][i] - K.o[p][i];
        shift_force(r, pa);
        shift_inertia(r, IA[b]);
#pragma unroll
        for (int e = 0; e < 6; e++) pA[p][e] += pa[e];
#pragma unroll
        for (int i = 0; i < 21; i++) IA[p][i] += IA[b][i];
        // U at the common origin for pass 3 and the constraint responses: [U_n + o_b x U_f; U_f]
#pragma unroll
        for (int j = 0; j < k; j++) {
            T x[3];
            cross3(K.o[b], Ul[j] + 3, x);
#pragma unroll
            for (int i = 0; i < 3; i++) { A.U[d0 + j][i] = Ul[j][i] + x[i]; A.U[d0 + j][3 + i] = Ul[j][3 + i]; }
        }
    }
    // ---- base (the torso's pivot is the common origin)
    chol6(IA[0], A.L0);
    T a[NB][6];
#pragma unroll
    for (int i = 0; i < 6; i++) a[0][i] = -pA[0][i];
    chol6_solve(A.L0, a[0]);
    // ---- pass 3: accelerations (common origin)
#pragma unroll
    for (int b = 1; b < NB; b++) {
        const int p = body_parent[b], k = body_ndof[b], d0 = body_dof0[b];
        T ap[6];
#pragma unroll
        for (int e = 0; e < 6; e++) ap[e] = a[p][e] + A.c[b][e];
        T r[3];
#pragma unroll
        for (int j = 0; j < k; j++) {
            T s = A.uu[d0 + j];
#pragma unroll
            for (int e = 0; e < 6; e++) s -= A.U[d0 + j][e] * ap[e];
            r[j] = s;
        }
#pragma unroll
        for (int i = 0; i < k; i++) {
            T s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += A.Dinv[b][3 * i + j] * r[j];
            acc[6 + d0 + i] = s;
        }
#pragma unroll
        for (int e = 0; e < 6; e++) a[b][e] = ap[e];
#pragma unroll
        for (int i = 0; i < k; i++) {
            T S[6];
            motion_col(K, b, d0 + i, S);
#pragma unroll
            for (int e = 0; e < 6; e++) a[b][e] += S[e] * acc[6 + d0 + i];
        }
    }
    T wxv[3];
    cross3(nu, nu + 3, wxv);
#pragma unroll
    for (int i = 0; i < 3; i++) { acc[i] = a[0][i]; acc[3 + i] = a[0][3 + i] + wxv[i]; }
}

// Response of the generalised velocity to a generalised impulse: spatial forces fa on body ba and fb on
// body bb (bb < 0: none) plus a unit joint impulse `jsign` on dof jd (jd < 0: none).  out[NV] = M^-1 J^T.
template <typename T>
__device__ inline void impulse_response(const Kin<T>& K, const Aba<T>& A, int ba, const T* fa, int bb, const T* fb,
                                        int jd, T jsign, T* out) {
    T pA[NB][6];
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int e = 0; e < 6; e++) pA[b][e] = 0;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        if (b == ba) {
#pragma unroll
            for (int e = 0; e < 6; e++) pA[b][e] -= fa[e];
        }
        if (b == bb) {
#pragma unroll
            for (int e = 0; e < 6; e++) pA[b][e] -= fb[e];
        }
    }
    T uq[NDOF];
#pragma unroll
    for (int b = NB - 1; b >= 1; b--) {
        const int p = body_parent[b], k = body_ndof[b], d0 = body_dof0[b];
#pragma unroll
        for (int j = 0; j < k; j++) {
            T S[6];
            motion_col(K, b, d0 + j, S);
            T s = (d0 + j == jd) ? jsign : T(0);
#pragma unroll
            for (int e = 0; e < 6; e++) s -= S[e] * pA[b][e];
            uq[d0 + j] = s;
        }
#pragma unroll
        for (int e = 0; e < 6; e++) {
            T s = pA[b][e];
#pragma unroll
            for (int i = 0; i < k; i++) {
                T w = 0;
#pragma unroll
                for (int j = 0; j < k; j++) w += A.Dinv[b][3 * i + j] * uq[d0 + j];
                s += A.U[d0 + i][e] * w;
            }
            pA[p][e] += s;
        }
    }
    T a[NB][6];
#pragma unroll
    for (int e = 0; e < 6; e++) a[0][e] = -pA[0][e];
    chol6_solve(A.L0, a[0]);
#pragma unroll
    for (int e = 0; e < 6; e++) out[e] = a[0][e];
#pragma unroll
    for (int b = 1; b < NB; b++) {
        const int p = body_parent[b], k = body_ndof[b], d0 = body_dof0[b];
        T r[3];
#pragma unroll
        for (int j = 0; j < k; j++) {
            T s = uq[d0 + j];
#pragma unroll
            for (int e = 0; e < 6; e++) s -= A.U[d0 + j][e] * a[p][e];
            r[j] = s;
        }
#pragma unroll
        for (int e = 0; e < 6; e++) a[b][e] = a[p][e];
#pragma unroll
        for (int i = 0; i < k; i++) {
            T s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += A.Dinv[b][3 * i + j] * r[j];
            out[6 + d0 + i] = s;
            T S[6];
            motion_col(K, b, d0 + i, S);
#pragma unroll
            for (int e = 0; e < 6; e++) a[b][e] += S[e] * s;
        }
    }
}

// J row (NV) for spatial force f at body b: base part = f, dof part = f . S_k on the path to the root
template <typename T>
__device__ inline void add_row_jacobian(const Kin<T>& K, int b, const T* f, T sgn, T* J) {
#pragma unroll
    for (int e = 0; e < 6; e++) J[e] += sgn * f[e];
#pragma unroll
    for (int bb = NB - 1; bb >= 1; bb--) {
        // is bb on the path root..b ?
        bool on = false;
        int x = b;
#pragma unroll
        for (int h = 0; h < NB; h++) {
            if (x == bb) on = true;
            x = x > 0 ? body_parent[x] : 0;
        }
        if (on) {
#pragma unroll
            for (int k = 0; k < body_ndof[bb]; k++) {
                const int d = body_dof0[bb] + k;
                T S[6];
                motion_col(K, bb, d, S);
                T s = 0;
#pragma unroll
                for (int e = 0; e < 6; e++) s += f[e] * S[e];
                J[6 + d] += sgn * s;
            }
        }
    }
}

// ------------------------------------------------------------------------------------- collision
// Ericson 5.1.9 closest points between segments (same algorithm as the oracle)
template <typename T>
__device__ inline void seg_seg(const T* p1, const T* q1, const T* p2, const T* q2, T* c1, T* c2) {
    T d1[3], d2[3], r[3];
#pragma unroll
    for (int i = 0; i < 3; i++) { d1[i] = q1[i] - p1[i]; d2[i] = q2[i] - p2[i]; r[i] = p1[i] - p2[i]; }
    T a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    T s, t;
    const T EPS = (T)1e-12;
    if (a <= EPS && e <= EPS) { s = t = 0; }
    else if (a <= EPS) { s = 0; t = clampT(f * prcp_geo(e), T(0), T(1)); }
    else {
        T c = dot3(d1, r);
        const T ia = prcp_geo(a);
        if (e <= EPS) { t = 0; s = clampT(-c * ia, T(0), T(1)); }
        else {
            T b = dot3(d1, d2), den = a * e - b * b;
            s = (den > EPS) ? clampT((b * f - c * e) * prcp_geo(den), T(0), T(1)) : T(0);
            t = (b * s + f) * prcp_geo(e);
            if (t < 0) { t = 0; s = clampT(-c * ia, T(0), T(1)); }
            else if (t > 1) { t = 1; s = clampT((b - c) * ia, T(0), T(1)); }
        }
    }
#pragma unroll
    for (int i = 0; i < 3; i++) { c1[i] = p1[i] + d1[i] * s; c2[i] = p2[i] + d2[i] * t; }
}

template <typename T>
__device__ inline void plane_space(const T* n, T* p, T* q) {  // btPlaneSpace1
    if (fabs(n[2]) > (T)0.7071067811865475244) {
        T a = n[1] * n[1] + n[2] * n[2], k = prsqrt(a);
        p[0] = 0; p[1] = -n[2] * k; p[2] = n[1] * k;
        q[0] = a * k; q[1] = -n[0] * p[2]; q[2] = n[0] * p[1];
    } else {
        T a = n[0] * n[0] + n[1] * n[1], k = prsqrt(a);
        p[0] = -n[1] * k; p[1] = n[0] * k; p[2] = 0;
        q[0] = -n[2] * p[1]; q[1] = n[2] * p[0]; q[2] = a * k;
    }
}

// ------------------------------------------------------------------------------------- one substep
// st: lane physics state in Real (47); rows: per-lane scratch; returns contact-overflow flag.
template <typename T>
__device__ inline int substep(const PhysParams& P, T* st, const T* tau, const Lane<T>& rows) {
    const T dt = (T)P.dt;
    Kin<T> K;
    forward_kinematics(st + 3, st + 13, K);
    T nu[NV];
#pragma unroll
    for (int i = 0; i < 3; i++) { nu[i] = st[10 + i]; nu[3 + i] = st[7 + i]; }
#pragma unroll
    for (int j = 0; j < NDOF; j++) nu[6 + j] = st[30 + j];

    Aba<T> A;
    T acc[NV];
    aba(P, K, nu, tau, A, acc);
    const T vmax = (T)P.max_coord_vel;
#pragma unroll
    for (int i = 0; i < NV; i++) nu[i] = clampT(nu[i] + dt * acc[i], -vmax, vmax);

    // ---- rows: limits [0, nl), normals [LIM, LIM+nc), friction [LIM+MAXC, LIM+MAXC+2nc)
    auto R = [&](int row, int e) -> T& { return rows.at(row * ROW_STRIDE + e); };
    enum { E_J = 0, E_M = NV, E_B = 2 * NV, E_LO, E_HI, E_LAM, E_MEFF, E_MU };
    int nl = 0;
#pragma unroll
    for (int j = 0; j < NDOF; j++) {
        const T q = st[13 + j];
#pragma unroll
        for (int side = 0; side < 2; side++) {
            const T pen = side == 0 ? q - (T)dof_lo[j] : (T)dof_hi[j] - q;
            if (pen <= 0) {
                const T sg = side == 0 ? T(1) : T(-1);
                T M[NV];
                impulse_response(K, A, -1, (const T*)nullptr, -1, (const T*)nullptr, j, sg, M);
                const int row = nl++;
                T jm = sg * M[6 + j];
#pragma unroll
                for (int e = 0; e < NV; e++) { R(row, E_J + e) = (e == 6 + j) ? sg : T(0); R(row, E_M + e) = M[e]; }
                R(row, E_B) = pen > (T)P.split_pen ? -pen * (T)P.erp_limit / dt : T(0);
                R(row, E_LO) = 0;
                R(row, E_HI) = (T)P.limit_max_impulse;
                R(row, E_LAM) = 0;
                R(row, E_MEFF) = T(1) / jm;
            }
        }
    }
    // ---- contacts: detect (unrolled, compile-time geometry) into the scratch list, then build rows
    auto C = [&](int c, int e) -> T& { return rows.at(MAXROWS * ROW_STRIDE + c * CON_STRIDE + e); };
    int nc = 0, overflow = 0;
    const int maxc = P.max_contacts;
    T gp1[NGEOM][3], gp2[NGEOM][3];
#pragma unroll
    for (int g = 0; g < NGEOM; g++) {
        const int b = geom_body[g];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            gp1[g][i] = K.o[b][i] + K.R[b][3 * i] * (T)geom_p1[3 * g] + K.R[b][3 * i + 1] * (T)geom_p1[3 * g + 1] +
                        K.R[b][3 * i + 2] * (T)geom_p1[3 * g + 2];
            gp2[g][i] = K.o[b][i] + K.R[b][3 * i] * (T)geom_p2[3 * g] + K.R[b][3 * i + 1] * (T)geom_p2[3 * g + 1] +
                        K.R[b][3 * i + 2] * (T)geom_p2[3 * g + 2];
        }
    }
    const T basez = st[2];
    auto push = [&](int ba, const T* pa, int bb, const T* pb, const T* n, T d) {
        if (nc >= maxc) { overflow = 1; return; }
        C(nc, 0) = (T)ba; C(nc, 1) = (T)bb;
#pragma unroll
        for (int i = 0; i < 3; i++) { C(nc, 2 + i) = pa[i]; C(nc, 5 + i) = pb[i]; C(nc, 8 + i) = n[i]; }
        C(nc, 11) = d;
        nc++;
    };
    // ground: every sphere (1 point) and capsule end (2 points) below the breaking threshold
#pragma unroll
    for (int g = 0; g < NGEOM; g++) {
#pragma unroll
        for (int e = 0; e < (geom_type[g] == 0 ? 1 : 2); e++) {
            const T* p = e == 0 ? gp1[g] : gp2[g];
            const T d = basez + p[2] - (T)geom_r[g];
            if (d < (T)P.contact_thresh) {
                T pa[3] = {p[0], p[1], p[2] - (T)geom_r[g]};
                T n[3] = {0, 0, 1};
                push(geom_body[g], pa, -1, pa, n, d);
            }
        }
    }
    if (P.self_collision) {
#pragma unroll
        for (int k = 0; k < NPAIR; k++) {
            const int ga = pair_a[k], gb = pair_b[k];
            T ca[3], cb[3], dv[3];
            seg_seg(gp1[ga], gp2[ga], gp1[gb], gp2[gb], ca, cb);
#pragma unroll
            for (int i = 0; i < 3; i++) dv[i] = ca[i] - cb[i];
            const T dist = sqrt(dot3(dv, dv));
            const T ra = (T)geom_r[ga], rb = (T)geom_r[gb];
            const T d = dist - ra - rb;
            if (d < (T)P.contact_thresh && dist > (T)1e-9) {
                T n[3], pa[3], pb[3];
                const T idist = T(1) / dist;
#pragma unroll
                for (int i = 0; i < 3; i++) {
                    n[i] = dv[i] * idist;
                    pa[i] = ca[i] - ra * n[i];
                    pb[i] = cb[i] + rb * n[i];
                }
                push(geom_body[ga], pa, geom_body[gb], pb, n, d);
            }
        }
    }
    // rows for each contact: normal (lambda >= 0) + two friction directions (box bounds +-mu*lambda_n)
#pragma unroll 1
    for (int c = 0; c < nc; c++) {
        const int ba = (int)C(c, 0), bb = (int)C(c, 1);
        T pa[3], pb[3], n[3];
#pragma unroll
        for (int i = 0; i < 3; i++) { pa[i] = C(c, 2 + i); pb[i] = C(c, 5 + i); n[i] = C(c, 8 + i); }
        const T d = C(c, 11);
        const T mu = bb >= 0 ? (T)P.mu_self : (T)P.mu_ground;
        // relative velocity of the contact points at nu* (friction direction)
        T Va[6], Vb[6];
#pragma unroll
        for (int e = 0; e < 6; e++) { Va[e] = nu[e]; Vb[e] = nu[e]; }
#pragma unroll
        for (int b2 = 1; b2 < NB; b2++) {
            bool ona = false, onb = false;
            int xa = ba, xb = bb < 0 ? 0 : bb;
#pragma unroll
            for (int h = 0; h < NB; h++) {
                if (xa == b2) ona = true;
                if (xb == b2) onb = true;
                xa = xa > 0 ? body_parent[xa] : 0;
                xb = xb > 0 ? body_parent[xb] : 0;
            }
#pragma unroll
            for (int k = 0; k < body_ndof[b2]; k++) {
                T S[6];
                motion_col(K, b2, body_dof0[b2] + k, S);
                const T qd = nu[6 + body_dof0[b2] + k];
#pragma unroll
                for (int e = 0; e < 6; e++) {
                    if (ona) Va[e] += S[e] * qd;
                    if (onb) Vb[e] += S[e] * qd;
                }
            }
        }
        T vr[3], va[3], vb[3] = {0, 0, 0};
        cross3(Va, pa, va);
#pragma unroll
        for (int i = 0; i < 3; i++) va[i] += Va[3 + i];
        if (bb >= 0) {
            cross3(Vb, pb, vb);
#pragma unroll
            for (int i = 0; i < 3; i++) vb[i] += Vb[3 + i];
        }
#pragma unroll
        for (int i = 0; i < 3; i++) vr[i] = va[i] - vb[i];
        const T vn = dot3(vr, n);
        T lat[3], t1[3], t2[3];
#pragma unroll
        for (int i = 0; i < 3; i++) lat[i] = vr[i] - n[i] * vn;
        const T l2 = dot3(lat, lat);
        if (l2 > (T)1e-12) {
            const T il = T(1) / sqrt(l2);
#pragma unroll
            for (int i = 0; i < 3; i++) t1[i] = lat[i] * il;
            cross3(t1, n, t2);
        } else {
            plane_space(n, t1, t2);
        }
#pragma unroll 1
        for (int f = 0; f < 3; f++) {
            const T* dir = f == 0 ? n : (f == 1 ? t1 : t2);
            T fa[6], fb[6], J[NV], M[NV];
            cross3(pa, dir, fa); fa[3] = dir[0]; fa[4] = dir[1]; fa[5] = dir[2];
            cross3(pb, dir, fb); fb[3] = -dir[0]; fb[4] = -dir[1]; fb[5] = -dir[2];
            fb[0] = -fb[0]; fb[1] = -fb[1]; fb[2] = -fb[2];   // fb = -[pb x dir; dir]
#pragma unroll
            for (int e = 0; e < NV; e++) J[e] = 0;
            add_row_jacobian(K, ba, fa, T(1), J);
            if (bb >= 0) add_row_jacobian(K, bb, fb, T(1), J);
            impulse_response(K, A, ba, fa, bb, fb, -1, T(0), M);
            T jm = 0;
            const int row = f == 0 ? MAX_LIMIT_ROWS + c : MAX_LIMIT_ROWS + MAXC + 2 * c + (f - 1);
#pragma unroll
            for (int e = 0; e < NV; e++) { R(row, E_J + e) = J[e]; R(row, E_M + e) = M[e]; jm += J[e] * M[e]; }
            R(row, E_B) = f == 0 ? (d > 0 ? -d / dt : (d > (T)P.split_pen ? -d * (T)P.erp_contact / dt : T(0))) : T(0);
            R(row, E_LO) = 0;
            R(row, E_HI) = (T)1e10;
            R(row, E_LAM) = 0;
            R(row, E_MEFF) = T(1) / jm;
            R(row, E_MU) = mu;
        }
    }

    // ---- PGS (btMultiBodyConstraintSolver order: limits, normals, frictions)
    auto solve_row = [&](int row) {
        T jv = 0;
#pragma unroll
        for (int e = 0; e < NV; e++) jv += R(row, E_J + e) * nu[e];
        const T lam = R(row, E_LAM);
        const T lnew = clampT(lam + R(row, E_MEFF) * (R(row, E_B) - jv), R(row, E_LO), R(row, E_HI));
        const T dl = lnew - lam;
        R(row, E_LAM) = lnew;
#pragma unroll
        for (int e = 0; e < NV; e++) nu[e] += R(row, E_M + e) * dl;
    };
#pragma unroll 1
    for (int it = 0; it < P.iters; it++) {
#pragma unroll 1
        for (int r = 0; r < nl; r++) solve_row(r);
#pragma unroll 1
        for (int c = 0; c < nc; c++) solve_row(MAX_LIMIT_ROWS + c);
#pragma unroll 1
        for (int c = 0; c < nc; c++) {
            const T ln = R(MAX_LIMIT_ROWS + c, E_LAM);
#pragma unroll 1
            for (int f = 0; f < 2; f++) {
                const int frow = MAX_LIMIT_ROWS + MAXC + 2 * c + f;
                const T mu = R(frow, E_MU);
                R(frow, E_LO) = -mu * ln;
                R(frow, E_HI) = mu * ln;
                solve_row(frow);
            }
        }
    }

    // ---- integrate positions (semi-implicit Euler; base orientation by Bullet's exponential map)
#pragma unroll
    for (int i = 0; i < 3; i++) { st[10 + i] = nu[i]; st[7 + i] = nu[3 + i]; st[i] += dt * nu[3 + i]; }
#pragma unroll
    for (int j = 0; j < NDOF; j++) { st[30 + j] = nu[6 + j]; st[13 + j] += dt * nu[6 + j]; }
    {
        const T* w = st + 10;
        T ang = sqrt(dot3(w, w)), ax[3];
        const T thr = (T)(0.25 * 3.14159265358979323846);
        if (ang * dt > thr) ang = thr / dt;
        if (ang < (T)0.001) {
            const T s = (T)0.5 * dt - dt * dt * dt * (T)0.020833333333 * ang * ang;
#pragma unroll
            for (int i = 0; i < 3; i++) ax[i] = w[i] * s;
        } else {
            const T s = sin((T)0.5 * ang * dt) / ang;
#pragma unroll
            for (int i = 0; i < 3; i++) ax[i] = w[i] * s;
        }
        const T dw = cos((T)0.5 * ang * dt);
        T* q = st + 3;
        T nq[4] = {dw * q[0] + ax[0] * q[3] + ax[1] * q[2] - ax[2] * q[1],
                   dw * q[1] + ax[1] * q[3] + ax[2] * q[0] - ax[0] * q[2],
                   dw * q[2] + ax[2] * q[3] + ax[0] * q[1] - ax[1] * q[0],
                   dw * q[3] - ax[0] * q[0] - ax[1] * q[1] - ax[2] * q[2]};
        const T nn = T(1) / sqrt(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
        for (int i = 0; i < 4; i++) q[i] = nq[i] * nn;
    }
    return overflow;
}

// world positions (relative to base COM) of the 33 parts; floor handled by the caller
template <typename T>
__device__ inline void part_positions(const Kin<T>& K, T (*pp)[3]) {
#pragma clang fp contract(on)   // per-expression fusion only: the same frames in every inlining context
#pragma unroll
    for (int k = 0; k < NPART; k++) {
        const int b = part_body[k];
        if (b < 0) { pp[k][0] = pp[k][1] = pp[k][2] = 0; continue; }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            T v = fmak(K.R[b][3 * i], part_p[3 * k], K.o[b][i]);
            v = fmak(K.R[b][3 * i + 1], part_p[3 * k + 1], v);
            pp[k][i] = fmak(K.R[b][3 * i + 2], part_p[3 * k + 2], v);
        }
    }
}

}  // namespace hk

// physics_group.h - cooperative (16 lanes per env) version of the humanoid substep.
//
// MI355X mapping: a 64-lane wavefront = 4 envs x 16 lanes; each env's working set lives in LDS
// (struct GroupLDS, ~10 KB fp32), so a CU holds 16 envs (4 blocks of one wave: one wave per SIMD, the CU's
// 160 KB; the kernel holds 512 VGPRs and spills 26 of them, 76 B of scratch per lane, tests/test_cpu_isa.py).
// Same algorithm and operation order as physics.h (the per-lane kernel,
// kept as the reference-shaped variant) except for the order of floating-point sums inside the
// element-parallel ABA backward pass and the 16-lane DPP reductions of the PGS row products.
//
//   FK              every lane (registers), lane 0 publishes R/o/u to LDS
//   ABA pass 1      lane b = body b: velocity, bias acceleration, spatial inertia, bias force
//   ABA pass 2      by tree level (4 steps, one body per 4-lane group), children summed by the parent
//   ABA pass 3      base on every lane, then by tree level (root -> leaves), groups integrate their dofs
//   limits/contacts lane-parallel candidate tests, ballot-compacted in the oracle's order
//   rows            one constraint row per lane: Jacobian + test-impulse response M^-1 J^T
//   PGS             rows in Bullet order; J.nu over the 16 lanes by DPP row_ror reductions
#pragma once
#include <utility>

#include "physics.h"
#include "terrain.h"

namespace hk {

constexpr int GL = 16;                       // lanes per env
// contacts: the first MAXC_LDS of an env's contact list live in LDS, the rest (rare: a lying humanoid with
// many self contacts) in the env's slice of its block's global spill region; the list holds every candidate
// (MAXC_G = 29 ground points + 24 heightfield ridge points + 66 geom pairs), so nothing is ever dropped
constexpr int MAXC_LDS = 16;
constexpr int MAXC_G = MAXC;                 // = NCAND_ALL (physics.h)
constexpr int CW = 12;                       // contact entry: ba, bb, pa[3], pb[3], n[3], d
// limit rows: one per violated side, and a dof violates at most one side (lo < hi for every dof).  17 slots instead
// of 34 also keep the per-env LDS stride off a multiple of 64 dwords (with 30 row slots, 34 made it exactly 2560
// dwords: the 4 envs of a wave then hit the same LDS bank on every same-field access)
constexpr int MAXL_G = NDOF;
constexpr bool limits_proper() {
    for (int d = 0; d < NDOF; d++)
        if (!(dof_lo[d] < dof_hi[d])) return false;
    return true;
}
static_assert(limits_proper(), "a dof with lo >= hi could violate both sides");
constexpr int MAXR_G = NDOF + 3 * MAXC_G;    // rows of one env: limits + (normal + 2 frictions) per contact
// constraint row layout (T units): J and M^-1 J^T interleaved per dof ([2q] = J_q, [2q+1] = (M^-1 J^T)_q), a
// zero pair (read by the lanes without a second velocity component), then two 16-byte scalar quads:
// b, hi, lambda, meff = 1/(J M^-1 J^T) and mu, q = meff * J . (M^-1 J^T of the predecessor row), next3, next3_ln
// (ints).
// lo is 0 for every row type and not stored.
constexpr int RO_Z = 2 * NV;          // zero pair
constexpr int RO_S0 = 2 * NV + 2;     // b, hi, lam, meff
constexpr int RO_S1 = 2 * NV + 6;     // mu, c, next3, next3_ln
constexpr int RO_LAM = RO_S0 + 2;
constexpr int RW = 2 * NV + 10;
static_assert(RO_S0 % 4 == 0 && RW % 4 == 0, "16-byte scalar quads");
constexpr int NCAND_GROUND = [] { int n = 0; for (int g = 0; g < NGEOM; g++) n += geom_type[g] == 0 ? 1 : 2; return n; }();
constexpr int NCAND = NCAND_GROUND + NPAIR;

// the model tables the cooperative kernel indexes by lane-varying body / dof / link / geom / candidate
// (compile-time-indexed constants come from model_gen.h directly)
template <typename T>
struct ModelTab {
    int dof0[NB], ndof[NB], nlink[NB], link0[NB];
    T mass[NB], com[NB][3], inertia[NB][9];
    T lo[NDOF], hi[NDOF], damp[NDOF];
    T lmass[NLINK], lcom[NLINK][3], linertia[NLINK][9];
    int gbody[NGEOM];
    T gr[NGEOM], gp1[NGEOM][3], gp2[NGEOM][3];
    int cand[NCAND];                     // a | b << 16; ground: (geom, -1 - endpoint), pair: (ga, gb)
    T gbr[NGEOM];                        // bounding-sphere radius about the segment midpoint: |p2-p1|/2 + r
    int act_dof[NACT];
    float act_gain[NACT];
    double act_gain_d[NACT];
};
__device__ inline int cand_a(int v) { return v & 0xffff; }
__device__ inline int cand_b(int v) { return v >> 16; }

constexpr double csqrt(double x) {   // constexpr Newton square root (model constants only)
    if (x <= 0) return 0;
    double r = x > 1 ? x : 1;
    for (int i = 0; i < 100; i++) r = 0.5 * (r + x / r);
    return r;
}

// ONX[x] bit b: body x is body b or one of its ancestors (x >= 1).  Indexed by the compile-time x of an
// unrolled loop and shifted by the lane-varying b, so "is x on b's path" costs one shift and no memory load
// (a lane-varying table lookup is a vector-memory load with its full latency on the dependency chain).
constexpr unsigned onx_mask(int x) {
    unsigned m = 0;
    for (int b = 0; b < NB; b++)
        for (int y = b; y > 0; y = body_parent[y])
            if (y == x) m |= 1u << b;
    return m;
}
__device__ inline bool on_path(int x, int b) {   // b < 0: no body
    return b >= 0 && ((onx_mask(x) >> (b & 31)) & 1u);
}
// small per-body / per-geom integers packed into 64-bit constants (field width W bits, entry i at bit W*i):
// a lane-indexed lookup is a shift and a mask instead of a vector-memory load
template <int W, int N>
constexpr unsigned long long pack_bits(const int (&v)[N], int off = 0) {
    unsigned long long m = 0;
    for (int i = 0; i < N - off && W * i < 64; i++) m |= (unsigned long long)v[off + i] << (W * i);
    return m;
}
__device__ inline int body_ndof_l(int b) { return (int)((pack_bits<2>(body_ndof) >> (2 * b)) & 3u); }
__device__ inline int body_dof0_l(int b) { return (int)((pack_bits<5>(body_dof0) >> (5 * b)) & 31u); }
// tree depth (torso 0) and parent (torso: itself) of each body, for lane-indexed lookups
struct TreeInfo { int depth[NB], parent0[NB], maxdepth; };
constexpr TreeInfo tree_info() {
    TreeInfo t{};
    t.maxdepth = 0;
    for (int b = 0; b < NB; b++) {
        int d = 0;
        for (int y = b; y > 0; y = body_parent[y]) d++;
        t.depth[b] = d;
        t.parent0[b] = b > 0 ? body_parent[b] : 0;
        t.maxdepth = d > t.maxdepth ? d : t.maxdepth;
    }
    return t;
}
constexpr TreeInfo TREE = tree_info();
static_assert(TREE.maxdepth < 8 && NB <= 21, "3-bit depth codes");
// (S^T IA S + dt damping)^-1 of body b packed k x k (row major) from DINV_OFF[b]: sum k^2 = 35 words, not NB x 9
struct DinvOff { int off[NB + 1]; };
constexpr DinvOff dinv_off() {
    DinvOff r{};
    r.off[0] = 0;
    for (int b = 0; b < NB; b++) r.off[b + 1] = r.off[b] + body_ndof[b] * body_ndof[b];
    return r;
}
constexpr DinvOff DINV = dinv_off();
constexpr int DINV_N = DINV.off[NB];
__device__ inline int body_depth_l(int b) { return (int)((pack_bits<3>(TREE.depth) >> (3 * b)) & 7u); }
__device__ inline int body_parent_l(int b) { return (int)((pack_bits<4>(TREE.parent0) >> (4 * b)) & 15u); }
// the hinge dofs on body b's root path (its ancestors' and its own, root to leaf = ascending dof order) as at most two
// contiguous runs: [0, e1) and [s2, s2 + len - e1)
struct PathRuns { int e1[NB], s2[NB], len[NB]; bool ok; };
constexpr PathRuns path_runs() {
    PathRuns r{};
    r.ok = true;
    for (int b = 0; b < NB; b++) {
        bool on[NDOF] = {};
        int len = 0;
        for (int y = b; y > 0; y = body_parent[y])
            for (int k = 0; k < body_ndof[y]; k++) { on[body_dof0[y] + k] = true; len++; }
        int e1 = 0;
        while (e1 < NDOF && on[e1]) e1++;
        int s2 = e1;
        while (s2 < NDOF && !on[s2]) s2++;
        if (len == e1) s2 = 0;
        for (int d = 0; d < NDOF; d++)
            if (on[d] != (d < e1 || (d >= s2 && d < s2 + len - e1))) r.ok = false;
        r.e1[b] = e1; r.s2[b] = s2; r.len[b] = len;
    }
    return r;
}
constexpr PathRuns PATHS = path_runs();
static_assert(PATHS.ok, "every root path is at most two contiguous dof runs, the first from dof 0");
constexpr int PATH_LEN_MAX = [] { int m = 0; for (int b = 0; b < NB; b++) m = PATHS.len[b] > m ? PATHS.len[b] : m; return m; }();
static_assert(PATH_LEN_MAX < 8 && NDOF < 32, "3-bit path lengths, 5-bit dof indices");
// the longest parent path (a body's parent velocity sums it)
constexpr int PPATH_MAX = [] { int m = 0; for (int b = 1; b < NB; b++) m = PATHS.len[body_parent[b]] > m ? PATHS.len[body_parent[b]] : m; return m; }();
__device__ inline int path_e1_l(int b) { return (int)((pack_bits<3>(PATHS.e1) >> (3 * b)) & 7u); }
__device__ inline int path_s2_l(int b) { return (int)((pack_bits<5>(PATHS.s2) >> (5 * b)) & 31u); }
__device__ inline int path_len_l(int b) { return (int)((pack_bits<3>(PATHS.len) >> (3 * b)) & 7u); }
struct LinkInfo { int nlink[NB], link0[NB]; };
constexpr LinkInfo link_info() {
    LinkInfo r{};
    for (int b = 0; b < NB; b++) { r.nlink[b] = 0; r.link0[b] = 0; }
    for (int l = NLINK - 1; l >= 0; l--) { r.nlink[link_body[l]]++; r.link0[link_body[l]] = l; }
    return r;
}
constexpr LinkInfo LINKS = link_info();
__device__ inline int body_nlink_l(int b) { return (int)((pack_bits<2>(LINKS.nlink) >> (2 * b)) & 3u); }
__device__ inline int body_link0_l(int b) { return (int)((pack_bits<4>(LINKS.link0) >> (4 * b)) & 15u); }
struct DofBodies { int b[NDOF]; };
constexpr DofBodies dof_bodies() {
    DofBodies r{};
    for (int x = 0; x < NB; x++)
        for (int k = 0; k < body_ndof[x]; k++) r.b[body_dof0[x] + k] = x;
    return r;
}
constexpr DofBodies DOFB = dof_bodies();
static_assert(NB <= 16 && NDOF <= 32, "4-bit body codes, two constants");
constexpr unsigned long long DOFB_LO = pack_bits<4>(DOFB.b), DOFB_HI = pack_bits<4>(DOFB.b, 16);
__device__ inline int dof_body_l(int d) {   // the body dof d moves: d < 16 from one constant, d >= 16 the other
    return d < 16 ? (int)((DOFB_LO >> (4 * (d & 15))) & 15u) : (int)((DOFB_HI >> (4 * (d - 16))) & 15u);
}
__device__ inline int geom_body_l(int g) {   // g < 16 from one constant, g = 16 the other
    return g < 16 ? (int)((pack_bits<4>(geom_body) >> (4 * (g & 15))) & 15u) : geom_body[16];
}
// geom radius: a 3-bit code per geom (7 distinct radii) selects among exact compile-time constants
struct RadiusCodes { int code[NGEOM]; double val[8]; int n; };
constexpr RadiusCodes radius_codes() {
    RadiusCodes r{};
    r.n = 0;
    for (int g = 0; g < NGEOM; g++) {
        int c = -1;
        for (int i = 0; i < r.n; i++) if (r.val[i] == geom_r[g]) c = i;
        if (c < 0) { c = r.n; r.val[r.n++] = geom_r[g]; }
        r.code[g] = c;
    }
    return r;
}
constexpr RadiusCodes RCODES = radius_codes();
static_assert(RCODES.n <= 8, "3-bit radius codes");
template <typename T>
__device__ __attribute__((always_inline)) inline T geom_r_l(int g) {
    const int c = (int)((pack_bits<3>(RCODES.code) >> (3 * g)) & 7u);
    T r = (T)RCODES.val[0];
#pragma unroll
    for (int i = 1; i < RCODES.n; i++) r = c == i ? (T)RCODES.val[i] : r;
    return r;
}

// contact candidates per (round, lane): 16-bit descriptors packed four lanes per 64-bit constant, so a
// lane-indexed candidate costs a few selects and shifts and neither a table load (whose latency sat on the
// chain of every round of every substep) nor registers held across the substep loop
constexpr int CC_GROUND = (NCAND_GROUND + 15) / 16, CC_PAIR = (NPAIR + 15) / 16;
struct CandDesc { unsigned long long g[CC_GROUND][4], p[CC_PAIR][4]; };
constexpr CandDesc cand_desc() {
    CandDesc d{};
    int gl[NCAND_GROUND] = {}, el[NCAND_GROUND] = {}, c = 0;
    for (int g = 0; g < NGEOM; g++)
        for (int e = 0; e < (geom_type[g] == 0 ? 1 : 2); e++) { gl[c] = g; el[c] = e; c++; }
    for (int r = 0; r < CC_GROUND; r++)
        for (int l = 0; l < 16; l++) {
            const int k = 16 * r + l;   // geom | endpoint << 5 | body << 6; 0xffff: none
            const unsigned long long v = k < NCAND_GROUND ? (unsigned)(gl[k] | el[k] << 5 | geom_body[gl[k]] << 6) : 0xffffu;
            d.g[r][l >> 2] |= v << (16 * (l & 3));
        }
    for (int r = 0; r < CC_PAIR; r++)
        for (int l = 0; l < 16; l++) {
            const int k = 16 * r + l;   // ga | gb << 5; 0xffff: none
            const unsigned long long v = k < NPAIR ? (unsigned)(pair_a[k] | pair_b[k] << 5) : 0xffffu;
            d.p[r][l >> 2] |= v << (16 * (l & 3));
        }
    return d;
}
constexpr CandDesc CDESC = cand_desc();
// heightfield ground: lane l of an env takes capsule l (geom order) for the ridge contacts (terrain.h)
constexpr int NCAPS = [] { int n = 0; for (int g = 0; g < NGEOM; g++) n += geom_type[g] == 0 ? 0 : 1; return n; }();
static_assert(NCAPS <= 16 && NCAPS * RIDGE_MAX + NCAND_GROUND + NPAIR == MAXC, "one capsule per lane; capacity");
struct CapDesc { unsigned long long c[4]; };
constexpr CapDesc cap_desc() {
    CapDesc d{};
    int l = 0;
    for (int g = 0; g < NGEOM; g++)
        if (geom_type[g] != 0) { d.c[l >> 2] |= (unsigned long long)(unsigned)(g | geom_body[g] << 6) << (16 * (l & 3)); l++; }
    for (; l < 16; l++) d.c[l >> 2] |= 0xffffull << (16 * (l & 3));
    return d;
}
constexpr CapDesc CAPDESC = cap_desc();
__device__ __attribute__((always_inline)) inline int lane16(int l, unsigned long long c0, unsigned long long c1,
                                                            unsigned long long c2, unsigned long long c3) {
    const int q = l >> 2;
    const unsigned long long c = q == 0 ? c0 : (q == 1 ? c1 : (q == 2 ? c2 : c3));
    return (int)((c >> (16 * (l & 3))) & 0xffffu);
}
// bounding radius |p2 - p1| / 2 + r: a 4-bit code per geom (10 distinct values) over exact constants
struct BrCodes { int code[NGEOM]; double val[16]; int n; };
constexpr BrCodes br_codes() {
    BrCodes r{};
    r.n = 0;
    for (int g = 0; g < NGEOM; g++) {
        double h2 = 0;
        for (int i = 0; i < 3; i++) h2 += (geom_p2[3 * g + i] - geom_p1[3 * g + i]) * (geom_p2[3 * g + i] - geom_p1[3 * g + i]);
        const double v = 0.5 * csqrt(h2) + geom_r[g];
        int c = -1;
        for (int i = 0; i < r.n; i++) if (r.val[i] == v) c = i;
        if (c < 0) { c = r.n; r.val[r.n++] = v; }
        r.code[g] = c;
    }
    return r;
}
constexpr BrCodes BRCODES = br_codes();
static_assert(BRCODES.n <= 16, "4-bit bounding-radius codes");
template <typename T>
__device__ __attribute__((always_inline)) inline T geom_br_l(int g) {
    const int c = g < 16 ? (int)((pack_bits<4>(BRCODES.code) >> (4 * (g & 15))) & 15u) : BRCODES.code[16];
    T r = (T)BRCODES.val[0];
#pragma unroll
    for (int i = 1; i < BRCODES.n; i++) r = c == i ? (T)BRCODES.val[i] : r;
    return r;
}

template <typename T>
constexpr ModelTab<T> make_tab() {
    ModelTab<T> m{};
    for (int b = 0; b < NB; b++) {
        m.dof0[b] = body_dof0[b]; m.ndof[b] = body_ndof[b];
        m.mass[b] = (T)body_mass[b];
        for (int i = 0; i < 3; i++) m.com[b][i] = (T)body_com[3 * b + i];
        for (int i = 0; i < 9; i++) m.inertia[b][i] = (T)body_inertia[9 * b + i];
        m.nlink[b] = 0; m.link0[b] = -1;
    }
    for (int l = 0; l < NLINK; l++) {
        const int b = link_body[l];
        if (m.link0[b] < 0) m.link0[b] = l;
        m.nlink[b]++;
        m.lmass[l] = (T)link_mass[l];
        for (int i = 0; i < 3; i++) m.lcom[l][i] = (T)link_com[3 * l + i];
        for (int i = 0; i < 9; i++) m.linertia[l][i] = (T)link_inertia[9 * l + i];
    }
    for (int d = 0; d < NDOF; d++) {
        m.lo[d] = (T)dof_lo[d]; m.hi[d] = (T)dof_hi[d];
        m.damp[d] = (T)dof_damping[d];
    }
    int c = 0;
    for (int g = 0; g < NGEOM; g++) {
        m.gbody[g] = geom_body[g]; m.gr[g] = (T)geom_r[g];
        for (int i = 0; i < 3; i++) { m.gp1[g][i] = (T)geom_p1[3 * g + i]; m.gp2[g][i] = (T)geom_p2[3 * g + i]; }
        double h2 = 0;
        for (int i = 0; i < 3; i++) h2 += (geom_p2[3 * g + i] - geom_p1[3 * g + i]) * (geom_p2[3 * g + i] - geom_p1[3 * g + i]);
        m.gbr[g] = (T)(0.5 * csqrt(h2) + geom_r[g]);
        for (int e = 0; e < (geom_type[g] == 0 ? 1 : 2); e++) { m.cand[c] = g | (int)((unsigned)(-1 - e) << 16); c++; }
    }
    for (int k = 0; k < NPAIR; k++) { m.cand[c] = pair_a[k] | (pair_b[k] << 16); c++; }
    for (int k = 0; k < NACT; k++) { m.act_dof[k] = hm::act_dof[k]; m.act_gain[k] = (float)hm::act_gain[k]; m.act_gain_d[k] = hm::act_gain[k]; }
    return m;
}

static __constant__ ModelTab<float> kTabF = make_tab<float>();   // per translation unit
static __constant__ ModelTab<double> kTabD = make_tab<double>();
template <typename T> __device__ inline const ModelTab<T>& tab();
#ifdef HUM_TAB_LDS   // measured slower than __constant__ (24.3M vs 25.1M env-steps/s): opt-in experiment
// fp32: the cooperative kernel indexes the tables by lane (body, dof, geom, candidate), which from
// __constant__ memory are per-lane vector-memory loads with L1/L2 latency on every dependent chain.  Each
// block keeps its own 2.9 KB LDS copy instead, filled once per launch by load_tab_lds.
static __shared__ ModelTab<float> sTabF;
template <> __device__ inline const ModelTab<float>& tab<float>() { return sTabF; }
#else
template <> __device__ inline const ModelTab<float>& tab<float>() { return kTabF; }
#endif
template <> __device__ inline const ModelTab<double>& tab<double>() { return kTabD; }
// The table through a pointer the compiler cannot see through: its constant-offset loads are then issued where they
// are used (scalar loads) instead of being hoisted out of the substep / step loops into registers live across them.
template <typename T>
__device__ __attribute__((always_inline)) inline const ModelTab<T>& tab_fresh() {
#ifdef HUM_TAB_LDS
    return tab<T>();
#else
    using CT = const __attribute__((address_space(4))) ModelTab<T>;
    CT* p = (CT*)&tab<T>();
    asm volatile("" : "+s"(p));
    return *(const ModelTab<T>*)p;
#endif
}

template <typename T>
__device__ inline void load_tab_lds() {   // block-wide; the caller's __syncthreads publishes it
#ifdef HUM_TAB_LDS
    if constexpr (sizeof(T) == 4) {
        static_assert(sizeof(ModelTab<float>) % 4 == 0, "word copy");
        const int* src = reinterpret_cast<const int*>(&kTabF);
        int* dst = reinterpret_cast<int*>(&sTabF);
        for (int w = threadIdx.x; w < (int)(sizeof(ModelTab<float>) / 4); w += blockDim.x) dst[w] = src[w];
    }
#endif
}

// rows kept in LDS; rows beyond spill to a per-env global region and the wave takes the slow PGS path
// (random-policy rollouts: p99 20 rows, > 30 in 0.04% of env-substeps; but the launch lasts as long as
// its slowest wave, so a smaller capacity costs more than its frequency suggests: 24 rows is 9% slower)
// 30 rows: 4 fp32 blocks of 4 envs take exactly the CU's 160 KB (29: 156.5 KB; 30 measured +0.3 % on the contact-rich
// split-impulse workload, tools/gpu/ab.sh).  Diagnostic builds with extra shared memory use 29 (Makefile).
#ifndef HUM_MAXR_LDS
#define HUM_MAXR_LDS 30
#endif

// Bounds-checked diagnostic build (-DHUM_BOUNDS_CHECK, csrc/Makefile target `bounds`; never the shipped library):
// the sites that were generic-pointer (flat) accesses until round 4 check their index against
// its slice; an index outside sets HUM_EFLAG_DIAG_BOUNDS and is clamped to the slice's first entry
#ifdef HUM_BOUNDS_CHECK
#define HUM_BOUNDS(ef, ok, fix) do { if (!(ok)) { (ef) |= HUM_EFLAG_DIAG_BOUNDS; fix; } } while (0)
#else
#define HUM_BOUNDS(ef, ok, fix) do {} while (0)
#endif

constexpr int MAXR_LDS = HUM_MAXR_LDS;

template <typename T>
struct GroupLDS {   // ~9.7 KB (fp32): 4 blocks of 4 envs per CU = one wavefront per SIMD
    T st[HUM_NSTATE + 1];
    T tau[NDOF + 3];
    T nu[NV + 1];
    T R[NB][9], o[NB][3], Sc[NDOF][6];   // Sc: motion subspace column [u; o x u] of each hinge (world axes)
    T U[NDOF][6], Dinv[DINV_N], L0[21];
    // body velocities of the ABA's velocity nu* (before the constraint solve), written by pass 3: the friction
    // rows' slip directions read them instead of re-summing the root path per row
    T Vs[NB][6];
    union {
        struct {   // articulated-body pass (dead once the accelerations are known)
            // IA rows padded to 24 words: 16-byte aligned, so a row moves in six 16-byte LDS accesses
            // c: bias accelerations at the common origin (pass 3), cl: about each body's pivot (pass 2)
            T V[NB][6], c[NB][6], cl[NB][6];
            alignas(16) T IA[NB][24];
            T pA[NB][6], uu[NDOF + 1];   // V: pass-3 body accelerations
        } aba;
        struct {   // contacts + constraint rows
            T gp[NGEOM][2][3];
            T con[MAXC_LDS][CW];
            alignas(16) T row[MAXR_LDS][RW];
            int rdesc[MAXL_G];   // limit rows: dof | side << 8
        } cr;
    } x;
};

static_assert(HUM_MAXR_LDS != 30 || 4 * sizeof(GroupLDS<float>) * 4 <= 160 * 1024,
              "four blocks of four fp32 envs must fit one CU's LDS");
static_assert((sizeof(GroupLDS<float>) / 4) % 64 != 0, "per-env LDS stride: not a multiple of the 64 banks");

template <typename T>
__device__ __attribute__((always_inline)) inline void load_sc(const GroupLDS<T>& S, int d, T* Sc) {
#pragma unroll
    for (int e = 0; e < 6; e++) Sc[e] = S.Sc[d][e];
}

// ---- block row pool.  The rows of a block's EPB_ envs are packed back to back (env 0's, then env 1's, ...)
// over its EPB_ * MAXR_LDS LDS row slots (slot s = row s % MAXR_LDS of env struct s / MAXR_LDS), so one env
// may hold more than MAXR_LDS rows while the block total fits: the random-policy per-env tail (> 30 rows in
// 0.04% of env-substeps) no longer sends a wave to the global spill path, which made it the launch's
// slowest wave.  Positions from P.lds_rows on go to the block's global spill region (never observed with a
// random policy; tests force it with hum_config.lds_rows).
template <typename T>
__device__ __attribute__((always_inline)) inline int pool_off(int p) {   // byte offset from the block's LDS array
    const int s = p / MAXR_LDS, i = p - s * MAXR_LDS;
    return s * (int)sizeof(GroupLDS<T>) + (int)offsetof(GroupLDS<T>, x.cr.row) + i * RW * (int)sizeof(T);
}
__host__ __device__ constexpr int grow_rows_per_block(int epb, int cap) { return epb * MAXR_G - cap; }
// a block's global spill region (T units): rows past the LDS pool, then each env's contacts past MAXC_LDS
__host__ __device__ constexpr long grow_block_size(int epb, int cap) {
    return (long)grow_rows_per_block(epb, cap) * RW + (long)epb * (MAXC_G - MAXC_LDS) * CW;
}
__host__ __device__ constexpr long gcon_offset(int epb, int cap, int ge) {
    return (long)grow_rows_per_block(epb, cap) * RW + (long)ge * (MAXC_G - MAXC_LDS) * CW;
}

// ---- diagnostics (never in the shipped library): -DHUM_PHASE_TIMING = per-phase s_memtime counters (global
// atomics: they slow the kernel and skew it between XCDs) + the per-block work log; -DHUM_WAVE_LOG = the work
// log alone (one plain store per block at its end: timing close to the shipped kernel)
#if defined(HUM_PHASE_TIMING) || defined(HUM_WAVE_LOG)
#define HUM_WLOG_ON 1
// per-block work log: [0] s_memtime duration, [1] PGS length, [2] row rounds, [3] narrow-phase rounds,
// [4] s_memrealtime duration, [5] s_memrealtime start, [6] HW_ID, [7] XCC_ID, [8 + k] phase k cycles (k 1-10;
// 11-23: optional sub-phase markers SUBPHASE(k), which split the time of the phase they sit in)
// (HUM_WAVE_LOG builds: accumulated in LDS by thread 0, written at the end)
constexpr int WLOG_W = 32;   // [8 + k]: phase k (1-10), sub-phase markers 11-23
__device__ unsigned g_wave_log[65536][WLOG_W];
template <int EPB_>
__device__ inline int env_max(int x) {   // max over the wave's envs of a per-env (group-uniform) value
    int m = __builtin_amdgcn_readlane(x, 0);
#pragma unroll
    for (int e = 1; e < EPB_; e++) m = max(m, __builtin_amdgcn_readlane(x, e * 16));
    return m;
}
#define WLOG(k, v)                                                               \
    do {                                                                         \
        const int v_ = (v);                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 65536) g_wave_log[blockIdx.x][k] += v_; \
    } while (0)
#else
#define WLOG(k, v) do { } while (0)
#endif
#ifdef HUM_PHASE_TIMING
__device__ unsigned long long g_phase_cycles[32];
#define PHASE(k)                                                                 \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();                \
            atomicAdd(&g_phase_cycles[k], t_ - t_last_);                         \
            t_last_ = t_;                                                        \
        }                                                                        \
    } while (0)
#define PHASE_INIT unsigned long long t_last_ = __builtin_amdgcn_s_memtime()
#elif defined(HUM_WAVE_LOG)
static __shared__ unsigned long long s_phase[24];
static __shared__ unsigned long long s_tlast;   // shared: markers also sit inside the env-logic functions
#define PHASE(k)                                                                 \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();                \
            s_phase[k] += t_ - s_tlast;                                          \
            s_tlast = t_;                                                        \
        }                                                                        \
    } while (0)
#define PHASE_INIT                                                               \
    do {                                                                         \
        if (threadIdx.x == 0) s_tlast = __builtin_amdgcn_s_memtime();           \
    } while (0)
#elif defined(HUM_PHASE_MARK)   // static ISA attribution (tools/isa_phases.py): asm comments at phase ends
#define PHASE(k) asm volatile("; @phase " #k ::: "memory")
#define PHASE_INIT do { } while (0)
#else
#define PHASE(k) do { } while (0)
#define PHASE_INIT do { } while (0)
#endif

// Lane-utilisation study (tools/lane_util.py; diagnostic builds only): -DHUM_STOP_AFTER=k ends every substep after
// phase k (0 = before FK; 9 = the whole substep), so SQ counters of builds k - 1 and k, stepped from the same saved
// states, differ by phase k's instructions and thread-cycles
#ifdef HUM_STOP_AFTER
#define HUM_STOP(k)                                                              \
    do {                                                                         \
        if constexpr (HUM_STOP_AFTER == (k)) return;                             \
    } while (0)
#else
#define HUM_STOP(k) do { } while (0)
#endif

#if defined(HUM_WAVE_LOG) && defined(HUM_SUBPHASE)   // finer split of a phase's time (tools/wave_log.py)
#define SUBPHASE(k) PHASE(k)
#elif defined(HUM_PHASE_MARK) && defined(HUM_SUBPHASE)   // static ISA attribution of the sub-phases
#define SUBPHASE(k) asm volatile("; @sub " #k ::: "memory")
#else
#define SUBPHASE(k) do { } while (0)
#endif
// HUM_SUBPHASE_PGS: the Delassus PGS's own split (markers 19-22) in place of the post-step ones; HUM_SUBPHASE_ROWS:
// the rows phase's split (markers 19-22, per row round: setup, Jacobian, articulated solve, coupling)
#define ROWS_SUBPHASE(k) do { } while (0)
#ifdef HUM_SUBPHASE_PGS
#define PGS_SUBPHASE(k) SUBPHASE(k)
#define POST_SUBPHASE(k) do { } while (0)
#elif defined(HUM_SUBPHASE_ROWS)
#define PGS_SUBPHASE(k) do { } while (0)
#define POST_SUBPHASE(k) do { } while (0)
#undef ROWS_SUBPHASE
#define ROWS_SUBPHASE(k) SUBPHASE(k)
#else
#define PGS_SUBPHASE(k) do { } while (0)
#define POST_SUBPHASE(k) SUBPHASE(k)
#endif

#ifdef HUM_CHECK_LINKS
__device__ unsigned g_check[8];
#endif
__device__ inline void wave_sync() {   // cross-lane LDS ordering inside one wavefront
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// phase boundary of the cooperative substep: a block is one wavefront (EPB_ envs x 16 lanes <= 64), so LDS ordering
// inside the wave suffices (no s_barrier, no drain of the wave's outstanding LDS writes).  The boundaries after the
// contacts and the rows keep __syncthreads: spilled contacts and rows cross lanes through global memory.
__device__ inline void phase_sync() { wave_sync(); }

__device__ inline float med3(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ inline double med3(double x, double lo, double hi) { return fmin(fmax(x, lo), hi); }

// 16-lane (DPP row) all-reduce sum
__device__ inline float row_sum(float v) {
    // update_dpp with old = 0 / bound_ctrl lets the compiler fold each step into one v_add_f32_dpp
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true));  // row_ror:8
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, true));  // row_ror:4
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, true));  // row_ror:2
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, true));  // row_ror:1
    return v;
}
template <int CTRL>
__device__ inline double mov_dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ inline double row_sum(double v) {
    v += mov_dpp_d<0x128>(v);
    v += mov_dpp_d<0x124>(v);
    v += mov_dpp_d<0x122>(v);
    v += mov_dpp_d<0x121>(v);
    return v;
}

// 6x6 Cholesky with the inverse of each pivot stored on the diagonal: the solves (base step, and one per
// constraint row in g_response) multiply instead of dividing (an IEEE fp32 divide is ~10 VALU)
template <typename T>
__device__ inline void chol6_inv(const T* A, T* L) {
#pragma unroll
    for (int j = 0; j < 6; j++) {
        T s = A[sidx(j, j)];
#pragma unroll
        for (int k = 0; k < j; k++) s -= L[j * (j + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
        const T inv = prsqrt_piv(s);
        L[j * (j + 1) / 2 + j] = inv;
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
__device__ inline void chol6_solve_inv(const T* L, T* b) {
#pragma unroll
    for (int i = 0; i < 6; i++) {
        T s = b[i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= L[i * (i + 1) / 2 + k] * b[k];
        b[i] = s * L[i * (i + 1) / 2 + i];
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        T s = b[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) s -= L[k * (k + 1) / 2 + i] * b[k];
        b[i] = s * L[i * (i + 1) / 2 + i];
    }
}

// ------------------------------------------------------------------------- test-impulse response
// M^-1 J^T by the articulated-body solve of physics.h::impulse_response, reading the ABA factorisation from LDS.
// the forward half: base acceleration from its articulated inertia, then root -> leaves
template <typename T>
__device__ __attribute__((always_inline)) inline void g_response_fwd(const GroupLDS<T>& S, const T* uq, T (&a)[NB][6], T* out) {
    {
        T L[21];
#pragma unroll
        for (int q = 0; q < 21; q++) L[q] = S.L0[q];
        chol6_solve_inv(L, a[0]);
    }
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
            for (int e = 0; e < 6; e++) s -= S.U[d0 + j][e] * a[p][e];
            r[j] = s;
        }
#pragma unroll
        for (int e = 0; e < 6; e++) a[b][e] = a[p][e];
#pragma unroll
        for (int i = 0; i < k; i++) {
            T s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += S.Dinv[DINV.off[b] + k * i + j] * r[j];
            out[6 + d0 + i] = s;
            const int d = d0 + i;
            T Sc[6];
            load_sc(S, d, Sc);
#pragma unroll
            for (int e = 0; e < 6; e++) a[b][e] += Sc[e] * s;
        }
    }
}


struct TreeKids { bool leaf[NB]; int last_kid[NB]; };   // last_kid: the highest-index child (processed first)
constexpr TreeKids tree_kids() {
    TreeKids t{};
    for (int b = 0; b < NB; b++) { t.leaf[b] = true; t.last_kid[b] = -1; }
    for (int b = 1; b < NB; b++) {
        t.leaf[body_parent[b]] = false;
        if (b > t.last_kid[body_parent[b]]) t.last_kid[body_parent[b]] = b;
    }
    return t;
}
constexpr TreeKids KIDS = tree_kids();
// The row's generalised impulse J^T drives the solve (physics.h::impulse_response injects the spatial forces on
// its two bodies instead: the same linear map).  No per-body force selects (400 fewer VALU per row, +2.5 % measured,
// profiles/r04_ab_rows.txt); the leaves receive no child contribution and each body's first child initialises its
// parent's accumulator.  Rounding: a joint's impulse is J_d - S_d . pA (two rounded terms, where the force form
// rounds S_d . (pA - f) once); measured over 512 lanes from identical states its fp32 error distribution is the
// force form's (tools/diag_fp32_ab.py, profiles/r04_fp32ab.txt).
template <typename T>
__device__ inline void g_response(const GroupLDS<T>& S, const T* J, T* out) {
    T pA[NB][6];   // the children's contributions to each body's articulated bias impulse
    T uq[NDOF];
#pragma unroll
    for (int b = NB - 1; b >= 1; b--) {
        const int p = body_parent[b], k = body_ndof[b], d0 = body_dof0[b];
#pragma unroll
        for (int j = 0; j < k; j++) {
            const int d = d0 + j;
            T s = J[6 + d];
            if (!KIDS.leaf[b]) {
                T Sc[6];
                load_sc(S, d, Sc);
#pragma unroll
                for (int e = 0; e < 6; e++) s -= Sc[e] * pA[b][e];
            }
            uq[d] = s;
        }
        T w[3];
#pragma unroll
        for (int i = 0; i < k; i++) {
            T t = 0;
#pragma unroll
            for (int j = 0; j < k; j++) t += S.Dinv[DINV.off[b] + k * i + j] * uq[d0 + j];
            w[i] = t;
        }
#pragma unroll
        for (int e = 0; e < 6; e++) {
            T s = KIDS.leaf[b] ? T(0) : pA[b][e];
#pragma unroll
            for (int i = 0; i < k; i++) s += S.U[d0 + i][e] * w[i];
            if (KIDS.last_kid[p] == b) pA[p][e] = s;
            else pA[p][e] += s;
        }
    }
    T a[NB][6];
#pragma unroll
    for (int e = 0; e < 6; e++) a[0][e] = J[e] - pA[0][e];
    g_response_fwd(S, uq, a, out);
}

// J row for a spatial force f on body b (generic: runtime b)
template <typename T>
__device__ inline void g_row_jacobian(const GroupLDS<T>& S, int b, const T* f, T sgn, T* J) {
#pragma unroll
    for (int e = 0; e < 6; e++) J[e] += sgn * f[e];
#pragma unroll
    for (int x = 1; x < NB; x++) {
        const bool on = on_path(x, b);
#pragma unroll
        for (int k = 0; k < body_ndof[x]; k++) {
            const int d = body_dof0[x] + k;
            T Sc[6];
            load_sc(S, d, Sc);
            T s = 0;
#pragma unroll
            for (int e = 0; e < 6; e++) s += f[e] * Sc[e];
            if (on) J[6 + d] += sgn * s;
        }
    }
}

// J row for spatial forces fa on body ba and fb on body bb (either < 0 = absent), one pass over the dofs
template <typename T>
__device__ inline void g_row_jacobian2(const GroupLDS<T>& S, int ba, const T* fa, int bb, const T* fb, T* J) {
#pragma unroll
    for (int e = 0; e < 6; e++) J[e] = (ba >= 0 ? fa[e] : T(0)) + (bb >= 0 ? fb[e] : T(0));
#pragma unroll
    for (int x = 1; x < NB; x++) {
        const bool ona = on_path(x, ba);
        const bool onb = on_path(x, bb);
#pragma unroll
        for (int k = 0; k < body_ndof[x]; k++) {
            const int d = body_dof0[x] + k;
            T Sc[6];
            load_sc(S, d, Sc);
            T sa = 0, sb = 0;
#pragma unroll
            for (int e = 0; e < 6; e++) { sa += fa[e] * Sc[e]; sb += fb[e] * Sc[e]; }
            J[6 + d] = (ona ? sa : T(0)) + (onb ? sb : T(0));
        }
    }
}

// ------------------------------------------------------------------------- constraint rows, wave-wide
// Row t of the wave's concatenated row list (env 0's rows, then env 1's, ...) goes to lane t % (16 EPB_):
// per-env counts are wave-uniform (readlane), so the env/row of a task is two compares away.
template <typename T>
__device__ __attribute__((always_inline)) void store_row(T* R, const T* J, const T* Mi, const T* sc, int next3,
                                                         int next3_ln, T qc = T(0)) {
#pragma unroll
    for (int q = 0; q < NV; q++) { R[2 * q] = J[q]; R[2 * q + 1] = Mi[q]; }
    R[RO_Z] = T(0); R[RO_Z + 1] = T(0);
    R[RO_S0] = sc[0]; R[RO_S0 + 1] = sc[2]; R[RO_S0 + 2] = sc[3]; R[RO_S0 + 3] = sc[4];
    R[RO_S1] = sc[5]; R[RO_S1 + 1] = qc;   // q = meff c (0 after a zero row; else from group_rows)
    *reinterpret_cast<int*>(R + RO_S1 + 2) = next3;
    *reinterpret_cast<int*>(R + RO_S1 + 3) = next3_ln;
}
template <typename T>
__device__ __attribute__((always_inline)) void store_row_global(T* R, const T* J, const T* Mi, const T* sc) {
    // spilled rows: nontemporal stores keep the compiler from merging this path with the LDS one into
    // generic (flat) stores
#pragma unroll
    for (int q = 0; q < NV; q++) { __builtin_nontemporal_store(J[q], R + 2 * q); __builtin_nontemporal_store(Mi[q], R + 2 * q + 1); }
    __builtin_nontemporal_store(sc[0], R + RO_S0);
    __builtin_nontemporal_store(sc[2], R + RO_S0 + 1);
    __builtin_nontemporal_store(sc[3], R + RO_S0 + 2);
    __builtin_nontemporal_store(sc[4], R + RO_S0 + 3);
    __builtin_nontemporal_store(sc[5], R + RO_S1);
}

// PGS pool layout of an env with nl limit rows and nc contacts (rows: limits, normals, 2 frictions per
// contact): zero rows (J = M^-1 J^T = b = bounds = lambda = c = 0: every update of one is lnew = dl = 0)
// between the normals and the frictions put each friction row at least PGS_AHEAD + 1 positions after its
// normal row, and trail the cycle up to PGS_AHEAD + 1 positions.  The PGS reads the row PGS_AHEAD ahead (and
// the lambda bounding it) while a row is solved, so every lambda it reads was stored before.
constexpr int PGS_AHEAD = 3;
__device__ inline int pool_gap(int nc) { return nc > 0 && nc < PGS_AHEAD + 1 ? PGS_AHEAD + 1 - nc : 0; }
__device__ inline int pool_used(int nl, int nc) { return nl + 3 * nc + pool_gap(nc); }
__device__ inline int pool_rows(int nl, int nc) {
    const int u = pool_used(nl, nc);
    return u < PGS_AHEAD + 1 ? PGS_AHEAD + 1 : u;
}
__device__ inline int pool_pos(int r, int nl, int nc) { return r < nl + nc ? r : r + pool_gap(nc); }   // real row r
__device__ inline bool pool_zero(int q, int nl, int nc) {   // position q holds a zero row
    return (q >= nl + nc && q < nl + nc + pool_gap(nc)) || q >= pool_used(nl, nc);
}
// PGS links (byte offsets from the block's LDS array, used only when the block's rows all fit in LDS) of
// pool position q of an env: the position PGS_AHEAD ahead in cyclic order, and the lambda bounding it - its
// normal row's for a friction row, its own otherwise (mu = 0 there)
template <typename T>
__device__ inline void pgs_link(int epos, int q, int nl, int nc, int& next3, int& next3_ln) {
    const int neff = pool_rows(nl, nc), f0 = nl + nc + pool_gap(nc);
    const int t = q + PGS_AHEAD < neff ? q + PGS_AHEAD : q + PGS_AHEAD - neff;   // (q + PGS_AHEAD) % neff: q < neff, PGS_AHEAD < neff
    const bool fric = t >= f0 && t < pool_used(nl, nc);
    next3 = pool_off<T>(epos + t);
    next3_ln = pool_off<T>(epos + (fric ? nl + ((t - f0) >> 1) : t)) + RO_LAM * (int)sizeof(T);
}

// The Delassus-form PGS (pgs_delassus below; -DHUM_DELASSUS builds only: measured slower) runs
// when every env of the wave has at most LMAX rows, the block's rows all sit in its LDS pool, and the wave is the
// benchmarked fp32 one of 4 envs (one MFMA wave).
constexpr int LMAX = NV;   // a row's J slots hold its Delassus row: LMAX <= NV
#ifdef HUM_DELASSUS
constexpr bool DELASSUS_ON = true;
#else
constexpr bool DELASSUS_ON = false;
#endif
template <typename T, int EPB_>
constexpr bool delassus_kernel() { return DELASSUS_ON && sizeof(T) == 4 && EPB_ == 4; }

template <typename T, int EPB_>
__device__ __attribute__((always_inline)) void group_rows(const PhysParams& P, GroupLDS<T>* shb, T* gblock, int nl, int nc,
                                                          const T dt, int& pbase, int& ptot, bool& lam, unsigned& ef) {
    const ModelTab<T>& M = tab_fresh<T>();
    const int lane = threadIdx.x & 63, cap = P.lds_rows;
    const T idt = T(1) / dt;
    // pre: task prefix (actual rows); pos: pool prefix (velocity form: short envs are padded with zero rows, see PGS;
    // Delassus form: the rows back to back, no padding)
    int cnt[EPB_], nls[EPB_], ncs[EPB_], pre[EPB_ + 1], pos[EPB_ + 1];
    pre[0] = 0;
    pos[0] = 0;
    int nmax = 0;
#pragma unroll
    for (int e = 0; e < EPB_; e++) {
        nls[e] = __builtin_amdgcn_readlane(nl, e * GL);
        ncs[e] = __builtin_amdgcn_readlane(nc, e * GL);
        cnt[e] = nls[e] + 3 * ncs[e];
        pre[e + 1] = pre[e] + cnt[e];
        nmax = max(nmax, cnt[e]);
    }
    lam = delassus_kernel<T, EPB_>() && pre[EPB_] <= cap && nmax <= LMAX;   // the Delassus-form PGS (wave-uniform)
#pragma unroll
    for (int e = 0; e < EPB_; e++) pos[e + 1] = pos[e] + (lam ? cnt[e] : pool_rows(nls[e], ncs[e]));
    pbase = 0;
#pragma unroll
    for (int q = 0; q < EPB_; q++)
        if (q == lane / GL) pbase = pos[q];
    ptot = pos[EPB_];
    const int total = pre[EPB_];
    WLOG(2, (total + EPB_ * GL - 1) / (EPB_ * GL));
    for (int t = lane; t < total; t += EPB_ * GL) {
        int e = 0;
#pragma unroll
        for (int q = 1; q < EPB_; q++) e += t >= pre[q] ? 1 : 0;
        int r = t, enl = nls[0], enc = ncs[0], epos = 0;
#pragma unroll
        for (int q = 0; q < EPB_; q++)
            if (q == e) { r = t - pre[q]; enl = nls[q]; enc = ncs[q]; epos = pos[q]; }
        const GroupLDS<T>& S = shb[e];
        const auto& C = S.x.cr;
        // every row type (limit / normal / friction) funnels into ONE test-impulse response call: the wave's
        // lanes hold mixed row types, so separate calls per branch would all execute
        T J[NV], Mi[NV], sc[7];
        int ba = -1, bb = -1, jd = -1;
        T fa[6] = {0, 0, 0, 0, 0, 0}, fb[6] = {0, 0, 0, 0, 0, 0}, jsign = 0;
        const bool lim = r < enl;
        if (lim) {
            const int d = C.rdesc[r] & 0xff, side = C.rdesc[r] >> 8;
#ifdef HUM_CHECK_LINKS
            if (d >= NDOF || side > 1) atomicAdd(&g_check[5], 1u);
#endif
            const T sg = side == 0 ? T(1) : T(-1);
            const T q = S.st[13 + d];
            const T pen = side == 0 ? q - M.lo[d] : M.hi[d] - q;
            jd = d;
            jsign = sg;
            sc[0] = pen > (T)P.split_pen ? -pen * (T)P.erp_limit * idt : T(0);
            sc[2] = (T)P.limit_max_impulse;
            sc[5] = 0;
        } else {
            const int cidx = r < enl + enc ? r - enl : (r - enl - enc) >> 1;
            const int f = r < enl + enc ? 0 : 1 + ((r - enl - enc) & 1);
            T ce[CW];
            if (cidx < MAXC_LDS) {   // LDS and global (spilled contact) through address-space-typed pointers: the
                                     // two loads are never merged into one flat load through a generic pointer
                const HUM_LDS T* lc = (const HUM_LDS T*)&C.con[cidx][0];
#pragma unroll
                for (int k = 0; k < CW; k++) ce[k] = lc[k];
            } else {
                int ci = cidx - MAXC_LDS, ce_env = e;   // the env's spill slice: MAXC_G - MAXC_LDS contacts
                HUM_BOUNDS(ef, ci >= 0 && ci < MAXC_G - MAXC_LDS && ce_env >= 0 && ce_env < EPB_, (ci = 0, ce_env = 0));
                const HUM_GLOBAL T* gc = (const HUM_GLOBAL T*)(gblock + gcon_offset(EPB_, cap, ce_env) + (long)ci * CW);
#pragma unroll
                for (int k = 0; k < CW; k++) ce[k] = __builtin_nontemporal_load(gc + k);
            }
            ba = (int)ce[0];
            bb = (int)ce[1];
            const T pa[3] = {ce[2], ce[3], ce[4]}, pb[3] = {ce[5], ce[6], ce[7]}, n[3] = {ce[8], ce[9], ce[10]};
            const T d = ce[11];
            T dir[3];
            if (f == 0) {
                dir[0] = n[0]; dir[1] = n[1]; dir[2] = n[2];
            } else {
                T Va[6], Vb[6], va[3], vb[3], vr[3];
#pragma unroll
                for (int e = 0; e < 6; e++) { Va[e] = S.Vs[ba][e]; Vb[e] = bb >= 0 ? S.Vs[bb >= 0 ? bb : 0][e] : T(0); }
                cross3(Va, pa, va);
                cross3(Vb, pb, vb);
#pragma unroll
                for (int i = 0; i < 3; i++) vr[i] = (va[i] + Va[3 + i]) - (vb[i] + Vb[3 + i]);
                const T vn = dot3(vr, n);
                T lat[3], t1[3], t2[3];
#pragma unroll
                for (int i = 0; i < 3; i++) lat[i] = vr[i] - n[i] * vn;
                const T l2 = dot3(lat, lat);
                if (l2 > (T)1e-12) {
                    const T il = prsqrt_row(l2);
#pragma unroll
                    for (int i = 0; i < 3; i++) t1[i] = lat[i] * il;
                    cross3(t1, n, t2);
                } else {
                    plane_space(n, t1, t2);
                }
#pragma unroll
                for (int i = 0; i < 3; i++) dir[i] = f == 1 ? t1[i] : t2[i];
            }
            cross3(pa, dir, fa); fa[3] = dir[0]; fa[4] = dir[1]; fa[5] = dir[2];
            if (bb >= 0) {
                cross3(pb, dir, fb);
                fb[0] = -fb[0]; fb[1] = -fb[1]; fb[2] = -fb[2]; fb[3] = -dir[0]; fb[4] = -dir[1]; fb[5] = -dir[2];
            }
            sc[0] = f == 0 ? (d > 0 ? -d * idt : (d > (T)P.split_pen ? -d * (T)P.erp_contact * idt : T(0))) : T(0);
            sc[2] = f == 0 ? (T)1e10 : T(0);   // friction rows: bounds come from mu * lambda_n in the PGS
            sc[5] = f == 0 ? T(0) : (bb >= 0 ? (T)P.mu_self : (T)P.mu_ground);   // friction rows only
        }
        ROWS_SUBPHASE(19);
        g_row_jacobian2(S, ba, fa, bb, fb, J);   // limit rows: ba = bb = -1 -> J = 0 (unit entry below)
#pragma unroll
        for (int k = 0; k < NDOF; k++)
            if (k == jd) J[6 + k] = jsign;
        ROWS_SUBPHASE(20);
        g_response(S, J, Mi);
        ROWS_SUBPHASE(21);
        T jm = 0;
#pragma unroll
        for (int q = 0; q < NV; q++) jm += J[q] * Mi[q];   // limit rows: sg * Mi[6 + d] (sg^2 = 1)
        sc[1] = 0;   // lo = 0 for every row type: the PGS reads this slot as its zero pad
        sc[3] = 0;
        sc[4] = prcp_row(jm);
        const int p = epos + (lam ? r : pool_pos(r, enl, enc));
        // coupling c_r = J_r . (M^-1 J^T)_pred(r) from the lane that solved the predecessor row in this round
        // (ds_bpermute); predecessors in another round are left to the LDS pass below.  The Delassus-form PGS stores
        // instead the row's velocity J_r . nu* (the constraint velocity its residual starts from) and, in the link slot,
        // the LDS offset of the lambda that bounds it (its normal row's for a friction row, its own otherwise)
        T qc = T(0);
        if (lam) {
#pragma unroll
            for (int q = 0; q < NV; q++) qc += J[q] * S.nu[q];
        } else
#ifndef HUM_COUPLING_LDS   // A/B: every coupling from the LDS pass below instead of the predecessor lane
        {
            const int qr = p - epos, qp = qr == 0 ? pool_rows(enl, enc) - 1 : qr - 1;
            const int rp = qp < enl + enc ? qp : qp - pool_gap(enc);
            const int tp = (t - r) + rp, t0 = t - lane;
            const bool here = !pool_zero(qp, enl, enc) && tp >= t0 && tp < t0 + EPB_ * GL;
            const int src = 4 * (here ? tp - t0 : lane);
            T c = 0;
#pragma unroll
            for (int q = 0; q < NV; q++) {
                T mp;
                if constexpr (sizeof(T) == 4) {
                    mp = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(Mi[q])));
                } else {
                    const long long b = __double_as_longlong(Mi[q]);
                    const int lo = __builtin_amdgcn_ds_bpermute(src, (int)(b & 0xffffffff));
                    const int hi = __builtin_amdgcn_ds_bpermute(src, (int)(b >> 32));
                    mp = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
                }
                c += J[q] * mp;
            }
            if (here) qc = c * sc[4];
        }
#else
        {}
#endif
        ROWS_SUBPHASE(22);
        if (p < cap) {
            int n3, n3ln;
            if (lam) {   // dense layout: the normal row of friction row r is row enl + (r - enl - enc) / 2
                n3 = 0;
                n3ln = pool_off<T>(r >= enl + enc ? epos + enl + ((r - enl - enc) >> 1) : p) + RO_LAM * (int)sizeof(T);
            } else {
                pgs_link<T>(epos, p - epos, enl, enc, n3, n3ln);   // (used only when all of the block's rows are in LDS)
            }
            store_row(reinterpret_cast<T*>(reinterpret_cast<char*>(shb) + pool_off<T>(p)), J, Mi, sc, n3, n3ln, qc);
        }
        else {
            store_row_global(gblock + (long)(p - cap) * RW, J, Mi, sc);
        }
    }
    // couplings c_r = J_r . (M^-1 J^T)_pred(r) (cyclic predecessor; 0 after a zero row) for the lookahead
    // PGS, which needs them only when the block's rows all sit in LDS: the rows whose predecessor another round
    // solved (more rows than lanes), from LDS
#ifdef HUM_COUPLING_LDS
    constexpr bool all_lds = true;
#else
    constexpr bool all_lds = false;
#endif
    if (!lam && pos[EPB_] <= cap && (all_lds || total > EPB_ * GL)) {   // rows whose predecessor another round solved
        wave_sync();
        for (int t = lane; t < total; t += EPB_ * GL) {
            int e = 0;
#pragma unroll
            for (int q = 1; q < EPB_; q++) e += t >= pre[q] ? 1 : 0;
            int r = t, epos = 0, enl = nls[0], enc = ncs[0];
#pragma unroll
            for (int q = 0; q < EPB_; q++)
                if (q == e) { r = t - pre[q]; epos = pos[q]; enl = nls[q]; enc = ncs[q]; }
            const int qr = pool_pos(r, enl, enc);
            const int qp = qr == 0 ? pool_rows(enl, enc) - 1 : qr - 1;
            const int tp = (t - r) + (qp < enl + enc ? qp : qp - pool_gap(enc));
            if (!pool_zero(qp, enl, enc) && (all_lds || tp / (EPB_ * GL) != t / (EPB_ * GL))) {
                T* Rr = reinterpret_cast<T*>(reinterpret_cast<char*>(shb) + pool_off<T>(epos + qr));
                const T* Rp = reinterpret_cast<const T*>(reinterpret_cast<const char*>(shb) + pool_off<T>(epos + qp));
                T c = 0;
                if constexpr (sizeof(T) == 4) {
                    // 16-byte reads of (J, M^-1 J^T) pair couples, all issued before the sum needs them (the pairwise
                    // scalar reads were issued two at a time, each pair waited for)
                    static_assert(RO_Z == 2 * NV && NV % 2 == 1, "the last quad holds pair NV - 1 and the zero pair");
                    using f4v = float __attribute__((ext_vector_type(4)));
                    f4v a4[(NV + 1) / 2], b4[(NV + 1) / 2];
#pragma unroll
                    for (int h = 0; h < (NV + 1) / 2; h++) {
                        a4[h] = reinterpret_cast<const f4v*>(Rr)[h];
                        b4[h] = reinterpret_cast<const f4v*>(Rp)[h];
                    }
#pragma unroll
                    for (int h = 0; h < (NV + 1) / 2; h++) asm volatile("" ::"v"(a4[h]), "v"(b4[h]));   // whole quads, in flight together
#pragma unroll
                    for (int h = 0; h < (NV + 1) / 2; h++) {
                        c += a4[h].x * b4[h].y;
                        if (2 * h + 1 < NV) c += a4[h].z * b4[h].w;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < NV; q++) c += Rr[2 * q] * Rp[2 * q + 1];
                }
                Rr[RO_S1 + 1] = c * Rr[RO_S0 + 3];   // q_r = meff_r c_r: the PGS scalar chain multiplies it by dl
            }
        }
    }
}


// f(std::integral_constant<int, k>) for k = 0 .. N-1 (an index usable as a constant expression, e.g. a DPP control)
template <typename F, int... K>
__device__ __attribute__((always_inline)) inline void static_for_impl(F&& f, std::integer_sequence<int, K...>) {
    (f(std::integral_constant<int, K>{}), ...);
}
template <int N, typename F>
__device__ __attribute__((always_inline)) inline void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ------------------------------------------------------------------------- PGS, Delassus form
// The same Gauss-Seidel sweep as the velocity-form PGS below (rows in Bullet order, P.iters iterations, friction bounds
// from the current normal impulse, nu += (M^-1 J^T)_k dl after every row update), restated so that the row-to-row
// chain needs no reduction: the constraint velocities w = J nu are carried per row,
//     row k:  lambda_k' = clamp(lambda_k + meff_k (b_k - w_k)),  dl = lambda_k' - lambda_k,  w += A[:, k] dl,
// with A = J M^-1 J^T (the Delassus matrix).  Lane l of an env owns the env's rows l and l + 16 (residual b - w,
// lambda and bounds in registers) and the generalised velocity components l and 16 + l; at step k the owner's dl reaches
// the env's 16 lanes by one DPP row_newbcast and every lane updates its two residuals and two velocity components with
// one fma each, reading A and M^-1 J^T four steps ahead from LDS: the chain is fma, med3, sub, broadcast, fma - no
// 16-lane J . nu reduction per row (4 DPP adds, the velocity form's).  A is formed per substep on the matrix cores:
// C = J (rows x 24) x (M^-1 J^T)^T by v_mfma_f32_16x16x4_f32 16 x 16 tiles (K = 23 padded with a zero), the 4 envs'
// chains interleaved, written over the rows' J slots (J . nu* was taken by group_rows).  The rows sit back to back in
// the pool (no zero rows): a friction row's normal is at least one step earlier, so its bound is read one step ahead.
template <int EPB_>
__device__ __attribute__((always_inline)) void pgs_delassus(const PhysParams& P, GroupLDS<float>* shb, GroupLDS<float>& S,
                                                             int nl, int nc, int pbase, int l, float& n0, float& n1) {
    static_assert(EPB_ == 4 && LMAX <= NV && LMAX <= 2 * GL, "one MFMA wave of 4 envs; a row's J slots hold its A row");
    using f4 = float __attribute__((ext_vector_type(4)));
    char* lds0 = reinterpret_cast<char*>(shb);
    const int lane = threadIdx.x & 63;
    int pe[EPB_], ne[EPB_], M = 0;
    {
        int acc = 0;
#pragma unroll
        for (int e = 0; e < EPB_; e++) {
            pe[e] = acc;
            ne[e] = __builtin_amdgcn_readlane(nl, e * GL) + 3 * __builtin_amdgcn_readlane(nc, e * GL);
            acc += ne[e];
            M = max(M, ne[e]);
        }
    }
    if (M == 0) return;   // wave-uniform: no constraint row in any env
    const bool TWOANY = M > GL;   // wave-uniform
    const int neff = nl + 3 * nc;
    const int dummy = (int)(reinterpret_cast<char*>(&S.nu[NV]) - lds0);   // an unused word: reads of 0, stray stores
    // finite reads standing in for absent rows (their updates are dl = 0): the env's rotation matrices (>= 46 words)
    const int finite = (int)(reinterpret_cast<char*>(&S.R[0][0]) - lds0);
    if (l == 0) S.nu[NV] = 0.f;
    // ---- A of every env: lane (lk, lr) supplies J / M^-1 J^T of row lr (+ 16) at k = 4 s + lk (rows past the env and
    //      k = 23 masked to 0); C[4 lk + q][lr] comes back.  Every operand is read before any A entry is written.
    const int lr = lane & 15, lk = lane >> 4;
    using f2 = float __attribute__((ext_vector_type(2)));
    f2 op[EPB_][2][6];
    auto load_ops = [&](int ti) {
#pragma unroll
        for (int e = 0; e < EPB_; e++) {
            const int r = lr + GL * ti;
            const bool rv = r < ne[e];
            const float* R = reinterpret_cast<const float*>(lds0 + (rv ? pool_off<float>(pe[e] + r) : finite));
#pragma unroll
            for (int s4 = 0; s4 < 6; s4++) {
                const int k = 4 * s4 + lk;
                const f2 jm = *reinterpret_cast<const f2*>(R + 2 * min(k, NV - 1));   // (J_k, (M^-1 J^T)_k)
                op[e][ti][s4] = rv && k < NV ? jm : f2{0.f, 0.f};
            }
        }
    };
    load_ops(0);
    if (TWOANY) load_ops(1);
    PGS_SUBPHASE(19);
    f4 c00[EPB_], c01[EPB_], c11[EPB_];
#pragma unroll
    for (int e = 0; e < EPB_; e++) c00[e] = c01[e] = c11[e] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 6; s4++)
#pragma unroll
        for (int e = 0; e < EPB_; e++)
            c00[e] = __builtin_amdgcn_mfma_f32_16x16x4f32(op[e][0][s4].x, op[e][0][s4].y, c00[e], 0, 0, 0);
    if (TWOANY) {
#pragma unroll
        for (int s4 = 0; s4 < 6; s4++)
#pragma unroll
            for (int e = 0; e < EPB_; e++) {
                c01[e] = __builtin_amdgcn_mfma_f32_16x16x4f32(op[e][0][s4].x, op[e][1][s4].y, c01[e], 0, 0, 0);
                c11[e] = __builtin_amdgcn_mfma_f32_16x16x4f32(op[e][1][s4].x, op[e][1][s4].y, c11[e], 0, 0, 0);
            }
    }
    PGS_SUBPHASE(20);
    // A[r][c] into row r's J slot 2 c (rows of the env, c < LMAX; columns past the env: the zeros C holds there)
#pragma unroll
    for (int e = 0; e < EPB_; e++) {
        auto put = [&](int r, int c, float v) {
            const bool ok = r < ne[e] && c < LMAX;
            *reinterpret_cast<float*>(lds0 + (ok ? pool_off<float>(pe[e] + r) + 2 * c * (int)sizeof(float) : dummy)) = v;
        };
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = 4 * lk + q;
            put(r, lr, c00[e][q]);
        }
        if (TWOANY) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = 4 * lk + q;
                put(r, GL + lr, c01[e][q]);
                put(GL + lr, r, c01[e][q]);   // A is symmetric: the (1, 0) tile is the (0, 1) one transposed
                put(GL + r, GL + lr, c11[e][q]);
            }
        }
    }
    // ---- the lane's rows l and l + 16: residual b - J nu*, bounds, LDS offsets of its A row, its lambda and the
    //      lambda bounding it (absent rows: zeros, the dummy word, finite stand-in reads)
    float r0, r1, me0, me1, hi0, hi1, mu0, mu1, lam0 = 0.f, lam1 = 0.f;
    int ao0, ao1, lno0, lno1, lmo0, lmo1;
    {
        auto row_in = [&](int q, float& rq, float& meq, float& hiq, float& muq, int& aoq, int& lnoq, int& lmoq) {
            const bool v = q < neff;
            const int off = v ? pool_off<float>(pbase + q) : finite;
            const float* R = reinterpret_cast<const float*>(lds0 + off);
            const f4 s0 = *reinterpret_cast<const f4*>(R + RO_S0), s1 = *reinterpret_cast<const f4*>(R + RO_S1);
            rq = v ? s0.x - s1.y : 0.f;   // b - J nu*
            hiq = v ? s0.y : 0.f;
            meq = v ? s0.w : 0.f;
            muq = v ? s1.x : 0.f;
            lnoq = v ? __float_as_int(s1.w) : dummy;
            lmoq = v ? off + RO_LAM * (int)sizeof(float) : dummy;
            aoq = off;
        };
        row_in(l, r0, me0, hi0, mu0, ao0, lno0, lmo0);
        row_in(GL + l, r1, me1, hi1, mu1, ao1, lno1, lmo1);
    }
    // the env's row k for the velocity updates: its (M^-1 J^T)_l / _(16 + l) words (absent rows: finite stand-ins)
    const int mo0 = (2 * l + 1) * (int)sizeof(float), mo1 = (l < NV - GL ? 2 * (GL + l) + 1 : RO_Z) * (int)sizeof(float);
    auto row_off = [&](int k) { return k < neff ? pool_off<float>(pbase + k) : finite; };
    wave_sync();   // the A entries
    PGS_SUBPHASE(21);
    // one sweep over the rows; TWO: some env of the wave has rows in slot 1 (> 16 rows).  Steps come in chunks of 4
    // straight-line steps (the wave-uniform row count is tested once per chunk: a step past an env's rows is a no-op
    // dl = 0), so the LDS reads and writes of a chunk are counted exactly by the waitcnts
    float v0 = n0, v1 = n1;
    auto sweep = [&](auto two_c) {
        constexpr bool TWO = decltype(two_c)::value;
        constexpr int AH = 4;   // A and M^-1 J^T entries read AH steps ahead
        float a0v[AH], a1v[AH], m0v[AH], m1v[AH], lnv = 0.f;
        auto fetch = [&](int k, int j) {
            a0v[j] = *reinterpret_cast<const float*>(lds0 + ao0 + 2 * k * (int)sizeof(float));
            if constexpr (TWO) a1v[j] = *reinterpret_cast<const float*>(lds0 + ao1 + 2 * k * (int)sizeof(float));
            const int ro = row_off(k);
            m0v[j] = *reinterpret_cast<const float*>(lds0 + ro + mo0);
            m1v[j] = *reinterpret_cast<const float*>(lds0 + ro + mo1);
        };
        static_for<AH>([&](auto jc) { fetch(decltype(jc)::value, decltype(jc)::value); });
        static_for<(LMAX + 3) / 4>([&](auto cc) {
            constexpr int c0 = 4 * decltype(cc)::value;
            if (c0 >= M || (!TWO && c0 >= GL)) return;   // wave-uniform
            static_for<4>([&](auto jc) {
                constexpr int k = c0 + decltype(jc)::value;
                if constexpr (k < LMAX && (TWO || k < GL)) {
                    constexpr bool hi_slot = k >= GL;
                    const float a0k = a0v[k % AH], a1k = TWO ? a1v[k % AH] : 0.f, m0k = m0v[k % AH], m1k = m1v[k % AH];
                    if constexpr (k + AH < LMAX) fetch(k + AH, k % AH);
                    const float ln = lnv;
                    const float mu = hi_slot ? mu1 : mu0, hc = hi_slot ? hi1 : hi0, me = hi_slot ? me1 : me0;
                    const float rr = hi_slot ? r1 : r0, lamv = hi_slot ? lam1 : lam0;
                    const float lsol = med3(fmaf(me, rr, lamv), -(mu * ln), fmaf(mu, ln, hc));   // == clamp: lo <= hi
                    const float dl = lsol - lamv;
                    const int di = __float_as_int(dl);
                    // row_newbcast: the owner's (lane k % 16 of each env) dl to its env's 16 lanes
                    const float dlb = __int_as_float(__builtin_amdgcn_update_dpp(di, di, 0x150 + (k & (GL - 1)), 0xF, 0xF,
                                                                                 false));
                    const float lnew = l == (k & (GL - 1)) ? lsol : lamv;
                    if constexpr (hi_slot) {
                        lam1 = lnew;
                        *reinterpret_cast<float*>(lds0 + lmo1) = lnew;
                    } else {
                        lam0 = lnew;
                        *reinterpret_cast<float*>(lds0 + lmo0) = lnew;
                    }
                    // the bounding lambda of step k + 1 (a friction row's normal is at least one step earlier: its
                    // lambda of this sweep was stored before)
                    if constexpr (k + 1 < LMAX)
                        lnv = *reinterpret_cast<const float*>(lds0 + (k + 1 < GL ? lno0 : lno1));
                    r0 = fmaf(-a0k, dlb, r0);
                    if constexpr (TWO) r1 = fmaf(-a1k, dlb, r1);
                    v0 = fmaf(m0k, dlb, v0);
                    v1 = fmaf(m1k, dlb, v1);
                }
            });
        });
    };
#pragma unroll 1
    for (int it = 0; it < P.iters; it++) {
        if (TWOANY) sweep(std::true_type{});
        else sweep(std::false_type{});
    }
    PGS_SUBPHASE(22);
    n0 = v0;
    n1 = v1;
}

// ------------------------------------------------------------------------- ABA pass 2, one tree level
// Level tables (body per 4-lane group): children are always processed in an earlier level.
constexpr int LVL_BODY[4][4] = {{4, 6, 8, 10}, {3, 5, 7, 9}, {2, 2, 2, 2}, {1, 1, 1, 1}};
constexpr int LVL_KID[4][4][2] = {{{-1, -1}, {-1, -1}, {-1, -1}, {-1, -1}},
                                  {{4, -1}, {6, -1}, {8, -1}, {10, -1}},
                                  {{3, 5}, {3, 5}, {3, 5}, {3, 5}},
                                  {{2, -1}, {2, -1}, {2, -1}, {2, -1}}};
template <int LV>
__device__ inline int lvl_sel(int g, int (*f)(int)) {   // per-group compile-time value
    const int v0 = f(LVL_BODY[LV][0]), v1 = f(LVL_BODY[LV][1]), v2 = f(LVL_BODY[LV][2]), v3 = f(LVL_BODY[LV][3]);
    return g == 0 ? v0 : (g == 1 ? v1 : (g == 2 ? v2 : v3));
}
// joint damping of the group's body's j-th dof (0 past its dof count), selected among compile-time constants
template <int LV, typename T>
__device__ __attribute__((always_inline)) inline T lvl_damp(int g, int j) {
    T v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int x = LVL_BODY[LV][i];
        v[i] = j < body_ndof[x] ? (T)dof_damping[body_dof0[x] + j] : T(0);
    }
    return g == 0 ? v[0] : (g == 1 ? v[1] : (g == 2 ? v[2] : v[3]));
}

// The inputs of a level's body that pass 1 (or the FK) wrote: loaded one level early, while the previous level
// computes, so the LDS latency of only the children's contributions stays on the level-to-level chain.
template <typename T>
struct AbaIn { T IA[21], pA[6], c[6], u[3][3], tau[3], qd[3], ob[3], op[3]; };
template <int LV>
constexpr int aba_km() {   // the level's largest dof count (1, 3, 1, 2): smaller bodies of the level are padded to it
    int m = 0;
    for (int i = 0; i < 4; i++) m = body_ndof[LVL_BODY[LV][i]] > m ? body_ndof[LVL_BODY[LV][i]] : m;
    return m;
}
template <typename T, int LV>
__device__ __attribute__((always_inline)) void aba_load(const GroupLDS<T>& S, const int g, AbaIn<T>& in) {
    const auto& A = S.x.aba;
    constexpr int KM = aba_km<LV>();
    const int b = lvl_sel<LV>(g, [](int x) { return x; });
    const int k = lvl_sel<LV>(g, [](int x) { return body_ndof[x]; });
    const int d0 = lvl_sel<LV>(g, [](int x) { return body_dof0[x]; });
#pragma unroll
    for (int q = 0; q < 21; q++) in.IA[q] = A.IA[b][q];
#pragma unroll
    for (int e = 0; e < 6; e++) { in.pA[e] = A.pA[b][e]; in.c[e] = A.cl[b][e]; }
    const int p = lvl_sel<LV>(g, [](int x) { return body_parent[x]; });
#pragma unroll
    for (int i = 0; i < 3; i++) { in.ob[i] = S.o[b][i]; in.op[i] = S.o[p][i]; }
#pragma unroll
    for (int j = 0; j < KM; j++) {
        const int d = j < k ? d0 + j : d0;
#pragma unroll
        for (int i = 0; i < 3; i++) in.u[j][i] = S.Sc[d][i];
        in.tau[j] = S.tau[d];
        in.qd[j] = S.nu[6 + d];
    }
}

// Levels 1 and 3 take their first (level 3: only) child's contribution from registers: that child is the body the same
// lane group updated one level earlier (kIA / kpa, the previous call's oIA / opa); only level 1 stores its result (the
// pelvis and the base read the thighs and upper arms from LDS; the base reads lwaist from registers).
template <typename T, int LV>
__device__ __attribute__((always_inline)) void group_aba_level(const PhysParams& P, GroupLDS<T>& S, const int g, const T dt,
                                                               const AbaIn<T>& in, const T* kIA, const T* kpa, T* oIA,
                                                               T* opa) {
    constexpr bool KREG = LV == 1 || LV == 3, STORE = LV == 1;   // level 3 (lwaist): the base reads it from registers
    auto& A = S.x.aba;
    constexpr int KM = aba_km<LV>();
    const int b = lvl_sel<LV>(g, [](int x) { return x; });
    const int k = lvl_sel<LV>(g, [](int x) { return body_ndof[x]; });
    const int d0 = lvl_sel<LV>(g, [](int x) { return body_dof0[x]; });
    T IA[21], pAb[6], cb[6], u[3][3], U[3][6], D[9], Di[9], uj[3], W[3][6];
#pragma unroll
    for (int q = 0; q < 21; q++) IA[q] = in.IA[q];
#pragma unroll
    for (int e = 0; e < 6; e++) { pAb[e] = in.pA[e]; cb[e] = in.c[e]; }
    auto add_kid = [&](int kid) {
#pragma unroll
        for (int q = 0; q < 21; q++) IA[q] += A.IA[kid][q];
#pragma unroll
        for (int e = 0; e < 6; e++) pAb[e] += A.pA[kid][e];
    };
    // every group of a level has the same number of kids (0, 1 or 2)
    static_assert(!KREG || (LVL_KID[LV][0][0] == LVL_BODY[LV - 1][0] && LVL_KID[LV][1][0] == LVL_BODY[LV - 1][1] &&
                            LVL_KID[LV][2][0] == LVL_BODY[LV - 1][2] && LVL_KID[LV][3][0] == LVL_BODY[LV - 1][3]),
                  "a register child is the body the same group updated one level earlier");
    if constexpr (KREG) {
#pragma unroll
        for (int q = 0; q < 21; q++) IA[q] += kIA[q];
#pragma unroll
        for (int e = 0; e < 6; e++) pAb[e] += kpa[e];
    } else if constexpr (LVL_KID[LV][0][0] >= 0)
        add_kid(g == 0 ? LVL_KID[LV][0][0] : (g == 1 ? LVL_KID[LV][1][0] : (g == 2 ? LVL_KID[LV][2][0] : LVL_KID[LV][3][0])));
    if constexpr (LVL_KID[LV][0][1] >= 0)
        add_kid(g == 0 ? LVL_KID[LV][0][1] : (g == 1 ? LVL_KID[LV][1][1] : (g == 2 ? LVL_KID[LV][2][1] : LVL_KID[LV][3][1])));
    // about the body's pivot its hinge columns are [u; 0]: U = IA[:, 0:3] u, D = u . U[0:3], S^T pA = u . pA[0:3]
#pragma unroll
    for (int j = 0; j < KM; j++) {
        const bool on = j < k;
#pragma unroll
        for (int i = 0; i < 3; i++) u[j][i] = on ? in.u[j][i] : T(0);
#pragma unroll
        for (int e = 0; e < 6; e++) U[j][e] = IA[sidx(e, 0)] * u[j][0] + IA[sidx(e, 1)] * u[j][1] + IA[sidx(e, 2)] * u[j][2];
        T t = in.tau[j] - dot3(u[j], pAb);
        if (P.joint_damping) t -= lvl_damp<LV, T>(g, j) * in.qd[j];
        uj[j] = on ? t : T(0);
    }
#pragma unroll
    for (int i = 0; i < KM; i++) {
#pragma unroll
        for (int j = 0; j < KM; j++) D[3 * i + j] = dot3(u[i], U[j]);
        const bool on = i < k;
        if (P.joint_damping) D[4 * i] += dt * lvl_damp<LV, T>(g, i);
        D[4 * i] = on ? D[4 * i] : T(1);   // identity pivot for padded dofs
    }
    // LDL^T of the block (physics.h::ldl_small); the downdate through Y = U L^-T, W = U Dinv for the bias force
    T Lf[9], idd[3], Y[3][6];
    ldl_small<T, KM>(D, Lf, idd, Di);
#pragma unroll
    for (int j = 0; j < KM; j++)
#pragma unroll
        for (int e = 0; e < 6; e++) {
            T t = 0, y = U[j][e];
#pragma unroll
            for (int i = 0; i < KM; i++) t += U[i][e] * Di[3 * i + j];
#pragma unroll
            for (int q = 0; q < j; q++) y -= Lf[3 * j + q] * Y[q][e];
            W[j][e] = t;
            Y[j][e] = y;
        }
    // Ia = IA - sum_j Y_j idd_j Y_j^T (in place), pa = pA + Ia c + W u
#pragma unroll
    for (int r = 0; r < 6; r++)
#pragma unroll
        for (int cc = r; cc < 6; cc++) {
            T t = IA[sidx(r, cc)];
#pragma unroll
            for (int j = 0; j < KM; j++) t -= Y[j][r] * idd[j] * Y[j][cc];
            IA[sidx(r, cc)] = t;
        }
    T pa[6];
    symmv(IA, cb, pa);
#pragma unroll
    for (int e = 0; e < 6; e++) {
        T t = pAb[e] + pa[e];
#pragma unroll
        for (int j = 0; j < KM; j++) t += W[j][e] * uj[j];
        pa[e] = t;
    }
    {   // to the parent's pivot
        T r[3];
#pragma unroll
        for (int i = 0; i < 3; i++) r[i] = in.ob[i] - in.op[i];
        shift_force(r, pa);
        shift_inertia(r, IA);
    }
    // contribution to the parent in the body's own (now dead) slots; factorisation for passes 3 / responses.
    // The 4 lanes of a group (and groups sharing a body) write identical values.
#pragma unroll
    for (int q = 0; q < 21; q++) {
        oIA[q] = IA[q];
        if constexpr (STORE) A.IA[b][q] = IA[q];
    }
#pragma unroll
    for (int e = 0; e < 6; e++) {
        opa[e] = pa[e];
        if constexpr (STORE) A.pA[b][e] = pa[e];
    }
#pragma unroll
    for (int j = 0; j < KM; j++) {
        if (j < k) {
            T x[3];   // U at the common origin (pass 3, the constraint responses): [U_n + o_b x U_f; U_f]
            cross3(in.ob, U[j] + 3, x);
#pragma unroll
            for (int e = 0; e < 3; e++) { S.U[d0 + j][e] = U[j][e] + x[e]; S.U[d0 + j][3 + e] = U[j][3 + e]; }
            A.uu[d0 + j] = uj[j];
        }
    }
    const int doff = lvl_sel<LV>(g, [](int x) { return DINV.off[x]; });
#pragma unroll
    for (int i = 0; i < KM; i++)
#pragma unroll
        for (int j = 0; j < KM; j++)
            if (i < k && j < k) S.Dinv[doff + k * i + j] = Di[3 * i + j];
}

// ------------------------------------------------------------------------- ABA pass 3, one tree level
// Root -> leaves: {lwaist, upper arms} -> {pelvis, lower arms} -> {thighs} -> {shins}; body accelerations
// travel through the dead pass-1 velocity slots A.V.  Each group integrates its own dofs into nu*
// (groups sharing a body compute and write identical values).
constexpr int FWD_BODY[4][4] = {{1, 7, 9, 9}, {2, 8, 10, 10}, {3, 5, 3, 5}, {4, 6, 4, 6}};
template <int LV>
constexpr int fwd_km() {
    int m = 0;
    for (int i = 0; i < 4; i++) m = body_ndof[FWD_BODY[LV][i]] > m ? body_ndof[FWD_BODY[LV][i]] : m;
    return m;
}
template <int LV, typename F>
__device__ __attribute__((always_inline)) inline int fwd_sel(int g, F f) {   // per-group compile-time value
    const int v0 = f(FWD_BODY[LV][0]), v1 = f(FWD_BODY[LV][1]), v2 = f(FWD_BODY[LV][2]), v3 = f(FWD_BODY[LV][3]);
    return g == 0 ? v0 : (g == 1 ? v1 : (g == 2 ? v2 : v3));
}
// a level's inputs from pass 2 and the FK (everything but the parent's acceleration and velocity), loaded one level
// early like pass 2's (AbaIn)
template <typename T>
struct FwdIn { T c[6], U[3][6], uu[3], Dinv[9], Sc[3][6], nu[3]; };
template <typename T, int LV>
__device__ __attribute__((always_inline)) void fwd_load(const GroupLDS<T>& S, const int g, FwdIn<T>& in) {
    const auto& A = S.x.aba;
    constexpr int KM = fwd_km<LV>();
    const int b = fwd_sel<LV>(g, [](int x) { return x; });
    const int k = fwd_sel<LV>(g, [](int x) { return body_ndof[x]; });
    const int d0 = fwd_sel<LV>(g, [](int x) { return body_dof0[x]; });
    const int doff = fwd_sel<LV>(g, [](int x) { return DINV.off[x]; });
#pragma unroll
    for (int e = 0; e < 6; e++) in.c[e] = A.c[b][e];
#pragma unroll
    for (int j = 0; j < KM; j++) {
        const int d = j < k ? d0 + j : d0;
#pragma unroll
        for (int e = 0; e < 6; e++) in.U[j][e] = S.U[d][e];
        in.uu[j] = A.uu[d];
        load_sc(S, d, in.Sc[j]);
        in.nu[j] = S.nu[6 + d];
#pragma unroll
        for (int i = 0; i < KM; i++) in.Dinv[3 * i + j] = i < k && j < k ? S.Dinv[doff + k * i + j] : T(0);   // padded: 0
    }
}
// Levels 0, 1 and 3 take the parent's acceleration and velocity from registers (pa / pv): the base (computed on every
// lane) or the body the same lane group solved one level earlier; level 2's pelvis children read them from LDS.
template <int LV>
constexpr bool fwd_parent_in_regs() {
    if (LV == 2) return false;
    for (int i = 0; i < 4; i++)
        if (body_parent[FWD_BODY[LV][i]] != (LV == 0 ? 0 : FWD_BODY[LV - 1][i])) return false;
    return true;
}
template <typename T, int LV>
__device__ __attribute__((always_inline)) void group_fwd_level(const PhysParams& P, GroupLDS<T>& S, const int g, const T dt,
                                                               const FwdIn<T>& in, const T* pa, const T* pv, T* oa,
                                                               T* ov) {
    constexpr bool PREG = LV != 2;
    static_assert(!PREG || fwd_parent_in_regs<LV>(), "a register parent is the base or this group's previous body");
    auto& A = S.x.aba;
    const int b = fwd_sel<LV>(g, [](int x) { return x; });
    const int p = fwd_sel<LV>(g, [](int x) { return body_parent[x]; });
    const int k = fwd_sel<LV>(g, [](int x) { return body_ndof[x]; });
    const int d0 = fwd_sel<LV>(g, [](int x) { return body_dof0[x]; });
    constexpr int KM = fwd_km<LV>();
    const T vmax = (T)P.max_coord_vel;
    T ap[6], r[3], ab[6], vs[6];
#pragma unroll
    for (int e = 0; e < 6; e++) {
        ap[e] = (PREG ? pa[e] : A.V[p][e]) + in.c[e];
        ab[e] = ap[e];
        vs[e] = PREG ? pv[e] : S.Vs[p][e];
    }
#pragma unroll
    for (int j = 0; j < KM; j++) {
        T t = in.uu[j];
#pragma unroll
        for (int e = 0; e < 6; e++) t -= in.U[j][e] * ap[e];
        r[j] = j < k ? t : T(0);
    }
#pragma unroll
    for (int i = 0; i < KM; i++) {
        T t = 0;
#pragma unroll
        for (int j = 0; j < KM; j++) t += in.Dinv[3 * i + j] * r[j];   // padded block: 0, r = 0
        const int d = i < k ? d0 + i : d0;
        const T qdd = i < k ? t : T(0);
#pragma unroll
        for (int e = 0; e < 6; e++) ab[e] += in.Sc[i][e] * qdd;
        const T nn = clampT(in.nu[i] + dt * qdd, -vmax, vmax);
        if (i < k) S.nu[6 + d] = nn;
        // the body's velocity of nu*: its parent's plus its own dofs, in root-path order (the sums a per-row path
        // walk would form, in the same order)
        const T qn = i < k ? nn : T(0);
#pragma unroll
        for (int e = 0; e < 6; e++) vs[e] += in.Sc[i][e] * qn;
    }
#pragma unroll
    for (int e = 0; e < 6; e++) { A.V[b][e] = ab[e]; S.Vs[b][e] = vs[e]; oa[e] = ab[e]; ov[e] = vs[e]; }
}

// ------------------------------------------------------------------------- one cooperative substep
// Called by all 64 lanes of the block (uniform control flow at every __syncthreads).
// ---- FK by root-to-leaf chains.  The tree (torso; lwaist - pelvis - thigh - shin twice; upper - lower arm twice) is
// four chains of at most four bodies: {1 2 3 4}, {7 8}, {9 10}, {1 2 5 6} (the fourth repeats lwaist and pelvis rather
// than waiting for them).  Lane l of an env is chain l >> 2, frame row l & 3 (row 3 idle): a row of a body's frame
// depends only on the same row of its parent's frame (M = R_p Roff, o = o_p + R_p toff, and the hinge rotations mix
// columns within a row), so 12 lanes walk the four chains in four dependent steps instead of lane 0 composing all ten
// bodies.  Every value is formed by the same operations as forward_kinematics_pre (zero constants skipped, the same
// contracted expressions): the frames are bit-identical.  At a chain depth every chain's body has the same dof count;
// the per-lane constants are selects among the four chains' compile-time values.  Opt-in (-DHUM_FK_CHAIN): bitwise
// equal to the serial FK but 1.9 % slower same-box (35.84 vs 36.54 M env-steps/s; wave log FK 19.1 K -> 26.8 K cycles
// per block-step, profiles/r05_fk_chain_ab.txt): the selects and zero-skip compares triple the FK's VALU instructions,
// and at one wave per SIMD a VALU instruction costs its issue slot whatever its exec mask.
constexpr int FK_CH[4][4] = {{1, 2, 3, 4}, {7, 8, -1, -1}, {9, 10, -1, -1}, {1, 2, 5, 6}};
constexpr double fk_roff(int dd, int ch, int k) { return FK_CH[ch][dd] < 0 ? 0.0 : body_Roff[9 * FK_CH[ch][dd] + k]; }
constexpr double fk_toff(int dd, int ch, int k) { return FK_CH[ch][dd] < 0 ? 0.0 : body_toff[3 * FK_CH[ch][dd] + k]; }
constexpr int fk_body(int dd, int ch) { return FK_CH[ch][dd]; }
constexpr int fk_dof(int dd, int ch, int k) { return FK_CH[ch][dd] < 0 ? 0 : body_dof0[FK_CH[ch][dd]] + k; }
constexpr int fk_ndof(int dd) { return body_ndof[FK_CH[0][dd]]; }
constexpr bool fk_uniform_axis(int dd, int k) {
    for (int c = 1; c < 4; c++)
        if (FK_CH[c][dd] >= 0 && dof_axis[fk_dof(dd, c, k)] != dof_axis[fk_dof(dd, 0, k)]) return false;
    return true;
}
constexpr bool fk_check() {   // same dof count across the chains at each depth
    for (int dd = 0; dd < 4; dd++)
        for (int c = 0; c < 4; c++)
            if (FK_CH[c][dd] >= 0 && body_ndof[FK_CH[c][dd]] != fk_ndof(dd)) return false;
    return true;
}
static_assert(NB == 11 && fk_check(), "FK chains: the humanoid tree of model_gen.h");
template <typename T>
__device__ __attribute__((always_inline)) inline T fk_sel(int ch, double v0, double v1, double v2, double v3) {
    return ch == 0 ? (T)v0 : (ch == 1 ? (T)v1 : (ch == 2 ? (T)v2 : (T)v3));
}
__device__ __attribute__((always_inline)) inline int fk_seli(int ch, int v0, int v1, int v2, int v3) {
    return ch == 0 ? v0 : (ch == 1 ? v1 : (ch == 2 ? v2 : v3));
}
// one row of rot_post (physics.h): the same expressions, the axis per lane
template <typename T>
__device__ __attribute__((always_inline)) inline void fk_rot_row(T* m, int ax, T c, T s) {
#pragma clang fp contract(on)   // per-expression fusion only, as rot_post
    const T mi = ax == 0 ? m[1] : (ax == 1 ? m[2] : m[0]);   // column (ax + 1) % 3
    const T mj = ax == 0 ? m[2] : (ax == 1 ? m[0] : m[1]);   // column (ax + 2) % 3
    const T ni = c * mi + s * mj;
    const T nj = -s * mi + c * mj;
    m[0] = ax == 0 ? m[0] : (ax == 1 ? nj : ni);
    m[1] = ax == 0 ? ni : (ax == 1 ? m[1] : nj);
    m[2] = ax == 0 ? nj : (ax == 1 ? ni : m[2]);
}
template <typename T, int AX>
__device__ __attribute__((always_inline)) inline void fk_rot_row_c(T* m, T c, T s) {
#pragma clang fp contract(on)
    constexpr int i = (AX + 1) % 3, j = (AX + 2) % 3;
    const T mi = m[i], mj = m[j];
    m[i] = c * mi + s * mj;
    m[j] = -s * mi + c * mj;
}
// chain depth DD for lane (ch, row): Rp / op = the parent's frame row in, the body's out; publishes it
template <typename T, int DD>
__device__ __attribute__((always_inline)) inline void fk_depth(GroupLDS<T>& S, const T* scs, int ch, int row, T* Rp, T& op) {
#pragma clang fp contract(on)
    const int b = fk_seli(ch, fk_body(DD, 0), fk_body(DD, 1), fk_body(DD, 2), fk_body(DD, 3));
    if (b < 0) return;
    T M[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {   // (R_p Roff)[row][c] as forward_kinematics_pre forms it
        const T c0 = fk_sel<T>(ch, fk_roff(DD, 0, c), fk_roff(DD, 1, c), fk_roff(DD, 2, c), fk_roff(DD, 3, c));
        const T c1 = fk_sel<T>(ch, fk_roff(DD, 0, 3 + c), fk_roff(DD, 1, 3 + c), fk_roff(DD, 2, 3 + c), fk_roff(DD, 3, 3 + c));
        const T c2 = fk_sel<T>(ch, fk_roff(DD, 0, 6 + c), fk_roff(DD, 1, 6 + c), fk_roff(DD, 2, 6 + c), fk_roff(DD, 3, 6 + c));
        T m = c0 == T(0) ? T(-0.0) : Rp[0] * c0;
        m = c1 == T(0) ? m : fma(Rp[1], c1, m);
        M[c] = c2 == T(0) ? m : fma(Rp[2], c2, m);
    }
    {
        const T t0 = fk_sel<T>(ch, fk_toff(DD, 0, 0), fk_toff(DD, 1, 0), fk_toff(DD, 2, 0), fk_toff(DD, 3, 0));
        const T t1 = fk_sel<T>(ch, fk_toff(DD, 0, 1), fk_toff(DD, 1, 1), fk_toff(DD, 2, 1), fk_toff(DD, 3, 1));
        const T t2 = fk_sel<T>(ch, fk_toff(DD, 0, 2), fk_toff(DD, 1, 2), fk_toff(DD, 2, 2), fk_toff(DD, 3, 2));
        T o = t0 == T(0) ? op : fma(Rp[0], t0, op);
        o = t1 == T(0) ? o : fma(Rp[1], t1, o);
        op = t2 == T(0) ? o : fma(Rp[2], t2, o);
    }
    const bool pub = ch != 3 || DD >= 2;   // chain 3 repeats lwaist and pelvis, which chain 0 publishes
    static_for<fk_ndof(DD)>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const int d = fk_seli(ch, fk_dof(DD, 0, k), fk_dof(DD, 1, k), fk_dof(DD, 2, k), fk_dof(DD, 3, k));
        const T sg = fk_sel<T>(ch, dof_sign[fk_dof(DD, 0, k)], dof_sign[fk_dof(DD, 1, k)], dof_sign[fk_dof(DD, 2, k)],
                               dof_sign[fk_dof(DD, 3, k)]);
        const T cs = scs[2 * d + 1], sn = sg * scs[2 * d];
        if constexpr (fk_uniform_axis(DD, k)) {
            constexpr int AX = dof_axis[fk_dof(DD, 0, k)];
            if (pub) S.Sc[d][row] = M[AX] * sg;
            fk_rot_row_c<T, AX>(M, cs, sn);
        } else {
            const int ax = fk_seli(ch, dof_axis[fk_dof(DD, 0, k)], dof_axis[fk_dof(DD, 1, k)], dof_axis[fk_dof(DD, 2, k)],
                                   dof_axis[fk_dof(DD, 3, k)]);
            if (pub) S.Sc[d][row] = (ax == 0 ? M[0] : (ax == 1 ? M[1] : M[2])) * sg;
            fk_rot_row(M, ax, cs, sn);
        }
    });
    if (pub) {
#pragma unroll
        for (int c = 0; c < 3; c++) S.R[b][3 * row + c] = M[c];
        S.o[b][row] = op;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) Rp[c] = M[c];
}

template <typename T, int EPB_, bool TERRAIN = false>   // TERRAIN: heightfield ground (hum_set_terrain)
__device__ __attribute__((always_inline)) void group_substep(const PhysParams& P, GroupLDS<T>* shb, const int ge,
                                                             T* gblock, const int l, unsigned& ef,
                                                             unsigned long long tkey,   // tkey: terrain 2
                                                             const bool frozen = false) {   // env takes no step
    static_assert(EPB_ * GL <= 64, "a block is one wavefront (phase_sync)");
    GroupLDS<T>& S = shb[ge];
    const ModelTab<T>& M = tab_fresh<T>();
    const T dt = (T)P.dt;
    PHASE_INIT;
    HUM_STOP(0);
    // ---- FK (every lane, registers); lane 0 publishes
    {
        // the 17 hinge angles' sin / cos once, one per lane (scratch: the ABA transients are dead until pass 1)
        T* scs = &S.x.aba.IA[0][0];
        for (int d = l; d < NDOF; d += GL) {
            T sn, cs;
            hinge_sincos(S.st[13 + d], &sn, &cs);
            scs[2 * d] = sn;
            scs[2 * d + 1] = cs;
        }
        wave_sync();
        SUBPHASE(11);
        T quat[4];
#pragma unroll
        for (int e = 0; e < 4; e++) quat[e] = S.st[3 + e];
#ifndef HUM_FK_CHAIN   // lane 0 composes every body (forward_kinematics_pre) and publishes
        Kin<T> K;
        forward_kinematics_pre(quat, scs, K);
        SUBPHASE(12);
        if (l == 0) {
#pragma unroll
            for (int b = 0; b < NB; b++) {
#pragma unroll
                for (int i = 0; i < 9; i++) S.R[b][i] = K.R[b][i];
#pragma unroll
                for (int i = 0; i < 3; i++) S.o[b][i] = K.o[b][i];
            }
#pragma unroll
            for (int d = 0; d < NDOF; d++)   // the hinge axes: the first half of the motion subspace columns
#pragma unroll
                for (int i = 0; i < 3; i++) S.Sc[d][i] = K.u[d][i];
        }
#else
        {   // -DHUM_FK_CHAIN (measured slower): lane (chain l >> 2, row l & 3) walks a chain
            const int ch = l >> 2, row = l & 3;
            if (row < 3) {
                T R0[9];
                quat_to_mat(quat, R0);
                T Rp[3], op = T(0);
#pragma unroll
                for (int c = 0; c < 3; c++) Rp[c] = row == 0 ? R0[c] : (row == 1 ? R0[3 + c] : R0[6 + c]);
                if (ch == 0) {
#pragma unroll
                    for (int c = 0; c < 3; c++) S.R[0][3 * row + c] = Rp[c];
                    S.o[0][row] = T(0);
                }
                fk_depth<T, 0>(S, scs, ch, row, Rp, op);
                fk_depth<T, 1>(S, scs, ch, row, Rp, op);
                fk_depth<T, 2>(S, scs, ch, row, Rp, op);
                fk_depth<T, 3>(S, scs, ch, row, Rp, op);
            }
        }
        SUBPHASE(12);
#endif
        if (l < 16) {   // generalised velocity
            S.nu[l] = l < 3 ? S.st[10 + l] : (l < 6 ? S.st[7 + l - 3] : S.st[30 + l - 6]);
            if (l < NV - 16) S.nu[16 + l] = S.st[30 + 10 + l];
        }
        wave_sync();
        for (int d = l; d < NDOF; d += GL) {   // motion subspace columns [u; o_b x u], one dof per lane
            const int b = dof_body_l(d);
            T ob[3], u[3];
#pragma unroll
            for (int i = 0; i < 3; i++) { ob[i] = S.o[b][i]; u[i] = S.Sc[d][i]; }
            cross3(ob, u, S.Sc[d] + 3);
        }
    }
    phase_sync();
    PHASE(1);
    HUM_STOP(1);
    // ---- ABA pass 1: lane b = body b
    if (l < NB) {
        const int b = l;
        T V[6];
        {   // parent velocity: the base velocity plus the parent's root-path dofs in path order (the sums a tree-depth
            // sweep forms, without its 4 synchronised steps; the torso: the base velocity itself)
            const int p = body_parent_l(b), e1 = path_e1_l(p), s2 = path_s2_l(p), n = path_len_l(p);
#pragma unroll
            for (int e = 0; e < 6; e++) V[e] = S.nu[e];
#pragma unroll
            for (int j = 0; j < PPATH_MAX; j++) {
                if (j < n) {
                    const int d = j < e1 ? j : s2 + (j - e1);
                    T Sc[6];
                    load_sc(S, d, Sc);
                    const T qd = S.nu[6 + d];
#pragma unroll
                    for (int e = 0; e < 6; e++) V[e] += Sc[e] * qd;
                }
            }
        }
        SUBPHASE(13);
        // passes 1 and 2 run about the body's own pivot o_b (physics.h::aba): the parent's velocity moved to o_b,
        // then the body's dofs, whose columns there are [u; 0]; bias acceleration sum_k V^(k) x [u_k qd_k; 0]
        T Rb[9], ob[3];
#pragma unroll
        for (int i = 0; i < 9; i++) Rb[i] = S.R[b][i];
#pragma unroll
        for (int i = 0; i < 3; i++) ob[i] = S.o[b][i];
        {
            T x[3];
            cross3(V, ob, x);
#pragma unroll
            for (int i = 0; i < 3; i++) V[3 + i] += x[i];
        }
        T cb[6] = {0, 0, 0, 0, 0, 0};
        const int k = body_ndof_l(b), d0 = body_dof0_l(b);
        for (int j = 0; j < k; j++) {
            const int d = d0 + j;
            const T qd = S.nu[6 + d];
            const T uq[3] = {S.Sc[d][0] * qd, S.Sc[d][1] * qd, S.Sc[d][2] * qd};
#pragma unroll
            for (int i = 0; i < 3; i++) V[i] += uq[i];
            T wx[3], vx[3];
            cross3(V, uq, wx);
            cross3(V + 3, uq, vx);
#pragma unroll
            for (int i = 0; i < 3; i++) { cb[i] += wx[i]; cb[3 + i] += vx[i]; }
        }
        T c3[3], Icw[9], IA[21], h[6], pA[6];
#pragma unroll
        for (int i = 0; i < 3; i++) c3[i] = Rb[3 * i] * M.com[b][0] + Rb[3 * i + 1] * M.com[b][1] + Rb[3 * i + 2] * M.com[b][2];
        {
            T RI[9];
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int cc = 0; cc < 3; cc++)
                    RI[3 * r + cc] = Rb[3 * r] * M.inertia[b][cc] + Rb[3 * r + 1] * M.inertia[b][3 + cc] + Rb[3 * r + 2] * M.inertia[b][6 + cc];
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int cc = 0; cc < 3; cc++) Icw[3 * r + cc] = RI[3 * r] * Rb[3 * cc] + RI[3 * r + 1] * Rb[3 * cc + 1] + RI[3 * r + 2] * Rb[3 * cc + 2];
        }
        spatial_inertia(M.mass[b], c3, Icw, IA);
        symmv(IA, V, h);
        crf(V, h, pA);
        const T mg = -M.mass[b] * (T)P.gravity;
        pA[0] -= c3[1] * mg;
        pA[1] -= -c3[0] * mg;
        pA[5] -= mg;
        SUBPHASE(14);
        for (int q = 0; q < body_nlink_l(b); q++) {   // Bullet per-link velocity damping
            const int lk = body_link0_l(b) + q;
            T cl[3], vc[3], Iw[9], wI[3];
#pragma unroll
            for (int i = 0; i < 3; i++) cl[i] = Rb[3 * i] * M.lcom[lk][0] + Rb[3 * i + 1] * M.lcom[lk][1] + Rb[3 * i + 2] * M.lcom[lk][2];
            cross3(V, cl, vc);
#pragma unroll
            for (int i = 0; i < 3; i++) vc[i] += V[3 + i];
            const T kv = (T)P.lin_damp * (T(1) + psqrt(dot3(vc, vc)));
            const T kw = (T)P.ang_damp * (T(1) + psqrt(dot3(V, V)));
            {
                T RI[9];
#pragma unroll
                for (int r = 0; r < 3; r++)
#pragma unroll
                    for (int cc = 0; cc < 3; cc++)
                        RI[3 * r + cc] = Rb[3 * r] * M.linertia[lk][cc] + Rb[3 * r + 1] * M.linertia[lk][3 + cc] + Rb[3 * r + 2] * M.linertia[lk][6 + cc];
#pragma unroll
                for (int r = 0; r < 3; r++)
#pragma unroll
                    for (int cc = 0; cc < 3; cc++) Iw[3 * r + cc] = RI[3 * r] * Rb[3 * cc] + RI[3 * r + 1] * Rb[3 * cc + 1] + RI[3 * r + 2] * Rb[3 * cc + 2];
            }
#pragma unroll
            for (int i = 0; i < 3; i++) wI[i] = Iw[3 * i] * V[0] + Iw[3 * i + 1] * V[1] + Iw[3 * i + 2] * V[2];
            const T m = M.lmass[lk];
            T F[3], n[3], cxF[3];
#pragma unroll
            for (int i = 0; i < 3; i++) { F[i] = -m * vc[i] * kv; n[i] = -wI[i] * kw; }
            cross3(cl, F, cxF);
#pragma unroll
            for (int i = 0; i < 3; i++) { pA[i] -= n[i] + cxF[i]; pA[3 + i] -= F[i]; }
        }
        T cx[3];   // the bias acceleration at the common origin for pass 3: v_O = v_b - w x o_b
        cross3(cb, ob, cx);
#pragma unroll
        for (int e = 0; e < 6; e++) {
            S.x.aba.cl[b][e] = cb[e];
            S.x.aba.c[b][e] = e < 3 ? cb[e] : cb[e] - cx[e - 3];
            S.x.aba.pA[b][e] = pA[e];
        }
#pragma unroll
        for (int q = 0; q < 21; q++) S.x.aba.IA[b][q] = IA[q];
    }
    phase_sync();
    PHASE(2);
    HUM_STOP(2);
    // ---- ABA pass 2 (leaves -> root) by tree level: 4 steps {shins, lower arms} -> {thighs, upper arms}
    //      -> pelvis -> lwaist instead of 10 sequential bodies.  In a step, lane group g (4 lanes) updates
    //      one body redundantly in registers (dof count padded to 3 with identity pivots, so every body runs
    //      the same branch-free code), sums its own articulated inertia/bias force with its children's
    //      contributions, and overwrites its IA/pA slots with its contribution to the parent (no longer
    //      needed itself).  The base step below sums the torso with lwaist and both upper arms.
    auto& A = S.x.aba;
    T kIA[21], kpa[6];   // the contribution to the parent of the body this group updated last (after level 3: lwaist)
    {
        AbaIn<T> in0, in1;
        aba_load<T, 0>(S, l >> 2, in0);
        aba_load<T, 1>(S, l >> 2, in1);
        group_aba_level<T, 0>(P, S, l >> 2, dt, in0, kIA, kpa, kIA, kpa);
        aba_load<T, 2>(S, l >> 2, in0);
        group_aba_level<T, 1>(P, S, l >> 2, dt, in1, kIA, kpa, kIA, kpa);
        wave_sync();   // level 2 (the pelvis) reads both thighs' contributions from LDS
        aba_load<T, 3>(S, l >> 2, in1);
        group_aba_level<T, 2>(P, S, l >> 2, dt, in0, kIA, kpa, kIA, kpa);
        group_aba_level<T, 3>(P, S, l >> 2, dt, in1, kIA, kpa, kIA, kpa);
    }
    phase_sync();
    PHASE(3);
    HUM_STOP(3);
    // ---- base + pass 3 (redundant on every lane); lane 0 publishes L0 and nu* = clamp(nu + dt acc)
    {
        // base (redundant on every lane), then the forward pass by tree level (root -> leaves, one body per
        // 4-lane group, see group_fwd_level); lane 0 integrates the base and publishes L0 (inverse-diagonal form)
        const T vmax = (T)P.max_coord_vel;
        FwdIn<T> fin0, fin1;
        fwd_load<T, 0>(S, l >> 2, fin0);   // read while the base solve runs
        T L[21], a0[6], IA0[21], nub[6];
#pragma unroll
        for (int q = 0; q < 21; q++) IA0[q] = A.IA[0][q] + kIA[q] + A.IA[7][q] + A.IA[9][q];   // torso + kids
        chol6_inv(IA0, L);
#pragma unroll
        for (int e = 0; e < 6; e++) a0[e] = -(A.pA[0][e] + kpa[e] + A.pA[7][e] + A.pA[9][e]);
        chol6_solve_inv(L, a0);
#pragma unroll
        for (int e = 0; e < 6; e++) nub[e] = S.nu[e];
        T nus[6];   // the base's nu*: the torso's velocity for the forward levels' body velocities
        {
            T wxv[3];
            cross3(nub, nub + 3, wxv);
#pragma unroll
            for (int i = 0; i < 3; i++) {
                nus[i] = clampT(nub[i] + dt * a0[i], -vmax, vmax);
                nus[3 + i] = clampT(nub[3 + i] + dt * (a0[3 + i] + wxv[i]), -vmax, vmax);
            }
        }
        if (l == 0) {
#pragma unroll
            for (int e = 0; e < 6; e++) { A.V[0][e] = a0[e]; S.Vs[0][e] = nus[e]; }
        }
        SUBPHASE(15);
        T fa[6], fv[6];   // acceleration and velocity of the body this group solved last
        fwd_load<T, 1>(S, l >> 2, fin1);
        group_fwd_level<T, 0>(P, S, l >> 2, dt, fin0, a0, nus, fa, fv);
        fwd_load<T, 2>(S, l >> 2, fin0);
        group_fwd_level<T, 1>(P, S, l >> 2, dt, fin1, fa, fv, fa, fv);
        wave_sync();   // level 2 (thighs) reads the pelvis from LDS
        fwd_load<T, 3>(S, l >> 2, fin1);
        group_fwd_level<T, 2>(P, S, l >> 2, dt, fin0, fa, fv, fa, fv);
        group_fwd_level<T, 3>(P, S, l >> 2, dt, fin1, fa, fv, fa, fv);
        if (l == 0) {
#pragma unroll
            for (int q = 0; q < 21; q++) S.L0[q] = L[q];
#pragma unroll
            for (int e = 0; e < 6; e++) S.nu[e] = nus[e];
        }
    }
    phase_sync();
    PHASE(4);
    HUM_STOP(4);
    // ---- geom endpoints (lane g; lane 0 also the 17th) and joint-limit scan
    auto& C = S.x.cr;
    // per-geom table for the contact phase, in the row storage the rows phase has not written yet (the survivor
    // list sits two rows above): endpoint sum and bounding radius (the broad phase's pair test reads two such
    // quads), then radius and body (ground points, narrow phase) - LDS reads instead of per-lane selects among
    // compile-time constants
    T* gsum = &C.row[MAXR_LDS - 6][0];
    static_assert(3 * RW >= 8 * NGEOM && MAXR_LDS >= 6, "three rows hold the contact phase's geom table");
    for (int g = l; g < NGEOM; g += GL) {
        const int b = geom_body_l(g);
        T e0[3], e1[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            e0[i] = S.o[b][i] + S.R[b][3 * i] * M.gp1[g][0] + S.R[b][3 * i + 1] * M.gp1[g][1] + S.R[b][3 * i + 2] * M.gp1[g][2];
            e1[i] = S.o[b][i] + S.R[b][3 * i] * M.gp2[g][0] + S.R[b][3 * i + 1] * M.gp2[g][1] + S.R[b][3 * i + 2] * M.gp2[g][2];
            C.gp[g][0][i] = e0[i];
            C.gp[g][1][i] = e1[i];
        }
#pragma unroll
        for (int i = 0; i < 3; i++) gsum[8 * g + i] = e0[i] + e1[i];
        gsum[8 * g + 3] = geom_br_l<T>(g);
        gsum[8 * g + 4] = geom_r_l<T>(g);
        gsum[8 * g + 5] = (T)b;
    }
    const int gbit = (threadIdx.x & 63) & ~(GL - 1);   // first lane of this group in the wave
    const unsigned long long lanemask_lt = (1ull << (threadIdx.x & 63)) - 1ull;
    int nl = 0;
#pragma unroll
    for (int rd = 0; rd < 2; rd++) {   // dofs 0..15, then dof 16 (lane 0)
        const int d = rd * GL + l;
        bool lowv = false, hiv = false;
        if (d < NDOF) {
            const T q = S.st[13 + d];
            lowv = (q - M.lo[d]) <= 0;
            hiv = (M.hi[d] - q) <= 0;
        }
        // each dof yields up to 2 rows (lower first); count per lane then prefix within the group
        const int cnt = (int)lowv + (int)hiv;
        const unsigned long long b1 = __ballot(cnt >= 1), b2 = __ballot(cnt >= 2);
        const unsigned long long gm1 = (b1 >> gbit) & 0xFFFFull, gm2 = (b2 >> gbit) & 0xFFFFull;
        const unsigned long long below = ((lanemask_lt >> gbit) & 0xFFFFull);
        const int pos = nl + __popcll(gm1 & below) + __popcll(gm2 & below);
        if (lowv) C.rdesc[pos] = d | (0 << 8);
        if (hiv) C.rdesc[pos + (int)lowv] = d | (1 << 8);
        nl += __popcll(gm1) + __popcll(gm2);
    }
    phase_sync();
    PHASE(5);
    HUM_STOP(5);
    // ---- contacts, compacted in candidate order (ground points, then geom pairs)
    const int maxc = P.max_contacts < MAXC_G ? P.max_contacts : MAXC_G;
    int nc = 0, over = 0;
    const T basez = S.st[2];
    const unsigned long long below16 = (lanemask_lt >> gbit) & 0xFFFFull;
    // the candidate descriptors below are loop-invariant: an opaque copy of the lane index keeps the
    // compiler from hoisting them out of the substep loop into registers held across every phase
    int lc = l;
    asm volatile("" : "+v"(lc));
    T* gcon = gblock + gcon_offset(EPB_, P.lds_rows, ge);   // this env's contacts past MAXC_LDS
    auto emit = [&](bool hit, int ba, int bb, const T* pa, const T* pb, const T* n, T d) {
        const unsigned long long bm = (__ballot(hit) >> gbit) & 0xFFFFull;
        const int pos = nc + __popcll(bm & below16);
        if (hit) {
            if (pos < maxc) {
                if (pos < MAXC_LDS) {
                    T* e = C.con[pos];
                    e[0] = (T)ba; e[1] = (T)bb;
#pragma unroll
                    for (int i = 0; i < 3; i++) { e[2 + i] = pa[i]; e[5 + i] = pb[i]; e[8 + i] = n[i]; }
                    e[11] = d;
                } else {
                    T* e = gcon + (long)(pos - MAXC_LDS) * CW;
                    __builtin_nontemporal_store((T)ba, e);
                    __builtin_nontemporal_store((T)bb, e + 1);
#pragma unroll
                    for (int i = 0; i < 3; i++) {
                        __builtin_nontemporal_store(pa[i], e + 2 + i);
                        __builtin_nontemporal_store(pb[i], e + 5 + i);
                        __builtin_nontemporal_store(n[i], e + 8 + i);
                    }
                    __builtin_nontemporal_store(d, e + 11);
                }
            } else {
                over = 1;
            }
        }
        nc += __popcll(bm);
    };
    if constexpr (!TERRAIN) {
#pragma unroll
        for (int r = 0; r < CC_GROUND; r++) {   // sphere / capsule end vs plane (cheap, exact)
            const int gd = lane16(lc, CDESC.g[r][0], CDESC.g[r][1], CDESC.g[r][2], CDESC.g[r][3]);
            bool hit = false;
            int ba = 0;
            T pa[3] = {0, 0, 0}, n[3] = {0, 0, 1}, d = 0;
            if (gd != 0xffff) {
                const int ga = gd & 31, e = (gd >> 5) & 1;
                const T gr = gsum[8 * ga + 4];
                const T* p = C.gp[ga][e];
                d = basez + p[2] - gr;
                hit = d < (T)P.contact_thresh;
                ba = gd >> 6;
                pa[0] = p[0]; pa[1] = p[1]; pa[2] = p[2] - gr;
            }
            emit(hit, ba, -1, pa, pa, n, d);
        }
    } else {
        // heightfield (terrain.h): the same candidates against the closest point of the terrain surface (a
        // separate kernel instantiation, so the plane kernel carries none of this code)
#pragma unroll 1
        for (int r = 0; r < CC_GROUND; r++) {
            const int gd = lane16(lc, CDESC.g[r][0], CDESC.g[r][1], CDESC.g[r][2], CDESC.g[r][3]);
            bool hit = false;
            int ba = 0;
            T pa[3] = {0, 0, 0}, n[3] = {0, 0, 1}, d = 0;
            if (gd != 0xffff) {
                const int ga = gd & 31, e = (gd >> 5) & 1;
                const T gr = gsum[8 * ga + 4];
                const T* p = C.gp[ga][e];
                const T cw[3] = {S.st[0] + p[0], S.st[1] + p[1], basez + p[2]};
                hit = terrain_contact<T>(P, tkey, cw, gr, n, d);
                ba = gd >> 6;
#pragma unroll
                for (int i = 0; i < 3; i++) pa[i] = p[i] - gr * n[i];
            }
            emit(hit, ba, -1, pa, pa, n, d);
        }
        // capsule axes across convex terrain edges (terrain.h ridge_contacts): lane l takes capsule l; slot 0 of every
        // capsule, then slot 1 (the oracle's order)
        {
            const int cd = lane16(lc, CAPDESC.c[0], CAPDESC.c[1], CAPDESC.c[2], CAPDESC.c[3]);
            T rn[RIDGE_MAX][3], rd[RIDGE_MAX], rt[RIDGE_MAX];
            int nr = 0;
            const int ga = cd & 31;
            if (cd != 0xffff) {
                const T* p1 = C.gp[ga][0];
                const T* p2 = C.gp[ga][1];
                const T aw[3] = {S.st[0] + p1[0], S.st[1] + p1[1], basez + p1[2]};
                const T bw[3] = {S.st[0] + p2[0], S.st[1] + p2[1], basez + p2[2]};
                nr = ridge_contacts<T>(P, tkey, aw, bw, gsum[8 * ga + 4], rn, rd, rt);
            }
#pragma unroll
            for (int slot = 0; slot < RIDGE_MAX; slot++) {
                const bool hit = slot < nr;
                T pa[3] = {0, 0, 0}, n[3] = {0, 0, 1}, d = 0;
                if (hit) {
                    const T* p1 = C.gp[ga][0];
                    const T* p2 = C.gp[ga][1];
                    const T gr = gsum[8 * ga + 4];
#pragma unroll
                    for (int i = 0; i < 3; i++) {
                        n[i] = rn[slot][i];
                        pa[i] = p1[i] + rt[slot] * (p2[i] - p1[i]) - gr * n[i];
                    }
                    d = rd[slot];
                }
                emit(hit, cd >> 6, -1, pa, pa, n, d);
            }
        }
    }
    if (P.self_collision) {
        // broad phase: bounding spheres about the segment midpoints (conservative margin), survivors listed
        // in pair order in the (not yet used) row storage; narrow phase (segment-segment) on survivors only
        int* surv = reinterpret_cast<int*>(&C.row[MAXR_LDS - 3][0]);
        const T reach = (T)P.contact_thresh + (T)1e-3;
        int ns = 0;
#pragma unroll
        for (int r = 0; r < CC_PAIR; r++) {
            const int pd = lane16(lc, CDESC.p[r][0], CDESC.p[r][1], CDESC.p[r][2], CDESC.p[r][3]);
            bool maybe = false;
            if (pd != 0xffff) {
                const int ga = pd & 31, gb = pd >> 5;
                T qa[4], qb[4], dm[3];
                if constexpr (sizeof(T) == 4) {
                    using f4v = float __attribute__((ext_vector_type(4)));
                    const f4v va = *reinterpret_cast<const f4v*>(gsum + 8 * ga), vb = *reinterpret_cast<const f4v*>(gsum + 8 * gb);
                    qa[0] = va.x; qa[1] = va.y; qa[2] = va.z; qa[3] = va.w;
                    qb[0] = vb.x; qb[1] = vb.y; qb[2] = vb.z; qb[3] = vb.w;
                } else {
#pragma unroll
                    for (int i = 0; i < 4; i++) { qa[i] = gsum[8 * ga + i]; qb[i] = gsum[8 * gb + i]; }
                }
#pragma unroll
                for (int i = 0; i < 3; i++) dm[i] = qa[i] - qb[i];   // (pa1 + pa2) - (pb1 + pb2)
                const T rr = qa[3] + qb[3] + reach;
                maybe = dot3(dm, dm) < T(4) * rr * rr;   // |ma - mb| < rr with ma = (p1 + p2) / 2
            }
            const unsigned long long bm = (__ballot(maybe) >> gbit) & 0xFFFFull;
            if (maybe) surv[ns + __popcll(bm & below16)] = pd;   // survivors in pair order: ga | gb << 5
            ns += __popcll(bm);
        }
        wave_sync();
        WLOG(3, (env_max<EPB_>(ns) + GL - 1) / GL);
        for (int r0 = 0; r0 < ns; r0 += GL) {
            const int j = r0 + l;
            bool hit = false;
            int ba = 0, bb = -1;
            T pa[3] = {0, 0, 0}, pb[3] = {0, 0, 0}, n[3] = {0, 0, 1}, d = 0;
            if (j < ns) {
                const int pd = surv[j], ga = pd & 31, gb = pd >> 5;
#ifdef HUM_CHECK_LINKS
                if ((unsigned)ga >= (unsigned)NGEOM || (unsigned)gb >= (unsigned)NGEOM) atomicAdd(&g_check[4], 1u);
#endif
                T ca[3], cb[3], dv[3];
                seg_seg(C.gp[ga][0], C.gp[ga][1], C.gp[gb][0], C.gp[gb][1], ca, cb);
#pragma unroll
                for (int i = 0; i < 3; i++) dv[i] = ca[i] - cb[i];
                const T dist = psqrt(dot3(dv, dv));
                const T ra = gsum[8 * ga + 4], rb = gsum[8 * gb + 4];
                d = dist - ra - rb;
                hit = d < (T)P.contact_thresh && dist > (T)1e-9;
                if (hit) {
                    const T idist = prcp_geo(dist);
#pragma unroll
                    for (int i = 0; i < 3; i++) {
                        n[i] = dv[i] * idist;
                        pa[i] = ca[i] - ra * n[i];
                        pb[i] = cb[i] + rb * n[i];
                    }
                }
                ba = (int)gsum[8 * ga + 5];
                bb = (int)gsum[8 * gb + 5];
            }
            emit(hit, ba, bb, pa, pb, n, d);
        }
    }
    if (nc > maxc) { nc = maxc; over = 1; }
    if (over) ef |= HUM_EFLAG_CONTACT_OVERFLOW;
    __syncthreads();
    PHASE(6);
    HUM_STOP(6);
    // ---- rows (limits, normals, frictions): Jacobian + test-impulse response, one row per lane, the rows of
    //      all EPB_ envs of the wave spread over its lanes (one round instead of max_e ceil(nrows_e / 16))
    const int nrows = nl + 3 * nc;
    int pbase, ptot;   // this env's first pool position, the block's pool positions in use
    bool lam;          // the Delassus-form PGS (wave-uniform)
    group_rows<T, EPB_>(P, shb, gblock, nl, nc, dt, pbase, ptot, lam, ef);
    const int cap = P.lds_rows;
    WLOG(1, env_max<EPB_>(nrows));
    __syncthreads();
    PHASE(7);
    HUM_STOP(7);
    // ---- PGS (lane l owns nu[l] and nu[16+l]).  Every lane recomputes lambda identically and only
    //      re-reads values it wrote itself, so no cross-lane LDS ordering is needed inside the loop.
    T n0 = S.nu[l], n1 = l < NV - GL ? S.nu[GL + l] : T(0);
#ifdef HUM_PHASE_TIMING
    {   // row statistics: slow-path waves, waves, rows per env, envs with > 24 / > 30 rows
        const unsigned long long slow = ptot > cap;
        if (threadIdx.x == 0) { atomicAdd(&g_phase_cycles[11], slow); atomicAdd(&g_phase_cycles[12], 1ull); }
        if (l == 0) {
            atomicAdd(&g_phase_cycles[13], (unsigned long long)nrows);
            atomicAdd(&g_phase_cycles[14], (unsigned long long)(nrows > 24));
            atomicAdd(&g_phase_cycles[15], (unsigned long long)(nrows > 30));
        }
    }
#endif
    bool delassus_done = false;
    if constexpr (delassus_kernel<T, EPB_>()) {
        if (lam) {   // wave-uniform
            pgs_delassus<EPB_>(P, shb, S, nl, nc, pbase, l, n0, n1);
            delassus_done = true;
        }
    }
    if (delassus_done) {
    }
#ifndef HUM_PGS_SLOW
    else if (ptot <= cap) {   // wave-uniform
#else
    else if (false) {
#endif
        // Common case (the block's rows all in its LDS pool).  Gauss-Seidel over the flattened (iteration,
        // row) sequence, restated for latency: with n_k the velocity before row k and dl_k its impulse change,
        //     J_k . n_k = J_k . n_(k-1) + dl_(k-1) c_k,    c_k = J_k . M^-1 J_(k-1)^T (precomputed per row),
        // so the 16-lane reduction of J_k . n_(k-1) runs while row k-1 is solved, and the row update
        //     lambda_k + meff_k (b_k - J_k . n_k) = P_k - q_k dl_(k-1),   P_k = lambda_k + meff_k (b_k - J_k . n_(k-1)),
        // with q_k = meff_k c_k stored per row and P_k formed as soon as the reduction lands: the row-to-row
        // dependency chain is 3 scalar ops (fma, med3, sub).  Row k+3 is read while row k is solved
        // (through a link stored in row k), two stages before its reduction needs it; the lambdas it reads were
        // stored earlier (LDS ops of a wave are ordered: the pool layout keeps a friction row >= 4 positions
        // after its normal row and a cycle >= 4 positions long, see pool_gap).
        // Branch-free bounds: lo = 0 for every row, normal and limit rows have mu = 0, friction rows hi = 0,
        // so [-mu ln, hi + mu ln] is exact for all.
        using T2 = typename std::conditional<sizeof(T) == 4, float2, double2>::type;
        struct RowRegs { T j0, m0, j1, m1, b, hi, lam, meff, mu, q; int next3, next3_ln; };
        const char* lds0 = reinterpret_cast<const char*>(shb);
        const int off0 = 2 * l * (int)sizeof(T), off1 = (l < NV - GL ? 2 * (GL + l) : RO_Z) * (int)sizeof(T);
        auto as_int = [](T v) -> int {
            if constexpr (sizeof(T) == 4) return __float_as_int(v);
            else return (int)(unsigned)__double_as_longlong(v);
        };
        auto load = [&](int off, RowRegs& d) {
            const char* R = lds0 + off;
            const T2 p0 = *reinterpret_cast<const T2*>(R + off0), p1 = *reinterpret_cast<const T2*>(R + off1);
            d.j0 = p0.x; d.m0 = p0.y; d.j1 = p1.x; d.m1 = p1.y;
            if constexpr (sizeof(T) == 4) {
                const float4 s0 = *reinterpret_cast<const float4*>(R + RO_S0 * sizeof(T));
                const float4 s1 = *reinterpret_cast<const float4*>(R + RO_S1 * sizeof(T));
                d.b = s0.x; d.hi = s0.y; d.lam = s0.z; d.meff = s0.w;
                d.mu = s1.x; d.q = s1.y; d.next3 = __float_as_int(s1.z); d.next3_ln = __float_as_int(s1.w);
            } else {
                const T* S0 = reinterpret_cast<const T*>(R) + RO_S0;
                d.b = S0[0]; d.hi = S0[1]; d.lam = S0[2]; d.meff = S0[3];
                d.mu = S0[4]; d.q = S0[5]; d.next3 = as_int(S0[6]); d.next3_ln = as_int(S0[7]);
            }
        };
        auto load_ln = [&](int ln_off) -> T { return *reinterpret_cast<const T*>(lds0 + ln_off); };
        const int neff = pool_rows(nl, nc);
        // the zero rows of the pool layout (positions reserved by group_rows): the gap after the normals and the
        // trailing rows up to the minimum cycle length (pool_zero), visited directly rather than by scanning the frictions
        {
            auto zero_row = [&](int z) {
                T* Z = reinterpret_cast<T*>(reinterpret_cast<char*>(shb) + pool_off<T>(pbase + z));
                int n3, n3ln;
                pgs_link<T>(pbase, z, nl, nc, n3, n3ln);
                Z[l] = T(0); Z[GL + l] = T(0); Z[2 * GL + l] = T(0);
                if (l < RW - 2 - 3 * GL) Z[3 * GL + l] = T(0);
                if (l == 0) *reinterpret_cast<int*>(Z + RO_S1 + 2) = n3;
                if (l == 1) *reinterpret_cast<int*>(Z + RO_S1 + 3) = n3ln;
            };
            const int g0 = nl + nc, g1 = g0 + pool_gap(nc), u = pool_used(nl, nc);   // u >= g1
            for (int z = g0; z < g1; z++) zero_row(z);
            for (int z = u; z < neff; z++) zero_row(z);
        }
        wave_sync();
        const int total = P.iters * neff;
#ifdef HUM_CHECK_LINKS
        // diagnostic: every link of the env's cycle is what pgs_link says
        if (l == 0) {
            for (int r = 0; r < neff; r++) {
                const char* R = lds0 + pool_off<T>(pbase + r);
                int e3, e3ln;
                pgs_link<T>(pbase, r, nl, nc, e3, e3ln);
                if (*reinterpret_cast<const int*>(R + (RO_S1 + 2) * sizeof(T)) != e3) atomicAdd(&g_check[0], 1u);
                if (*reinterpret_cast<const int*>(R + (RO_S1 + 3) * sizeof(T)) != e3ln) atomicAdd(&g_check[1], 1u);
            }
            if (pbase + neff > ptot || ptot > cap) atomicAdd(&g_check[2], 1u);
            atomicAdd(&g_check[3], 1u);
        }
#endif
        {
            // one wave-uniform trip count (the longest env's, in whole rounds of 4 stages): an env past its
            // own count keeps cycling its rows with updates masked to dl = 0, so the loop has no divergent exits.
            // Rounds below the shortest env's count need no mask (tmin): they run a copy of the stage without it.
            int tmax = total, tmin = total;
#pragma unroll
            for (int e = 0; e < EPB_; e++) {
                tmax = max(tmax, __builtin_amdgcn_readlane(total, e * GL));
                tmin = min(tmin, __builtin_amdgcn_readlane(total, e * GL));
            }
            tmin &= ~3;
            RowRegs A, B, C, D;
            int oA = pool_off<T>(pbase), oB = pool_off<T>(pbase + 1), oC = pool_off<T>(pbase + 2), oD;
            load(oA, A);
            load(oB, B);
            load(oC, C);
            // positions 0..2 are never friction rows (mu = 0): their bounds need no lambda
            T lnA = T(0), lnB = T(0), lnC = T(0), lnD;
            // P of the row being solved, from its reduction one stage earlier (the first row's here)
            T pA = fma(A.meff, A.b - row_sum(A.j0 * n0 + A.j1 * n1), A.lam), pB, pC, pD, dlp = T(0);
            // one stage: X (row k) is solved, Y's (row k+1) reduction runs, W (row k+3) is read; Z is row k+2
            // (HUM_PGS_STUDY_*: timing-only diagnostic builds for the stall attribution of DESIGN.md section 7 - the
            // 16-lane DPP reduction replaced by four dependent plain adds, the row-ahead LDS loads by register copies;
            // their results are meaningless, the trip counts are the real ones)
#ifdef HUM_PGS_STUDY_NODPP
            auto rsum = [](T v) { v += v; v += v; v += v; v += v; return v; };
#else
            auto rsum = [](T v) { return row_sum(v); };
#endif
            auto stage = [&](auto masked, int kk, const RowRegs& X, const RowRegs& Y, RowRegs& W, const RowRegs& Z, int oX,
                             int& oW, T pX, T& pY, T lnX, T& lnW) {
                oW = X.next3;
#ifdef HUM_PGS_STUDY_NOLOAD
                W = Z;
                W.next3 = X.next3;
                lnW = lnX;
#else
                load(oW, W);
                lnW = load_ln(X.next3_ln);
#endif
                // the row-ahead loads issue at the top of their stage: ALU work may cross this point, LDS ops may not
                __builtin_amdgcn_sched_barrier(0x407);
                pY = fma(Y.meff, Y.b - rsum(Y.j0 * n0 + Y.j1 * n1), Y.lam);
                const T lo = -(X.mu * lnX), hi = X.hi + X.mu * lnX;
                const T tX = fma(-X.q, dlp, pX);
                const T lsol = med3(tX, lo, hi);   // == clamp: lo <= hi always
                T lnew = lsol;
                if constexpr (decltype(masked)::value) lnew = kk < total ? lsol : X.lam;
                *reinterpret_cast<T*>(const_cast<char*>(lds0) + oX + RO_LAM * sizeof(T)) = lnew;
                const T dl = lnew - X.lam;
                // the same fma twice, spelled differently: SLP would pack the two into a v_pk_fma_f32 on an
                // (m0, m1) register pair, which the (J, M^-1 J^T) pair loads never deliver adjacent: the copies
                // that build the pair waited on the row loads just issued (two exposed LDS latencies per round)
                n0 = fma(X.m0, dl, n0);
                n1 += X.m1 * dl;
                dlp = dl;
                // the row read one stage earlier (Z) must have landed by the end of this one: keeps the scheduler
                // from sinking its loads next to their first use, where the LDS latency was exposed (+1.1 %), and
                // gives them a whole stage to land (pinning the row read in this stage instead, with the loads at
                // the stage top: -0.4 %; every field of the row and its bounding lambda pinned: no change;
                // profiles/r04_ab_rows.txt)
                asm volatile("" ::"v"(Z.j0), "v"(Z.m0), "v"(Z.j1), "v"(Z.m1), "v"(Z.b), "v"(Z.meff));
            };
            auto round = [&](auto masked, int k) {
                stage(masked, k, A, B, D, C, oA, oD, pA, pB, lnA, lnD);
                stage(masked, k + 1, B, C, A, D, oB, oA, pB, pC, lnB, lnA);
                stage(masked, k + 2, C, D, B, A, oC, oB, pC, pD, lnC, lnB);
                stage(masked, k + 3, D, A, C, B, oD, oC, pD, pA, lnD, lnC);
            };
            int k = 0;
            // two rounds per iteration: the scheduler sinks a round's last row-ahead loads to the loop end, where the
            // next iteration's first stage waits for them (lgkmcnt(0)); with 8 stages per iteration half as many
            // loads cross the back edge (+0.5 %, profiles/r03_pgs_sched_ab.txt; pinning the loads with
            // sched_barrier instead measured -0.5 %)
            for (; k + 8 <= tmin; k += 8) {
                round(std::false_type{}, k);
                round(std::false_type{}, k + 4);
            }
            for (; k < tmin; k += 4) round(std::false_type{}, k);
            for (; k < tmax; k += 4) round(std::true_type{}, k);
        }
    } else {
        // the block's rows overflow its LDS pool: plain loop over pool positions (LDS or global spill region).  Each
        // access is an LDS or a global one chosen per value, never one through a generic pointer that may point at
        // either (a flat access)
        auto rd = [&](int p, int w) -> T {
            HUM_BOUNDS(ef, p >= 0 && p < EPB_ * MAXR_G, p = 0);   // the LDS pool, then the block's spill rows
            if (p < cap) return ((const HUM_LDS T*)((const HUM_LDS char*)shb + pool_off<T>(p)))[w];
            return __builtin_nontemporal_load((const HUM_GLOBAL T*)(gblock + (long)(p - cap) * RW) + w);
        };
        auto wr = [&](int p, int w, T v) {
            HUM_BOUNDS(ef, p >= 0 && p < EPB_ * MAXR_G, p = 0);
            if (p < cap) ((HUM_LDS T*)((HUM_LDS char*)shb + pool_off<T>(p)))[w] = v;
            else __builtin_nontemporal_store(v, (HUM_GLOBAL T*)(gblock + (long)(p - cap) * RW) + w);
        };
        auto solve = [&](int p, int r) {
            T lo = T(0), hi = rd(p, RO_S0 + 1);
            if (r >= nl + nc) {   // friction bounds from the normal impulse of the same contact
                const T mu = rd(p, RO_S1);
                const T ln = rd(pbase + pool_pos(nl + ((r - nl - nc) >> 1), nl, nc), RO_LAM);
                lo = -mu * ln;
                hi = mu * ln;
            }
            const T part = rd(p, 2 * l) * n0 + (l < NV - GL ? rd(p, 2 * (GL + l)) * n1 : T(0));
            const T m0 = rd(p, 2 * l + 1), m1 = l < NV - GL ? rd(p, 2 * (GL + l) + 1) : T(0);
            const T jv = row_sum(part);
            const T lam = rd(p, RO_LAM);
            const T lnew = clampT(lam + rd(p, RO_S0 + 3) * (rd(p, RO_S0) - jv), lo, hi);
            const T dl = lnew - lam;
            wr(p, RO_LAM, lnew);
            n0 += m0 * dl;
            n1 += m1 * dl;
        };
        for (int it = 0; it < P.iters; it++)
            for (int r = 0; r < nrows; r++) solve(pbase + pool_pos(r, nl, nc), r);
    }
    PHASE(8);
    HUM_STOP(8);
    S.nu[l] = n0;
    if (l < NV - GL) S.nu[GL + l] = n1;
    // ---- integrate (lanes split the state), lane 0 the quaternion.  A frozen env (no action this round, a
    //      non-finite action, or the hierarchical env's high-level turn) rides along with the wave and keeps its state.
    if (!frozen) {
        if (l < 3) { S.st[10 + l] = S.nu[l]; S.st[7 + l] = S.nu[3 + l]; S.st[l] += dt * S.nu[3 + l]; }
        for (int j = l; j < NDOF; j += GL) { S.st[30 + j] = S.nu[6 + j]; S.st[13 + j] += dt * S.nu[6 + j]; }
        if (l == 0) {
            T w[3] = {S.nu[0], S.nu[1], S.nu[2]};
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
            T q[4] = {S.st[3], S.st[4], S.st[5], S.st[6]};
            T nq[4] = {dw * q[0] + ax[0] * q[3] + ax[1] * q[2] - ax[2] * q[1],
                       dw * q[1] + ax[1] * q[3] + ax[2] * q[0] - ax[0] * q[2],
                       dw * q[2] + ax[2] * q[3] + ax[0] * q[1] - ax[1] * q[0],
                       dw * q[3] - ax[0] * q[0] - ax[1] * q[1] - ax[2] * q[2]};
            const T nn = T(1) / sqrt(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
            for (int i = 0; i < 4; i++) S.st[3 + i] = nq[i] * nn;
        }
    }
    phase_sync();
    PHASE(9);
}

}  // namespace hk

// lab.cpp - host build of the product's per-lane physics (imitation-learning-rl_amd/csrc/physics.h) for the fp32
// accuracy study: the kernel's formulation stepped on the CPU in float and in double, so
// formulation changes can be measured against the fp64 / fp32 oracle from identical states without a GPU.
//
// The host float build is not bitwise the GPU kernel (the GPU's v_rcp_f32 / v_rsq_f32 approximations, a different
// sincosf, its own fma contraction) but carries the same formulation's rounding; tools/fp32lab/lab.py compares the
// error ratios (kernel / same-lane fp32 envelope) it shows with the GPU's.
//
// exported: lab_step_f32 / lab_step_f64 (one env step, 4 substeps, state in place, tau in dof order)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define __device__
#define __host__
#define __forceinline__ inline
// host stand-ins for the physics-only hardware approximations (physics.h prcp / psqrt / prsqrt): exact here
#define __builtin_amdgcn_rcpf(x) (1.0f / (x))
#define __builtin_amdgcn_sqrtf(x) sqrtf(x)
#define __builtin_amdgcn_rsqf(x) (1.0f / sqrtf(x))
using std::sqrt;
using std::sin;
using std::cos;
using std::fabs;
using std::fma;

#include "../../imitation-learning-rl_amd/csrc/physics.h"

using namespace hk;

static PhysParams params() {
    PhysParams P{};
    P.dt = 0.0165 / 4; P.nsub = 4; P.gravity = 9.8; P.iters = 5; P.erp_contact = 0.9; P.erp_limit = 0.2;
    P.mu_ground = 1.6; P.mu_self = 4.0; P.contact_thresh = 0.02; P.lin_damp = 0.04; P.ang_damp = 0.04;
    P.split_pen = -0.04;
    P.limit_max_impulse = 100; P.max_coord_vel = 100; P.max_contacts = MAXC; P.self_collision = 1;
    P.joint_damping = 1; P.lds_rows = 0; P.terrain = 0;
    return P;
}

template <typename T>
static void step(double* st_d, const double* tau_d) {
    static thread_local std::vector<T> scratch(SCRATCH_PER_LANE);
    const PhysParams P = params();
    T st[47], tau[NDOF];
    for (int e = 0; e < 47; e++) st[e] = (T)st_d[e];
    for (int d = 0; d < NDOF; d++) tau[d] = (T)tau_d[d];
    Lane<T> rows{scratch.data(), 1};
    for (int s = 0; s < P.nsub; s++) substep(P, st, tau, rows);
    for (int e = 0; e < 47; e++) st_d[e] = (double)st[e];
}

extern "C" {
void lab_step_f32(double* st, const double* tau) { step<float>(st, tau); }
void lab_step_f64(double* st, const double* tau) { step<double>(st, tau); }
}

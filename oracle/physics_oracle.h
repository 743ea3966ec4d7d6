/* ORACLE - test infrastructure only (see physics_oracle.c).  Parameters and entry points of the fp64 CPU
 * physics restatement, shared by physics_oracle.c and env_oracle.c. */
#pragma once

typedef struct {
    double dt;              /* substep */
    int nsub;               /* substeps per env step */
    double gravity;
    int iters;              /* PGS iterations */
    double erp_contact, erp_limit, mu_ground, mu_self, contact_thresh;
    double lin_damp, ang_damp, limit_max_impulse;
    int max_contacts;
    int self_collision;
    int joint_damping;      /* 0: ignore MJCF joint damping, 1: implicit per substep (default) */
    double max_coord_vel;   /* btMultiBody::m_maxCoordinateVelocity clamp in applyDeltaVeeMultiDof */
    /* ground (hum_set_terrain): 0 = plane z = 0, 1 = heightfield hf, 2 = CustomScene random blocks from
       terrain_key (humanoid.py:68-144) */
    int terrain;
    const float* hf;        /* terrain 1: heights, vertex (i, j) = hf[i + j * hf_w] */
    int hf_w, hf_l;
    double hf_s[3], hf_o[3], hf_mid;
    unsigned long long terrain_key;
    double split_pen;       /* Bullet split impulse (m_splitImpulsePenetrationThreshold -0.04): a limit / contact row
                               penetrating deeper gets no position bias (btMultiBodyConstraintSolver never applies
                               m_rhsPenetration to multibodies) */
} om_params;

void om_default_params(om_params* P);
/* one env step of physics: state (47) in place; tau_motor[17] in dof order */
void om_step(const om_params* P, double* st, const double* tau_motor, int* ncontact_out);
void om_parts(const double* st, double* out /* [OM_NPART][3] */);

"""The physics oracle's multibody dynamics against first principles (CPU).

PyBullet is absent, so nothing the reference holds pins `oracle/physics_oracle.c` ("parity vs PyBullet
unpinned").  What CAN be pinned without it is that the restatement's dynamics core is Newtonian mechanics of the
reference's MJCF humanoid: the mass matrix (Jacobian form, `mass_matrix`), the articulated-body recursion (`aba`,
an independent algorithm, incl. its velocity-product and gyroscopic terms), and the integrator (`substep`).
The checks use only the model's masses, COM offsets and inertias (`oracle/humanoid_links.json`, compiled from the
reference's XML) and the oracle's forward kinematics (`om_link_frames`):

* kinetic energy: 1/2 nu^T H nu equals the sum over links of 1/2 m |v_c|^2 + 1/2 w^T I w, the link velocities
  differentiated numerically from the kinematics;
* the base rows of H are the total mass and the system COM;
* H . aba(q, 0, tau) = [0; tau] (the two algorithms invert each other);
* from rest under gravity with arbitrary joint torques, the momentum rate is the gravity wrench (internal torques
  cancel), and with no torques every link falls alike (no joint or angular acceleration);
* in motion with no gravity, torques or damping: energy, linear momentum and angular momentum are conserved by the
  ABA's accelerations (the velocity terms H-dot from finite differences), and with torques and gravity the power
  balance dT/dt = tau . qd + g . P holds;
* one substep without contacts or limits is semi-implicit Euler of the ABA (velocities first, then positions, the
  base orientation by the exponential map), and a body released at rest free-falls exactly: z_n = z0 - g dt^2
  n(n+1)/2;
* the constraint rows' impulses (H(q0) (nu' - nu_free) after one substep): joint-limit impulses act on the violated
  joints only, push them back into range, stay within limit_max_impulse and leave both momenta alone; self-contact
  impulses are equal and opposite (no net force); the ground only pushes (net impulse up) and its horizontal part
  stays inside the friction box's bound sqrt(2) mu times the vertical part;
* over 0.1 s of free tumbling the energy and momentum drift halves with every halving of dt (first-order
  consistency of the substep);
* static equilibrium: dropped onto the plane, or onto a 15 degree heightfield slope (friction holding it), and
  left to settle, the ground's impulse over 32 substeps is vertical and the weight's.

Bullet's link damping (0.04, default on) and MJCF joint damping are switched off where a conservation law is
checked; contact, limit and damping semantics stay hypotheses about Bullet.  The GPU kernel
is tied to this oracle by the parity tests (fp64 kernel vs oracle), so these laws carry over to it.
"""
import ctypes
import os
import sys

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle as O  # noqa: E402

LINKS = O.LINKS["links"]
NL = len(LINKS)
MASS = np.array([lk["mass"] for lk in LINKS])
COM = np.array([lk["com"] for lk in LINKS])
INERTIA = np.array([lk["inertia"] for lk in LINKS]).reshape(NL, 3, 3)
MTOT = MASS.sum()
G = 9.8


def params(gravity=0.0, damping=False):
    P = O.default_params()
    P.gravity = gravity
    if not damping:
        P.lin_damp = P.ang_damp = 0.0
        P.joint_damping = 0
    P.self_collision = 0
    return P


def frames(st):
    R = np.zeros(NL * 9)
    x = np.zeros(NL * 3)
    O.lib().om_link_frames(O._p(np.ascontiguousarray(st, dtype=np.float64)), O._p(R), O._p(x))
    return R.reshape(NL, 3, 3), x.reshape(NL, 3)


def link_coms(st):
    R, x = frames(st)
    return x + np.einsum("lij,lj->li", R, COM), R


def nu_of(st):
    """Generalised velocity in the oracle's order: base angular (world), base COM linear (world), joint rates."""
    return np.concatenate([st[10:13], st[7:10], st[30:47]])


def advance(st, h):
    """The configuration moved along the state's own velocity for time h (base: translation, world-frame
    exponential map; joints: linear) - the tangent curve used for numerical derivatives."""
    s = st.copy()
    s[0:3] += h * st[7:10]
    s[3:7] = (Rotation.from_rotvec(h * st[10:13]) * Rotation.from_quat(st[3:7])).as_quat()
    s[13:30] += h * st[30:47]
    return s


def random_state(rng, moving=True, z=5.0):
    """A pose 5 m above the plane (no ground contact), joints in the middle 60 % of their ranges (no limit rows),
    random orientation; random base and joint velocities when moving."""
    st = np.zeros(O.NSTATE)
    st[0:3] = [rng.uniform(-1, 1), rng.uniform(-1, 1), z]
    st[3:7] = Rotation.random(random_state=rng).as_quat()
    mid, half = (O.LO + O.HI) / 2, (O.HI - O.LO) / 2
    st[13:30] = mid + 0.6 * half * rng.uniform(-1, 1, 17)
    if moving:
        st[7:10] = rng.normal(0, 1.0, 3)
        st[10:13] = rng.normal(0, 1.5, 3)
        st[30:47] = rng.normal(0, 2.0, 17)
    return st


def skew(a):
    return np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])


@pytest.mark.parametrize("seed", range(6))
def test_mass_matrix_is_the_links_kinetic_energy(seed):
    rng = np.random.default_rng(seed)
    st = random_state(rng)
    H = O.mass_matrix(st)
    assert np.allclose(H, H.T, rtol=0, atol=1e-12 * np.abs(H).max())
    assert np.linalg.eigvalsh(H).min() > 0
    nu = nu_of(st)
    h = 1e-5
    cp, Rp = link_coms(advance(st, h))
    cm, Rm = link_coms(advance(st, -h))
    T = 0.0
    for lk in range(NL):
        if MASS[lk] <= 0:
            continue
        v = (cp[lk] - cm[lk]) / (2 * h)
        w = Rotation.from_matrix(Rp[lk] @ Rm[lk].T).as_rotvec() / (2 * h)
        Rl = link_coms(st)[1][lk]
        T += 0.5 * MASS[lk] * v @ v + 0.5 * w @ (Rl @ INERTIA[lk] @ Rl.T) @ w
    assert abs(0.5 * nu @ H @ nu - T) < 1e-8 * T, (0.5 * nu @ H @ nu, T)


@pytest.mark.parametrize("seed", range(4))
def test_mass_matrix_base_rows_are_total_mass_and_com(seed):
    st = random_state(np.random.default_rng(100 + seed))
    H = O.mass_matrix(st)
    c = (MASS[:, None] * link_coms(st)[0]).sum(0) / MTOT
    np.testing.assert_allclose(H[3:6, 3:6], MTOT * np.eye(3), rtol=0, atol=1e-12 * MTOT)
    np.testing.assert_allclose(H[0:3, 3:6], MTOT * skew(c - st[0:3]), rtol=0, atol=1e-12 * MTOT)


@pytest.mark.parametrize("seed", range(4))
def test_aba_inverts_the_mass_matrix(seed):
    """At rest with no gravity and no damping the ABA's accelerations solve H qdd = [0; tau] - two independent
    algorithms (recursive articulated inertias vs Jacobian-summed H) agree."""
    rng = np.random.default_rng(200 + seed)
    st = random_state(rng, moving=False)
    tau = rng.normal(0, 50, 17)
    acc = O.aba(st, tau, params(gravity=0.0))
    r = O.mass_matrix(st) @ acc - np.concatenate([np.zeros(6), tau])
    assert np.abs(r).max() < 1e-10 * np.abs(tau).max()


@pytest.mark.parametrize("seed", range(4))
def test_momentum_rate_from_rest_is_the_gravity_wrench(seed):
    """From rest, whatever the joint torques (internal forces): dP/dt = M g and dL/dt about the base COM =
    M (c - x0) x g.  With no torques every link falls alike: no joint and no angular acceleration."""
    rng = np.random.default_rng(300 + seed)
    st = random_state(rng, moving=False)
    g = np.array([0, 0, -G])
    H = O.mass_matrix(st)
    c = (MASS[:, None] * link_coms(st)[0]).sum(0) / MTOT
    for tau in (rng.normal(0, 50, 17), np.zeros(17)):
        acc = O.aba(st, tau, params(gravity=G))
        rate = H[0:6] @ acc
        np.testing.assert_allclose(rate[3:6], MTOT * g, rtol=0, atol=1e-10 * MTOT * G)
        np.testing.assert_allclose(rate[0:3], MTOT * np.cross(c - st[0:3], g), rtol=0, atol=1e-10 * MTOT * G)
    np.testing.assert_allclose(acc[0:3], 0, atol=1e-12)
    np.testing.assert_allclose(acc[3:6], g, rtol=0, atol=1e-12)
    np.testing.assert_allclose(acc[6:], 0, atol=1e-11)


def _rates(st, tau, gravity):
    """(dT/dt, dP/dt, dL_O/dt) along the ABA's accelerations: d/dt (H nu) = H nudot + Hdot nu, Hdot by a central
    difference along the motion; L_O about the world origin = L_x0 + x0 x P."""
    nu = nu_of(st)
    acc = O.aba(st, tau, params(gravity=gravity))
    H = O.mass_matrix(st)
    h = 1e-6
    Hd = (O.mass_matrix(advance(st, h)) - O.mass_matrix(advance(st, -h))) / (2 * h)
    p = H @ nu
    pd = H @ acc + Hd @ nu
    Td = nu @ H @ acc + 0.5 * nu @ Hd @ nu
    P, Pd = p[3:6], pd[3:6]
    Ld = pd[0:3] + np.cross(st[7:10], P) + np.cross(st[0:3], Pd)
    return Td, Pd, Ld, H, nu, acc


@pytest.mark.parametrize("seed", range(6))
def test_free_motion_conserves_energy_and_momentum(seed):
    """No gravity, no torques, no damping, tumbling with every joint moving: the ABA's velocity-product and
    gyroscopic terms keep T, P and L_O constant (their rates vanish against the rates' own scale)."""
    st = random_state(np.random.default_rng(400 + seed))
    Td, Pd, Ld, H, nu, acc = _rates(st, np.zeros(17), 0.0)
    scale = np.abs(nu @ H @ acc)   # the size of either half of dT/dt
    assert scale > 1.0
    assert abs(Td) < 1e-7 * scale, (Td, scale)
    assert np.abs(Pd).max() < 1e-7 * np.abs(H[3:6] @ acc).max()
    assert np.abs(Ld).max() < 1e-7 * np.abs(H[0:3] @ acc).max()


@pytest.mark.parametrize("seed", range(4))
def test_power_balance_with_torques_and_gravity(seed):
    """dT/dt = tau . qd + g . P (the motors' and gravity's power), dP/dt = M g, dL_O/dt = M c x g."""
    rng = np.random.default_rng(500 + seed)
    st = random_state(rng)
    tau = rng.normal(0, 50, 17)
    g = np.array([0, 0, -G])
    Td, Pd, Ld, H, nu, acc = _rates(st, tau, G)
    P = (H @ nu)[3:6]
    power = tau @ st[30:47] + g @ P
    scale = np.abs(nu @ H @ acc) + abs(power)
    assert abs(Td - power) < 1e-7 * scale, (Td, power)
    np.testing.assert_allclose(Pd, MTOT * g, rtol=0, atol=1e-7 * MTOT * G)
    c = (MASS[:, None] * link_coms(st)[0]).sum(0) / MTOT
    np.testing.assert_allclose(Ld, MTOT * np.cross(c, g), rtol=0, atol=1e-6 * MTOT * G * (1 + np.abs(c).max()))


def _one_substep(st, tau, gravity):
    P = params(gravity=gravity)
    P.nsub = 1
    out = O.phys_step(st, tau, P)
    nc = ctypes.c_int(0)
    O.lib().om_step(ctypes.byref(P), O._p(st.copy()), O._p(np.ascontiguousarray(tau, dtype=np.float64)),
                    ctypes.byref(nc))
    return out, P, nc.value


@pytest.mark.parametrize("seed", range(4))
def test_substep_is_semi_implicit_euler_of_the_aba(seed):
    """Away from the ground and the joint limits, one substep is: nu' = nu + dt aba(q, nu, tau); q' = q + dt nu'
    (joints, base position), base orientation exp(dt w') applied in the world frame."""
    rng = np.random.default_rng(600 + seed)
    st = random_state(rng)
    tau = rng.normal(0, 50, 17)
    out, P, nc = _one_substep(st, tau, G)
    assert nc == 0
    dt = P.dt
    nu1 = nu_of(st) + dt * O.aba(st, tau, P)
    np.testing.assert_allclose(nu_of(out), nu1, rtol=0, atol=1e-12 * np.abs(nu1).max())
    np.testing.assert_allclose(out[0:3], st[0:3] + dt * nu1[3:6], rtol=0, atol=1e-13)
    np.testing.assert_allclose(out[13:30], st[13:30] + dt * nu1[6:], rtol=0, atol=1e-13)
    q1 = (Rotation.from_rotvec(dt * nu1[0:3]) * Rotation.from_quat(st[3:7])).as_quat()
    assert min(np.abs(out[3:7] - q1).max(), np.abs(out[3:7] + q1).max()) < 1e-12


def test_free_fall_from_rest_is_exact():
    """Released at rest 5 m up with no torques: every substep adds -g dt to the vertical velocity and then moves
    by it, so after n substeps z = z0 - g dt^2 n (n + 1) / 2 and vz = -g dt n; pose and joints stay put."""
    st = random_state(np.random.default_rng(7), moving=False)
    P = params(gravity=G)
    P.nsub = 40
    out = O.phys_step(st, np.zeros(17), P)
    n, dt = 40, P.dt
    assert abs(out[2] - (st[2] - G * dt * dt * n * (n + 1) / 2)) < 1e-12
    assert abs(out[9] + G * dt * n) < 1e-12
    np.testing.assert_allclose(out[0:2], st[0:2], atol=1e-13)
    np.testing.assert_allclose(out[7:9], 0, atol=1e-13)
    np.testing.assert_allclose(out[10:13], 0, atol=1e-12)
    np.testing.assert_allclose(out[13:30], st[13:30], atol=1e-12)
    np.testing.assert_allclose(out[30:47], 0, atol=1e-11)
    assert min(np.abs(out[3:7] - st[3:7]).max(), np.abs(out[3:7] + st[3:7]).max()) < 1e-12


def test_default_damping_only_dissipates():
    """With Bullet's link damping and the MJCF joint damping on (the env's defaults), no gravity and no torques,
    the kinetic energy falls at every substep."""
    st = random_state(np.random.default_rng(11))
    P = params(gravity=0.0, damping=True)
    P.nsub = 1
    T = []
    for _ in range(30):
        nu = nu_of(st)
        T.append(0.5 * nu @ O.mass_matrix(st) @ nu)
        st = O.phys_step(st, np.zeros(17), P)
    assert all(b < a for a, b in zip(T, T[1:])), T


def _constraint_impulse(st, P):
    """One substep of the oracle; returns (H(q0) (nu1 - nu_free), contacts): the generalised impulse the constraint
    rows (limits, contacts) applied, nu_free = nu0 + dt aba being the velocity before the constraint phase."""
    P.nsub = 1
    nu_free = nu_of(st) + P.dt * O.aba(st, np.zeros(17), P)
    out = O.phys_step(st, np.zeros(17), P)
    return O.mass_matrix(st) @ (nu_of(out) - nu_free), O.contacts(st, P)


@pytest.mark.parametrize("seed", range(4))
def test_limit_impulses_are_internal_and_act_on_their_joints_only(seed):
    """Joints pushed past their limits (moving further out), no gravity / contacts: the limit rows' impulse is
    e_j lambda_j on the violated joints only - pushing back into range, at most limit_max_impulse - and moves
    neither the linear nor the angular momentum of the body."""
    rng = np.random.default_rng(700 + seed)
    st = random_state(rng)
    lo_j, hi_j = rng.choice(17, 6, replace=False).reshape(2, 3)
    st[13 + lo_j] = O.LO[lo_j] - rng.uniform(0.005, 0.03, 3)
    st[13 + hi_j] = O.HI[hi_j] + rng.uniform(0.005, 0.03, 3)
    st[30 + lo_j] = -np.abs(st[30 + lo_j])
    st[30 + hi_j] = np.abs(st[30 + hi_j])
    P = params(gravity=0.0)
    imp, con = _constraint_impulse(st, P)
    assert len(con) == 0
    scale = np.abs(imp).max()
    assert scale > 1e-3
    assert np.abs(imp[0:6]).max() < 1e-10 * scale
    others = np.setdiff1d(np.arange(17), np.concatenate([lo_j, hi_j]))
    assert np.abs(imp[6 + others]).max() < 1e-10 * scale
    # a row's impulse is >= 0 (it may end at 0 when the other rows' impulses already turned the joint around)
    assert (imp[6 + lo_j] > -1e-12 * scale).all() and (imp[6 + hi_j] < 1e-12 * scale).all()
    assert np.abs(imp[6:]).max() <= P.limit_max_impulse * (1 + 1e-12)


def _self_contact_state(rng):
    P = params()
    P.self_collision = 1
    for _ in range(2000):
        st = random_state(rng)
        st[13:30] = rng.uniform(O.LO + 1e-3, O.HI - 1e-3)   # any pose in range: limbs often cross each other
        con = O.contacts(st, P)
        if len(con) >= 2 and (con[:, 2] < 0).any():   # at least one pair overlapping (not only speculative)
            return st
    raise AssertionError("no self-contact pose found")


@pytest.mark.parametrize("seed", range(4))
def test_self_contact_impulses_conserve_linear_momentum(seed):
    """Self-collision contacts (geom pairs of the same body) apply equal and opposite impulses: with no gravity and
    the ground far below, the constraint impulse's base force rows vanish (Newton's third law through the
    contact rows' Jacobians, normal and friction rows alike)."""
    rng = np.random.default_rng(800 + seed)
    st = _self_contact_state(rng)
    P = params(gravity=0.0)
    P.self_collision = 1
    imp, con = _constraint_impulse(st, P)
    assert len(con) >= 2 and (con[:, 1] >= 0).all()
    scale = np.abs(imp).max()
    assert scale > 1e-4
    assert np.abs(imp[3:6]).max() < 1e-10 * scale


@pytest.mark.parametrize("seed", range(4))
def test_ground_impulses_push_up_within_the_friction_cone(seed):
    """Falling onto the plane (gravity on, lowest part 1 cm into it, moving down and sideways): the ground's net
    impulse points up (normal rows clamped at >= 0) and its horizontal part is bounded by sqrt(2) mu times its
    vertical part (each contact's two friction rows are clamped to mu times that contact's final normal impulse)."""
    rng = np.random.default_rng(900 + seed)
    st = random_state(rng, z=0.0)
    st[2] -= O.parts(st)[:32, 2].min() + 0.01
    st[7:10] = [rng.uniform(-1, 1), rng.uniform(-1, 1), -1.0]
    P = params(gravity=G)
    imp, con = _constraint_impulse(st, P)
    assert len(con) >= 1 and (con[:, 1] < 0).all()
    J = imp[3:6]
    assert J[2] > 0.1
    mu = P.mu_ground
    assert np.hypot(J[0], J[1]) <= np.sqrt(2) * mu * J[2] * (1 + 1e-9)


@pytest.mark.parametrize("seed", [40, 41, 44])
def test_integrator_drift_is_first_order(seed):
    """Free tumbling motion for 0.1 s (no gravity, torques, damping or contacts; joint rates small enough that no
    limit is reached) at dt, dt/2, dt/4, dt/8: the drift of the kinetic energy and of the linear momentum halves
    with every halving of dt - the substep is a consistent first-order integrator of the conserving dynamics
    (semi-implicit Euler).  (Seeds whose drift is far above rounding at dt/8.)"""
    st0 = random_state(np.random.default_rng(seed))
    st0[30:47] *= 0.25
    H0, nu0 = O.mass_matrix(st0), nu_of(st0)
    E0, P0 = 0.5 * nu0 @ H0 @ nu0, (H0 @ nu0)[3:6]
    dE, dP = [], []
    for div in (1, 2, 4, 8):
        P = params(gravity=0.0)
        P.dt, P.nsub = 0.0165 / 4 / div, 1
        st = st0.copy()
        for _ in range(int(round(0.1 / P.dt))):
            st = O.phys_step(st, np.zeros(17), P)
            assert ((st[13:30] >= O.LO) & (st[13:30] <= O.HI)).all()
        H, nu = O.mass_matrix(st), nu_of(st)
        dE.append(abs(0.5 * nu @ H @ nu - E0) / E0)
        dP.append(np.abs((H @ nu)[3:6] - P0).max())
    for d in (dE, dP):
        assert d[-1] > 1e-9
        for a, b in zip(d, d[1:]):
            assert 1.8 < a / b < 2.2, d


def lying_states():
    """Four poses lying on the plane (on the back, front and both sides), 5 cm above it, at rest."""
    out = []
    for k, (ax, ang) in enumerate((("y", 90), ("y", -90), ("x", 90), ("x", -90))):
        st = random_state(np.random.default_rng(3 + k), moving=False, z=0.0)
        st[3:7] = Rotation.from_euler(ax, ang, degrees=True).as_quat()
        st[2] -= O.parts(st)[:32, 2].min() - 0.05
        out.append(st)
    return out


def ground_impulse_over(states_fn):
    """The constraint impulse's base force rows summed over consecutive substeps, each substep's H(q) (nu' - nu_free)
    with the env's default physics (damping on).  states_fn() yields (state, next substep's state) pairs."""
    P1 = O.default_params()
    P1.nsub = 1
    tot = np.zeros(3)
    s = None
    for s, out in states_fn():
        nu_free = nu_of(s) + P1.dt * O.aba(s, np.zeros(17), P1)
        tot += (O.mass_matrix(s) @ (nu_of(out) - nu_free))[3:6]
    return tot


@pytest.mark.parametrize("pose", range(4))
def test_resting_on_the_plane_the_ground_carries_the_weight(pose):
    """Static equilibrium: dropped 5 cm onto the plane and left for 400 env steps (6.6 s, default physics, zero
    torques), the ground's impulse over the next 32 substeps (8 env steps: the settled body still rocks slightly
    from substep to substep) is the weight's, M g 32 dt, within 1 %, with a horizontal part under 2 % of it."""
    st = lying_states()[pose]
    P = O.default_params()
    for _ in range(400):
        st = O.phys_step(st, np.zeros(17), P)
    P1 = O.default_params()
    P1.nsub = 1

    def steps():
        s = st.copy()
        for _ in range(32):
            out = O.phys_step(s, np.zeros(17), P1)
            yield s, out
            s = out
    J = ground_impulse_over(steps)
    w = MTOT * G * 32 * P1.dt
    assert abs(J[2] / w - 1) < 0.01, J[2] / w
    assert np.hypot(J[0], J[1]) < 0.02 * J[2]


SLOPE = 0.27   # a 15 degree planar heightfield z = SLOPE x + 0.3 (below the box friction's tan = mu = 1.6)


def slope_terrain(w=64, l=64):
    i, j = np.meshgrid(np.arange(w), np.arange(l), indexing="xy")   # vertex (i, j) at heights[i + j w]
    h = (SLOPE * (i - (w - 1) / 2) + 0.3).astype(np.float32).reshape(-1)
    return O.Terrain(O.TERRAIN_HEIGHTFIELD, heights=h, w=w, l=l, origin=(0.0, 0.0, 0.0))


def lying_on_slope(ter):
    out = []
    for st in lying_states():
        st = st.copy()
        st[2] += SLOPE * st[0] + 0.3 - ter.mid
        out.append(st)
    return out


@pytest.mark.parametrize("pose", range(4))
def test_resting_on_a_slope_friction_holds_the_weight(pose):
    """Static equilibrium on a 15 degree heightfield slope: the contact normals lean downhill, so only friction can
    make the ground's force cancel gravity - after 400 env steps the ground's impulse over 32 substeps is vertical
    and equal to the weight's within 1 % (its horizontal part under 1 % of it)."""
    ter = slope_terrain()
    st = lying_on_slope(ter)[pose]
    P = ter.apply(O.default_params())
    for _ in range(400):
        st = O.phys_step(st, np.zeros(17), P)
    P1 = ter.apply(O.default_params())
    P1.nsub = 1
    con = O.contacts(st, P1)
    nz = con[con[:, 1] < 0][:, 7:10]
    np.testing.assert_allclose(nz, np.tile([-SLOPE, 0, 1] / np.hypot(SLOPE, 1), (len(nz), 1)), atol=1e-6)

    def steps():
        s = st.copy()
        for _ in range(32):
            out = O.phys_step(s, np.zeros(17), P1)
            yield s, out
            s = out
    J = ground_impulse_over(steps)
    w = MTOT * G * 32 * P1.dt
    assert abs(J[2] / w - 1) < 0.01, J[2] / w
    assert np.hypot(J[0], J[1]) < 0.01 * J[2], J

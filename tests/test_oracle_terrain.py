"""CPU tests of the heightfield ground restatement (oracle/physics_oracle.c terrain_contact, oracle.Terrain):
LowLevelHumanoidEnv(useCustomEnv=True)'s CustomScene (/root/reference/humanoid.py:68-144).

Parity vs PyBullet's btHeightfieldTerrainShape collision is unpinned (pybullet absent, no fixture); these tests
pin the restatement's geometry to closed forms: a flat heightfield is the plane, a planar (tilted) heightfield
gives the plane's normal and signed distance whatever the diagonal, and the random terrain follows
CustomScene.episode_restart's layout (2 x 2 blocks in [0, 0.5), four flat centre blocks)."""
import ctypes

import numpy as np
import pytest
from scipy.spatial.transform import Rotation as R

import oracle as O
from ilrl_amd.clips import load_clip


def _states(n, seed=3, spread=0.0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        st = np.zeros(O.NSTATE)
        st[3:7] = R.random(random_state=int(rng.integers(1 << 30))).as_quat()
        st[13:30] = rng.uniform(O.LO, O.HI)
        p = O.parts(st)
        st[2] = -p[:32, 2].min() + rng.uniform(-0.05, 0.01)
        st[0:2] = rng.uniform(-spread, spread, 2)
        out.append(st)
    return out


def _params(terrain, key=0):
    return terrain.apply(O.default_params(), key)


def test_flat_heightfield_is_the_plane():
    flat = O.Terrain(O.TERRAIN_HEIGHTFIELD, heights=np.zeros(64 * 64), w=64, l=64, origin=(0.0, 0.0, 0.0))
    n_total = 0
    for st in _states(40, spread=3.0):
        cp = O.contacts(st)
        ct = O.contacts(st, _params(flat))
        gp = cp[cp[:, 1] < 0]
        gt = ct[ct[:, 1] < 0]
        assert len(gp) == len(gt)
        n_total += len(gp)
        np.testing.assert_array_equal(gp[:, 0], gt[:, 0])
        np.testing.assert_allclose(gt[:, 2], gp[:, 2], atol=1e-12)      # signed distance
        np.testing.assert_allclose(gt[:, 4:7], gp[:, 4:7], atol=1e-12)  # contact point on the body
        np.testing.assert_allclose(gt[:, 7:10], gp[:, 7:10], atol=1e-9)  # normal (0, 0, 1)
        # self contacts unaffected
        np.testing.assert_array_equal(cp[cp[:, 1] >= 0], ct[ct[:, 1] >= 0])
        # and a whole physics step agrees
        tau = np.zeros(17)
        np.testing.assert_allclose(O.phys_step(st, tau, _params(flat)), O.phys_step(st, tau), atol=1e-9)
    assert n_total > 40


@pytest.mark.parametrize("slope", [(0.1, 0.0), (0.05, -0.08)])
def test_planar_heightfield_normal_and_distance(slope):
    """z = sx x + sy y + 0.3 sampled on the vertices: both diagonals lie in the plane, so every contact has the
    plane's normal and signed distance (centre below the surface included)."""
    w = l = 64
    i, j = np.meshgrid(np.arange(w), np.arange(l), indexing="xy")   # i along x
    x, y = i - (w - 1) / 2, j - (l - 1) / 2
    h = (slope[0] * x + slope[1] * y + 0.3).astype(np.float32).reshape(-1)   # h[i + j * w]
    t = O.Terrain(O.TERRAIN_HEIGHTFIELD, heights=h, w=w, l=l, origin=(0.0, 0.0, 0.0))
    nrm = np.array([-slope[0], -slope[1], 1.0])
    nrm /= np.linalg.norm(nrm)
    seen = 0
    for st in _states(30, spread=5.0, seed=9):
        st[2] += slope[0] * st[0] + slope[1] * st[1] + 0.3 - t.mid
        c = O.contacts(st, _params(t))
        c = c[c[:, 1] < 0]
        for row in c:
            seen += 1
            np.testing.assert_allclose(row[7:10], nrm, atol=1e-6)
            # contact point on the sphere = centre - r n; its signed distance to the plane is d
            pa = row[4:7]
            zplane = slope[0] * pa[0] + slope[1] * pa[1] + (0.3 - t.mid)
            # distance of pa from the plane along the normal, measured through the vertical offset
            np.testing.assert_allclose((pa[2] - zplane) * nrm[2], row[2], atol=2e-6)
    assert seen > 20


def test_random_block_terrain_layout():
    key = O.next_terrain_key(0, O.lane_key(5, 3))
    hb = np.array([[O.random_block_height(key, bi, bj) for bi in range(128)] for bj in range(128)])
    assert hb.dtype == np.float32
    assert (hb >= 0).all() and (hb < 0.5).all()
    assert (hb[63:65, 63:65] == 0).all()
    assert 0.2 < hb.mean() < 0.3 and hb.std() > 0.1          # U(0, 0.5): mean 0.25, sd 0.144
    key2 = O.next_terrain_key(key, O.lane_key(5, 3))
    assert key2 != key and O.random_block_height(key2, 10, 10) != O.random_block_height(key, 10, 10)


def test_custom_env_rollout_resets_terrain():
    """OracleLowLevelEnv over CustomScene's random terrain: every reset draws a new terrain, steps run and
    generate ground contacts against it."""
    env = O.OracleLowLevelEnv(load_clip("motion08_03"), seed=2, terrain=O.Terrain(O.TERRAIN_RANDOM_BLOCKS))
    keys = []
    rng = np.random.default_rng(0)
    for ep in range(3):
        env.reset()
        keys.append(env.terrain_key)
        for _ in range(5):
            obs, rew, done, _ = env.step(rng.uniform(-1, 1, 17).astype(np.float32))
            assert np.isfinite(obs).all() and np.isfinite(rew)
    assert len(set(keys)) == 3
    # a state over a raised block touches the terrain at its height, not at z = 0
    st = _states(1, seed=4)[0]
    bi, bj = 70, 70   # vertices 140..141 -> x, y in [12.5, 13.5]
    hblk = float(O.random_block_height(keys[-1], bi, bj))
    st[0] = st[1] = 2 * bi - 127.5 + 0.5
    st[2] += hblk
    c = O.contacts(st, _params(env.terrain, keys[-1]))
    g = c[c[:, 1] < 0]
    assert len(g) > 0
    assert np.all(np.abs(g[:, 4 + 2] - (hblk + g[:, 2])) < 0.2)


# ------------------------------------------------------------------ capsule bodies across terrain edges (ridges)
def _roof(w=64, l=64, x0=0.5, top=0.3, slope=0.2, sign=1.0):
    """z = top - sign * slope * |x - x0| sampled on the vertices (x = i - (w - 1) / 2): a straight ridge (sign 1) or
    valley (sign -1) along y at the vertex column x0; every cell is planar, so the only non-flat edges are the
    column's vertical edges."""
    i, j = np.meshgrid(np.arange(w), np.arange(l), indexing="xy")
    x = i - (w - 1) / 2
    h = (top - sign * slope * np.abs(x - x0)).astype(np.float32).reshape(-1)
    return O.Terrain(O.TERRAIN_HEIGHTFIELD, heights=h, w=w, l=l, origin=(0.0, 0.0, 0.0))


def _surface_z(t, x):
    return float(np.float32(0.3 - 0.2 * abs(x - 0.5))) - t.mid


@pytest.mark.parametrize("gap", [0.0, 0.01, -0.01])
def test_capsule_across_a_ridge_touches_it(gap):
    """A horizontal capsule lying across the ridge (axis x in [-0.2, 1.2], y 0.3) at `gap` above its surface: the
    end caps are 0.14 m above the facets (no contact), and the ridge gives exactly one contact at x = 0.5 with the
    closed-form normal (0, 0, 1) and signed distance gap."""
    t = _roof()
    P = t.apply(O.default_params())
    r = 0.04
    zc = _surface_z(t, 0.5) + r + gap
    a, b = np.array([-0.2, 0.3, zc]), np.array([1.2, 0.3, zc])
    for end in (a, b):   # the end caps see nothing within contact range
        n, d = np.zeros(3), np.zeros(1)
        f = O.lib().om_terrain_contact
        dp = ctypes.POINTER(ctypes.c_double)
        f.argtypes = [ctypes.POINTER(O.OmParams), dp, ctypes.c_double, dp, dp]
        assert f(ctypes.byref(P), O._p(end), r, O._p(n), O._p(d)) == 0
    rc = O.ridge_contacts(a, b, r, P)
    assert len(rc) == 1
    nrm, d, tt = rc[0]
    np.testing.assert_allclose(nrm, [0, 0, 1], atol=1e-12)
    assert abs(d - gap) < 1e-9
    assert abs(tt - 0.7 / 1.4) < 1e-9


def test_capsule_across_a_ridge_tilted_and_valley():
    t = _roof()
    P = t.apply(O.default_params())
    r = 0.04
    # tilted across the ridge, one end resting on the left facet: the end cap and the ridge both touch
    za = _surface_z(t, 0.1)
    a = np.array([0.1, 0.3, za + r / np.cos(np.arctan(0.2)) + 1e-3])
    b = np.array([0.9, 0.3, _surface_z(t, 0.5) + r + 0.005 + 0.4 * 0.02])
    rc = O.ridge_contacts(a, b, r, P)
    assert len(rc) == 1 and 0.4 < rc[0][2] < 0.6
    # a valley (concave edge): no ridge contact anywhere along the axis; the end caps carry the contacts, one on
    # each facet with that facet's normal (-/+0.2, 0, 1)/|.| and the closed-form distance
    v = _roof(sign=-1.0)
    Pv = v.apply(O.default_params())
    zv = float(np.float32(0.3 + 0.2 * 0.7)) - v.mid
    a, b = np.array([-0.2, 0.3, zv]), np.array([1.2, 0.3, zv])
    assert O.ridge_contacts(a, b, r, Pv) == []
    f = O.lib().om_terrain_contact
    dp = ctypes.POINTER(ctypes.c_double)
    f.argtypes = [ctypes.POINTER(O.OmParams), dp, ctypes.c_double, dp, dp]
    for end, sx in ((a, -1.0), (b, 1.0)):
        n, d = np.zeros(3), np.zeros(1)
        assert f(ctypes.byref(Pv), O._p(end), r, O._p(n), O._p(d)) == 1
        want = np.array([sx * -0.2, 0.0, 1.0]) / np.sqrt(1.04)
        np.testing.assert_allclose(n, want, atol=1e-6)
        # the end sits on its facet's surface height: distance to the facet plane = height gap x cos(slope) - r
        zs = float(np.float32(0.3 + 0.2 * abs(end[0] - 0.5))) - v.mid
        np.testing.assert_allclose(d[0], (end[2] - zs) / np.sqrt(1.04) - r, atol=1e-6)
    # parallel to the ridge (never crossing an edge's interior transversally): the ridge line itself is the minimum
    # all along, so the closest points fall at an axis end - the end caps' contacts, no ridge contact
    zr = _surface_z(t, 0.5) + r + 0.005
    assert O.ridge_contacts(np.array([0.5, -0.3, zr]), np.array([0.5, 0.3, zr]), r, P) == []


def test_capsule_on_flat_and_planar_heightfields_has_no_ridge_contacts():
    """Flat and tilted planar heightfields have no convex edge: whole-state contacts equal the plane's (flat) and
    every ground contact keeps the plane's normal (tilted), ridge path included (the two tests above)."""
    w = l = 64
    i, j = np.meshgrid(np.arange(w), np.arange(l), indexing="xy")
    h = (0.05 * (i - (w - 1) / 2) - 0.08 * (j - (l - 1) / 2) + 0.3).astype(np.float32).reshape(-1)
    for hh in (np.zeros(w * l, np.float32), h):
        t = O.Terrain(O.TERRAIN_HEIGHTFIELD, heights=hh, w=w, l=l, origin=(0.0, 0.0, 0.0))
        P = t.apply(O.default_params())
        rng = np.random.default_rng(1)
        for _ in range(50):
            a = rng.uniform([-5, -5, -0.5], [5, 5, 1.0])
            b = a + rng.uniform(-0.3, 0.3, 3)
            assert O.ridge_contacts(a, b, 0.05, P) == []


def _surface_height(terrain, key, x, y):
    """world z of the heightfield surface at (x, y): the cell's triangle (diamond subdivision) interpolated"""
    u, v = x + (terrain.w - 1) / 2, y + (terrain.l - 1) / 2
    ci, cj = int(np.floor(u)), int(np.floor(v))
    fa, fb = u - ci, v - cj

    def hz(i, j):
        h = float(O.random_block_height(key, i >> 1, j >> 1)) if terrain.mode == O.TERRAIN_RANDOM_BLOCKS else \
            float(terrain.heights[i + j * terrain.w])
        return h - terrain.mid + terrain.origin[2]
    z00, z10, z01, z11 = hz(ci, cj), hz(ci + 1, cj), hz(ci, cj + 1), hz(ci + 1, cj + 1)
    if (ci + cj) % 2 == 0:   # split (0,0)-(1,1)
        return z00 + fb * (z01 - z00) + fa * (z11 - z01) if fb >= fa else z00 + fa * (z10 - z00) + fb * (z11 - z10)
    return z00 + fa * (z10 - z00) + fb * (z01 - z00) if fa + fb <= 1 else z11 + (1 - fa) * (z01 - z11) + (1 - fb) * (z10 - z11)


def test_random_blocks_limbs_across_block_edges():
    """CustomScene's random block terrain: humanoid states placed over block edges produce ridge contacts (limbs
    across a raised block's top edge).  Each sits on the terrain surface with its normal from the surface to the
    capsule axis, and the whole-state contact list holds the end caps, then the ridge contacts slot-major
    (slot 0 of every capsule in geom order, then slot 1), then the self contacts."""
    terrain = O.Terrain(O.TERRAIN_RANDOM_BLOCKS)
    key = O.next_terrain_key(0, O.lane_key(7, 1))
    P = terrain.apply(O.default_params(), key)
    seen = 0
    rng = np.random.default_rng(5)
    for st in _states(1000, seed=11, spread=20.0):
        x, y = st[0], st[1]
        hs = [float(O.random_block_height(key, (int(np.floor(x + 127.5)) + di) >> 1, (int(np.floor(y + 127.5)) + dj) >> 1))
              for di in (-1, 0, 1, 2) for dj in (-1, 0, 1, 2)]
        st[2] += max(hs) - terrain.mid + terrain.origin[2] + rng.uniform(-0.06, 0.0)
        segs = O.geom_segments(st)
        ends, ridges = [], [[], []]
        for g in range(17):
            p1, p2, r, typ = segs[g, :3], segs[g, 3:6], segs[g, 6], segs[g, 7]
            for p in ((p1,) if typ == 0 else (p1, p2)):
                n, d = np.zeros(3), np.zeros(1)
                if O.lib().om_terrain_contact(ctypes.byref(P), O._p(np.ascontiguousarray(p)), ctypes.c_double(r),
                                              O._p(n), O._p(d)):
                    ends.append(g)
            if typ == 1:
                for k, (n, d, t) in enumerate(O.ridge_contacts(p1, p2, r, P)):
                    ridges[k].append((g, n, d, t))
                    s = p1 + t * (p2 - p1)
                    pb = s - (r + d) * n   # the terrain point
                    assert abs(pb[2] - _surface_height(terrain, key, pb[0], pb[1])) < 1e-9
                    assert 0 < t < 1 and d < P.contact_thresh
        c = O.contacts(st, P)
        g_rows = c[c[:, 1] < 0]
        rl = ridges[0] + ridges[1]
        assert len(g_rows) == len(ends) + len(rl)
        for row, (g, n, d, t) in zip(g_rows[len(ends):], rl):
            np.testing.assert_allclose(row[7:10], n, atol=1e-12)
            assert abs(row[2] - d) < 1e-12
        seen += len(rl)
    print("ridge contacts", seen)
    assert seen >= 10, seen


def test_ridge_contact_invariants_random_capsules():
    """Every ridge contact of random capsules over CustomScene's blocks satisfies the model's invariants: a unit
    normal, its axis point clear of both end caps (t L > 0.02 and (1 - t) L > 0.02), the terrain point on the surface
    at signed distance d from the capsule (|s - pb| = r + d along n; when the axis point is inside the terrain, the
    face-normal branch's projection onto the plane under it), d below the contact threshold, at most two per capsule
    and none within 0.02 m of another along the axis."""
    terrain = O.Terrain(O.TERRAIN_RANDOM_BLOCKS)
    key = O.next_terrain_key(0, O.lane_key(3, 9))
    P = terrain.apply(O.default_params(), key)
    rng = np.random.default_rng(21)
    found = 0
    for _ in range(4000):
        c = rng.uniform([-30, -30, 0.0], [30, 30, 0.0])
        c[2] = _surface_height(terrain, key, c[0], c[1]) + rng.uniform(0.0, 0.12)
        half = rng.uniform(0.05, 0.25)
        d = rng.normal(size=3)
        d[2] *= 0.2   # mostly lying
        d /= np.linalg.norm(d)
        a, b, r = c - half * d, c + half * d, rng.uniform(0.03, 0.06)
        rc = O.ridge_contacts(a, b, r, P)
        assert len(rc) <= 2
        L = 2 * half
        ts = []
        for n, dist, t in rc:
            found += 1
            assert abs(np.linalg.norm(n) - 1) < 1e-12
            assert t * L > 0.02 - 1e-12 and (1 - t) * L > 0.02 - 1e-12
            assert dist < P.contact_thresh
            s = a + t * (b - a)
            pb = s - (r + dist) * n
            if s[2] > _surface_height(terrain, key, s[0], s[1]):   # the closest-point branch: pb on the surface
                assert abs(pb[2] - _surface_height(terrain, key, pb[0], pb[1])) < 1e-9
            else:   # axis point inside the terrain: the face-normal branch projects onto the plane under s
                assert abs(pb[2] - _surface_height(terrain, key, pb[0], pb[1])) < 1e-3
            ts.append(t)
        if len(ts) == 2:
            assert abs(ts[0] - ts[1]) * L >= 0.02
    assert found >= 20, found

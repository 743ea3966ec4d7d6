"""CPU tests of the heightfield ground restatement (oracle/physics_oracle.c terrain_contact, oracle.Terrain):
LowLevelHumanoidEnv(useCustomEnv=True)'s CustomScene (/root/reference/humanoid.py:68-144).

Parity vs PyBullet's btHeightfieldTerrainShape collision is unpinned (pybullet absent, no fixture); these tests
pin the restatement's geometry to closed forms: a flat heightfield is the plane, a planar (tilted) heightfield
gives the plane's normal and signed distance whatever the diagonal, and the random terrain follows
CustomScene.episode_restart's layout (2 x 2 blocks in [0, 0.5), four flat centre blocks)."""
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

"""GPU tests of the C-ABI contract details (include/humanoid_env.h): lanes without an action are left
untouched (hier send_actions), out-of-range resetFromFrame start frames are flagged without touching the lane,
and captured step graphs see changed predefined courses / lane modes (they are re-captured)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.hier_env import HierVecEnv  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402


@pytest.mark.parametrize("kernel", [1, 0])
def test_hier_skip_lanes_untouched(kernel):
    n = 16
    env = HierVecEnv(n, seed=2, kernel=kernel)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    # one high step everywhere, then low steps with every third lane absent from the action dict
    env.step(torch.rand(n, 2, device="cuda", generator=g) * 2 - 1, None, agent=np.ones(n, np.uint8))
    p0, b0 = env.get_state()
    sel = np.zeros(n, np.uint8)
    sel[::3] = N.HUM_AGENT_SEL_SKIP
    agents, *_ = env.step(None, torch.rand(n, 17, device="cuda", generator=g) * 2 - 1, agent=sel)
    agents = agents.cpu().numpy()
    p1, b1 = env.get_state()
    skip = sel == N.HUM_AGENT_SEL_SKIP
    assert (agents[skip] == 0).all() and (agents[~skip] != 0).all()
    np.testing.assert_array_equal(p1[skip], p0[skip])
    np.testing.assert_array_equal(b1[skip], b0[skip])
    assert (np.abs(p1[~skip] - p0[~skip]).max(axis=1) > 0).all()
    env.close()


def test_start_frame_out_of_range_flagged():
    env = HumanoidVecEnv(4, clips=("motion09_03",), seed=1)
    env.reset()
    p0, b0 = env.get_state()
    npos = env.clips[0].pos.shape[0]
    sf = torch.tensor([5, npos, npos + 100, 7], dtype=torch.int32, device="cuda")
    env.reset(start_frame=sf)
    p1, b1 = env.get_state()
    assert env.error_flags() & N.HUM_EFLAG_BAD_START_FRAME
    np.testing.assert_array_equal(p1[1:3], p0[1:3])
    np.testing.assert_array_equal(b1[1:3], b0[1:3])
    assert b1[0, N.BK["frame"]] == 7 and b1[3, N.BK["frame"]] == 9   # resetFromFrame + incFrame(2)
    env.close()


def _graph_step(env, a, k):
    rc = N.lib().hum_step_graph(env.h, N.ctypes.c_void_p(a.data_ptr()), N.ctypes.c_void_p(env.obs.data_ptr()),
                                N.ctypes.c_void_p(env.reward.data_ptr()), N.ctypes.c_void_p(env.done.data_ptr()),
                                N.ctypes.c_void_p(env.frame.data_ptr()), N.HUM_STEP_AUTORESET,
                                N.ctypes.c_void_p(env.obs_reset.data_ptr()), k)
    assert rc == 0


def test_graph_recaptured_after_predefined_targets_change():
    """step_graph, then set_predefined_targets (frees and reallocates the course), then step_graph again: the
    graph must not replay the freed course; results equal the eager path."""
    n = 64
    envs = [HumanoidVecEnv(n, clips=("motion08_03",), seed=9) for _ in range(2)]
    course1 = np.array([[0.3, 0.0, 0.0], [0.6, 0.1, 0.0]])
    course2 = np.array([[0.2, 0.2, 0.0], [0.4, -0.3, 0.0], [0.1, 0.1, 0.0]])
    for e in envs:
        e.set_predefined_targets(course1)
        e.set_modes(predefined=True)
        e.reset()
    a = (torch.rand(n, 17, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3)) * 0.3).contiguous()
    for step in range(2):
        if step == 1:
            for e in envs:
                e.set_predefined_targets(course2)
        for _ in range(6):
            envs[0].step(a, autoreset=True)
        torch.cuda.synchronize()
        _graph_step(envs[1], a, 6)
        envs[1].sync()
        p0, b0 = envs[0].get_state()
        p1, b1 = envs[1].get_state()
        np.testing.assert_array_equal(p0, p1)
        np.testing.assert_array_equal(b0, b1)
    for e in envs:
        e.close()


def test_load_clip_csv_on_device_equals_packed_clip():
    """hum_load_clip_csv (runtime 4-CSV ingestion, pandas-identical parse) uploads the same tables as the
    packed .clip path: identical rollouts."""
    from ilrl_amd.clips import CSV_DIR
    n = 64
    envs = [HumanoidVecEnv(n, clips=("motion08_03", "motion13_13"), seed=4) for _ in range(2)]
    for cid, name in enumerate(("motion08_03", "motion13_13")):
        assert N.lib().hum_load_clip_csv(envs[1].h, cid, CSV_DIR.encode(), name.encode()) == 0
    g = torch.Generator(device="cuda").manual_seed(6)
    acts = [(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1).contiguous() for _ in range(20)]
    for e in envs:
        e.reset()
        for a in acts:
            e.step(a, autoreset=True)
    p0, b0 = envs[0].get_state()
    p1, b1 = envs[1].get_state()
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(b0, b1)
    assert N.lib().hum_load_clip_csv(envs[1].h, 0, CSV_DIR.encode(), b"nope") != 0
    assert b"cannot open" in N.lib().hum_last_error()
    for e in envs:
        e.close()


def _p(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return N.ctypes.c_void_p(x.ctypes.data)
    return N.ctypes.c_void_p(x.data_ptr())


@pytest.mark.parametrize("k", [1, 3])
def test_host_io_equals_device_path(k):
    """HUM_STEP_HOST_IO (buffers may be host or device pointers, flag): host numpy buffers give the
    device path's results bit for bit, and rows the step leaves unwritten (obs_reset of lanes not done) keep the
    caller's values."""
    n = 64
    envs = [HumanoidVecEnv(n, clips=("motion02_04",), seed=21) for _ in range(2)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(2)
    for it in range(6):
        a = rng.uniform(-1, 1, (k, n, 17)).astype(np.float32)
        dev = envs[0].step_k(torch.as_tensor(a, device="cuda"), autoreset=True)
        obs = np.zeros((k, n, 70), np.float32)
        rew = np.zeros((k, n), np.float32)
        done = np.zeros((k, n), np.uint8)
        frame = np.zeros((k, n), np.int32)
        orst = np.full((k, n, 70), 7.0, np.float32)
        rc = N.lib().hum_step_k(envs[1].h, _p(a), _p(obs), _p(rew), _p(done), _p(frame),
                                N.HUM_STEP_AUTORESET | N.HUM_STEP_HOST_IO, _p(orst), k, None)
        assert rc == 0, N.lib().hum_last_error()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(obs, dev[0].cpu().numpy())
        np.testing.assert_array_equal(rew, dev[1].cpu().numpy())
        np.testing.assert_array_equal(done, dev[2].cpu().numpy())
        np.testing.assert_array_equal(frame, dev[3].cpu().numpy())
        dm = done.astype(bool)
        np.testing.assert_array_equal(orst[dm], dev[4].cpu().numpy()[dm])
        assert (orst[~dm] == 7.0).all()
    p0, b0 = envs[0].get_state()
    p1, b1 = envs[1].get_state()
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(b0, b1)
    for e in envs:
        e.close()


def test_hier_host_io_equals_device_path():
    n = 32
    envs = [HierVecEnv(n, seed=3) for _ in range(2)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(4)
    for it in range(12):
        ah = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        al = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
        dev = [x.cpu().numpy() for x in envs[0].step(ah, al, autoreset=True)]
        agents = np.zeros(n, np.uint8)
        oh = np.zeros((n, 44), np.float32)
        ol = np.zeros((n, 70), np.float32)
        rh = np.zeros(n, np.float32)
        rl = np.zeros(n, np.float32)
        done = np.zeros(n, np.uint8)
        frame = np.zeros(n, np.int32)
        rc = N.lib().hum_hier_step(envs[1].h, _p(ah), _p(al), None, _p(agents), _p(oh), _p(ol), _p(rh), _p(rl),
                                   _p(done), _p(frame), N.HUM_STEP_AUTORESET | N.HUM_STEP_HOST_IO, None, None)
        assert rc == 0, N.lib().hum_last_error()
        np.testing.assert_array_equal(agents, dev[0])
        hi, lo = (agents & N.HUM_AGENT_HIGH) != 0, (agents & N.HUM_AGENT_LOW) != 0
        np.testing.assert_array_equal(oh[hi], dev[1][hi])
        np.testing.assert_array_equal(ol[lo], dev[2][lo])
        np.testing.assert_array_equal(rh, dev[3])
        np.testing.assert_array_equal(rl, dev[4])
        np.testing.assert_array_equal(done, dev[5])
    p0, b0 = envs[0].get_state()
    p1, b1 = envs[1].get_state()
    inv = {v: k for k, v in N.BK.items()}
    for i, c in np.argwhere(b0 != b1)[:10]:
        print("lane %d book %d (%s): %r vs %r" % (i, c, inv.get(c), b0[i, c], b1[i, c]))
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(b0, b1)
    for e in envs:
        e.close()


def test_check_finite_returns_error_status():
    """HUM_STEP_CHECK_FINITE: a non-finite action is an error status of the call itself (humanoid.py:55 assert);
    the lane is not stepped, the others are, and the sticky bit is consumed."""
    n = 16
    env = HumanoidVecEnv(n, clips=("motion02_04",), seed=5)
    env.reset()
    p0, b0 = env.get_state()
    a = np.random.default_rng(0).uniform(-1, 1, (n, 17)).astype(np.float32)
    a[3, 4] = np.nan
    obs = np.zeros((n, 70), np.float32)
    rew = np.zeros(n, np.float32)
    done = np.zeros(n, np.uint8)
    rc = N.lib().hum_step(env.h, _p(a), _p(obs), _p(rew), _p(done), None,
                          N.HUM_STEP_HOST_IO | N.HUM_STEP_CHECK_FINITE, None, None)
    assert rc == N.HUM_ERR_ARG
    assert b"non-finite action" in N.lib().hum_last_error()
    p1, b1 = env.get_state()
    np.testing.assert_array_equal(p1[3], p0[3])
    np.testing.assert_array_equal(b1[3], b0[3])
    assert (np.abs(p1[np.arange(n) != 3] - p0[np.arange(n) != 3]).max(axis=1) > 0).all()
    assert env.error_flags() & N.HUM_EFLAG_NONFINITE_ACTION == 0
    a[3, 4] = 0.5
    rc = N.lib().hum_step(env.h, _p(a), _p(obs), _p(rew), _p(done), None,
                          N.HUM_STEP_HOST_IO | N.HUM_STEP_CHECK_FINITE, None, None)
    assert rc == N.HUM_OK
    # a non-finite action of an earlier UNCHECKED step leaves the sticky bit set; a later checked call whose own
    # actions are finite still succeeds (the bit is cleared on the stream before its launch)
    a[5, 0] = np.inf
    assert N.lib().hum_step(env.h, _p(a), _p(obs), _p(rew), _p(done), None, N.HUM_STEP_HOST_IO, None, None) == N.HUM_OK
    assert env.error_flags() & N.HUM_EFLAG_NONFINITE_ACTION
    a[5, 0] = 0.25
    assert N.lib().hum_step(env.h, _p(a), _p(obs), _p(rew), _p(done), None,
                            N.HUM_STEP_HOST_IO | N.HUM_STEP_CHECK_FINITE, None, None) == N.HUM_OK
    g = torch.zeros(n, 17, device="cuda")
    assert N.lib().hum_step_graph(env.h, _p(g), _p(env.obs), _p(env.reward), _p(env.done), None,
                                  N.HUM_STEP_CHECK_FINITE, None, 2) == N.HUM_ERR_ARG
    env.close()


def test_gym_view_raises_past_the_velocity_table():
    """motion13_13 has 120 velocity rows for 220 pose rows: the reference's JointSpeedRadSec.iloc[frame] raises
    IndexError once the frame reaches 120 (low_level_env.py:208, :310, :345); the single-env view raises likewise
    (vector / bench handles keep the clamped row and flag HUM_EFLAG_VEL_ROW)."""
    from ilrl_amd.low_level_env import LowLevelHumanoidEnv
    env = LowLevelHumanoidEnv(reference_name="motion13_13", seed=1)
    env.resetFromFrame(startFrame=115)          # frame 117
    env.step(np.zeros(17, np.float32))          # frame 119
    with pytest.raises(IndexError):
        env.step(np.zeros(17, np.float32))      # getLowLevelObs at frame 121
    with pytest.raises(IndexError):
        env.step(np.zeros(17, np.float32))      # calcJointVelScore at frame 121
    with pytest.raises(IndexError):
        env.resetFromFrame(startFrame=118)      # obs row 120
    env.resetFromFrame(startFrame=10)
    o, r, d, _ = env.step(np.zeros(17, np.float32))
    assert np.isfinite(o).all()
    env.close()

"""GPU parity: the HIP kernel (through the C-ABI) vs the reference's golden vectors and the CPU oracle.

Every golden scenario (tests/golden/make_golden.py, produced by the real reference env module) is
replayed as ONE launch with one lane per recorded step: lane t gets the recorded physics state and the
bookkeeping the reference held before step t, and the recorded action.

* injected physics (HUM_STEP_SKIP_PHYSICS): lane physics = the reference's post-step state -> the
  kernel's env logic (obs, reward, done, frame, target, ...) must equal the reference's;
* full physics: lane physics = pre-step state -> kernel physics vs the fp64 oracle physics.

Tolerances (stated per quantity below): done / frame / timestep / target decisions bit-exact;
fp64 kernel: obs within 1 float32 ulp, reward 1e-9; fp32 kernel with injected physics: obs within 1e-6 + 2 float32
ulps of the reference value and <= 1e-5 absolute (measured max 6.5e-6 = half an ulp of a 145 rad/s
table velocity, the float32 output format) - the Euler-angle obs (1, 2, 6, 7) add 2^-22 / cos(pitch) for the float32
quaternion - reward 1e-4 (measured 1.3e-6).  Full fp32 physics step vs the fp64 oracle ("fp32
step bound"): obs <= 2.5e-4, reward <= 1e-5, done / frame exact on well-conditioned states (tests/test_gpu_scale.py).
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from conftest import scenarios
from golden_replay import rec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.clips import load_clip  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

SCEN = ["motion02_04_l0", "motion02_04_l1", "motion02_04_l2", "motion08_03_l0", "motion08_03_l1", "motion08_03_l2",
        "motion09_03_l0", "motion09_03_l1", "motion09_03_l2", "motion13_13_f10", "motion13_13_f60", "yaw45_scaled",
        "debug_true", "teleport_target", "teleport_far", "predefined_course", "timestep_limit", "frame_wrap"]


def book_rows(r, t_idx):
    """HUM_NBOOK rows holding the reference bookkeeping BEFORE each step t in t_idx."""
    seed, lane, _, debug, _, _, _ = [int(x) for x in r["meta"]]
    key = O.legacy_lane_key(seed, lane)   # the stream the fixtures' recorded draws came from
    out = np.zeros((len(t_idx), N.HUM_NBOOK))
    for row, t in enumerate(t_idx):
        src = (lambda k: r["book0_" + k]) if t == 0 else (lambda k: r["book_" + k][t - 1])
        b = out[row]
        b[N.BK["frame"]] = src("frame")
        b[N.BK["cur_timestep"]] = r["cur_timestep_pre"][t]
        b[N.BK["rng_counter"]] = src("rng_counter")
        b[N.BK["predefinedTargetIndex"]] = src("predefinedTargetIndex")
        for k in ("target", "starting_robot_pos", "robot_pos", "starting_ep_pos"):
            b[N.BK[k]:N.BK[k] + 3] = src(k)
        b[N.BK["walk_target"]:N.BK["walk_target"] + 2] = src("walk_target")
        for k in ("highLevelDegTarget", "lowTargetScore", "deltaJoints", "deltaVelJoints", "bodyPostureScore",
                  "electricityScore", "jointLimitScore", "aliveReward", "delta_lowTargetScore"):
            b[N.BK[k]] = src(k)
        b[N.BK["clip"]] = 0
        b[N.BK["mode"]] = (N.HUM_MODE_DEBUG if debug else 0) | (N.HUM_MODE_PREDEFINED if len(r["predefined"]) else 0)
        b[N.BK["rng_key_lo"]] = key & 0xFFFFFFFF
        b[N.BK["rng_key_hi"]] = key >> 32
    return out


def run_scenario(r, precision, skip_physics, kernel=1, **physics):
    T = len(r["reward"])
    # the fixtures were made under numpy 2.2 (NEP 50 float32 scalar arithmetic, include/humanoid_env.h)
    env = HumanoidVecEnv(T, clips=(str(r["clip"]),), precision=precision, kernel=kernel, numpy_semantics=N.HUM_NUMPY_2,
                         **physics)
    if len(r["predefined"]):
        env.set_predefined_targets(r["predefined"])
    phys = r["state_post"] if skip_physics else r["state_pre"]
    env.set_state(phys, book_rows(r, range(T)))
    obs, rew, done, frame = env.step(r["action"], skip_physics=skip_physics)
    out = dict(obs=obs.cpu().numpy(), rew=rew.cpu().numpy(), done=done.cpu().numpy().astype(bool),
               frame=frame.cpu().numpy())
    out["aux"] = env.get_aux().cpu().numpy()
    out["phys"], out["book"] = env.get_state()
    env.close()
    return out


def f32_ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


@pytest.mark.parametrize("kernel", [1, 0])
@pytest.mark.parametrize("name", SCEN)
def test_env_logic_matches_reference_fp64(golden, name, kernel):
    """Injected physics, fp64 kernel: env logic equals the reference's golden outputs."""
    r = rec(golden, name)
    o = run_scenario(r, "fp64", skip_physics=True, kernel=kernel)
    np.testing.assert_array_equal(o["done"], r["done"])
    np.testing.assert_array_equal(o["frame"], r["book_frame"].astype(np.int32))
    np.testing.assert_array_equal(o["book"][:, N.BK["cur_timestep"]], r["book_cur_timestep"])
    np.testing.assert_array_equal(o["book"][:, N.BK["rng_counter"]], r["book_rng_counter"])
    assert f32_ulp_diff(o["obs"], r["obs"]).max() <= 1, "obs beyond 1 float32 ulp"
    np.testing.assert_allclose(o["rew"], r["reward"], rtol=1e-6, atol=1e-6)   # f32 output of an f64 sum
    for k in ("target", "starting_robot_pos", "starting_ep_pos"):   # starting_ep_pos: R13 (:221-222, :277-289)
        np.testing.assert_allclose(o["book"][:, N.BK[k]:N.BK[k] + 3], r["book_" + k], rtol=0, atol=1e-12, err_msg=k)
    # calcEndPointScore (R12, low_level_env.py:361-382) as the reference returns it after each step: aux columns
    np.testing.assert_allclose(o["aux"][:, N.AUX.index("endPointScore")], r["endpoint_score"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(o["aux"][:, N.AUX.index("endPointScoreExp")], r["endpoint_score_exp"], rtol=1e-6,
                               atol=1e-7)
    assert (o["aux"][:, N.AUX.index("deltaEndPoints")] == 0).all()   # the reference attribute stays 0 (:445)
    np.testing.assert_allclose(o["book"][:, N.BK["robot_pos"]:N.BK["robot_pos"] + 3], r["book_robot_pos"], atol=1e-12)
    for k in ("lowTargetScore", "deltaJoints", "deltaVelJoints", "bodyPostureScore", "electricityScore",
              "jointLimitScore", "aliveReward", "delta_lowTargetScore", "highLevelDegTarget"):
        np.testing.assert_allclose(o["book"][:, N.BK[k]], r["book_" + k], rtol=1e-12, atol=1e-12, err_msg=k)


@pytest.mark.parametrize("kernel", [1, 0])
@pytest.mark.parametrize("name", SCEN)
def test_env_logic_matches_reference_fp32(golden, name, kernel):
    """Injected physics, fp32 kernel (the benchmarked build): FK in fp32."""
    r = rec(golden, name)
    o = run_scenario(r, "fp32", skip_physics=True, kernel=kernel)
    np.testing.assert_array_equal(o["done"], r["done"])
    np.testing.assert_array_equal(o["frame"], r["book_frame"].astype(np.int32))
    err = np.abs(o["obs"] - r["obs"])
    bound = 1e-6 + 2.0 ** -22 * np.abs(r["obs"])
    # the fp32 state's base quaternion is rounded to float32 (half an ulp per component); the Euler angles
    # (getEulerFromQuaternion: pitch = asin, roll / yaw = atan2 of terms that vanish at gimbal lock) amplify that
    # by 1 / cos(pitch), and angle_to_target (obs 1, 2) inherits the yaw's error
    cp = np.maximum(np.cos(r["obs"][:, 7].astype(np.float64)), 1e-3)
    for k in (1, 2, 6, 7):
        bound[:, k] += 2.0 ** -22 / cp
    assert (err <= bound).all(), "obs beyond 1e-6 + 2 float32 ulps (+ the Euler angles' quaternion conditioning)"
    assert (err[:, [0] + list(range(3, 6)) + list(range(8, 70))] <= 1e-5).all()
    np.testing.assert_allclose(o["rew"], r["reward"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(o["book"][:, N.BK["target"]:N.BK["target"] + 3], r["book_target"], atol=1e-5)
    np.testing.assert_allclose(o["aux"][:, N.AUX.index("endPointScoreExp")], r["endpoint_score_exp"], atol=1e-5)


@pytest.mark.parametrize("kernel", [1, 0])
@pytest.mark.parametrize("name", SCEN)
def test_physics_fp64_matches_oracle(golden, name, kernel):
    """Full step, fp64 kernel physics (world-frame ABA, merged multi-dof bodies) vs the fp64 oracle
    (local-frame ABA over pybullet's 32-link layout, H^-1 J^T responses)."""
    r = rec(golden, name)
    o = run_scenario(r, "fp64", skip_physics=False, kernel=kernel)
    err = np.abs(o["phys"] - r["state_post"])
    assert err.max() < 1e-6, "max state err %.3g at %s" % (err.max(), np.unravel_index(err.argmax(), err.shape))
    np.testing.assert_array_equal(o["done"], r["done"])
    np.testing.assert_allclose(o["obs"], r["obs"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(o["rew"], r["reward"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("lds_rows", [1, 7])
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_physics_row_spill_path_matches_oracle(golden, precision, lds_rows):
    """Cooperative kernel with its block row pool capped at lds_rows: the rows past the cap take the global
    spill path of the PGS (1 = all but one row of every block, 7 = a mix of LDS and global rows)."""
    errs = []
    for name in scenarios(golden):
        r = rec(golden, name)
        o = run_scenario(r, precision, skip_physics=False, kernel=1, lds_rows=lds_rows)
        if precision == "fp64":
            err = np.abs(o["phys"] - r["state_post"])
            assert err.max() < 1e-6, "%s: max state err %.3g" % (name, err.max())
            np.testing.assert_array_equal(o["done"], r["done"])
        errs.append(np.abs(o["obs"] - r["obs"]).max(axis=1))
    assert np.median(np.concatenate(errs)) < 1e-3


@pytest.mark.parametrize("kernel", [1, 0])
def test_physics_fp32_matches_oracle_statistics(golden, kernel):
    """Full step, fp32 kernel physics vs fp64 oracle over every recorded step of every scenario."""
    errs, rerr, dmis, n = [], [], 0, 0
    for name in scenarios(golden):
        r = rec(golden, name)
        o = run_scenario(r, "fp32", skip_physics=False, kernel=kernel)
        errs.append(np.abs(o["obs"] - r["obs"]).max(axis=1))
        rerr.append(np.abs(o["rew"] - r["reward"]))
        dmis += int((o["done"] != r["done"]).sum())
        n += len(r["reward"])
    errs, rerr = np.concatenate(errs), np.concatenate(rerr)
    print("fp32 physics: steps=%d obs err p50=%.2e p99=%.2e max=%.2e; reward err p50=%.2e p99=%.2e; done mismatches=%d"
          % (n, np.median(errs), np.percentile(errs, 99), errs.max(), np.median(rerr), np.percentile(rerr, 99), dmis))
    out = os.environ.get("ILRL_PARITY_OUT")    # summary for bench.py's "parity" object (copied into profiles/)
    if out:
        os.makedirs(out, exist_ok=True)
        json.dump({"vs": "fp64 CPU oracle (PyBullet absent: parity vs PyBullet unpinned)", "kernel": kernel,
                   "precision": "fp32", "steps": n, "obs_max_abs_err": float(errs.max()),
                   "obs_p50_abs_err": float(np.median(errs)), "obs_p99_abs_err": float(np.percentile(errs, 99)),
                   "reward_max_abs_err": float(rerr.max()), "reward_p99_abs_err": float(np.percentile(rerr, 99)),
                   "done_mismatches": dmis}, open(os.path.join(out, "parity_fp32_kernel%d.json" % kernel), "w"), indent=1)
    assert errs.max() <= 2.5e-4          # measured 8.0e-5 (kernel 1) / 1.1e-4 (kernel 0)
    assert rerr.max() <= 1e-5            # measured 1.3e-6
    assert dmis == 0


@pytest.mark.parametrize("kernel", [1, 0])
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_reset_matches_oracle(precision, kernel):
    """reset()/resetFromFrame with lane RNG draws: kernel vs oracle (low_level_env.py:224-305)."""
    clip = load_clip("motion08_03")
    n = 64
    env = HumanoidVecEnv(n, clips=(clip,), seed=123, precision=precision, kernel=kernel)
    yaw = np.linspace(-90, 90, n)
    sf = np.where(np.arange(n) % 2 == 0, -1, np.arange(n) % clip.max_frame - 5).astype(np.int32)
    sf = np.where(sf < 0, -1, np.abs(sf))
    obs = env.reset(start_frame=torch.as_tensor(sf, device="cuda"), reset_yaw=torch.as_tensor(yaw, device="cuda"))
    obs = obs.cpu().numpy()
    phys, book = env.get_state()
    tol = 1e-12 if precision == "fp64" else 1e-5
    for i in range(n):
        o = O.OracleLowLevelEnv(clip, seed=123, lane=i)
        ref = o.reset(resetYaw=yaw[i]) if sf[i] < 0 else o.resetFromFrame(int(sf[i]), resetYaw=yaw[i])
        assert book[i, N.BK["frame"]] == o.frame
        np.testing.assert_allclose(book[i, N.BK["target"]:N.BK["target"] + 3], o.target, atol=1e-12)
        np.testing.assert_allclose(phys[i], o.state, atol=tol * 10, rtol=1e-6)
        np.testing.assert_allclose(obs[i], ref, atol=2e-5 if precision == "fp32" else 1e-6, rtol=1e-5)
    env.close()


@pytest.mark.parametrize("kernel", [1, 0])
def test_rollout_properties_at_scale(kernel):
    """4096 lanes x 200 auto-reset steps (bench shape): finite, frames/timesteps consistent."""
    n = 4096
    env = HumanoidVecEnv(n, clips=("motion02_04",), seed=5, kernel=kernel)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    prev_t = np.zeros(n)
    for t in range(200):
        a = torch.rand(n, 17, device="cuda", generator=g) * 2 - 1
        obs, rew, done, frame = env.step(a, autoreset=True)
    torch.cuda.synchronize()
    phys, book = env.get_state()
    assert np.isfinite(phys).all() and torch.isfinite(obs).all() and torch.isfinite(rew).all()
    fr = book[:, N.BK["frame"]]
    assert (fr >= 0).all() and (fr < 297).all()
    assert (book[:, N.BK["cur_timestep"]] <= 200).all()
    assert (env.error_flags() & N.HUM_EFLAG_NONFINITE_ACTION) == 0
    env.close()


def test_graph_replay_equals_eager():
    n = 256
    e1 = HumanoidVecEnv(n, clips=("motion09_03",), seed=9)
    e2 = HumanoidVecEnv(n, clips=("motion09_03",), seed=9)
    e1.reset(); e2.reset()
    a = (torch.rand(n, 17, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 2 - 1).contiguous()
    for _ in range(8):
        e1.step(a, autoreset=True)
    torch.cuda.synchronize()
    rc = N.lib().hum_step_graph(e2.h, N.ctypes.c_void_p(a.data_ptr()), N.ctypes.c_void_p(e2.obs.data_ptr()),
                                N.ctypes.c_void_p(e2.reward.data_ptr()), N.ctypes.c_void_p(e2.done.data_ptr()),
                                N.ctypes.c_void_p(e2.frame.data_ptr()), N.HUM_STEP_AUTORESET,
                                N.ctypes.c_void_p(e2.obs_reset.data_ptr()), 8)
    assert rc == 0
    torch.cuda.synchronize()
    p1, b1 = e1.get_state()
    p2, b2 = e2.get_state()
    np.testing.assert_array_equal(p1, p2)
    np.testing.assert_array_equal(b1, b2)
    e1.close(); e2.close()


@pytest.mark.parametrize("kernel", [1, 0])
def test_nonfinite_action_flagged(kernel):
    env = HumanoidVecEnv(5, clips=("motion09_03",), kernel=kernel)
    env.reset()
    a = torch.zeros(5, 17, device="cuda")
    a[2, 5] = float("nan")
    env.step(a)
    assert env.error_flags() & N.HUM_EFLAG_NONFINITE_ACTION
    assert env.done[2].item() == 1
    ph, _ = env.get_state()
    assert np.isfinite(ph).all()
    env.close()


def test_gym_view_and_vector_env():
    from ilrl_amd.low_level_env import HumanoidVectorEnv, LowLevelHumanoidEnv
    e = LowLevelHumanoidEnv(reference_name="motion09_03")
    o = e.reset()
    assert o.shape == (70,) and o.dtype == np.float64
    o, r, d, info = e.step(np.zeros(17, np.float32))
    assert isinstance(r, float) and isinstance(d, bool) and info == {}
    assert e.cur_timestep == 1 and e.target.shape == (3,)
    with pytest.raises(AssertionError):
        e.step(np.full(17, np.nan, np.float32))
    e.close()
    v = HumanoidVectorEnv(8, reference_name="motion09_03")
    obs = v.vector_reset()
    assert len(obs) == 8
    for _ in range(5):
        obs, rews, dones, infos = v.vector_step(np.zeros((8, 17), np.float32))
        for i, d in enumerate(dones):
            if d:
                assert v.reset_at(i).shape == (70,)
    u = v.get_unwrapped()[0]
    for attr in ("deltaJoints", "deltaEndPoints", "lowTargetScore", "deltaVelJoints", "bodyPostureScore",
                 "highTargetScore", "driftScore", "baseReward", "aliveReward", "electricityScore", "jointLimitScore",
                 "robot_pos"):
        getattr(u, attr)


def test_results_independent_of_sharding_at_bench_size():
    """Size-independent property at the bench shape: 4096 lanes on one handle == two 2048-lane handles with
    lane_offset (the multi-GPU layout) after 60 auto-reset steps - bitwise, lane by lane."""
    n = 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    acts = [(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1).contiguous() for _ in range(60)]
    full = HumanoidVecEnv(n, clips=("motion02_04",), seed=11)
    half = [HumanoidVecEnv(n // 2, clips=("motion02_04",), seed=11, lane_offset=k * n // 2) for k in range(2)]
    full.reset()
    for h in half:
        h.reset()
    for a in acts:
        full.step(a, autoreset=True)
        for k, h in enumerate(half):
            h.step(a[k * n // 2:(k + 1) * n // 2].contiguous(), autoreset=True)
    pf, bf = full.get_state()
    for k, h in enumerate(half):
        ph, bh = h.get_state()
        np.testing.assert_array_equal(pf[k * n // 2:(k + 1) * n // 2], ph)
        np.testing.assert_array_equal(bf[k * n // 2:(k + 1) * n // 2], bh)
    full.close()
    for h in half:
        h.close()


def test_four_clip_round_robin_rollout():
    """Config 3: the four clips round-robin per lane; frames stay inside each clip, motion13_13 lanes that walk
    past its 120-row velocity table are flagged (the reference raises IndexError there)."""
    from ilrl_amd.clips import CLIP_NAMES
    n = 1024
    env = HumanoidVecEnv(n, clips=CLIP_NAMES, seed=3)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(2)
    for t in range(150):
        env.step((torch.rand(n, 17, device="cuda", generator=g) * 2 - 1) * 0.5, autoreset=True)
    phys, book = env.get_state()
    assert np.isfinite(phys).all()
    clip = book[:, N.BK["clip"]].astype(int)
    np.testing.assert_array_equal(clip, np.arange(n) % 4)
    frame = book[:, N.BK["frame"]]
    for c, name in enumerate(CLIP_NAMES):
        mf = load_clip(name).max_frame
        assert (frame[clip == c] < mf - 1).all() and (frame[clip == c] >= 0).all(), name
    assert env.error_flags() & N.HUM_EFLAG_VEL_ROW   # motion13_13 frames >= 120 were reached
    env.close()


def test_rollout_deterministic():
    n = 2048
    outs = []
    for _ in range(2):
        env = HumanoidVecEnv(n, clips=("motion08_03",), seed=5)
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(9)
        for t in range(40):
            env.step(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
        outs.append(env.get_state())
        env.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_in_kernel_autoreset_equals_explicit_reset(precision):
    """The step kernel's auto-reset (start frame drawn by lane 0, the reset pose's hinge sin / cos computed
    across the env's lanes) leaves exactly the state, bookkeeping and reset obs that step-without-reset
    followed by hum_reset (reset_kernel, one thread per lane) produces from the same RNG counters."""
    import torch
    n = 256
    a_env = HumanoidVecEnv(n, clips=("motion02_04",), seed=11, precision=precision)
    b_env = HumanoidVecEnv(n, clips=("motion02_04",), seed=11, precision=precision)
    a_env.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    checked = 0
    for s in range(60):
        act = (torch.rand(n, 17, device="cuda", generator=g) * 2 - 1).contiguous()
        phys, book = a_env.get_state()
        b_env.set_state(phys, book)
        _, _, done_a, _ = a_env.step(act, autoreset=True)
        done_a = done_a.cpu().numpy().astype(bool)
        obs_reset_a = a_env.obs_reset.cpu().numpy().copy()
        pa, ba = a_env.get_state()
        _, _, done_b, _ = b_env.step(act, autoreset=False)
        np.testing.assert_array_equal(done_b.cpu().numpy().astype(bool), done_a)
        if done_a.any():
            obs_b = b_env.reset(mask=done_a.astype(np.uint8)).cpu().numpy()
            np.testing.assert_array_equal(obs_reset_a[done_a], obs_b[done_a])
            checked += int(done_a.sum())
        pb, bb = b_env.get_state()
        np.testing.assert_array_equal(pa, pb)
        bad = np.nonzero((ba != bb).any(axis=0))[0]
        names = {v: k for k, v in N.BK.items()}
        assert len(bad) == 0, "book columns differ: %s (lanes %s, max %.3g)" % (
            [names.get(int(c), int(c)) for c in bad], np.nonzero((ba != bb).any(axis=1))[0][:8], np.abs(ba - bb).max())
    a_env.close()
    b_env.close()
    assert checked > 0, "no lane finished an episode"


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_numpy_semantics_alive_threshold(precision):
    """calcAliveReward at the 0.75 boundary (tests/golden/golden_numpy.npz, the reference's own method under
    NumPy 2.2): HUM_NUMPY_2 decides in float32 like the fixture, HUM_NUMPY_1 in float64."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_numpy.npz"), allow_pickle=False)
    xs = g["obs0"]
    n = len(xs)
    for sem in (N.HUM_NUMPY_2, N.HUM_NUMPY_1):
        env = HumanoidVecEnv(n, clips=("motion02_04",), seed=4, precision=precision, numpy_semantics=sem)
        env.reset(start_frame=torch.full((n,), 20, dtype=torch.int32, device="cuda"))
        phys, book = env.get_state()
        phys[:, 2] = xs.astype(np.float64) + 0.8   # obs[0] = float32(z - 0.8) = x (fp64 state)
        env.set_state(phys, book)
        obs, _, _, _ = env.step(torch.zeros(n, 17, device="cuda"), skip_physics=True)
        obs0 = obs[:, 0].cpu().numpy()
        _, book = env.get_state()
        alive = book[:, N.BK["aliveReward"]]
        if precision == "fp64":
            np.testing.assert_array_equal(obs0, xs)
            if sem == N.HUM_NUMPY_2:
                np.testing.assert_array_equal(alive, g["alive"])
        want = [2.0 if ((float(x) + 0.8 > 0.75) if sem == N.HUM_NUMPY_1 else (x + np.float32(0.8) > np.float32(0.75)))
                else -1.0 for x in obs0]
        np.testing.assert_array_equal(alive, want)
        env.close()


@pytest.mark.parametrize("kernel", [1, 0])
@pytest.mark.parametrize("start_from_ref,init_vel", [(False, True), (True, False), (False, False)])
def test_reset_from_frame_switches_match_oracle(start_from_ref, init_vel, kernel):
    """resetFromFrame(startFromRef, initVel) (low_level_env.py:247-305): startFromRef=False keeps the frame and
    leaves the joints at flat_env.reset()'s U(-0.1, 0.1); initVel=False gives no starting base velocity."""
    clip = load_clip("motion09_03")
    n = 32
    env = HumanoidVecEnv(n, clips=(clip,), seed=77, precision="fp64", kernel=kernel)
    env.reset()
    yaw = np.linspace(-60, 60, n)
    obs = env.reset(start_frame=torch.full((n,), 12, dtype=torch.int32, device="cuda"),
                    reset_yaw=torch.as_tensor(yaw, device="cuda"), start_from_ref=start_from_ref,
                    init_vel=init_vel).cpu().numpy()
    phys, book = env.get_state()
    env.close()
    for i in range(n):
        o = O.OracleLowLevelEnv(clip, seed=77, lane=i)
        o.reset()
        ref = o.resetFromFrame(12, resetYaw=yaw[i], startFromRef=start_from_ref, initVel=init_vel)
        assert book[i, N.BK["frame"]] == o.frame
        np.testing.assert_allclose(phys[i], o.state, atol=1e-12, rtol=0)
        np.testing.assert_allclose(obs[i], ref, atol=1e-6, rtol=1e-6)
        if not init_vel or not start_from_ref:
            assert (phys[i, 7:10] == 0).all()
        if not start_from_ref:
            assert (np.abs(phys[i, 13:30]) <= 0.1).all() and (phys[i, 30:47] == 0).all()

"""GPU parity at the benchmark's full size (BASELINE configs 2, 3 and 5) and on contact-heavy states.

* 4096 lanes x 200 auto-reset steps of config 2 (motion02_04) and config 3 (the four clips round-robin per
  lane), uniform random actions: no contact is ever dropped (HUM_EFLAG_CONTACT_OVERFLOW stays clear), and a
  sample of 64 lanes per clip, taken mid-rollout, steps exactly like the oracle (oracle.phys_step + the oracle
  env logic, low_level_env.py:475-526) from the lane's injected state, bookkeeping and RNG stream.
* config 5 (the two-level env, hier_env.py:355-366, 538-642): 4096 lanes x 200 auto-reset agent transitions,
  then 64 lanes whose next transition is a high-level one and 64 whose next is a low-level (physics) one step
  once more on the GPU and in oracle_hier.OracleHierEnv from the injected state, bookkeeping and RNG stream.
* contact-heavy states (>= 17 contacts: past the 16 the cooperative kernel keeps in LDS) step like the oracle,
  so the global contact spill path is exact; a lowered max_contacts still flags its overflow.

Tolerances: frame, timestep and the RNG counter bit-exact everywhere.  fp64 kernel: state 1e-6 after a full
step (different but exact formulations), obs 1e-5, reward 1e-5, done exact.  fp32 kernel
(the benchmarked build) vs the fp64 oracle over ONE step from the identical state, held to the error of the
oracle's own physics run in float arithmetic from that state (the fp32 yardstick): see FP32_LANE_QUANTILES
and SENS_BOUND below.  A k = 32 variant steps the benchmark's launch shape (hum_step_k, 4096 lanes).
"""
import json
import os

import numpy as np
import pytest

import oracle as O
import oracle_hier as OH
from oracle_inject import BK, contact_heavy_states, oracle_from_lane

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.clips import CLIP_NAMES, load_clip  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

# one fp32 env step vs the fp64 oracle from the same state ("fp32 step bound").  The yardstick
# is the oracle's own physics instantiated in float arithmetic (oracle/physics_oracle_f32.c) stepped from the same
# state: its distance from the fp64 oracle is the rounding error intrinsic to an fp32 step of this algorithm
# (measured: up to 2.5e-4 in the joint speeds, above SURVEY's 1e-5 - no fp32 step of this physics meets 1e-5).  The
# lane's envelope is that error's max over FP32_REALISATIONS fp32-oracle steps: from the lane's state and from the
# state perturbed by 2^-24 relative (one float32 rounding of the input, which an fp32 step cannot resolve).
#
# The gate is PER LANE (round 5): on every well-conditioned lane and obs block (the 8 body terms, the 17 joint
# positions, the 17 joint speeds) the ratio kernel error / the same lane's envelope is formed, and over FP32_LANES
# lanes its quantiles must stay within FP32_LANE_QUANTILES - the kernel's typical error no larger than the yardstick's
# and its tail (p90, p99) within 1.5x and 3x of it.  Targets stated before the measurement, met by
# the pivot-local ABA (physics.h::aba); the round-4 world-frame ABA measured p90 2.75 / p99 7.8 on joint speeds and
# fails it.  The per-lane error is heavy-tailed (a lane on the edge of a limit or contact switch: max ratios 4 - 12
# for every build) so the maximum is bounded absolutely instead (FP32_ABS_MAX: twice the largest fp32-oracle
# envelope measured over 2048 lanes, tools/fp32lab).  The 28 clip-table values differ only by their float32 output
# rounding (<= FP32_FLOOR).  Over ALL lanes (ill-conditioned ones included) the reward stays within max(1e-4, 2 x the
# envelope's).
FP32_FLOOR = {"obs": 1e-5, "reward": 1e-5}
FP32_RATIO = 1.5
FP32_REALISATIONS = 4
FP32_LANES = 512   # config 5's physics transitions; configs 2 (k = 1 and k = 32) and 3 twice as many
# The floor of these ratios: another fp32 realisation of the oracle itself against the 4-realisation envelope measures
# p50 0.72, p90 1.2, p99 1.9 - 2.3, max 3 - 4.4 on joint speeds (512 and 2048 lanes, the bench's states); the p99 over
# 512 lanes (the 5th largest ratio) varies by +-0.5 between state samples for one build, hence 1024 lanes for config 2.
FP32_LANE_QUANTILES = {50: 1.0, 90: 1.5, 99: 3.0}
# ratio denominators below this are raised to it: errors under ~1 float32 ulp of an O(1) observation are not compared
FP32_LANE_FLOOR = 1e-7
FP32_ABS_MAX = {"body": 1e-4, "joint_pos": 1e-4, "joint_vel": 6e-4}
# the fixed bound the short-scenario tests (the hier golden scenarios, terrain) still use: 2x round 2's worst
# measured conditioned error
FP32_BOUND = {"obs_max": 1e-4, "reward_max": 1e-5}
OBS_BLOCKS = {"body": np.arange(0, 8), "joint_pos": np.arange(8, 42, 2), "joint_vel": np.arange(9, 42, 2),
              "clip_table": np.arange(42, 70)}
# Conditioning: a lane whose oracle step moves its obs by more than SENS_BOUND when the input state is perturbed by
# 2^-24 relative (float32 rounding) sits at a discontinuity of the model (a joint limit or contact switching on within
# that margin; Bullet's limits and contacts act only when violated / within the threshold).  There float32 vs float64
# rounding inside the step can switch it too, so the error is the model's; such lanes are counted, not bounded.
SENS_BOUND = 1e-5
# measured 4 - 10 of 64 per clip sample (joints resting on their limits after 200 random-action steps); every
# excluded lane is checked instead through the fp64 kernel stepped from the identical state (FP64_BOUND): the
# exclusion is the model's discontinuity, not the fp32 kernel's
MAX_ILL_FRACTION = 0.2
FP64_BOUND = {"obs_max": 1e-5, "reward_max": 1e-5, "state_max": 1e-6}


def unit_quat(phys):
    """The states with the base quaternion renormalised in float64.  An fp32 state's quaternion is unit only to
    float32 rounding (|q|^2 - 1 ~ 1e-7), so its rotation matrix is orthogonal only to that; the kernel (world-frame
    spatial algebra) and the oracle (local-frame, pybullet's link layout) use R^T as R^-1 in different places and
    the dynamics amplify the 1e-7 difference by up to ~1e7 on stiff states (measured: fp64 kernel vs oracle 1.2e-4
    from a raw fp32 state, 1e-12 from the same state renormalised).  The fp64 cross-check starts from these."""
    p = np.array(phys, dtype=np.float64, copy=True)
    p[..., 3:7] /= np.linalg.norm(p[..., 3:7], axis=-1, keepdims=True)
    return p


def _sample_lanes(book, c, name, per_clip, n):
    lanes = np.nonzero(book[:, BK["clip"]].astype(int) == c)[0]
    if name == "motion13_13":   # the reference raises IndexError past the 120-row velocity table
        lanes = lanes[book[lanes, BK["frame"]] + 2 < 120]
    idx = np.linspace(0, len(lanes) - 1, min(per_clip, len(lanes))).astype(int)
    return lanes[idx]


def rollout_and_compare(clips, precision, n=4096, steps=200, per_clip=64, seed=21, k=1):
    """k = 1: the rollout and the compared step are hum_step launches.  k > 1: the bench's launch shape - the rollout
    runs in hum_step_k launches of k env steps and the compared step is the first row of a k-step launch (its state
    after that step is not observable, so the state comparison is skipped)."""
    env = HumanoidVecEnv(n, clips=clips, seed=seed, precision=precision)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(4)
    if k == 1:
        for _ in range(steps):
            env.step(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
    else:
        for _ in range(steps // k):
            env.step_k(torch.rand(k, n, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
    flags = env.error_flags()
    phys, book = env.get_state()
    a = np.random.default_rng(5).uniform(-1, 1, (n, 17)).astype(np.float32)
    if k == 1:
        obs, rew, done, frame = [x.cpu().numpy() for x in env.step(torch.as_tensor(a, device="cuda"))]
        phys2, book2 = env.get_state()
    else:
        ak = torch.rand(k, n, 17, device="cuda", generator=g) * 2 - 1
        ak[0] = torch.as_tensor(a, device="cuda")
        obs, rew, done, frame, _ = [x[0].cpu().numpy() for x in env.step_k(ak, autoreset=True)]
        phys2, book2 = None, None
    env.close()
    # the fp64 kernel from the identical state, base quaternion renormalised (checks the lanes the fp32 bound
    # excludes; see unit_quat)
    physn = unit_quat(phys)
    env64 = HumanoidVecEnv(n, clips=clips, seed=seed, precision="fp64",
                           kernel=int(os.environ.get("ILRL_FP64_CHECK_KERNEL", "1")))   # diagnostics: 0 = per-lane
    env64.set_state(physn, book)
    obs64, rew64, done64, _ = [x.cpu().numpy() for x in env64.step(torch.as_tensor(a, device="cuda"))]
    phys64, _ = env64.get_state()
    env64.close()
    st = {"obs": [], "rew": [], "done": [], "state": [], "sens": [], "frame_ok": True, "lanes": 0,
          "obs64": [], "rew64": [], "done64": [], "state64": [], "obs_vec": [], "obs_vec_o32": [], "rew_o32": [],
          "obs_vec_o32env": [], "rew_o32env": []}
    prng = np.random.default_rng(6)
    prng32 = np.random.default_rng(7)
    for c, name in enumerate(clips):
        clip = load_clip(name)
        for i in _sample_lanes(book, c, name, per_clip, n):
            o = oracle_from_lane(clip, phys[i], book[i])
            ro, rr, rd, _ = o.step(a[i])
            st["obs"].append(np.abs(obs[i] - ro).max())
            st["obs_vec"].append(np.abs(obs[i] - ro))
            st["rew"].append(abs(float(rew[i]) - rr))
            st["done"].append(bool(done[i]) != rd)
            if phys2 is not None:
                st["state"].append(np.abs(phys2[i] - o.state).max())
            # the fp32 yardstick: the oracle's physics in float arithmetic from the same state (realisation 0) and
            # from the state perturbed by one float32 rounding (the envelope)
            env_o, env_r = np.zeros(70), 0.0
            for rz in range(FP32_REALISATIONS):
                pst = phys[i] if rz == 0 else phys[i] * (1 + 2.0 ** -24 * prng32.choice([-1.0, 1.0], 47))
                r32o, r32r, _, _ = oracle_from_lane(clip, pst, book[i], phys_precision="fp32").step(a[i])
                if rz == 0:
                    st["obs_vec_o32"].append(np.abs(r32o - ro))
                    st["rew_o32"].append(abs(r32r - rr))
                env_o, env_r = np.maximum(env_o, np.abs(r32o - ro)), max(env_r, abs(r32r - rr))
            st["obs_vec_o32env"].append(env_o)
            st["rew_o32env"].append(env_r)
            o64 = oracle_from_lane(clip, physn[i], book[i])
            ro64, rr64, rd64, _ = o64.step(a[i])
            st["obs64"].append(np.abs(obs64[i] - ro64).max())
            st["rew64"].append(abs(float(rew64[i]) - rr64))
            st["done64"].append(bool(done64[i]) != rd64)
            st["state64"].append(np.abs(phys64[i] - o64.state).max())
            p = oracle_from_lane(clip, phys[i] * (1 + 2.0 ** -24 * prng.choice([-1.0, 1.0], 47)), book[i])
            st["sens"].append(np.abs(p.step(a[i])[0] - ro).max())
            st["frame_ok"] &= int(frame[i]) == o.frame
            if book2 is not None:
                st["frame_ok"] &= int(book2[i, BK["cur_timestep"]]) == o.cur_timestep
                st["frame_ok"] &= int(book2[i, BK["rng_counter"]]) == o.rng.counter
            st["lanes"] += 1
    return flags, {k: (np.array(v) if isinstance(v, list) else v) for k, v in st.items()}


def _quantiles(r):
    return {"p50": float(np.median(r)), "p90": float(np.percentile(r, 90)), "p99": float(np.percentile(r, 99)),
            "max": float(r.max()), "lanes": int(len(r))}


def _summary(tag, st):
    good = st["sens"] <= SENS_BOUND
    s = {"lanes": st["lanes"], "obs_max": float(st["obs"].max()), "obs_p99": float(np.percentile(st["obs"], 99)),
         "obs_p50": float(np.median(st["obs"])), "reward_max": float(st["rew"].max()),
         "reward_p99": float(np.percentile(st["rew"], 99)), "done_mismatch": int(st["done"].sum()),
         "state_max": float(st["state"].max()) if len(st["state"]) else None,
         "state_p50": float(np.median(st["state"])) if len(st["state"]) else None,
         "ill_conditioned": int((~good).sum()), "obs_max_conditioned": float(st["obs"][good].max()),
         "reward_max_conditioned": float(st["rew"][good].max()),
         "done_mismatch_conditioned": int(st["done"][good].sum()), "sens_max": float(st["sens"].max())}
    if "obs64" in st and len(st["obs64"]):
        s["fp64_kernel_same_state"] = {"obs_max": float(st["obs64"].max()), "reward_max": float(st["rew64"].max()),
                                       "state_max": float(st["state64"].max()), "done_mismatch": int(st["done64"].sum()),
                                       "obs_max_ill_conditioned": float(st["obs64"][~good].max(initial=0))}
    if len(st.get("obs_vec_o32", [])):
        # per obs component and block, well-conditioned lanes: the kernel vs the fp32 oracle (both vs the fp64 oracle)
        kv, ov, ev = st["obs_vec"][good], st["obs_vec_o32"][good], st["obs_vec_o32env"][good]
        rms = lambda x: float(np.sqrt(np.mean(np.square(x)))) if len(x) else 0.0
        s["fp32_oracle"] = {
            "obs_max_conditioned": float(ov.max()), "reward_max_conditioned": float(st["rew_o32"][good].max()),
            "obs_max": float(st["obs_vec_o32"].max()), "reward_max": float(st["rew_o32"].max()),
            "envelope": {"realisations": FP32_REALISATIONS, "obs_max_conditioned": float(ev.max()),
                         "reward_max_conditioned": float(st["rew_o32env"][good].max()),
                         "reward_max": float(st["rew_o32env"].max())},
            "reward_rms_conditioned": {"kernel": rms(st["rew"][good]), "fp32_oracle": rms(st["rew_o32"][good])},
            "blocks": {b: {"kernel": float(kv[:, ix].max()), "fp32_oracle": float(ov[:, ix].max()),
                           "fp32_envelope": float(ev[:, ix].max()), "kernel_rms": rms(kv[:, ix].max(1)),
                           "fp32_oracle_rms": rms(ov[:, ix].max(1)), "kernel_p50": float(np.median(kv[:, ix].max(1))),
                           "fp32_oracle_p50": float(np.median(ov[:, ix].max(1))),
                           "lanes_kernel": [float(x) for x in kv[:, ix].max(1)],
                           "lanes_fp32_oracle": [float(x) for x in ov[:, ix].max(1)],
                           "lanes_fp32_envelope": [float(x) for x in ev[:, ix].max(1)],
                           "lane_ratio": _quantiles(kv[:, ix].max(1) / np.maximum(ev[:, ix].max(1), FP32_LANE_FLOOR))}
                       for b, ix in OBS_BLOCKS.items()},
            "per_component": {"kernel": [float(x) for x in kv.max(0)], "fp32_oracle": [float(x) for x in ov.max(0)],
                              "fp32_envelope": [float(x) for x in ev.max(0)]}}
    print(tag, json.dumps(s))
    out = os.environ.get("ILRL_PARITY_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        json.dump(s, open(os.path.join(out, "parity_scale_%s.json" % tag), "w"), indent=1)
    return s


@pytest.mark.parametrize("config,precision,k", [("c2", "fp32", 1), ("c2", "fp64", 1), ("c3", "fp32", 1),
                                               ("c3", "fp64", 1), ("c2", "fp32", 32)])
def test_full_size_rollout_no_drop_and_sample_matches_oracle(config, precision, k):
    """k = 32: the benchmark's launch shape (4096 lanes, 32 env steps per hum_step_k launch)."""
    clips = ("motion02_04",) if config == "c2" else tuple(CLIP_NAMES)
    # fp32: the per-block maxima are compared over FP32_LANES lanes (per clip: 64 for the four-clip config 3)
    per_clip = 2 * FP32_LANES // len(clips) if precision == "fp32" else 64
    flags, st = rollout_and_compare(clips, precision, steps=192 if k > 1 else 200, k=k, per_clip=per_clip)
    assert flags & N.HUM_EFLAG_CONTACT_OVERFLOW == 0, "a contact was dropped"
    assert flags & N.HUM_EFLAG_NONFINITE_ACTION == 0
    assert st["lanes"] >= per_clip * len(clips) - (per_clip if config == "c3" else 0)
    assert st["frame_ok"], "frame / timestep / RNG counter differ from the oracle"
    s = _summary("%s_%s%s" % (config, precision, "_k%d" % k if k > 1 else ""), st)
    if precision == "fp64":
        assert s["state_max"] < 1e-6
        assert s["obs_max"] < 1e-5 and s["reward_max"] < 1e-5
        assert s["done_mismatch"] == 0
    else:
        _check_fp32(s)


def _check_fp32(s):
    o32 = s.get("fp32_oracle")
    if o32 is not None:   # per obs block and the reward, against the fp32 yardstick
        for b, v in o32["blocks"].items():
            if b == "clip_table":   # float32 output rounding of the float64 table values only
                assert v["kernel"] <= FP32_FLOOR["obs"], (b, v)
                continue
            q = v["lane_ratio"]
            for pct, bound in FP32_LANE_QUANTILES.items():
                assert q["p%d" % pct] <= bound, (b, "p%d" % pct, q)
            assert v["kernel"] <= FP32_ABS_MAX[b], (b, v["kernel"])
        env = o32["envelope"]
        assert s["reward_max_conditioned"] <= max(FP32_FLOOR["reward"], FP32_RATIO * env["reward_max_conditioned"])
        assert s["reward_max"] <= max(1e-4, 2 * env["reward_max"]), (s["reward_max"], env)
    assert s["done_mismatch_conditioned"] == 0
    assert s["ill_conditioned"] <= MAX_ILL_FRACTION * s["lanes"]
    f64 = s["fp64_kernel_same_state"]   # every lane incl. the excluded ones: the model, not the kernel
    assert f64["obs_max"] <= FP64_BOUND["obs_max"] and f64["reward_max"] <= FP64_BOUND["reward_max"]
    assert f64["state_max"] <= FP64_BOUND["state_max"] and f64["done_mismatch"] == 0


@pytest.mark.parametrize("kernel", [1, 0])
def test_contact_heavy_states_match_oracle_fp64(kernel):
    """>= 17 contacts per env (the cooperative kernel's LDS list holds 16): the spill path is exact."""
    states, counts = contact_heavy_states(64)
    assert counts.max() >= 20
    n = len(states)
    env = HumanoidVecEnv(n, clips=("motion02_04",), seed=3, precision="fp64", kernel=kernel)
    env.reset()
    _, book = env.get_state()
    env.set_state(states, book)
    a = np.random.default_rng(8).uniform(-1, 1, (n, 17)).astype(np.float32)
    env.step(torch.as_tensor(a, device="cuda"))
    phys, _ = env.get_state()
    flags = env.error_flags()
    env.close()
    assert flags & N.HUM_EFLAG_CONTACT_OVERFLOW == 0
    for i in range(n):
        ref = O.phys_step(states[i], O.motor_torques(a[i]))
        err = np.abs(phys[i] - ref).max()
        assert err < 1e-6, "lane %d (%d contacts): state err %.3g" % (i, counts[i], err)


def test_lowered_contact_cap_flags_overflow():
    states, _ = contact_heavy_states(8)
    env = HumanoidVecEnv(8, clips=("motion02_04",), seed=3, max_contacts=8)
    env.reset()
    _, book = env.get_state()
    env.set_state(states, book)
    env.step(torch.zeros(8, 17, device="cuda"))
    assert env.error_flags() & N.HUM_EFLAG_CONTACT_OVERFLOW
    env.close()


# ------------------------------------------------------------------------------------------ config 5 (hier)
def _agents_of(robs):
    return (N.HUM_AGENT_HIGH if OH.HIGH in robs else 0) | (N.HUM_AGENT_LOW if OH.LOW in robs else 0)


def hier_rollout_and_compare(precision, n=4096, steps=200, per_kind=64, seed=23):
    """per_kind lanes of each transition kind (an int, or {1: high-level, 0: low-level}); the fp32 test takes
    FP32_LANES low-level (physics) transitions for the per-lane gate and HIER_HIGH_LANES high-level ones, which take no
    physics step and are held to their own absolute bound (HIER_HIGH_BOUND)"""
    if isinstance(per_kind, int):
        per_kind = {1: per_kind, 0: per_kind}
    from ilrl_amd.hier_env import HierVecEnv, HIER_CLIP
    clip = load_clip(HIER_CLIP)
    env = HierVecEnv(n, seed=seed, precision=precision)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(9)
    for _ in range(steps):
        env.step(torch.rand(n, 2, device="cuda", generator=g) * 2 - 1,
                 torch.rand(n, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
    flags = env.error_flags()
    phys, book = env.get_state()
    rng = np.random.default_rng(15)
    ah = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    al = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
    T = lambda x: torch.as_tensor(x, device="cuda")
    outs = {}
    for prec, e in ((precision, env), ("fp64", None)):
        if e is None:   # the fp64 kernel from the identical state, base quaternion renormalised (unit_quat)
            e = HierVecEnv(n, seed=seed, precision="fp64")
            e.set_state(unit_quat(phys), book)
        res = [x.cpu().numpy() for x in e.step(T(ah), T(al))]
        outs[prec if e is env else "f64"] = res + list(e.get_state())
        e.close()
    agents, oh, ol, rh, rl, done, frame, phys2, book2 = outs[precision]
    a64, oh64, ol64, rh64, rl64, d64, _, p64, _ = outs["f64"]
    expect = book[:, BK["expect_high"]].astype(int)
    st = {k: [] for k in ("obs", "rew", "done", "state", "sens", "obs64", "rew64", "done64", "state64", "kind",
                          "obs_vec", "obs_vec_o32", "rew_o32", "obs_vec_o32env", "rew_o32env")}
    st["exact_ok"], st["lanes"] = True, 0
    prng = np.random.default_rng(16)
    prng32 = np.random.default_rng(17)
    for kind in (1, 0):   # high-level transition, low-level (physics) transition
        lanes = np.nonzero(expect == kind)[0]
        assert len(lanes) >= per_kind[kind]
        for i in lanes[np.linspace(0, len(lanes) - 1, per_kind[kind]).astype(int)]:
            act = {OH.HIGH: ah[i]} if kind else {OH.LOW: al[i]}
            o = OH.OracleHierEnv.from_lane(clip, phys[i], book[i], BK)
            robs, rrew, rdone, _ = o.step(act)
            ag = _agents_of(robs)
            st["exact_ok"] &= int(agents[i]) == ag and int(a64[i]) == ag
            st["exact_ok"] &= int(frame[i]) == o.selected_motion_frame
            for k, v in (("cur_timestep", o.cur_timestep), ("rng_counter", o.rng.counter),
                         ("steps_remaining_at_level", o.steps_remaining_at_level),
                         ("num_high_level_steps", o.num_high_level_steps)):
                st["exact_ok"] &= int(book2[i, BK[k]]) == int(v)

            def errs(obs_h, obs_l, r_h, r_l, robs, rrew):
                e = 0.0
                if OH.HIGH in robs:
                    e = max(e, float(np.abs(obs_h[i] - robs[OH.HIGH]).max()))
                if OH.LOW in robs:
                    e = max(e, float(np.abs(obs_l[i] - robs[OH.LOW]).max()))
                r = max(abs(float(r_h[i]) - float(rrew.get(OH.HIGH, 0))), abs(float(r_l[i]) - float(rrew.get(OH.LOW, 0))))
                return e, r
            eo, er = errs(oh, ol, rh, rl, robs, rrew)
            # per low-obs component, and the fp32 yardstick (the oracle's physics in float arithmetic)
            lowvec = lambda ob: np.abs(ob - robs[OH.LOW]) if OH.LOW in robs else np.zeros(70)
            st["obs_vec"].append(lowvec(ol[i]))
            env_o, env_r = np.zeros(70), 0.0
            for rz in range(FP32_REALISATIONS):
                pst = phys[i] if rz == 0 else phys[i] * (1 + 2.0 ** -24 * prng32.choice([-1.0, 1.0], 47))
                robs32, rrew32, _, _ = OH.OracleHierEnv.from_lane(clip, pst, book[i], BK, phys_precision="fp32").step(act)
                vo = lowvec(robs32[OH.LOW]) if OH.LOW in robs32 else np.zeros(70)
                vr = max(abs(float(rrew32.get(a_, 0)) - float(rrew.get(a_, 0))) for a_ in (OH.HIGH, OH.LOW))
                if rz == 0:
                    st["obs_vec_o32"].append(vo)
                    st["rew_o32"].append(vr)
                env_o, env_r = np.maximum(env_o, vo), max(env_r, vr)
            st["obs_vec_o32env"].append(env_o)
            st["rew_o32env"].append(env_r)
            o64 = OH.OracleHierEnv.from_lane(clip, unit_quat(phys[i]), book[i], BK)   # the fp64 cross-check's
            robs64, rrew64, rdone64, _ = o64.step(act)
            eo64, er64 = errs(oh64, ol64, rh64, rl64, robs64, rrew64)
            st["obs"].append(eo)
            st["rew"].append(er)
            st["done"].append(bool(done[i]) != rdone["__all__"])
            st["state"].append(float(np.abs(phys2[i] - o.state).max()))
            st["obs64"].append(eo64)
            st["rew64"].append(er64)
            st["done64"].append(bool(d64[i]) != rdone64["__all__"])
            st["state64"].append(float(np.abs(p64[i] - o64.state).max()))
            if kind:
                st["sens"].append(0.0)   # no physics: no discontinuity
            else:
                p = OH.OracleHierEnv.from_lane(clip, phys[i] * (1 + 2.0 ** -24 * prng.choice([-1.0, 1.0], 47)), book[i],
                                               BK)
                pobs = p.step(act)[0]
                st["sens"].append(max(float(np.abs(pobs[k] - robs[k]).max()) for k in robs if k in pobs))
            st["kind"].append(kind)
            st["lanes"] += 1
    return flags, {k: (np.array(v) if isinstance(v, list) else v) for k, v in st.items()}


def _subset(st, m):
    """the per-lane entries of a rollout_and_compare / hier_rollout_and_compare record restricted to mask m"""
    out = {k: (v[m] if isinstance(v, np.ndarray) and v.shape[:1] == m.shape else v) for k, v in st.items()}
    out["lanes"] = int(m.sum())
    return out


# config 5's high-level transitions take no physics step: their outputs (high obs 44, both rewards) come from the
# unchanged state through calc_state / the drift score, so an fp32 kernel is held to SURVEY's tolerances directly
HIER_HIGH_LANES = 128
HIER_HIGH_BOUND = {"obs_max": 1e-5, "reward_max": 1e-5}


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_hier_full_size_rollout_sample_matches_oracle(precision):
    """Config 5 at full size: 4096 lanes, 200 auto-reset transitions, then high-level and low-level transitions vs
    the oracle from the injected lane state (hier_env.py:355-366, 538-642).  fp32: the per-lane gate runs over the
    FP32_LANES low-level (physics) transitions only - the high-level ones have no physics error and would dilute its
    quantiles - and the high-level ones are bounded absolutely (HIER_HIGH_BOUND)."""
    per_kind = {1: HIER_HIGH_LANES, 0: FP32_LANES} if precision == "fp32" else 64
    flags, st = hier_rollout_and_compare(precision, per_kind=per_kind)
    assert flags & (N.HUM_EFLAG_CONTACT_OVERFLOW | N.HUM_EFLAG_NONFINITE_ACTION) == 0
    assert st["exact_ok"], "agents / frame / timestep / RNG counter / level counters differ from the oracle"
    if precision == "fp32":
        high = st["kind"] == 1
        sh = _summary("c5_fp32_high", _subset(st, high))
        assert sh["obs_max"] <= HIER_HIGH_BOUND["obs_max"], sh["obs_max"]
        assert sh["reward_max"] <= HIER_HIGH_BOUND["reward_max"], sh["reward_max"]
        assert sh["done_mismatch"] == 0
        s = _summary("c5_fp32", _subset(st, ~high))   # physics transitions only
        assert s["lanes"] >= FP32_LANES
        _check_fp32(s)
        return
    s = _summary("c5_%s" % precision, st)
    if precision == "fp64":
        assert s["state_max"] < FP64_BOUND["state_max"]
        assert s["obs_max"] < FP64_BOUND["obs_max"] and s["reward_max"] < FP64_BOUND["reward_max"]
        assert s["done_mismatch"] == 0
    else:
        _check_fp32(s)

"""The hierarchical CPU oracle (oracle/oracle_hier.py) reproduces the reference HierarchicalHumanoidEnv's own
outputs bit-exactly (golden vectors made by importing /root/reference/hier_env.py under stubs,
tests/golden/make_golden_hier.py)."""
import numpy as np
import pytest

import oracle as O
import oracle_hier as OH
from golden_replay import ScriptedRNG, rec
from ilrl_amd.clips import load_clip

HIER_SCEN = ["hier_l0", "hier_l1", "hier_l2", "hier_l3", "hier_full_actions", "hier_from_frame", "hier_debug",
             "hier_teleport_target", "hier_teleport_far", "hier_predefined", "hier_timestep_limit", "hier_frame_wrap"]
HIER_BOOK = ["selected_motion_frame", "cur_timestep", "highLevelDegTarget", "lowTargetScore", "deltaJoints",
             "deltaVelJoints", "bodyPostureScore", "electricityScore", "jointLimitScore", "aliveReward",
             "delta_lowTargetScore", "predefinedTargetIndex", "highTargetScore", "driftScore", "cumulative_driftScore",
             "delta_highTargetScore", "cumulative_aliveReward", "steps_remaining_at_level", "num_high_level_steps"]
HIER_VEC = ["target", "starting_robot_pos", "robot_pos", "starting_ep_pos"]


def replay_oracle_hier(r):
    env = OH.OracleHierEnv(load_clip("motion09_03"), rng=ScriptedRNG(r["draws"]), numpy_semantics=O.NUMPY_2)
    seed, lane, act_seed, debug, reset_yaw, start_frame, ts_off = [int(x) for x in r["meta"]]
    if len(r["predefined"]):
        env.usePredefinedTarget = True
        env.predefinedTarget = r["predefined"].copy()
    obs0 = env.reset() if start_frame < 0 else env.resetFromFrame(start_frame, resetYaw=reset_yaw)
    out = {"obs0": obs0[OH.HIGH], "state0": env.state.copy(), "book": [], "state_post": []}
    for k in ("has_high", "has_low", "obs_high", "obs_low", "rew_high", "rew_low", "done"):
        out[k] = []
    for t in range(len(r["done"])):
        env.state = r["state_pre"][t].copy()
        env.cur_timestep = int(r["cur_timestep_pre"][t])
        act = {OH.HIGH: r["action_high"][t]} if r["agent"][t] else {OH.LOW: r["action_low"][t]}
        obs, rew, done, _ = env.step(act, debug=bool(debug))
        out["has_high"].append(OH.HIGH in obs)
        out["has_low"].append(OH.LOW in obs)
        out["obs_high"].append(obs.get(OH.HIGH, np.zeros(44)))
        out["obs_low"].append(obs.get(OH.LOW, np.zeros(70)))
        out["rew_high"].append(float(rew.get(OH.HIGH, 0.0)))
        out["rew_low"].append(float(rew.get(OH.LOW, 0.0)))
        out["done"].append(done["__all__"])
        out["state_post"].append(env.state.copy())
        b = {k: float(getattr(env, k)) for k in HIER_BOOK}
        b.update({k: np.array(getattr(env, k), dtype=np.float64) for k in HIER_VEC})
        b["walk_target"] = np.array(env.walk_target)
        b["body_xyz"] = np.array(env.body_xyz[:2])
        out["book"].append(b)
    return out


@pytest.fixture(scope="session")
def golden_hier():
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_hier.npz"),
                   allow_pickle=False)


@pytest.mark.parametrize("name", HIER_SCEN)
def test_hier_oracle_matches_reference(golden_hier, name):
    r = rec(golden_hier, name)
    o = replay_oracle_hier(r)
    np.testing.assert_array_equal(o["obs0"], r["obs0"])
    np.testing.assert_array_equal(o["state0"], r["state0"])
    np.testing.assert_array_equal(np.array(o["state_post"]), r["state_post"])
    for k in ("has_high", "has_low", "obs_high", "obs_low", "rew_high", "rew_low", "done"):
        np.testing.assert_array_equal(np.array(o[k]), r[k], err_msg=k)
    for k in HIER_BOOK + HIER_VEC + ["walk_target", "body_xyz"]:
        got = np.array([b[k] for b in o["book"]], dtype=np.float64)
        np.testing.assert_array_equal(got, r["book_" + k].astype(np.float64), err_msg=k)


def test_hier_golden_covers_protocol(golden_hier):
    """The fixtures exercise every branch of low_level_step's return (hier_env.py:624-641) and checkTarget."""
    agents, hh, hl, dn = [], [], [], []
    for name in HIER_SCEN:
        r = rec(golden_hier, name)
        agents.append(r["agent"]); hh.append(r["has_high"]); hl.append(r["has_low"]); dn.append(r["done"])
    agents, hh, hl, dn = map(np.concatenate, (agents, hh, hl, dn))
    low = agents == 0
    assert (low & hl & ~hh).any()            # ordinary low step
    assert (low & hh & ~hl & ~dn).any()      # level hand-back to the high agent
    assert (low & hh & hl & dn).any()        # episode end
    assert (rec(golden_hier, "hier_teleport_target")["draws"].shape[0]) >= 3

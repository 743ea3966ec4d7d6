#!/usr/bin/env python3
"""Generate golden vectors for the hierarchical env from the REAL reference module (survey container only).

`/root/reference/hier_env.py` (HierarchicalHumanoidEnv, a two-agent RLlib MultiAgentEnv) and its helper
`math_util.py` are imported unmodified, with the same stub modules `make_golden.py` installs for the absent
third-party packages (gym, pybullet, pybullet_envs, ray): the flat env's physics is the fp64 oracle, the robot
is the reference's own `CustomHumanoidRobot`, the unseeded `np.random.default_rng()` (hier_env.py:89) is a
recording wrapper around the counter-based lane RNG.

A scenario drives the multi-agent protocol the way RLlib does: after reset only "high_level_agent" acts; its
step returns the low-level obs; the low agent acts until the env hands control back (every 5 low steps,
hier_env.py:631-636) or the episode ends.  Per call we record the acting agent, its action, the physics state
before/after, the returned obs/rew dicts, done["__all__"] and the full bookkeeping.  Output:
`tests/golden/golden_hier.npz` (data only - no reference source is stored).

Usage: python tests/golden/make_golden_hier.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (stubs, fake flat env, recording RNG)

BOOK = ["selected_motion_frame", "cur_timestep", "highLevelDegTarget", "lowTargetScore", "deltaJoints",
        "deltaVelJoints", "bodyPostureScore", "electricityScore", "jointLimitScore", "aliveReward",
        "delta_lowTargetScore", "predefinedTargetIndex", "highTargetScore", "driftScore", "cumulative_driftScore",
        "delta_highTargetScore", "cumulative_aliveReward", "steps_remaining_at_level", "num_high_level_steps"]
VEC = ["target", "starting_robot_pos", "robot_pos", "starting_ep_pos"]
HIGH, LOW = "high_level_agent", "low_level_agent"


def snapshot(env):
    d = {k: float(getattr(env, k)) for k in BOOK}
    for k in VEC:
        d[k] = np.array(getattr(env, k), dtype=np.float64).copy()
    d["walk_target"] = np.array([env.flat_env.robot.walk_target_x, env.flat_env.robot.walk_target_y], dtype=np.float64)
    d["body_xyz"] = np.array(env.flat_env.robot.body_xyz[:2], dtype=np.float64)
    d["rng_counter"] = float(env.rng.r.counter)
    return d


def run_scenario(name, seed, lane, calls, act_seed, start_frame=None, reset_yaw=0, debug=False, teleport=None,
                 predefined=None, timestep_offset=0, high_scale=1.0, low_scale=1.0):
    import hier_env
    from humanoid import CustomHumanoidRobot
    env = hier_env.HierarchicalHumanoidEnv(customRobot=CustomHumanoidRobot())
    env.rng = MG.RecordingRNG(seed, lane)
    if predefined is not None:
        env.usePredefinedTarget = True
        env.predefinedTarget = np.array(predefined, dtype=np.float64)
    if start_frame is None:
        obs0 = env.reset()
    else:
        obs0 = env.resetFromFrame(startFrame=start_frame, resetYaw=reset_yaw)
    rec = {"obs0": np.array(obs0[HIGH], dtype=np.float64), "state0": env.flat_env.state.copy()}
    for k, v in snapshot(env).items():
        rec["book0_" + k] = np.asarray(v)
    if timestep_offset:
        env.cur_timestep += timestep_offset
    arng = np.random.default_rng(act_seed)
    keys = ["agent", "action_high", "action_low", "state_pre", "state_post", "cur_timestep_pre", "has_high", "has_low",
            "obs_high", "obs_low", "rew_high", "rew_low", "done", "teleported"]
    out = {k: [] for k in keys}
    books = []
    agent = HIGH
    for t in range(calls):
        ah = (arng.uniform(-1, 1, 2) * high_scale).astype(np.float32)
        al = (arng.uniform(-1, 1, 17) * low_scale).astype(np.float32)
        tele = 0
        if teleport is not None and t in teleport:
            off = teleport[t]   # inject a base position near the target (checkTarget / done-by-distance)
            st = env.flat_env.state
            st[0] = env.target[0] + off[0]
            st[1] = env.target[1] + off[1]
            tele = 1
        out["cur_timestep_pre"].append(env.cur_timestep)
        out["state_pre"].append(env.flat_env.state.copy())
        n_tau = len(env.flat_env.torque_log)
        obs, rew, done, _ = env.step({agent: ah if agent == HIGH else al}, debug=debug)
        assert len(env.flat_env.torque_log) == n_tau + (agent == LOW)
        out["agent"].append(1 if agent == HIGH else 0)
        out["action_high"].append(ah)
        out["action_low"].append(al)
        out["state_post"].append(env.flat_env.state.copy())
        out["has_high"].append(HIGH in obs)
        out["has_low"].append(LOW in obs)
        out["obs_high"].append(np.array(obs[HIGH], dtype=np.float64) if HIGH in obs else np.zeros(44))
        out["obs_low"].append(np.array(obs[LOW], dtype=np.float64) if LOW in obs else np.zeros(70))
        assert (HIGH in rew) == (HIGH in obs) and (LOW in rew) == (LOW in obs)
        out["rew_high"].append(float(rew[HIGH]) if HIGH in rew else 0.0)
        out["rew_low"].append(float(rew[LOW]) if LOW in rew else 0.0)
        out["done"].append(bool(done["__all__"]))
        out["teleported"].append(tele)
        books.append(snapshot(env))
        if done["__all__"]:
            break
        agent = HIGH if HIGH in obs else LOW   # the agent that received an observation acts next
    for k, v in out.items():
        rec[k] = np.array(v)
    for k in books[0]:
        rec["book_" + k] = np.array([b[k] for b in books])
    rec["meta"] = np.array([seed, lane, act_seed, int(debug), reset_yaw, -1 if start_frame is None else start_frame,
                            timestep_offset], dtype=np.int64)
    rec["draws"] = np.array(env.rng.log, dtype=np.int64).reshape(-1, 3)
    rec["predefined"] = np.array(predefined if predefined is not None else np.zeros((0, 3)), dtype=np.float64)
    nh = int(np.sum(rec["agent"]))
    print("%-22s calls=%3d high=%2d done=%s draws=%d frame_end=%d" % (name, len(out["done"]), nh, out["done"][-1],
                                                                  len(env.rng.log), int(rec["book_selected_motion_frame"][-1])))
    return {name + "/" + k: v for k, v in rec.items()}


def main():
    MG.install_stubs()
    allrec = {}
    S = []
    for lane in range(4):
        S.append(dict(name="hier_l%d" % lane, seed=21, lane=lane, calls=90, act_seed=200 + lane, low_scale=0.4))
    S.append(dict(name="hier_full_actions", seed=22, lane=0, calls=60, act_seed=210))
    S.append(dict(name="hier_from_frame", seed=23, lane=0, calls=40, act_seed=211, start_frame=30, reset_yaw=30,
                  low_scale=0.3))
    S.append(dict(name="hier_debug", seed=24, lane=0, calls=70, act_seed=212, debug=True, start_frame=0, low_scale=0.5))
    S.append(dict(name="hier_teleport_target", seed=25, lane=0, calls=40, act_seed=213, low_scale=0.3,
                  teleport={4: (0.2, -0.1), 11: (0.3, 0.3), 19: (-0.45, 0.1), 26: (0.0, 0.5)}))
    S.append(dict(name="hier_teleport_far", seed=26, lane=0, calls=12, act_seed=214, teleport={5: (9.0, 0.0)}))
    S.append(dict(name="hier_predefined", seed=27, lane=0, calls=40, act_seed=215, start_frame=0, debug=True,
                  predefined=[[0, 5, 0], [5, 5, 0], [5, 0, 0], [0, 0, 0]], low_scale=0.3,
                  teleport={3: (0.1, 0.1), 9: (-0.2, 0.0), 16: (0.0, 0.3)}))
    S.append(dict(name="hier_timestep_limit", seed=28, lane=0, calls=8, act_seed=216, start_frame=5,
                  timestep_offset=2997, low_scale=0.2))
    S.append(dict(name="hier_frame_wrap", seed=29, lane=0, calls=14, act_seed=217, start_frame=82, low_scale=0.2))
    for s in S:
        name = s.pop("name")
        allrec.update(run_scenario(name, **s))
    out = os.path.join(HERE, "golden_hier.npz")
    np.savez_compressed(out, **allrec)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()

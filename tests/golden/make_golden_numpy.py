#!/usr/bin/env python3
"""Golden vectors for the two float32-scalar expressions whose result depends on NumPy's promotion rules,
taken from the REAL reference methods (imported under the stubs of make_golden.py, in this container only):

* `LowLevelHumanoidEnv.calcAliveReward` (low_level_env.py:384-387): `cur_obs[0] + initial_z > 0.75` for
  float32 obs[0] values straddling the threshold (obs[0] = -0.05 and its float32 neighbours);
* `CustomHumanoidRobot.apply_action` (humanoid.py:54-60): the torques it sets for float32 actions.

This image has NumPy 2.2 (NEP 50: float32 scalar op Python float stays float32), so the fixture pins the
HUM_NUMPY_2 semantics; the NumPy 1.x results (float64 promotion, the reference's era) are restated by the
oracle and are parity-unpinned here (no NumPy 1.x in the image).  Output: tests/golden/golden_numpy.npz.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402


def main():
    MG.install_stubs()
    import low_level_env
    from humanoid import CustomHumanoidRobot
    env = low_level_env.LowLevelHumanoidEnv(reference_name="motion02_04", customRobot=CustomHumanoidRobot())
    env.rng = MG.RecordingRNG(0, 0)
    env.resetFromFrame(startFrame=10)
    xs = [np.float32(-0.05)]
    for direction in (1, -1):
        x = np.float32(-0.05)
        for _ in range(8):
            x = np.nextafter(x, np.float32(direction))
            xs.append(x)
    xs += [np.float32(v) for v in (-0.04, -0.06, 0.0, -0.7, 0.3)]
    xs = np.array(sorted(xs), dtype=np.float32)
    alive = []
    for x in xs:
        obs = np.array(env.cur_obs, dtype=np.float32).copy()
        obs[0] = x
        env.cur_obs = obs
        alive.append(env.calcAliveReward())
    rng = np.random.default_rng(3)
    acts = np.concatenate([rng.uniform(-1.5, 1.5, (16, 17)), np.eye(17)[:4] * 0.37]).astype(np.float32)
    torques = []
    for a in acts:
        env.flat_env.robot.apply_action(a)
        torques.append(env.flat_env.torque.copy())
        env.flat_env.torque[:] = 0
    out = os.path.join(HERE, "golden_numpy.npz")
    np.savez_compressed(out, obs0=xs, alive=np.array(alive, dtype=np.int64), action=acts,
                        torque=np.array(torques), numpy_version=np.array(np.__version__))
    print("wrote", out, "alive:", dict(zip([repr(x) for x in xs], alive)))


if __name__ == "__main__":
    main()

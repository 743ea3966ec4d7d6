"""Diagnostics: the margins of tests/test_gpu_dynamics.py's bounds (worst measured / bound per check and precision)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "imitation-learning-rl_amd"))
import test_oracle_dynamics as D  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

O, DT = D.O, 0.0165 / 4
for prec in ("fp64", "fp32"):
    rel = 1e-7 if prec == "fp64" else 3e-4
    n = 32
    env = HumanoidVecEnv(n, seed=3, precision=prec, lin_damp=0.0, ang_damp=0.0, joint_damping=0, self_collision=0,
                         substeps=1, dt_env=DT, gravity=0.0)
    env.reset()
    rng = np.random.default_rng(9)
    env.set_state(phys=np.array([D.random_state(rng) for _ in range(n)]))
    s0, _ = env.get_state()
    act = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
    act[: n // 2] = 0
    env.step(act, autoreset=False)
    s1, _ = env.get_state()
    env.close()
    worst = [0.0, 0.0, 0.0]
    for i in range(n):
        tau = O.motor_torques(act[i].astype(np.float64))
        nu0, acc = D.nu_of(s0[i]), (D.nu_of(s1[i]) - D.nu_of(s0[i])) / DT
        H = O.mass_matrix(s0[i])
        h = 1e-6
        Hd = (O.mass_matrix(D.advance(s0[i], h)) - O.mass_matrix(D.advance(s0[i], -h))) / (2 * h)
        pd = H @ acc + Hd @ nu0
        P = (H @ nu0)[3:6]
        Ld = pd[0:3] + np.cross(s0[i, 7:10], P) + np.cross(s0[i, 0:3], pd[3:6])
        Td = nu0 @ H @ acc + 0.5 * nu0 @ Hd @ nu0
        power = tau @ s0[i, 30:47]
        worst[0] = max(worst[0], abs(Td - power) / (rel * (abs(nu0 @ H @ acc) + abs(power))))
        worst[1] = max(worst[1], np.abs(pd[3:6]).max() / (rel * np.abs(H[3:6] @ acc).max()))
        worst[2] = max(worst[2], np.abs(Ld).max() / (10 * rel * (np.abs(H[0:3] @ acc).max()
                                                                 + np.abs(np.cross(s0[i, 0:3], H[3:6] @ acc)).max())))
    print(prec, "free motion: worst / bound (power, P, L):", ["%.3g" % w for w in worst])

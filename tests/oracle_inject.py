"""Test helpers: an oracle env (oracle/oracle.py) holding exactly a kernel lane's state, and seeded
contact-heavy physics states.  Test infrastructure only (the oracle is the checker)."""
import numpy as np
from scipy.spatial.transform import Rotation as R

import oracle as O
from ilrl_amd import _native as N

BK = N.BK


def oracle_from_lane(clip, phys, book, phys_precision="fp64"):
    """OracleLowLevelEnv whose physics state, bookkeeping and RNG stream are one lane's hum_get_state rows
    (phys_precision "fp32": the oracle's physics in float arithmetic, the fp32 yardstick)."""
    return O.OracleLowLevelEnv.from_lane(clip, phys, book, BK, phys_precision=phys_precision)


def contact_heavy_states(n, min_contacts=17, seed=1):
    """n physics states (random orientation and joint angles, lowest part pressed up to 12 cm into the
    ground, a random twist and spin) with at least `min_contacts` contact candidates under the oracle's
    detector: they exercise the contact spill path (more than the 16 contacts the kernel keeps in LDS)."""
    rng = np.random.default_rng(seed)
    out, counts = [], []
    while len(out) < n:
        st = np.zeros(O.NSTATE)
        st[3:7] = R.random(random_state=int(rng.integers(1 << 30))).as_quat()
        st[13:30] = rng.uniform(O.LO, O.HI)
        p = O.parts(st)
        st[2] = -p[:32, 2].min() + rng.uniform(-0.12, 0.0)
        st[7:13] = rng.uniform(-0.5, 0.5, 6)
        st[30:47] = rng.uniform(-1, 1, 17)
        c = len(O.contacts(st))
        if c >= min_contacts:
            out.append(st)
            counts.append(c)
    return np.array(out), np.array(counts)

"""The RLlib drop-in adapters return exactly what the raw C-ABI path returns (they only move data between the
device and RLlib's per-env Python objects): HumanoidVectorEnv.vector_step / reset_at (RLlib 1.2 VectorEnv,
train_config.py:13-15,321) and HierarchicalVectorEnv.poll / send_actions / try_reset (BaseEnv, train_config.py:18-20,
320), each against a HumanoidVecEnv / HierVecEnv of the same seed stepped with the same actions - obs, rewards,
dones bitwise, the reset rows of done envs equal to the launch's auto-reset rows, actions handed over as RLlib does
(a list of per-env rows / {env_id: {agent_id: action}})."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.hier_env import HIGH, LOW, HierarchicalVectorEnv, HierVecEnv  # noqa: E402
from ilrl_amd.low_level_env import HumanoidVectorEnv  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402


@pytest.mark.parametrize("n", [512, 37])
def test_vector_env_equals_raw_path(n):
    va = HumanoidVectorEnv(n, reference_name="motion02_04", seed=9)
    raw = HumanoidVecEnv(n, clips=("motion02_04",), seed=9)
    o0 = va.vector_reset()
    np.testing.assert_array_equal(np.stack(o0), raw.reset().cpu().numpy())
    rng = np.random.default_rng(3)
    resets = 0
    for s in range(60):
        a = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
        obs, rew, done, info = va.vector_step(list(a) if s % 2 else a)
        ro, rr, rd, _ = [x.cpu().numpy() for x in raw.step(torch.as_tensor(a, device="cuda"), autoreset=True)]
        rres = raw.obs_reset.cpu().numpy()
        assert len(obs) == len(rew) == len(done) == len(info) == n and all(i == {} for i in info)
        np.testing.assert_array_equal(np.stack(obs), ro)
        np.testing.assert_array_equal(np.array(rew, np.float32), rr)
        assert done == rd.astype(bool).tolist() and all(type(x) is bool for x in done)
        assert all(type(x) is float for x in rew)
        for i in np.flatnonzero(rd):
            np.testing.assert_array_equal(va.reset_at(int(i)), rres[i])
            resets += 1
    assert resets > 0
    va.venv.close()
    raw.close()


def test_vector_env_refuses_non_finite_actions():
    va = HumanoidVectorEnv(8, seed=1)
    va.vector_reset()
    a = np.zeros((8, 17), np.float32)
    a[3, 5] = np.nan
    with pytest.raises(AssertionError):
        va.vector_step(list(a))
    va.venv.close()


@pytest.mark.parametrize("n", [256, 37])
def test_base_env_equals_raw_path(n):
    be = HierarchicalVectorEnv(n, seed=4)
    raw = HierVecEnv(n, seed=4)
    obs, rew, dones, infos, _ = be.poll()
    ro = raw.reset().cpu().numpy()
    assert set(obs) == set(range(n))
    np.testing.assert_array_equal(np.stack([obs[i][HIGH] for i in range(n)]), ro.astype(np.float64))
    cur = dict(obs)   # every env's latest observation dict (skipped envs keep theirs)
    rng = np.random.default_rng(5)
    skip_seen = resets = 0
    for s in range(40):
        ah = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        al = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
        acts, agent = {}, np.full(n, N.HUM_AGENT_SEL_SKIP, np.uint8)
        for i, ob in cur.items():
            if s % 7 == 3 and i % 5 == 0:   # RLlib did not act on this env this round
                skip_seen += 1
                continue
            if HIGH in ob:
                acts[i], agent[i] = {HIGH: ah[i]}, 1
            else:
                acts[i], agent[i] = {LOW: al[i]}, 0
        be.send_actions(acts)
        obs, rew, dones, infos, _ = be.poll()
        ag, oh, ol, rh, rl, dn, _ = [x.cpu().numpy() for x in raw.step(ah, al, agent=agent, autoreset=True)]
        rres = raw.obs_high_reset.cpu().numpy()
        assert set(obs) == set(acts)
        for i in acts:
            want_o, want_r = {}, {}
            if ag[i] & N.HUM_AGENT_HIGH:
                want_o[HIGH], want_r[HIGH] = oh[i].astype(np.float64), float(rh[i])
            if ag[i] & N.HUM_AGENT_LOW:
                want_o[LOW], want_r[LOW] = ol[i].astype(np.float64), float(rl[i])
            assert set(obs[i]) == set(want_o) and rew[i] == want_r and set(infos[i]) == set(want_o)
            for k in want_o:
                np.testing.assert_array_equal(obs[i][k], want_o[k])
            assert dones[i] == {"__all__": bool(dn[i])}
            if dn[i]:
                r = be.try_reset(i)
                np.testing.assert_array_equal(r[HIGH], rres[i].astype(np.float64))
                cur[i] = r
                resets += 1
            else:
                cur[i] = obs[i]
    assert skip_seen > 0 and resets > 0
    be.stop()
    raw.close()

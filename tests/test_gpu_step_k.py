"""Multi-step launches (hum_step_k / hum_hier_step_k, include/humanoid_env.h) equal k single-step launches
bitwise: every per-step output row, the auto-reset observations, the final physics state and bookkeeping, and
the error flags - for both kernels, both precisions, round-robin clips, random terrain, the non-finite action
path (lane not stepped) and the hierarchical env with and without an explicit agent selector."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.clips import CLIP_NAMES  # noqa: E402
from ilrl_amd.hier_env import HierVecEnv  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402


def _actions(k, n, width, seed, nonfinite=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = (torch.rand(k, n, width, device="cuda", generator=g) * 2 - 1).contiguous()
    if nonfinite:   # humanoid.py:55 assert: the lane is not stepped at that step only
        a[3, 5, 2] = float("nan")
        a[7, 9, 0] = float("inf")
    return a


def _same_state(e0, e1):
    p0, b0 = e0.get_state()
    p1, b1 = e1.get_state()
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(b0, b1)


CASES = [dict(kernel=1, precision="fp32"), dict(kernel=1, precision="fp64"), dict(kernel=0, precision="fp32"),
         dict(kernel=1, precision="fp32", clips="all"), dict(kernel=1, precision="fp32", terrain=True),
         dict(kernel=1, precision="fp32", nonfinite=True), dict(kernel=0, precision="fp64", nonfinite=True)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join("%s=%s" % kv for kv in c.items()))
def test_step_k_equals_k_steps(case):
    n, k = 256, 12
    clips = tuple(CLIP_NAMES) if case.get("clips") == "all" else ("motion02_04",)
    envs = [HumanoidVecEnv(n, clips=clips, seed=11, precision=case["precision"], kernel=case["kernel"])
            for _ in range(2)]
    for e in envs:
        if case.get("terrain"):
            e.set_terrain(N.HUM_TERRAIN_RANDOM_BLOCKS)
        e.reset()
    acts = _actions(k, n, 17, 3, case.get("nonfinite", False))
    rows = []
    for t in range(k):
        envs[0].obs_reset.zero_()
        o, r, d, f = envs[0].step(acts[t], autoreset=True)
        rows.append([x.clone() for x in (o, r, d, f, envs[0].obs_reset)])
    out = envs[1].step_k(acts, autoreset=True)
    torch.cuda.synchronize()
    for t in range(k):
        o, r, d, f, orst = rows[t]
        assert torch.equal(out[0][t], o), t
        assert torch.equal(out[1][t], r), t
        assert torch.equal(out[2][t], d), t
        assert torch.equal(out[3][t], f), t
        dm = d.bool()
        assert torch.equal(out[4][t][dm], orst[dm]), t
    assert int(sum(int(x[2].sum()) for x in rows)) > 0   # some lanes were reset inside the launch
    _same_state(*envs)
    f0, f1 = envs[0].error_flags(), envs[1].error_flags()
    assert f0 == f1
    assert bool(f0 & N.HUM_EFLAG_NONFINITE_ACTION) == bool(case.get("nonfinite"))
    for e in envs:
        e.close()


@pytest.mark.parametrize("kernel,precision,selector", [(1, "fp32", False), (1, "fp32", True), (1, "fp64", True),
                                                       (0, "fp32", False)])
def test_hier_step_k_equals_k_steps(kernel, precision, selector):
    n, k = 128, 14
    envs = [HierVecEnv(n, seed=5, precision=precision, kernel=kernel) for _ in range(2)]
    for e in envs:
        e.reset()
    ah = _actions(k, n, 2, 7)
    al = _actions(k, n, 17, 8)
    sel = None
    if selector:   # RLlib send_actions with lanes absent at some transitions (HUM_AGENT_SEL_SKIP)
        rng = np.random.default_rng(0)
        sel = np.zeros((k, n), np.uint8)
        sel[0] = 1                                  # every lane expects the high level after reset
        sel[1:] = rng.choice([0, 0, 0, N.HUM_AGENT_SEL_SKIP], size=(k - 1, n)).astype(np.uint8)
    rows = []
    for t in range(k):
        envs[0].obs_high_reset.zero_()
        out = envs[0].step(ah[t], al[t], agent=None if sel is None else sel[t], autoreset=True)
        rows.append([x.clone() for x in out] + [envs[0].obs_high_reset.clone()])
    outk = envs[1].step_k(ah, al, agent=sel, autoreset=True)
    torch.cuda.synchronize()
    for t in range(k):
        agents, oh, ol, rh, rl, done, frame, ohr = rows[t]
        assert torch.equal(outk[0][t], agents), t
        hi = (agents & N.HUM_AGENT_HIGH) != 0
        lo = (agents & N.HUM_AGENT_LOW) != 0
        assert torch.equal(outk[1][t][hi], oh[hi]), t
        assert torch.equal(outk[2][t][lo], ol[lo]), t
        present = agents != 0   # skipped lanes write nothing but agents = 0
        for j, ref in ((3, rh), (4, rl), (5, done), (6, frame)):
            assert torch.equal(outk[j][t][present], ref[present]), (t, j)
        dm = done.bool()
        assert torch.equal(outk[7][t][dm], ohr[dm]), t
    _same_state(*envs)
    for e in envs:
        e.close()


def test_step_k_rejects_bad_arguments():
    env = HumanoidVecEnv(16, seed=1)
    env.reset()
    a = _actions(2, 16, 17, 1)
    o = torch.zeros(2, 16, 70, device="cuda")
    r = torch.zeros(2, 16, device="cuda")
    d = torch.zeros(2, 16, dtype=torch.uint8, device="cuda")
    p = lambda t: N.ctypes.c_void_p(t.data_ptr())
    assert N.lib().hum_step_k(env.h, p(a), p(o), p(r), p(d), None, 0, None, 0, None) == N.HUM_ERR_ARG
    assert N.lib().hum_step_k(env.h, p(a), p(o), p(r), p(d), None, 64, None, 2, None) == N.HUM_ERR_ARG
    assert N.lib().hum_step_k(env.h, p(a), p(o), p(r), p(d), None, 0, None, 2, None) == N.HUM_OK
    env.close()

"""CPU tests of the Python drop-in surface (no GPU, no Ray in this image): with stub `gym` / `ray.rllib`
modules in place the env classes subclass the real framework bases (RLlib 1.2's BaseEnv.to_base_env only
drives VectorEnv / BaseEnv subclasses directly, train_config.py:13-20,320-321), and registration creators give
every env copy its own RNG stream (the reference's envs each own an unseeded default_rng, low_level_env.py:84)."""
import importlib
import sys
import types

import pytest


class _EnvContext(dict):
    """ray.rllib.env.env_context.EnvContext: a dict with worker_index / vector_index attributes."""

    def __init__(self, d, worker_index, vector_index=0):
        super().__init__(d)
        self.worker_index, self.vector_index = worker_index, vector_index


@pytest.fixture
def stub_frameworks(monkeypatch):
    class VectorEnv:
        def __init__(self, observation_space, action_space, num_envs):
            self.observation_space, self.action_space, self.num_envs = observation_space, action_space, num_envs

    class BaseEnv:
        pass

    class Env:
        pass

    mods = {"ray": {}, "ray.rllib": {}, "ray.rllib.env": {}, "ray.rllib.env.vector_env": {"VectorEnv": VectorEnv},
            "ray.rllib.env.base_env": {"BaseEnv": BaseEnv}, "gym": {"Env": Env}}
    for name, attrs in mods.items():
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        monkeypatch.setitem(sys.modules, name, m)
    import ilrl_amd.hier_env as H
    import ilrl_amd.low_level_env as L
    L2 = importlib.reload(L)
    H2 = importlib.reload(H)
    yield L2, H2, VectorEnv, BaseEnv, Env
    monkeypatch.undo()
    importlib.reload(L)
    importlib.reload(H)


def test_classes_subclass_framework_bases(stub_frameworks):
    L, H, VectorEnv, BaseEnv, Env = stub_frameworks
    assert issubclass(L.HumanoidVectorEnv, VectorEnv)
    assert issubclass(H.HierarchicalVectorEnv, BaseEnv)
    assert issubclass(L.LowLevelHumanoidEnv, Env)
    for name in ("vector_reset", "reset_at", "vector_step", "get_unwrapped"):
        assert callable(getattr(L.HumanoidVectorEnv, name))
    for name in ("poll", "send_actions", "try_reset", "get_unwrapped"):
        assert callable(getattr(H.HierarchicalVectorEnv, name))


def test_without_frameworks_bases_are_object():
    import ilrl_amd.low_level_env as L
    if "ray" in sys.modules or "gym" in sys.modules:
        pytest.skip("a real ray / gym is importable")
    assert L.HumanoidVectorEnv.__mro__[1] is object


def test_registration_seeds_are_distinct():
    from ilrl_amd.low_level_env import env_seed
    # no seed: OS entropy per env (the reference's unseeded default_rng)
    assert env_seed(None)[0] != env_seed(None)[0]
    # explicit seed: copies differ by their RLlib worker / vector index (global lane ranges never overlap)
    offs = {env_seed(_EnvContext({"seed": 5}, w, v), 1024)[1] for w in range(7) for v in range(3)}
    assert len(offs) == 21
    assert {env_seed(_EnvContext({"seed": 5}, w, 0), 1024)[0] for w in range(7)} == {5}
    lanes = sorted(env_seed(_EnvContext({"seed": 5}, w, 0), 1024)[1] for w in range(7))
    assert all(b - a >= 1024 for a, b in zip(lanes, lanes[1:]))


def test_bench_launch_sizes_cover_exactly_the_requested_steps():
    """bench.py times exactly --steps env steps (the driver's contract) whatever --k is: whole launches of k, then
    one shorter launch for the remainder."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for steps in (1, 7, 20, 31, 32, 33, 100, 1000):
        for k in (1, 8, 32, 64):
            sz = bench.launch_sizes(steps, k)
            assert sum(sz) == steps and all(0 < x <= k for x in sz) and all(x == k for x in sz[:-1])
    assert bench.launch_sizes(0, 32) == []


def test_bench_drain_plan_replays_the_same_action_rows():
    """bench.launch_plan(drain=True) (the chunked copy-engine gather): the last launch's final fifth runs as its own
    launch over the SAME rows of the same action block, so the trajectory is the unsplit plan's; every launch stays
    inside one block of k rows (and so inside one gather fragment, G a multiple of k)."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    assert bench.launch_plan(20, 32, drain=True) == [(0, 0, 16), (0, 16, 4)]
    assert bench.launch_plan(1000, 32, drain=True)[-3:] == [(30, 0, 32), (31, 0, 6), (31, 6, 2)]
    assert bench.launch_plan(1, 32, drain=True) == [(0, 0, 1)]
    for steps in (1, 2, 7, 20, 31, 32, 33, 100, 1000):
        for k in (1, 8, 32, 64):
            base = bench.launch_plan(steps, k)
            assert [kk for _, _, kk in base] == bench.launch_sizes(steps, k)
            plan = bench.launch_plan(steps, k, drain=True)
            rows = [(b, r) for b, o, kk in plan for r in range(o, o + kk)]
            assert rows == [(b, r) for b, o, kk in base for r in range(o, o + kk)]
            assert all(0 <= o and o + kk <= k and kk > 0 for _, o, kk in plan)


def test_register_envs_vectorised_by_default(monkeypatch):
    """register_envs() registers the N-lane creators by default (one launch per sampler step for all of a worker's
    envs): HumanoidBulletEnv-v0-Low -> make_env_low_vec, HumanoidBulletEnv-v0-Hier -> make_env_hier_vec; with
    vectorised=False the reference's one-env-per-call creators (train_config.py:13-20,320-321)."""
    reg = {}
    for name in ("ray", "ray.tune"):
        monkeypatch.setitem(sys.modules, name, types.ModuleType(name))
    r = types.ModuleType("ray.tune.registry")
    r.register_env = lambda name, fn: reg.__setitem__(name, fn)
    monkeypatch.setitem(sys.modules, "ray.tune.registry", r)
    import ilrl_amd.hier_env as H
    import ilrl_amd.low_level_env as L
    assert L.register_envs() == "HumanoidBulletEnv-v0-Low" and reg["HumanoidBulletEnv-v0-Low"] is L.make_env_low_vec
    assert H.register_envs() == "HumanoidBulletEnv-v0-Hier" and reg["HumanoidBulletEnv-v0-Hier"] is H.make_env_hier_vec
    L.register_envs(vectorised=False)
    H.register_envs(vectorised=False)
    assert reg["HumanoidBulletEnv-v0-Low"] is L.make_env_low and reg["HumanoidBulletEnv-v0-Hier"] is H.make_env_hier

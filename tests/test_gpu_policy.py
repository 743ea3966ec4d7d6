"""On-GPU policy inference (csrc/policy.hip, v_mfma_f32_16x16x4_f32) vs a plain PyTorch fp32 reference of the
same network, and the device-resident rollout loop vs the same loop driven step by step from Python.

Tolerance: the MFMA computes each output as a k-ordered fp32 fma chain, torch's matmul in another order; after
two tanh layers the action means agree to 2e-5 absolute (fp32 rounding of K = 256 dot products)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.hier_env import HierVecEnv  # noqa: E402
from ilrl_amd.policy import DevicePolicy, hier_rollout, reference_mean  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402


@pytest.mark.parametrize("n", [1, 17, 4096, 65536 + 77])   # the last: 4 row tiles per block (policy.hip), ragged end
def test_policy_mean_matches_torch_fp32(n):
    pol = DevicePolicy.random_init(seed=3)
    pol.w["b1"][:] = np.linspace(-0.3, 0.3, 256)   # non-zero biases exercise every term
    pol.close()
    pol = DevicePolicy(pol.w, seed=3)
    g = torch.Generator(device="cuda").manual_seed(n)
    obs = (torch.randn(n, 70, device="cuda", generator=g) * 2).contiguous()
    mean = torch.empty(n, 17, device="cuda")
    act = pol.act(obs, mean_out=mean)
    ref = reference_mean(pol.w, obs)
    assert (mean - ref).abs().max().item() < 2e-5
    torch.testing.assert_close(act, ref.clamp(-1, 1), atol=2e-5, rtol=0)
    if n > 4096:   # the 4-tile blocks equal the 1-tile kernel row for row (the same k-ordered MFMA chains)
        m1 = torch.empty(4096, 17, device="cuda")
        pol.act(obs[-4096:].contiguous(), mean_out=m1)
        assert torch.equal(m1, mean[-4096:])
    pol.close()


def test_policy_done_lanes_read_reset_obs_and_exploration_noise():
    n = 2048
    pol = DevicePolicy.random_init(seed=5, log_std=-2.0)
    g = torch.Generator(device="cuda").manual_seed(1)
    obs = torch.randn(n, 70, device="cuda", generator=g)
    obs_r = torch.randn(n, 70, device="cuda", generator=g)
    done = (torch.rand(n, device="cuda", generator=g) < 0.3).to(torch.uint8)
    mean = torch.empty(n, 17, device="cuda")
    pol.act(obs, obs_r, done, mean_out=mean)
    want = torch.where(done.bool()[:, None], obs_r, obs)
    assert (mean - reference_mean(pol.w, want)).abs().max().item() < 2e-5
    a1 = pol.act(want, explore=True, step=7, mean_out=mean)
    a2 = pol.act(want, explore=True, step=7)
    a3 = pol.act(want, explore=True, step=8)
    assert torch.equal(a1, a2) and not torch.equal(a1, a3)   # counter-based: (seed, lane, step, index)
    z = ((a1 - mean) / np.exp(-2.0))[(a1.abs() < 1)]        # unclipped samples: standard normal noise
    assert abs(z.mean().item()) < 0.02 and abs(z.std().item() - 1) < 0.02
    pol.close()


def test_rollout_equals_python_loop():
    """hum_rollout (policy -> step with auto-reset, k launches pairs on one stream) == the same loop from Python.
    The recorded actions are the samples before clip_actions (what RLlib's SampleBatch keeps for PPO's likelihood
    ratio); the env steps on their clip.  reset() clears `done`: no manual zeroing before the rollout,
    even after a previous episode left done lanes."""
    n, k = 512, 24
    pol = DevicePolicy.random_init(seed=9)
    envs = [HumanoidVecEnv(n, clips=("motion02_04",), seed=2) for _ in range(2)]
    for e in envs:
        e.done.fill_(1)   # stale flags from an earlier episode
        e.reset()
    tr = pol.rollout(envs[0], k, explore=True, step0=100)
    e = envs[1]
    act = torch.empty(n, 17, device="cuda")
    raw = torch.empty(n, 17, device="cuda")
    for t in range(k):
        inp = torch.where(e.done.bool()[:, None], e.obs_reset, e.obs).clone()
        torch.testing.assert_close(tr["obs"][t], inp, atol=0, rtol=0)
        pol.act(e.obs, e.obs_reset, e.done, explore=True, step=100 + t, out=act, raw_out=raw)
        torch.testing.assert_close(tr["actions"][t], raw, atol=0, rtol=0)
        torch.testing.assert_close(tr["actions"][t].clamp(-1, 1), act, atol=0, rtol=0)
        e.step(act, autoreset=True)
        torch.testing.assert_close(tr["rewards"][t], e.reward, atol=0, rtol=0)
        assert torch.equal(tr["dones"][t], e.done)
    p0, b0 = envs[0].get_state()
    p1, b1 = envs[1].get_state()
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(b0, b1)
    assert tr["dones"].sum().item() > 0
    assert (tr["actions"].abs() > 1).any()   # samples past the Box bound are recorded unclipped
    for x in envs:
        x.close()
    pol.close()


@pytest.mark.parametrize("k", [1, 16])
def test_fused_rollout_equals_policy_kernel_and_step_k(k):
    """hum_rollout_fused (the policy inside the multi-step env kernel) vs its two halves run separately: every
    recorded sample equals the standalone policy kernel's on the recorded input (the same k-ordered fp32 fma
    chains), and replaying the clipped samples through hum_step_k from the same start state reproduces the recorded
    rewards, dones, next inputs and final state bitwise.  Both auto-reset paths of the fused kernel run: both envs
    are first stepped identically until some lanes end done, so the first fused step takes the reset observation
    of those lanes (done_in set), and with k = 16 lanes also finish inside the launch (their reset observation is
    read back from LDS at the next step); a second fused rollout continues from the first one's done flags."""
    n = 512
    pol = DevicePolicy.random_init(seed=9)
    envs = [HumanoidVecEnv(n, clips=("motion02_04",), seed=2) for _ in range(2)]
    g = torch.Generator(device="cuda").manual_seed(3)
    pre = [torch.rand(n, 17, device="cuda", generator=g) * 2 - 1 for _ in range(40)]
    for e in envs:
        e.done.fill_(1)
        e.reset()
        for t in range(40):
            e.step(pre[t], autoreset=True)
    assert envs[0].done.any(), "no lane ends the warm-up done: the done_in path would not run"
    done_inside = False
    e = envs[1]
    want0 = torch.where(e.done.bool()[:, None], e.obs_reset, e.obs).clone()
    for rnd in range(2):
        tr = pol.rollout(envs[0], k, explore=True, step0=100 + rnd * k, fused=True)
        torch.testing.assert_close(tr["obs"][0], want0, atol=0, rtol=0)   # done_in lanes took their reset obs
        act = torch.empty(n, 17, device="cuda")
        raw = torch.empty(n, 17, device="cuda")
        worst = 0.0
        for t in range(k):
            pol.act(tr["obs"][t], explore=True, step=100 + rnd * k + t, out=act, raw_out=raw)
            worst = max(worst, (tr["actions"][t] - raw).abs().max().item())
        print("fused policy vs policy kernel (round %d): max |sample diff| %.3g" % (rnd, worst))
        assert worst == 0.0
        torch.testing.assert_close(envs[0]._act_buf, tr["actions"][k - 1].clamp(-1, 1), atol=0, rtol=0)
        obs_k, rew_k, done_k, _, rst_k = e.step_k(tr["actions"].clamp(-1, 1).contiguous(), autoreset=True)
        torch.testing.assert_close(tr["rewards"], rew_k, atol=0, rtol=0)
        assert torch.equal(tr["dones"], done_k)
        done_inside |= bool(done_k[:-1].any())
        for t in range(k - 1):
            want = torch.where(done_k[t].bool()[:, None], rst_k[t], obs_k[t])
            torch.testing.assert_close(tr["obs"][t + 1], want, atol=0, rtol=0)
        torch.testing.assert_close(envs[0].obs, obs_k[k - 1], atol=0, rtol=0)
        torch.testing.assert_close(envs[0].reward, rew_k[k - 1], atol=0, rtol=0)
        assert torch.equal(envs[0].done, done_k[k - 1])
        # the reset observation of lanes done at the launch's last step (the next launch's done_in input)
        last = done_k[k - 1].bool()
        torch.testing.assert_close(envs[0].obs_reset[last], rst_k[k - 1][last], atol=0, rtol=0)
        want0 = torch.where(last[:, None], rst_k[k - 1], obs_k[k - 1]).clone()
        p0, b0 = envs[0].get_state()
        p1, b1 = e.get_state()
        np.testing.assert_array_equal(p0, p1)
        np.testing.assert_array_equal(b0, b1)
    if k > 1:
        assert done_inside, "no lane finished inside a launch: the in-launch reset path did not run"
    for x in envs:
        x.close()
    pol.close()


@pytest.mark.parametrize("n_in,n_out", [(44, 2), (70, 17), (5, 32)])
def test_policy_shapes_match_torch_fp32(n_in, n_out):
    """hum_policy_create_ex: the same network at other widths (44 -> 2 = the high-level policy)."""
    pol = DevicePolicy.random_init(seed=4, n_in=n_in, n_out=n_out)
    pol.w["b3"][:] = np.linspace(-0.2, 0.2, n_out)
    pol.close()
    pol = DevicePolicy(pol.w, seed=4, n_in=n_in, n_out=n_out)
    obs = torch.randn(300, n_in, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2)) * 2
    mean = torch.empty(300, n_out, device="cuda")
    act = pol.act(obs, mean_out=mean)
    ref = reference_mean(pol.w, obs)
    assert (mean - ref).abs().max().item() < 2e-5
    torch.testing.assert_close(act, ref.clamp(-1, 1), atol=2e-5, rtol=0)
    with pytest.raises(ValueError):
        pol.act(torch.zeros(4, n_in + 1, device="cuda"))
    pol.close()


def test_hier_rollout_equals_python_loop():
    """hum_hier_rollout (config 5's two-level sampler: high policy, low policy, hum_hier_step with auto-reset per
    transition) == the same loop driven from Python through hum_policy_act + hum_hier_step, bitwise: policy inputs
    (done lanes: their auto-reset high observation), raw samples, the agent that acted, returned agents, both
    rewards, done and the final state.  Two calls in a row: the second starts from the first one's done flags."""
    n, k = 512, 20
    high = DevicePolicy.random_init_high(seed=11)
    low = DevicePolicy.random_init(seed=9)
    envs = [HierVecEnv(n, seed=4) for _ in range(2)]
    for e in envs:
        e.reset()
    e = envs[1]
    ah, rah = torch.empty(n, 2, device="cuda"), torch.empty(n, 2, device="cuda")
    al, ral = torch.empty(n, 17, device="cuda"), torch.empty(n, 17, device="cuda")
    expect_high = torch.ones(n, dtype=torch.bool, device="cuda")   # after reset every lane's next agent is the high one
    seen = torch.zeros(3, dtype=torch.int64)
    for rnd in range(2):
        tr = hier_rollout(envs[0], high, low, k, explore=True, step0=50 + rnd * k)
        for t in range(k):
            step = 50 + rnd * k + t
            torch.testing.assert_close(tr["obs_high"][t], torch.where(e.done.bool()[:, None], e.obs_high_reset,
                                                                      e.obs_high), atol=0, rtol=0)
            torch.testing.assert_close(tr["obs_low"][t], e.obs, atol=0, rtol=0)
            high.act(e.obs_high, e.obs_high_reset, e.done, explore=True, step=step, out=ah, raw_out=rah)
            low.act(e.obs, explore=True, step=step, out=al, raw_out=ral)
            torch.testing.assert_close(tr["act_high"][t], rah, atol=0, rtol=0)
            torch.testing.assert_close(tr["act_low"][t], ral, atol=0, rtol=0)
            want = torch.where(expect_high, N.HUM_AGENT_HIGH, N.HUM_AGENT_LOW).to(torch.uint8)
            assert torch.equal(tr["acted"][t], want)
            agents, _, _, rh, rl, done, _ = e.step(ah, al, autoreset=True)
            assert torch.equal(tr["agents"][t], agents) and torch.equal(tr["done"][t], done)
            torch.testing.assert_close(tr["rew_high"][t], rh, atol=0, rtol=0)
            torch.testing.assert_close(tr["rew_low"][t], rl, atol=0, rtol=0)
            expect_high = ((agents & N.HUM_AGENT_HIGH) != 0) | (done != 0)
            seen += torch.stack([(tr["acted"][t] == N.HUM_AGENT_HIGH).sum(), (tr["acted"][t] == N.HUM_AGENT_LOW).sum(),
                                 done.sum()]).cpu()
        for name in ("obs_high", "obs_high_reset", "obs", "done", "agents", "reward_high", "reward"):
            a0, a1 = getattr(envs[0], name), getattr(e, name)
            if name == "obs_high_reset":   # rows of lanes that reset at the last transition
                m = e.done.bool()
                a0, a1 = a0[m], a1[m]
            torch.testing.assert_close(a0, a1, atol=0, rtol=0, msg=name)
        p0, b0 = envs[0].get_state()
        p1, b1 = e.get_state()
        np.testing.assert_array_equal(p0, p1)
        np.testing.assert_array_equal(b0, b1)
    assert (seen > 0).all(), "high and low transitions and auto-resets must all occur: %s" % seen.tolist()
    for x in envs:
        x.close()
    high.close()
    low.close()


@pytest.mark.parametrize("n,k", [(510, 20), (512, 1)])
def test_hier_rollout_fused_equals_hier_rollout(n, k):
    """hum_hier_rollout_fused (both networks inside the env kernel, each only for the lanes that act with it) ==
    hum_hier_rollout bitwise on everything the acting agent produces: its policy inputs and raw samples, acted,
    agents, both rewards, done, the env buffers and the final state.  Both envs are first driven through the same
    unfused rollouts so lanes are out of phase (waves whose four envs expect different agents run both networks);
    n = 510 leaves the last wave two envs short."""
    high = DevicePolicy.random_init_high(seed=11)
    low = DevicePolicy.random_init(seed=9)
    envs = [HierVecEnv(n, seed=4) for _ in range(2)]
    for e in envs:
        e.reset()
        for rnd in range(3):
            hier_rollout(e, high, low, 16, explore=True, step0=rnd * 16, trajectories=False)
    mixed = done_seen = 0
    for rnd in range(40 // k if k < 20 else 3):
        step0 = 100 + rnd * k
        tu = hier_rollout(envs[1], high, low, k, explore=True, step0=step0)
        tf = hier_rollout(envs[0], high, low, k, explore=True, step0=step0, fused=True)
        for f in ("acted", "agents", "rew_high", "rew_low", "done"):
            assert torch.equal(tf[f], tu[f]), f
        hi = tu["acted"] == N.HUM_AGENT_HIGH
        lo = tu["acted"] == N.HUM_AGENT_LOW
        for f, m in (("obs_high", hi), ("act_high", hi), ("obs_low", lo), ("act_low", lo)):
            torch.testing.assert_close(tf[f][m], tu[f][m], atol=0, rtol=0, msg=f)
        w = tu["acted"][:, : n // 4 * 4].view(k, -1, 4)
        mixed += int(((w == N.HUM_AGENT_HIGH).any(-1) & (w == N.HUM_AGENT_LOW).any(-1)).sum())
        done_seen += int(tu["done"].sum())
        for name in ("obs_high", "obs", "done", "agents", "reward_high", "reward"):
            torch.testing.assert_close(getattr(envs[0], name), getattr(envs[1], name), atol=0, rtol=0, msg=name)
        m = envs[1].done.bool()
        torch.testing.assert_close(envs[0].obs_high_reset[m], envs[1].obs_high_reset[m], atol=0, rtol=0)
        torch.testing.assert_close(envs[0]._act_high_buf[hi[-1]], envs[1]._act_high_buf[hi[-1]], atol=0, rtol=0)
        torch.testing.assert_close(envs[0]._act_low_buf[lo[-1]], envs[1]._act_low_buf[lo[-1]], atol=0, rtol=0)
        p0, b0 = envs[0].get_state()
        p1, b1 = envs[1].get_state()
        np.testing.assert_array_equal(p0, p1)
        np.testing.assert_array_equal(b0, b1)
    print("fused hier rollout: %d mixed wave-transitions, %d dones" % (mixed, done_seen))
    assert mixed > 0, "no wave held envs expecting different agents: the two-network path did not run"
    assert done_seen > 0, "no auto-reset inside the compared rollouts"
    for x in envs:
        assert x.error_flags() == 0
        x.close()
    high.close()
    low.close()


def test_fused_rollout_mean_trace():
    """hum_rollout_fused_ex's mean trace: every recorded mean equals the standalone policy kernel's mean on the
    recorded input bitwise, the other outputs equal a run without the trace (same start state), and
    sample_batch_columns with the recorded means equals the recomputing call bitwise."""
    n, k = 512, 16
    pol = DevicePolicy.random_init(seed=9)
    envs = [HumanoidVecEnv(n, clips=("motion02_04",), seed=2) for _ in range(2)]
    for e in envs:
        e.reset()
    tm = pol.rollout(envs[0], k, explore=True, step0=7, fused=True, means=True)
    tp = pol.rollout(envs[1], k, explore=True, step0=7, fused=True)
    for f in ("obs", "actions", "rewards", "dones"):
        assert torch.equal(tm[f], tp[f]), f
    mean = torch.empty(n, 17, device="cuda")
    for t in range(k):
        pol.act(tm["obs"][t], explore=False, out=torch.empty(n, 17, device="cuda"), mean_out=mean)
        torch.testing.assert_close(tm["means"][t], mean, atol=0, rtol=0)
    c0 = pol.sample_batch_columns(tm["obs"], tm["actions"])
    c1 = pol.sample_batch_columns(tm["obs"], tm["actions"], mean=tm["means"])
    for f in ("action_dist_inputs", "action_logp"):
        torch.testing.assert_close(c1[f], c0[f], atol=0, rtol=0, msg=f)
    with pytest.raises(ValueError):
        pol.rollout(envs[1], k, fused=False, means=True)
    for x in envs:
        x.close()
    pol.close()


def test_hier_rollout_fused_mean_traces():
    """hum_hier_rollout_fused_ex: on each transition the acting agent's recorded mean equals its policy kernel's
    mean on the recorded input bitwise, and the trajectory equals a fused run without the traces."""
    n, k = 512, 20
    high = DevicePolicy.random_init_high(seed=11)
    low = DevicePolicy.random_init(seed=9)
    envs = [HierVecEnv(n, seed=4) for _ in range(2)]
    for e in envs:
        e.reset()
    tm = hier_rollout(envs[0], high, low, k, explore=True, step0=3, fused=True, means=True)
    tp = hier_rollout(envs[1], high, low, k, explore=True, step0=3, fused=True)
    hi = tm["acted"] == N.HUM_AGENT_HIGH
    lo = tm["acted"] == N.HUM_AGENT_LOW
    assert hi.any() and lo.any()
    for f in ("acted", "agents", "rew_high", "rew_low", "done"):
        assert torch.equal(tm[f], tp[f]), f
    for f, m in (("obs_high", hi), ("act_high", hi), ("obs_low", lo), ("act_low", lo)):
        torch.testing.assert_close(tm[f][m], tp[f][m], atol=0, rtol=0, msg=f)
    for pol, obs, mt, m, no in ((high, tm["obs_high"], tm["mean_high"], hi, 2), (low, tm["obs_low"], tm["mean_low"], lo, 17)):
        rows = obs[m]
        mean = torch.empty(rows.shape[0], no, device="cuda")
        pol.act(rows.contiguous(), explore=False, out=torch.empty_like(mean), mean_out=mean)
        torch.testing.assert_close(mt[m], mean, atol=0, rtol=0)
    for x in envs:
        assert x.error_flags() == 0
        x.close()
    high.close()
    low.close()


def test_hier_rollout_fused_without_trajectory():
    """No trajectory rows: the per-transition agents / rewards / done go to the handle's scratch (grown on demand),
    and the env buffers and the state still equal the per-transition loop's, call after call."""
    n = 256
    high = DevicePolicy.random_init_high(seed=3)
    low = DevicePolicy.random_init(seed=5)
    envs = [HierVecEnv(n, seed=8) for _ in range(2)]
    for e in envs:
        e.reset()
    for rnd, k in enumerate((8, 24, 8)):   # the scratch grows, then is reused
        hier_rollout(envs[0], high, low, k, explore=True, step0=rnd * 32, trajectories=False, fused=True)
        hier_rollout(envs[1], high, low, k, explore=True, step0=rnd * 32, trajectories=False)
        for name in ("obs_high", "obs", "done", "agents", "reward_high", "reward"):
            torch.testing.assert_close(getattr(envs[0], name), getattr(envs[1], name), atol=0, rtol=0, msg=name)
        p0, b0 = envs[0].get_state()
        p1, b1 = envs[1].get_state()
        np.testing.assert_array_equal(p0, p1)
        np.testing.assert_array_equal(b0, b1)
    for x in envs:
        x.close()
    high.close()
    low.close()


def test_hier_rollout_fused_rejects_other_kernels():
    high = DevicePolicy.random_init_high(seed=1)
    low = DevicePolicy.random_init(seed=1)
    env = HierVecEnv(64, seed=1, precision="fp64")
    env.reset()
    with pytest.raises(N.NativeError, match="hum_hier_rollout_fused"):
        hier_rollout(env, high, low, 2, fused=True)
    env.close()
    high.close()
    low.close()


def test_hier_rollout_rejects_wrong_shapes():
    env = HierVecEnv(64, seed=1)
    env.reset()
    low = DevicePolicy.random_init(seed=1)
    with pytest.raises(N.NativeError, match="hum_hier_rollout"):
        hier_rollout(env, low, low, 2)
    env.close()
    low.close()


def test_fused_rollout_rejects_other_kernels():
    pol = DevicePolicy.random_init(seed=1)
    env = HumanoidVecEnv(64, clips=("motion02_04",), seed=2, precision="fp64")
    env.reset()
    with pytest.raises(N.NativeError, match="hum_rollout_fused"):
        pol.rollout(env, 4, fused=True)
    env.close()
    pol.close()


def test_sample_batch_columns_match_torch_fp32():
    """The SampleBatch columns RLlib's sampler records (action_dist_inputs, action_logp, vf_preds) for a fused
    rollout's recorded inputs and samples: the value branch and the policy mean against plain PyTorch fp32, the
    log-density against torch.distributions.Normal summed over the action dimensions."""
    n, k = 512, 8
    pol = DevicePolicy.random_init(seed=9)
    vpol = DevicePolicy.random_init_value(seed=12)
    vpol.w["b3"][:] = 0.3
    vpol.close()
    vpol = DevicePolicy(vpol.w, n_out=1)
    env = HumanoidVecEnv(n, clips=("motion02_04",), seed=2)
    env.reset()
    tr = pol.rollout(env, k, explore=True, step0=3, fused=True)
    cols = pol.sample_batch_columns(tr["obs"], tr["actions"], value=vpol)
    obs = tr["obs"].reshape(-1, 70)
    mean = reference_mean(pol.w, obs)
    vf = reference_mean(vpol.w, obs)[:, 0]
    std = torch.exp(torch.as_tensor(pol.w["log_std"], device="cuda"))
    logp = torch.distributions.Normal(mean, std).log_prob(tr["actions"].reshape(-1, 17)).sum(-1)
    assert cols["action_dist_inputs"].shape == (k, n, 34) and cols["vf_preds"].shape == (k, n)
    torch.testing.assert_close(cols["action_dist_inputs"].reshape(-1, 34)[:, :17], mean, atol=2e-5, rtol=0)
    torch.testing.assert_close(cols["action_dist_inputs"].reshape(-1, 34)[:, 17:], torch.log(std).expand(len(obs), 17))
    torch.testing.assert_close(cols["vf_preds"].reshape(-1), vf, atol=2e-5, rtol=0)
    # action_logp: (1) against the same log-density evaluated in float64 from the columns' OWN mean - the fp32
    # rounding of a 17-term sum of terms up to |t| (17 x 2^-24 x max |t| per row, plus the float32 output); (2) against
    # torch's from the torch mean, within what the mean's own 2e-5 difference moves it: sum_k |z_k| / std_k x 2e-5
    lp = cols["action_logp"].reshape(-1).double()
    a64 = tr["actions"].reshape(-1, 17).double()
    m64 = cols["action_dist_inputs"].reshape(-1, 34)[:, :17].double()
    s64 = std.double()
    terms = -0.5 * ((a64 - m64) / s64) ** 2 - torch.log(s64) - 0.5 * np.log(2 * np.pi)
    own = terms.sum(-1)
    tol_own = 17 * 2.0 ** -24 * terms.abs().max(-1).values + 2.0 ** -24 * own.abs() + 1e-6
    assert ((lp - own).abs() <= tol_own).all(), float(((lp - own).abs() - tol_own).max())
    dz = ((a64 - mean.double()) / s64 ** 2).abs().sum(-1)   # |d logp / d mean| summed over the 17 dimensions
    tol_mean = 2e-5 * dz + 17 * 2.0 ** -24 * terms.abs().max(-1).values + tol_own
    assert ((lp - logp.double()).abs() <= tol_mean).all(), float(((lp - logp.double()).abs() - tol_mean).max())
    env.close()
    pol.close()
    vpol.close()


def test_value_branch_from_rllib_weight_names():
    rng = np.random.default_rng(0)
    names = {"default_policy/fc_value_1/kernel": (70, 256), "default_policy/fc_value_1/bias": (256,),
             "default_policy/fc_value_2/kernel": (256, 256), "default_policy/fc_value_2/bias": (256,),
             "default_policy/value_out/kernel": (256, 1), "default_policy/value_out/bias": (1,),
             "default_policy/fc_1/kernel": (70, 256)}
    w = {k: rng.standard_normal(s).astype(np.float32) * 0.05 for k, s in names.items()}
    v = DevicePolicy.value_from_rllib_weights(w)
    assert v.n_out == 1 and np.array_equal(v.w["w3"], w["default_policy/value_out/kernel"])
    obs = torch.randn(64, 70, device="cuda")
    got = torch.empty(64, 1, device="cuda")
    v.act(obs, mean_out=got)
    ref = reference_mean(v.w, obs)
    assert (got - ref).abs().max().item() < 2e-5
    v.close()


def test_rllib_weight_names():
    """from_rllib_weights picks the policy branch of an RLlib 1.2 TF FullyConnectedNetwork weight dict."""
    rng = np.random.default_rng(0)
    d = {"default_policy/fc_1/kernel": rng.standard_normal((70, 256)), "default_policy/fc_1/bias": np.zeros(256),
         "default_policy/fc_2/kernel": rng.standard_normal((256, 256)), "default_policy/fc_2/bias": np.zeros(256),
         "default_policy/fc_out/kernel": rng.standard_normal((256, 17)), "default_policy/fc_out/bias": np.zeros(17),
         "default_policy/log_std": np.zeros(17), "default_policy/fc_value_1/kernel": np.zeros((70, 256)),
         "default_policy/value_out/kernel": np.zeros((256, 1))}
    pol = DevicePolicy.from_rllib_weights(d)
    np.testing.assert_array_equal(pol.w["w2"], d["default_policy/fc_2/kernel"].astype(np.float32))
    pol.close()

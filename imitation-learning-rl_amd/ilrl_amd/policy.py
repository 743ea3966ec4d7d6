"""On-GPU policy inference and device-resident sampler loops over the C-ABI
(include/humanoid_env.h: hum_policy_create_ex / hum_policy_act / hum_rollout / hum_rollout_fused /
hum_hier_rollout).

The network is the reference's PPO policy (train_config.py:107-111: RLlib 1.2 FullyConnectedNetwork,
fcnet_hiddens [256, 256], fcnet_activation tanh, free_log_std True): action mean =
W3 tanh(W2 tanh(W1 obs + b1) + b2) + b3, sampled as DiagGaussian(mean, exp(log_std)) and clipped to the
action Box (RLlib clip_actions).  Weights come from `from_rllib_weights` (the dict a TF policy's
get_weights() returns, exported where Ray runs) or `random_init` (RLlib's normc initialisers; benchmarks).
Two shapes: the low-level policy 70 -> 17 and the hierarchical env's high-level policy 44 -> 2 (train_config.py:
23-27, 262-298), which `hier_rollout` drives together on a HierVecEnv (BASELINE config 5).
The reference's trained checkpoints are pickles that the safe loaders refuse, so no
trained weights ship here.
"""
import ctypes

import numpy as np

from . import _native as N

H = 256


def _fp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _normc(rng, shape, std):
    """RLlib's normc_initializer: normal columns scaled to norm `std`."""
    w = rng.standard_normal(shape).astype(np.float32)
    return (w * std / np.sqrt(np.square(w).sum(axis=0, keepdims=True))).astype(np.float32)


class DevicePolicy:
    """The policy network on one GPU (weights fp32, TF kernel layout [in][out]); n_in -> n_out = 70 -> 17 (the
    low-level policy) or 44 -> 2 (the high-level one)."""

    KEYS = ("w1", "b1", "w2", "b2", "w3", "b3", "log_std")

    def __init__(self, weights, device=0, seed=0, n_in=N.HUM_NOBS, n_out=N.HUM_NACT):
        import torch
        self.torch = torch
        self.device = torch.device("cuda", device)
        self.n_in, self.n_out = n_in, n_out
        shapes = {"w1": (n_in, H), "b1": (H,), "w2": (H, H), "b2": (H,), "w3": (H, n_out),
                  "b3": (n_out,), "log_std": (n_out,)}
        self.w = {}
        for k in self.KEYS:
            a = np.ascontiguousarray(weights.get(k, np.zeros(shapes[k])), dtype=np.float32)
            if a.shape != shapes[k]:
                raise ValueError("%s: shape %s, expected %s" % (k, a.shape, shapes[k]))
            self.w[k] = a
        h = ctypes.c_void_p()
        L = N.lib()
        if callable(L.hum_policy_create_ex):
            N.check(L.hum_policy_create_ex(device, n_in, n_out, *[_fp(self.w[k]) for k in self.KEYS],
                                           ctypes.c_uint64(seed), ctypes.byref(h)), "hum_policy_create")
        else:   # ILRL_AMD_AB: a library older than ABI 10 has only the (70, 17) entry point
            if (n_in, n_out) != (N.HUM_NOBS, N.HUM_NACT):
                raise N.NativeError("hum_policy_create_ex missing from %s" % N.LIB_PATH)
            N.check(L.hum_policy_create(device, *[_fp(self.w[k]) for k in self.KEYS], ctypes.c_uint64(seed),
                                        ctypes.byref(h)), "hum_policy_create")
        self.h = h

    @classmethod
    def random_init(cls, seed=0, device=0, log_std=-0.5, n_in=N.HUM_NOBS, n_out=N.HUM_NACT):
        rng = np.random.default_rng(seed)
        w = {"w1": _normc(rng, (n_in, H), 1.0), "b1": np.zeros(H), "w2": _normc(rng, (H, H), 1.0),
             "b2": np.zeros(H), "w3": _normc(rng, (H, n_out), 0.01), "b3": np.zeros(n_out),
             "log_std": np.full(n_out, log_std)}
        return cls(w, device=device, seed=seed, n_in=n_in, n_out=n_out)

    @classmethod
    def random_init_high(cls, seed=0, device=0, log_std=-0.5):
        """The hierarchical env's high-level policy shape (44 -> 2)."""
        return cls.random_init(seed=seed, device=device, log_std=log_std, n_in=N.HUM_NOBS_HIGH, n_out=N.HUM_NACT_HIGH)

    @classmethod
    def from_rllib_weights(cls, weights, device=0, seed=0, n_in=N.HUM_NOBS, n_out=N.HUM_NACT):
        """From a TF FullyConnectedNetwork's get_weights() dict (variable name -> array): the policy branch
        fc_1, fc_2, fc_out and the free log_std variable (value-branch variables are ignored).  The name mapping
        follows RLlib 1.2's naming; it is not exercised against a real checkpoint here (no Ray in this image)."""
        def pick(sub):
            hits = [k for k in weights if sub in k and "value" not in k]
            if len(hits) != 1:
                raise KeyError("expected exactly one variable matching %r, got %s" % (sub, hits))
            return np.asarray(weights[hits[0]])
        w = {"w1": pick("fc_1/kernel"), "b1": pick("fc_1/bias"), "w2": pick("fc_2/kernel"), "b2": pick("fc_2/bias"),
             "w3": pick("fc_out/kernel"), "b3": pick("fc_out/bias"), "log_std": pick("log_std")}
        w["log_std"] = w["log_std"].reshape(-1)
        return cls(w, device=device, seed=seed, n_in=n_in, n_out=n_out)

    @classmethod
    def value_from_rllib_weights(cls, weights, device=0, n_in=N.HUM_NOBS):
        """The value branch of the same TF FullyConnectedNetwork (RLlib 1.2 PPO: vf_share_layers False, so
        fc_value_1 -> fc_value_2 -> value_out, tanh, the same hidden sizes) as a 1-output network: act(...,
        mean_out=v) gives the value predictions (SampleBatch VF_PREDS).  Name mapping as from_rllib_weights."""
        def pick(sub):
            hits = [k for k in weights if sub in k]
            if len(hits) != 1:
                raise KeyError("expected exactly one variable matching %r, got %s" % (sub, hits))
            return np.asarray(weights[hits[0]])
        w = {"w1": pick("fc_value_1/kernel"), "b1": pick("fc_value_1/bias"), "w2": pick("fc_value_2/kernel"),
             "b2": pick("fc_value_2/bias"), "w3": pick("value_out/kernel"), "b3": pick("value_out/bias")}
        return cls(w, device=device, n_in=n_in, n_out=1)

    @classmethod
    def random_init_value(cls, seed=0, device=0, n_in=N.HUM_NOBS):
        """A value branch with RLlib's initialisers (normc 1.0 hidden, 0.01 output), for benchmarks and tests."""
        rng = np.random.default_rng(seed)
        w = {"w1": _normc(rng, (n_in, H), 1.0), "b1": np.zeros(H), "w2": _normc(rng, (H, H), 1.0), "b2": np.zeros(H),
             "w3": _normc(rng, (H, 1), 0.01), "b3": np.zeros(1)}
        return cls(w, device=device, seed=seed, n_in=n_in, n_out=1)

    def sample_batch_columns(self, obs, actions, value=None, out=None, mean=None, valid=None):
        """The policy-side SampleBatch columns RLlib's sampler records per step, for recorded policy inputs obs
        [..., n_in] and raw samples actions [..., n_out] (device; e.g. a rollout's trajectory, any leading shape):
        action_dist_inputs [..., 2 n_out] (the DiagGaussian's mean and log_std), action_logp [...] (log-density of
        the raw sample) and, given the value branch `value` (a 1-output DevicePolicy), vf_preds [...].  One
        policy launch (and one value launch) over all rows: within a fragment the weights are fixed, so this equals
        what the per-step compute_actions records.  out: a dict of the same tensors to write into.  mean: the policy
        means of these rows when the rollout already recorded them (rollout / hier_rollout with means=True: bitwise
        what the policy launch would give), so no policy launch runs.
        valid: a bool mask of the leading shape marking the rows that hold a real transition.  A fused hierarchical
        rollout (hier_rollout(fused=True)) leaves the non-acting agent's obs / act / mean rows unwritten, so their
        columns would be computed from stale or uninitialised memory: pass valid = (acted & HUM_AGENT_x) != 0 there;
        the invalid rows' columns are written as zeros."""
        t = self.torch
        lead = tuple(obs.shape[:-1])
        R = int(np.prod(lead)) if lead else 1
        o2 = obs.reshape(R, self.n_in)
        out = out if out is not None else {}
        if mean is None:
            mean = t.empty(R, self.n_out, dtype=t.float32, device=self.device)
            scratch = t.empty(R, self.n_out, dtype=t.float32, device=self.device)   # the clipped actions (unused)
            self.act(o2, explore=False, out=scratch, mean_out=mean)
        else:
            mean = mean.reshape(R, self.n_out)
        if getattr(self, "_log_std_dev", None) is None:   # uploaded once (no host copy per call)
            self._log_std_dev = t.as_tensor(self.w["log_std"], device=self.device)
        log_std = self._log_std_dev
        adi = out.get("action_dist_inputs")
        if adi is None:
            adi = t.empty(lead + (2 * self.n_out,), dtype=t.float32, device=self.device)
        adi.view(R, 2 * self.n_out)[:, :self.n_out].copy_(mean)
        adi.view(R, 2 * self.n_out)[:, self.n_out:].copy_(log_std.expand(R, self.n_out))
        # DiagGaussian.logp (RLlib): -0.5 sum(((x - mean) / std)^2) - 0.5 log(2 pi) n_out - sum(log_std)
        z = (actions.reshape(R, self.n_out) - mean) * t.exp(-log_std)
        logp = -0.5 * (z * z).sum(-1) - 0.5 * np.log(2.0 * np.pi) * self.n_out - log_std.sum()
        lp = out.get("action_logp")
        if lp is None:
            lp = t.empty(lead, dtype=t.float32, device=self.device)
        vm = None
        if valid is not None:
            vm = valid.reshape(R).to(t.bool)
            logp = t.where(vm, logp, t.zeros((), dtype=logp.dtype, device=logp.device))
            adi.view(R, 2 * self.n_out).masked_fill_(~vm[:, None], 0.0)
        lp.view(R).copy_(logp)
        res = {"action_dist_inputs": adi, "action_logp": lp}
        if value is not None:
            if value.n_in != self.n_in or value.n_out != 1:
                raise ValueError("sample_batch_columns: the value branch must map n_in -> 1")
            vf = out.get("vf_preds")
            if vf is None:
                vf = t.empty(lead, dtype=t.float32, device=self.device)
            value.act(o2, explore=False, out=t.empty(R, 1, dtype=t.float32, device=self.device), mean_out=vf.view(R, 1))
            if vm is not None:
                vf.view(R).masked_fill_(~vm, 0.0)
            res["vf_preds"] = vf
        return res

    def close(self):
        if getattr(self, "h", None):
            N.lib().hum_policy_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def act(self, obs, obs_reset=None, done=None, explore=False, step=0, out=None, mean_out=None, raw_out=None):
        """actions [n,n_out] (device, clipped to the Box) for device observations obs [n,n_in] (done lanes read
        obs_reset); raw_out receives the samples before clip_actions (RLlib's SampleBatch actions)."""
        t = self.torch
        n = obs.shape[0]
        if obs.shape[1] != self.n_in:
            raise ValueError("obs must be [n, %d], got %s" % (self.n_in, tuple(obs.shape)))
        act = out if out is not None else t.empty(n, self.n_out, dtype=t.float32, device=self.device)
        p = lambda x: ctypes.c_void_p(x.data_ptr()) if x is not None else None
        N.check(N.lib().hum_policy_act_ex(self.h, p(obs), p(obs_reset), p(done), n, p(act), p(mean_out), None,
                                          p(raw_out), int(bool(explore)), ctypes.c_uint64(step), self._stream()),
                "hum_policy_act")
        return act

    def rollout(self, venv, k, explore=True, step0=0, trajectories=True, fused=False, out=None, means=False):
        """k sampler steps (policy -> env step with auto-reset) on venv's lanes, all on the device with no host
        round trip.  venv.obs must hold the current observation (after venv.reset()).  Returns the trajectory
        tensors {obs [k,n,70] (policy inputs), actions [k,n,17] (the samples before clip_actions, as RLlib records
        them), rewards [k,n], dones [k,n]} (or {}).  fused: one launch with the policy inside the step kernel
        (hum_rollout_fused; cooperative fp32 handles with 4 envs per block on the plane).  out: a dict of the same
        tensors to write into (reused across calls, e.g. by a timed loop) instead of fresh ones.  means (fused only):
        also means [k,n,17], the policy's mean per step as the in-kernel network forms it (hum_rollout_fused_ex), for
        sample_batch_columns(..., mean=...)."""
        t = self.torch
        n = venv.n
        if means and not (fused and trajectories):
            raise ValueError("rollout: means=True needs fused=True and trajectories=True")
        if not hasattr(venv, "_act_buf"):
            venv._act_buf = t.zeros(n, N.HUM_NACT, dtype=t.float32, device=venv.device)
        tr = {}
        if trajectories:
            shapes = {"obs": ((N.HUM_NOBS,), t.float32), "actions": ((N.HUM_NACT,), t.float32),
                      "rewards": ((), t.float32), "dones": ((), t.uint8)}
            if means:
                shapes["means"] = ((N.HUM_NACT,), t.float32)
            for f, (sh, dt) in shapes.items():
                x = out.get(f) if out else None
                if x is None:
                    x = t.empty((k, n) + sh, dtype=dt, device=venv.device)
                elif tuple(x.shape) != (k, n) + sh or x.dtype != dt or x.device != venv.device or not x.is_contiguous():
                    raise ValueError("rollout: out[%r] must be a contiguous %s tensor of shape %s on %s"
                                     % (f, dt, (k, n) + sh, venv.device))
                tr[f] = x
        p = lambda x: ctypes.c_void_p(x.data_ptr()) if x is not None else None
        args = (venv.h, self.h, k, int(bool(explore)), ctypes.c_uint64(step0), p(venv.obs), p(venv.obs_reset),
                p(venv.done), p(venv.reward), p(venv._act_buf), p(tr.get("obs")), p(tr.get("actions")),
                p(tr.get("rewards")), p(tr.get("dones")))
        if means:
            N.check(N.lib().hum_rollout_fused_ex(*args, p(tr["means"]), venv._stream()), "hum_rollout_fused_ex")
        else:
            fn = N.lib().hum_rollout_fused if fused else N.lib().hum_rollout
            N.check(fn(*args, venv._stream()), "hum_rollout_fused" if fused else "hum_rollout")
        return tr


def _hier_traj_shapes():
    import torch as t
    f32, u8 = t.float32, t.uint8
    return {"acted": ((), u8), "obs_high": ((N.HUM_NOBS_HIGH,), f32), "act_high": ((N.HUM_NACT_HIGH,), f32),
            "obs_low": ((N.HUM_NOBS,), f32), "act_low": ((N.HUM_NACT,), f32), "agents": ((), u8),
            "rew_high": ((), f32), "rew_low": ((), f32), "done": ((), u8)}


def hier_traj_buffers(n, k, device, means=False):
    """Fresh trajectory tensors for hier_rollout(..., out=..., means=means) of k transitions on n lanes."""
    import torch as t
    out = {f: t.empty((k, n) + sh, dtype=dt, device=device) for f, (sh, dt) in _hier_traj_shapes().items()}
    if means:
        out["mean_high"] = t.empty(k, n, N.HUM_NACT_HIGH, dtype=t.float32, device=device)
        out["mean_low"] = t.empty(k, n, N.HUM_NACT, dtype=t.float32, device=device)
    return out


def hier_rollout(venv, high, low, k, explore=True, step0=0, trajectories=True, fused=False, out=None, means=False):
    """k transitions of the two-level env venv (a HierVecEnv after reset()) with the high-level policy `high`
    (44 -> 2) and the low-level policy `low` (70 -> 17), all on the device (hum_hier_rollout): per transition each
    lane steps with the action of the agent it expects.  venv's buffers carry the state between calls (obs_high /
    obs_high_reset / obs / done / agents / rewards).  Returns the trajectory {acted [k,n] (HUM_AGENT_HIGH / _LOW),
    obs_high [k,n,44], act_high [k,n,2], obs_low [k,n,70], act_low [k,n,17] (raw samples), agents [k,n],
    rew_high [k,n], rew_low [k,n], done [k,n]} (or {}).
    fused: one launch with both networks inside the env kernel (hum_hier_rollout_fused; the obs / act rows of the
    agent that did not act on a lane are left unwritten).  out: a dict of the same tensors to write into (reused
    across calls, e.g. by a timed loop) instead of fresh ones.  means (fused only): also mean_high [k,n,2] and
    mean_low [k,n,17], the acting agent's policy mean per transition (hum_hier_rollout_fused_ex; the other agent's
    rows unwritten), for sample_batch_columns(..., mean=...)."""
    import torch as t
    n, dev = venv.n, venv.device
    if means and not (fused and trajectories):
        raise ValueError("hier_rollout: means=True needs fused=True and trajectories=True")
    if not hasattr(venv, "_act_high_buf"):
        venv._act_high_buf = t.zeros(n, N.HUM_NACT_HIGH, dtype=t.float32, device=dev)
        venv._act_low_buf = t.zeros(n, N.HUM_NACT, dtype=t.float32, device=dev)
    tr = {}
    if trajectories:
        shapes = dict(_hier_traj_shapes())
        if means:
            shapes["mean_high"] = ((N.HUM_NACT_HIGH,), t.float32)
            shapes["mean_low"] = ((N.HUM_NACT,), t.float32)
        for f, (sh, dt) in shapes.items():
            x = out.get(f) if out else None
            if x is None:
                x = t.empty((k, n) + sh, dtype=dt, device=dev)
            elif tuple(x.shape) != (k, n) + sh or x.dtype != dt or x.device != dev or not x.is_contiguous():
                raise ValueError("hier_rollout: out[%r] must be a contiguous %s tensor of shape %s on %s"
                                 % (f, dt, (k, n) + sh, dev))
            tr[f] = x
    p = lambda x: x.data_ptr() if x is not None else None
    io = N.HumHierIO(p(venv.obs_high), p(venv.obs_high_reset), p(venv.obs), p(venv.done), p(venv.agents),
                     p(venv.reward_high), p(venv.reward), p(venv._act_high_buf), p(venv._act_low_buf))
    traj = N.HumHierTraj(*[p(tr.get(f)) for f, _ in N.HumHierTraj._fields_]) if trajectories else None
    args = (venv.h, high.h, low.h, k, int(bool(explore)), ctypes.c_uint64(step0), ctypes.byref(io),
            ctypes.byref(traj) if traj is not None else None)
    if means:
        N.check(N.lib().hum_hier_rollout_fused_ex(*args, p(tr["mean_high"]), p(tr["mean_low"]), venv._stream()),
                "hum_hier_rollout_fused_ex")
    else:
        fn = "hum_hier_rollout_fused" if fused else "hum_hier_rollout"
        N.check(getattr(N.lib(), fn)(*args, venv._stream()), fn)
    return tr


def reference_mean(w, obs):
    """The same network in plain PyTorch fp32 (tests' reference): the action mean."""
    import torch
    T = lambda k: torch.as_tensor(w[k], dtype=torch.float32, device=obs.device)
    h1 = torch.tanh(obs @ T("w1") + T("b1"))
    h2 = torch.tanh(h1 @ T("w2") + T("b2"))
    return h2 @ T("w3") + T("b3")

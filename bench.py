#!/usr/bin/env python3
"""Benchmark: env steps/s of the HIP humanoid imitation env (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4096 lanes per GPU, low-level imitation on motion02_04, uniform
random actions in [-1,1] (pre-generated pool, device resident, a fresh [n,17] action row for every env
step), auto-reset of done lanes inside the launch.  A "step" = one env step of every lane (4 physics substeps +
observation + imitation reward + bookkeeping); `--k K` env steps run per hum_step_k launch (outputs written
per step, [K, n, ...]), and every rate below is per env-step.  Multi-GPU: one process per GPU, lanes sharded
by rank (global lane ids -> identical per-lane streams regardless of N), no data-path collective -> weak
scaling; the trajectory gather (`--gather-every G`, default k when WORLD_SIZE > 1: the last G steps' obs / action /
reward / done rows of every rank gathered to rank 0 every G env steps, the only collective the path has)
runs asynchronously beside the next launches and is completed inside the timed region.

Prints ONE JSON line on rank 0.  Every number in it is measured in this run except `roofline.traffic`
(PMC bytes, profiles/pmc_traffic.json, from a rocprofv3 --pmc pass of this same command) and the static FLOP
count per env-step (profiles/r06_flops_per_env_step.json, tools/flop_count.py).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))

# algorithmic HBM bytes per env-step: action 17 x f32 read; physics state 47 x f32 read + write;
# bookkeeping 24 words x 4 B read + write; obs 70 x f32, reward f32, frame i32, done u8 written = 925 B.
BYTES_PER_STEP_ALGO = 17 * 4 + 2 * 47 * 4 + 2 * 24 * 4 + 70 * 4 + 4 + 4 + 1
# the kernel's actual layout per env-step: bookkeeping 23 f64 + 8 i32 instead of 24 words
BYTES_PER_STEP_LAYOUT = 2 * 47 * 4 + 2 * (23 * 8 + 8 * 4) + 17 * 4 + 70 * 4 + 4 + 1 + 4
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3       # MI355X FP32 vector (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector
K_DEFAULT = 32                 # env steps per launch (hum_step_k), DESIGN.md section 5 (k sweep)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--lanes", type=int, default=4096, help="env lanes per GPU")
    ap.add_argument("--clip", default="motion02_04", help="clip name, or 'all' = the four CMU clips round-robin per "
                                                          "lane (BASELINE config 3)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--block", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="CPU baseline threads (0 = the job's host cores)")
    ap.add_argument("--phys", action="append", default=[], help="physics override k=v (hum_config field), diagnostics")
    ap.add_argument("--hier", action="store_true",
                    help="config 5: HierarchicalHumanoidEnv two-level rollout (hum_hier_step), clip motion09_03")
    ap.add_argument("--gather-every", type=int, default=None,
                    help="trajectory gather to rank 0 of the last G env steps every G env steps (G %% k == 0); default "
                         "k when WORLD_SIZE > 1 (the learner's trajectory feed, SURVEY 8(e)), 0 = none")
    ap.add_argument("--k", type=int, default=K_DEFAULT, help="env steps per launch (hum_step_k)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise torch.distributed and run every collective (barriers, the timing all-reduce, the "
                         "gather) even with one rank: the RCCL code path on a one-GPU box, where RCCL refuses two ranks "
                         "on one device")
    ap.add_argument("--transport", default="dma", choices=["dma", "collective"],
                    help="the trajectory gather's transport for N > 1: dma = rank 0 pulls every launch's rows of "
                         "every rank's packed fragment with the SDMA copy engines over IPC-mapped buffers "
                         "(parallel.DmaGather: no compute unit, so it overlaps the next launch; the run ends on a short "
                         "drain launch, launch_plan); collective = one dist.gather per fragment (RCCL kernels, which "
                         "wait for the env launch to leave the CUs)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo: host-staged, tests)")
    ap.add_argument("--dump-gather", default=None,
                    help="rank 0: save every gathered trajectory fragment to this .npz (tests)")
    ap.add_argument("--dump-lane-stride", type=int, default=1,
                    help="with --dump-gather: keep every S-th global lane only (bounds host memory at 32768 lanes)")
    ap.add_argument("--policy", action="store_true",
                    help="closed loop: actions from the on-GPU policy network (random-init weights, exploration "
                         "noise) inside the timed loop, SURVEY 8(f) rank 2")
    ap.add_argument("--fused", action="store_true",
                    help="with --policy: one hum_rollout_fused launch per --k steps (the policy inside the env kernel) "
                         "instead of a policy launch + an env launch per step")
    ap.add_argument("--sample-batch", action="store_true",
                    help="with --fused --policy (or --hier --policy): after every rollout launch also form the policy "
                         "columns RLlib's sampler records - action_dist_inputs, action_logp and vf_preds from a "
                         "value branch of the same shape (random-init) - over the launch's rows")
    ap.add_argument("--no-secondary", action="store_true", help="skip the fp64 / parity side measurements")
    ap.add_argument("--terrain", default="plane", choices=["plane", "random"],
                    help="ground: the stadium plane (the reference's default scene) or LowLevelHumanoidEnv(useCustomEnv="
                         "True)'s CustomScene random block terrain, a new one per lane at every reset (humanoid.py:68-144; "
                         "its own kernel instantiation, heightfield contacts incl. capsule ridges)")
    ap.add_argument("--adapter", action="store_true",
                    help="time the RLlib drop-in path instead of the raw C-ABI launches: HumanoidVectorEnv.vector_step + "
                         "reset_at per done lane (RLlib 1.2 VectorEnv), or with --hier HierarchicalVectorEnv.poll / "
                         "send_actions / try_reset (BaseEnv); host-side numpy actions as RLlib hands them over, one launch "
                         "per sampler step (k = 1)")
    return ap.parse_args()


def host_cores():
    """Host cores this job may use: the box's CPU share (OMP_NUM_THREADS / MAX_JOBS are set to it on the GPU
    box; os.cpu_count() there reports the whole machine), else the affinity mask."""
    for k in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def cpu_baseline(seconds, threads):
    """CPU baseline (PyBullet absent -> the build's C restatement with OpenMP over the job's host
    cores): oracle/env_oracle.c (fp64 physics restatement + the env logic, bit-identical to the Python oracle) with
    one lane per thread stepping uniform random actions, reset on done."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import env_oracle as EO
    from ilrl_amd.clips import load_clip
    steps, wall = EO.bench(load_clip("motion02_04"), threads, seconds)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "oracle/env_oracle.c (fp64 C restatement of physics + env logic, OpenMP; PyBullet absent) on "
                      "motion02_04, %d threads (the job's host cores) x %.0f s of uniform-random-action steps with "
                      "resets (%d steps)" % (threads, seconds, steps)}


def parity_sample(env, clips, per_clip=64, seed=5, sens_bound=1e-5):
    """CPU checker leg (after the timed region): from the benchmark's own mid-rollout state, step once more on the
    GPU (no auto-reset) with the benchmarked fp32 kernel AND with the fp64 kernel given the identical state, and
    compare a sample of lanes per clip with the fp64 oracle stepped from the same injected state (fp64 C physics +
    the env logic).  Each lane's conditioning is measured too: the oracle stepped again from the state perturbed by
    2^-24 relative (float32 rounding) - a joint limit or contact that switches on within that margin makes the step
    discontinuous, and such lanes are reported apart (the error there is the model's, not the kernel's)."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from ilrl_amd import _native as N
    from ilrl_amd.clips import load_clip
    from ilrl_amd.vec_env import HumanoidVecEnv
    phys, book = env.get_state()
    n = env.n
    a = np.random.default_rng(seed).uniform(-1, 1, (n, 17)).astype(np.float32)
    at = torch.as_tensor(a, device=env.device)
    obs, rew, done, frame = [x.cpu().numpy() for x in env.step(at)]
    # the fp64 kernel from the same state with the base quaternion renormalised in float64 (an fp32 state's is unit
    # only to float32 rounding, which the kernel's and the oracle's formulations of R^-1 treat differently; see
    # tests/test_gpu_scale.py::unit_quat), compared with the oracle from that same renormalised state
    physn = phys.copy()
    physn[:, 3:7] /= np.linalg.norm(physn[:, 3:7], axis=1, keepdims=True)
    env64 = HumanoidVecEnv(n, clips=clips, seed=0, device=env.device.index, precision="fp64")
    env64.set_state(physn, book)
    obs64, rew64, done64, _ = [x.cpu().numpy() for x in env64.step(at)]
    st64, _ = env64.get_state()
    env64.close()
    prng = np.random.default_rng(seed + 1)
    eo, er, e64, r64, s64, sens, dm, fm, dm64, lanes = [], [], [], [], [], [], 0, 0, 0, 0
    for c, name in enumerate(clips):
        idx = np.nonzero(book[:, N.BK["clip"]].astype(int) == c)[0]
        if name == "motion13_13":   # the reference raises IndexError past the 120-row velocity table
            idx = idx[book[idx, N.BK["frame"]] + 2 < 120]
        clip = load_clip(name)
        for i in idx[np.linspace(0, len(idx) - 1, min(per_clip, len(idx))).astype(int)]:
            o = O.OracleLowLevelEnv.from_lane(clip, phys[i], book[i], N.BK)
            ro, rr, rd, _ = o.step(a[i])
            eo.append(float(np.abs(obs[i] - ro).max()))
            er.append(abs(float(rew[i]) - rr))
            o64 = O.OracleLowLevelEnv.from_lane(clip, physn[i], book[i], N.BK)
            ro64, rr64, rd64, _ = o64.step(a[i])
            e64.append(float(np.abs(obs64[i] - ro64).max()))
            r64.append(abs(float(rew64[i]) - rr64))
            s64.append(float(np.abs(st64[i] - o64.state).max()))
            dm += int(bool(done[i]) != rd)
            dm64 += int(bool(done64[i]) != rd64)
            fm += int(int(frame[i]) != o.frame)
            p = O.OracleLowLevelEnv.from_lane(clip, phys[i] * (1 + 2.0 ** -24 * prng.choice([-1.0, 1.0], 47)), book[i],
                                              N.BK)
            sens.append(float(np.abs(p.step(a[i])[0] - ro).max()))
            lanes += 1
    eo, er, sens = np.array(eo), np.array(er), np.array(sens)
    good = sens <= sens_bound
    return {"vs": "fp64 CPU oracle, one env step from the benchmark's own mid-rollout lane states (PyBullet absent: "
                  "parity vs PyBullet unpinned)", "lanes": lanes,
            "obs_max_abs_err": float(eo.max()), "obs_p99_abs_err": float(np.percentile(eo, 99)),
            "reward_max_abs_err": float(er.max()), "done_mismatches": dm, "frame_mismatches": fm,
            "ill_conditioned_lanes": int((~good).sum()),
            "obs_max_abs_err_conditioned": float(eo[good].max()) if good.any() else None,
            "reward_max_abs_err_conditioned": float(er[good].max()) if good.any() else None,
            "conditioning": "oracle obs change under a 2^-24 relative input perturbation > %g" % sens_bound,
            "fp64_kernel": {"from": "the same states, base quaternion renormalised in float64", "obs_max_abs_err": float(max(e64)), "reward_max_abs_err": float(max(r64)),
                            "state_max_abs_err": float(max(s64)), "done_mismatches": dm64}}


def _actions_desc(a):
    if a.hier and a.policy:
        return ("on-GPU policies of both levels in the loop (random-init 44-256-256-2 high-level and 70-256-256-17 "
                "low-level tanh MLPs + Gaussian exploration, %s)" % ("hum_hier_rollout_fused" if a.fused
                                                                      else "hum_hier_rollout"))
    if a.policy:
        return "on-GPU policy actions (random-init 70-256-256-17 tanh MLP + Gaussian exploration) in the loop"
    return "uniform random actions (a fresh row per env step)"


def _load_json(path):
    try:
        return json.load(open(os.path.join(REPO, path)))
    except Exception:
        return None


def _pools(a, dev, n, k, rank):
    """16 device-resident action blocks [k, n, 17] (and [k, n, 2] high-level headings for --hier), a fresh row per
    env step; launch s reads block s % 16."""
    import torch
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [(torch.rand(k, n, 17, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
    hpool = [(torch.rand(k, n, 2, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)] if a.hier else None
    return pool, hpool


def launch_sizes(steps, k):
    """Env steps per launch: whole launches of k, then one shorter launch for the remainder, so that exactly `steps`
    env steps run (the driver's --steps need not be a multiple of k)."""
    return [k] * (steps // k) + ([steps % k] if steps % k else [])


def launch_plan(steps, k, drain=False):
    """The timed launches as (action block, first row in it, env steps): launch_sizes' launches, block b of the
    device-resident action pool for launch b.  drain (the chunked copy-engine gather): the last launch's final fifth
    is split off into its own launch - same action rows, same trajectory bit for bit - so that what the gather still
    moves after the last launch ends is that short launch's rows, while the rest of the last launch's rows travel
    during it (a chunk's pull takes ~a fifth of the launch time that produced it)."""
    plan = [(b, 0, kk) for b, kk in enumerate(launch_sizes(steps, k))]
    if drain and plan and plan[-1][2] >= 2:
        b, _, kk = plan.pop()
        d = max(1, round(kk / 5))
        plan += [(b, 0, kk - d), (b, kk - d, d)]
    return plan


def run(a, world, rank, dev, n, precision, steps, warmup, phys, k=None):
    """Build the env, warm up, time `steps` env steps in launches of k.  Returns (env, wall_max_s, kernel_ms per
    env step, low_steps, gather_s, gathered, the timed launches' sizes)."""
    import torch
    import torch.distributed as dist
    k = k or a.k
    plan, wsizes = launch_plan(steps, k), launch_sizes(warmup, k)
    sizes = [p[2] for p in plan]
    launches, wlaunches = len(sizes), len(wsizes)
    pool, hpool = _pools(a, dev, n, k, rank)
    G = a.gather_every if a.dist and not a.policy else 0
    if G and G % k:
        raise SystemExit("--gather-every must be a multiple of --k")
    soff = [0]   # --policy: launches before the timed ones (the timed launch s is launch soff + s of the run)
    ring = [None]   # the launch's output buffers (packed into the gather fragment right after the launch)
    rem_out = {}   # output buffers of the shorter remainder launches, by size
    if a.hier:
        from ilrl_amd.hier_env import HierVecEnv
        env = HierVecEnv(n, seed=0, device=dev.index, lane_offset=rank * n, precision=precision, block_size=a.block,
                         **phys)

        def step(s, kk=k, o=0):
            j = s % len(ring)
            if kk < k:   # the remainder launch (or the drain launches: rows o .. o + kk of block s)
                return env.step_k(hpool[s % 16][o:o + kk], pool[s % 16][o:o + kk], autoreset=True,
                                  out=rem_out.get(kk))
            ring[j] = env.step_k(hpool[s % 16], pool[s % 16], autoreset=True, out=ring[j])
        if a.policy:   # config 5 closed loop: both levels' policies on the device (hum_hier_rollout[_fused])
            from ilrl_amd.policy import DevicePolicy, hier_rollout, hier_traj_buffers
            from ilrl_amd import _native as N
            high = DevicePolicy.random_init_high(seed=17 + rank, device=dev.index)
            low = DevicePolicy.random_init(seed=7 + rank, device=dev.index)
            traj_out = {}   # by launch size: the trajectory rows, reused launch to launch (allocated before the clock)
            mtr = bool(a.sample_batch and a.fused)   # the fused kernel records the policy means (no recompute)
            acted = {}      # by launch number: the agent that acted per (transition, lane), counted after the clock

            def traj_bufs(kk, s):
                o = dict(traj_out.setdefault(kk, hier_traj_buffers(n, kk, dev, means=mtr)))
                o["acted"] = acted.setdefault(s + soff[0], torch.empty(kk, n, dtype=torch.uint8, device=dev))
                return o

            vhigh = vlow = None
            if a.sample_batch:
                vhigh = DevicePolicy.random_init_value(seed=27 + rank, device=dev.index, n_in=44)
                vlow = DevicePolicy.random_init_value(seed=37 + rank, device=dev.index)
            cols_out = {}

            def step(s, kk=k, o=0):   # launch numbers (and the exploration noise's step index) continue past the warm-up
                tr = hier_rollout(env, high, low, kk, explore=True, step0=(s + soff[0]) * k, trajectories=True,
                                  fused=a.fused, out=traj_bufs(kk, s), means=mtr)
                if a.sample_batch:   # both agents' columns; rows of the agent that did not act are zeroed
                    ch, cl = cols_out.setdefault(kk, ({}, {}))
                    acted_k = tr["acted"]
                    ch.update(high.sample_batch_columns(tr["obs_high"], tr["act_high"], value=vhigh, out=ch,
                                                        mean=tr.get("mean_high"),
                                                        valid=(acted_k & N.HUM_AGENT_HIGH) != 0))
                    cl.update(low.sample_batch_columns(tr["obs_low"], tr["act_low"], value=vlow, out=cl,
                                                       mean=tr.get("mean_low"),
                                                       valid=(acted_k & N.HUM_AGENT_LOW) != 0))
                return tr
            env._bench_acted = acted
    else:
        from ilrl_amd.clips import CLIP_NAMES
        from ilrl_amd.vec_env import HumanoidVecEnv
        clips = tuple(CLIP_NAMES) if a.clip == "all" else (a.clip,)
        env = HumanoidVecEnv(n, clips=clips, seed=0, device=dev.index, lane_offset=rank * n, precision=precision,
                             block_size=a.block, **phys)
        if a.terrain == "random":
            from ilrl_amd import _native as N
            env.set_terrain(N.HUM_TERRAIN_RANDOM_BLOCKS)

        def step(s, kk=k, o=0):
            j = s % len(ring)
            if kk < k:   # the remainder launch (or the drain launches: rows o .. o + kk of block s)
                return env.step_k(pool[s % 16][o:o + kk], autoreset=True, out=rem_out.get(kk))
            ring[j] = env.step_k(pool[s % 16], autoreset=True, out=ring[j])
        if a.policy:
            from ilrl_amd.policy import DevicePolicy
            pol = DevicePolicy.random_init(seed=7 + rank, device=dev.index)
            actbuf = torch.zeros(n, 17, device=dev)

            def step(s, kk=1, o=0):
                pol.act(env.obs, env.obs_reset, env.done, explore=True, step=s + soff[0], out=actbuf)
                return env.step(actbuf, autoreset=True)
            if a.fused:   # the policy inside the multi-step env kernel (hum_rollout_fused), trajectories recorded
                traj_out = {}   # by launch size, reused launch to launch

                vpol = DevicePolicy.random_init_value(seed=27 + rank, device=dev.index) if a.sample_batch else None
                cols_out = {}

                def step(s, kk=k, _o=0):
                    o = traj_out.get(kk)
                    tr = pol.rollout(env, kk, explore=True, step0=(s + soff[0]) * k, trajectories=True, fused=True,
                                     out=o, means=a.sample_batch)
                    traj_out.setdefault(kk, tr)
                    if a.sample_batch:   # the means recorded by the fused kernel: no policy recompute
                        c = cols_out.setdefault(kk, {})
                        c.update(pol.sample_batch_columns(tr["obs"], tr["actions"], value=vpol, out=c,
                                                          mean=tr["means"]))
                    return tr
    env.reset()
    env.done.zero_()
    for w in range(wlaunches):
        step(w, wsizes[w])
    gather_s, gathered, tg = 0.0, [], None
    gdiag = os.environ.get("ILRL_GATHER_DIAG", "")   # diagnostics: "pack" = packing only, "comm" = the gather only
    if G:   # the trajectory gather: static shapes, packed step-major fragments, asynchronous (parallel.TrajectoryGather)
        from ilrl_amd.parallel import DmaGather, TrajectoryGather, shard
        o = ring[0] if ring[0] is not None else env.step_k_out(k)
        ring[0] = o
        cols = (o[2], o[4], o[5]) if a.hier else (o[0], o[1], o[2])   # obs (hier: low-level), reward, done
        fields = [("obs", tuple(cols[0].shape[2:]), cols[0].dtype), ("act", (17,), pool[0].dtype),
                  ("reward", tuple(cols[1].shape[2:]), cols[1].dtype), ("done", tuple(cols[2].shape[2:]), cols[2].dtype)]
        counts = [shard(n * world, world, r)[1] for r in range(world)]
        if a.transport == "dma":
            from ilrl_amd.parallel import DmaUnavailable
            try:
                tg = DmaGather(fields, counts, G, dev)
            except DmaUnavailable as e:   # every rank alike: the collective transport, recorded in the line
                print("bench: %s; falling back to --transport collective" % e, file=sys.stderr, flush=True)
                a.transport = "collective (dma unavailable: %s)" % str(e)[:200]
                tg = TrajectoryGather(fields, counts, G, dev)
        else:
            tg = TrajectoryGather(fields, counts, G, dev)
        tg.start(0)   # communicator setup (RCCL point-to-point pairs) outside the timed region
        tg.wait()
        if isinstance(tg, DmaGather):   # per-launch chunks: end on a short drain launch
            plan = launch_plan(steps, k, drain=True)
            sizes, launches = [p[2] for p in plan], len(plan)
            a.drain = plan[-1][2] if len(plan) > len(launch_sizes(steps, k)) else None
    soff[0] = wlaunches
    if a.hier and a.policy:   # the timed launches' trajectory buffers
        for s, kk in enumerate(sizes):
            traj_bufs(kk, s)
    elif a.policy and a.fused:
        for kk in set(sizes):
            if kk not in traj_out:
                traj_out[kk] = {"obs": torch.empty(kk, n, 70, device=dev), "actions": torch.empty(kk, n, 17, device=dev),
                                "rewards": torch.empty(kk, n, device=dev),
                                "dones": torch.empty(kk, n, dtype=torch.uint8, device=dev)}
                if a.sample_batch:
                    traj_out[kk]["means"] = torch.empty(kk, n, 17, device=dev)
    if not a.policy:
        # every output buffer the timed launches write exists before the clock starts (a warmup shorter than k, e.g.
        # the driver's --steps 20 --warmup 5, never ran a launch of the timed shape: its allocation and zero fill
        # were timed)
        for j in range(len(ring)):
            if ring[j] is None:
                ring[j] = env.step_k_out(k)
        for kk in set(sizes):
            if kk < k:
                rem_out[kk] = env.step_k_out(kk)
    torch.cuda.synchronize(dev)
    if a.dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    done_steps = 0
    for s, (b, ro, kk) in enumerate(plan):
        step(b, kk, ro)
        if tg is not None:
            th = time.perf_counter()
            slot, f0 = (done_steps // G) % 2, done_steps % G   # the fragment slot, the launch's first step in it
            o = ring[0] if kk == k else rem_out[kk]   # the launch's outputs (full, remainder or drain launch)
            cols = (o[2], o[4], o[5]) if a.hier else (o[0], o[1], o[2])
            act = pool[b % 16][ro:ro + kk]
            final = (done_steps + kk) % G == 0 or s == launches - 1   # a full fragment, or the last one
            if gdiag != "comm":
                tg.pack(slot, f0, {"obs": cols[0], "act": act, "reward": cols[1], "done": cols[2]})
            if gdiag != "pack":
                tg.commit(slot, f0, f0 + kk, final)
                if final and a.dump_gather:   # tests: rank 0 keeps the fragment (synchronous)
                    tg.wait(slot)
                    got = tg.result(slot)
                    if got is not None:
                        gathered.append([got[f][::a.dump_lane_stride].cpu() for f in ("obs", "act", "reward", "done")])
            gather_s += time.perf_counter() - th
        done_steps += kk
    if tg is not None:
        tg.wait()   # the last fragments' gathers complete inside the timed region
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if a.dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps   # per env step, on the launch stream (torch's current)
    if getattr(tg, "trace", None):   # diagnostics (ILRL_DMA_TRACE=1): the chunks' timeline against the clock
        print("dma-trace: " + json.dumps([(e, c, round((t - t0) * 1e3, 4)) for e, c, t in tg.trace] +
                                         [("timed_end", 0, round(wall * 1e3, 4))]), file=sys.stderr, flush=True)
    if tg is not None and hasattr(tg, "close"):   # outside the timed region: unmap the peers' buffers (collective)
        tg.close()
    wall = _all_reduce(world, dev, a.backend, wall, dist.ReduceOp.MAX) if a.dist else wall
    low_steps = None
    if a.hier and a.policy:   # physics env-steps in the timed region: the low-level transitions the rollouts recorded
        from ilrl_amd import _native as N
        low_steps = float(sum(int((env._bench_acted[wlaunches + s] == N.HUM_AGENT_LOW).sum().item())
                              for s in range(launches)))
    elif a.hier:   # physics env-steps in the timed region: replay the same deterministic sequence and count them
        low_steps = float(count_hier_low_steps(a, dev, n, precision, plan, wsizes, k, phys, rank))
        if a.dist:
            low_steps = _all_reduce(world, dev, a.backend, low_steps, dist.ReduceOp.SUM)   # all ranks
    return env, wall, kern_ms, low_steps, gather_s, gathered, sizes


def _all_reduce(world, dev, backend, x, op):
    """One float reduced over the ranks (a host tensor for gloo, a device tensor for RCCL)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=op)
    return float(t.item())


def count_hier_low_steps(a, dev, n, precision, plan, wsizes, k, phys, rank):
    """Lanes that take a low-level (physics) step in each transition of the timed launches: a lane acts high next
    iff its last outputs carried the high-level obs (level hand-back, or done -> auto-reset)."""
    import torch
    from ilrl_amd import _native as N
    from ilrl_amd.hier_env import HierVecEnv
    pool, hpool = _pools(a, dev, n, k, rank)
    env = HierVecEnv(n, seed=0, device=dev.index, lane_offset=rank * n, precision=precision, block_size=a.block, **phys)
    env.reset()
    expect_high = torch.ones(n, dtype=torch.bool, device=dev)
    low = 0
    # the same launches as run(): warm-up launch w reads pool block w % 16, timed launch (b, o, kk) rows o .. o + kk
    # of block b % 16
    seq = [(w, 0, kk, False) for w, kk in enumerate(wsizes)] + [(b, o, kk, True) for b, o, kk in plan]
    for s, o, kk, timed in seq:
        out = env.step_k(hpool[s % 16][o:o + kk], pool[s % 16][o:o + kk], autoreset=True)
        agents, done = out[0], out[5]
        for t in range(kk):
            if timed:
                low += int((~expect_high).sum().item())
            expect_high = ((agents[t] & N.HUM_AGENT_HIGH) != 0) | (done[t] != 0)
    env.close()
    return low


def run_adapter(a, dev, n):
    """The path a reference user's RLlib sampler drives (train_config.py:13-29,320-321): per sampler step the
    policy's actions arrive as host numpy rows, one env launch runs, and the results go back as per-env Python
    objects; done envs are then reset through reset_at / try_reset (served from the launch's auto-reset rows).
    Actions are pre-drawn host arrays (the policy is RLlib's, outside this path); everything the adapter does -
    the action upload, the launch, the copies back, the per-env lists / dicts, the resets - is timed."""
    import numpy as np
    import torch
    rng = np.random.default_rng(1234)
    steps, warm = a.steps, a.warmup
    t_adapter = 0.0
    if not a.hier:
        from ilrl_amd.low_level_env import HumanoidVectorEnv
        venv = HumanoidVectorEnv(n, reference_name=a.clip, seed=0, device=dev.index)
        pool = [list(rng.uniform(-1, 1, (n, 17)).astype(np.float32)) for _ in range(16)]   # RLlib: a list of rows
        venv.vector_reset()
        phys_steps, resets = 0, 0

        def step(s):
            nonlocal resets
            obs, rew, done, info = venv.vector_step(pool[s % 16])
            for i in np.flatnonzero(done):
                venv.reset_at(int(i))
                resets += 1
            return n
        for w in range(warm):
            step(w)
        resets = 0
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for s in range(steps):
            phys_steps += step(s)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        env = venv.venv
        desc = "HumanoidVectorEnv.vector_step (RLlib 1.2 VectorEnv) + reset_at per done env"
        transitions = phys_steps
    else:
        from ilrl_amd.hier_env import HIGH, LOW, HierarchicalVectorEnv
        venv = HierarchicalVectorEnv(n, seed=0, device=dev.index)
        hp = [rng.uniform(-1, 1, (n, 2)).astype(np.float32) for _ in range(16)]
        lp = [rng.uniform(-1, 1, (n, 17)).astype(np.float32) for _ in range(16)]
        phys_steps = transitions = resets = 0
        t_dict = [0.0]

        def step(s):   # RLlib 1.2's sampler: poll, reset the done envs, act on every returned agent obs
            nonlocal phys_steps, transitions, resets
            obs, rew, dones, infos, _ = venv.poll()
            for i, d in dones.items():
                if d["__all__"]:
                    obs[i] = venv.try_reset(i)
                    resets += 1
            th = time.perf_counter()
            acts, h, l = {}, hp[s % 16], lp[s % 16]
            for i, ob in obs.items():   # the policy's output, one dict per acting agent (RLlib's work, not the adapter's)
                acts[i] = {HIGH: h[i]} if HIGH in ob else {LOW: l[i]}
            nlow = sum(1 for ad in acts.values() if LOW in ad)
            t_dict[0] += time.perf_counter() - th
            venv.send_actions(acts)
            phys_steps += nlow
            transitions += len(acts)
        for w in range(warm):
            step(w)
        torch.cuda.synchronize(dev)
        t_dict[0] = 0.0
        phys_steps = transitions = resets = 0
        t0 = time.perf_counter()
        for s in range(steps):
            step(s)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0 - t_dict[0]
        env = venv.venv
        desc = ("HierarchicalVectorEnv.poll / send_actions / try_reset (RLlib 1.2 BaseEnv); the harness's per-env "
                "action dicts (RLlib's work) excluded: %.4f s" % t_dict[0])
    out = {"metric": "env steps/sec at N parallel humanoids, 1/2/4/8 MI355X; obs/reward max-abs-err vs PyBullet",
           "value": phys_steps / wall, "unit": "env-steps/s", "n_gpus": 1, "steps": steps, "warmup": warm,
           "ms_per_step": wall / steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": a.precision.replace("fp", "f"), "data": "synthetic",
           "config": {"workload": "RLlib drop-in adapter: %s, %s, %d envs, uniform random host actions, k = 1" % (
               desc, a.clip, n), "adapter": True, "envs_per_gpu": n, "clip": a.clip, "hier": bool(a.hier)},
           "resets": resets, "agent_transitions_per_s": transitions / wall, "error_flags": env.error_flags()}
    print(json.dumps(out), flush=True)
    venv.stop() if a.hier else venv.venv.close()


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    a.dist = world > 1 or a.force_dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; ranks beyond the visible devices share them (tests on a one-GPU box)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    if a.dist:
        if "RANK" not in os.environ:   # --force-dist outside torch.distributed.run: a one-rank group of its own
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(sk.getsockname()[1]))
            sk.close()
        torch.cuda.set_device(dev)
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    n = a.lanes
    phys = {}
    for kv in a.phys:
        key, v = kv.split("=")
        phys[key] = float(v) if "." in v else int(v)
    if a.hier:
        from ilrl_amd.hier_env import HIER_CLIP
        a.clip = HIER_CLIP
    if a.policy and not a.fused and not a.hier:
        a.k = 1   # closed loop: the policy acts on every step's observation, one launch each
    if a.k < 1:
        raise SystemExit("--k must be >= 1")
    if a.adapter:
        return run_adapter(a, dev, n)
    if a.terrain != "plane":   # the in-run parity sample and the secondary legs are the plane workload's
        a.no_secondary = True
    if a.gather_every is None:
        a.gather_every = a.k if world > 1 and not a.policy else 0
    env, wall_max, kern_ms, low_steps, gather_s, gathered, sizes = run(a, world, rank, dev, n, a.precision, a.steps,
                                                                       a.warmup, phys)
    flags = env.error_flags()
    if rank == 0 and a.dump_gather and gathered:
        import numpy as np
        names = ("obs", "act", "reward", "done")
        np.savez(a.dump_gather, **{"%s_%d" % (nm, j): g[c].numpy() for j, g in enumerate(gathered)
                                   for c, nm in enumerate(names)})
    if rank == 0:
        base, drain = launch_sizes(a.steps, a.k), getattr(a, "drain", None)   # the plan before the drain split
        total = n * world * a.steps
        phys_steps_per_step = (low_steps / world / a.steps) if a.hier else n   # per GPU, per env step
        value = (low_steps if a.hier else total) / wall_max
        flops_j = _load_json("profiles/r06_flops_per_env_step.json")
        flops = flops_j["flops_per_env_step_mean"] if flops_j else None
        achieved = phys_steps_per_step * BYTES_PER_STEP_ALGO / (kern_ms * 1e-3) / 1e9
        traffic = None
        tj = _load_json("profiles/pmc_traffic.json") or {}
        tkey = "%s_%d_%s_k%d" % ("hier" if a.hier else a.clip, n, a.precision, a.k)
        if tkey in tj:
            traffic = tj[tkey]["bytes_per_env_step"] * phys_steps_per_step
        out = {
            "metric": "env steps/sec at N parallel humanoids, 1/2/4/8 MI355X; obs/reward max-abs-err vs PyBullet",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": wall_max / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.precision.replace("fp", "f"), "data": "synthetic",
            "config": {"workload": ("HumanoidBulletEnv-v0-Hier two-level rollout (high heading every 5 low steps), "
                                    if a.hier else "HumanoidBulletEnv-v0-Low step+reward, ") +
                                   "%s, %d envs/GPU, %s, auto-reset, %s env steps per %s" % (
                                       a.clip, n, _actions_desc(a),
                                       "/".join(str(s) for s in sorted(set(base), reverse=True)),
                                       ("hum_hier_rollout_fused launch (both networks inside the env kernel)"
                                        if a.fused else
                                        "hum_hier_rollout call (2 policy launches + 1 env launch per transition)")
                                       if a.hier and a.policy else "launch") +
                                   (" (the last launch's final %d steps run as a separate drain launch: the "
                                    "trajectory gather's per-launch chunks, bench.launch_plan)" % drain if drain else ""),
                       "fused": bool(a.policy and a.fused),
                       "sample_batch_columns": bool(a.policy and a.sample_batch),
                       "envs_per_gpu": n, "clip": a.clip, "k": a.k, "terrain": a.terrain,
                       # the launches the timed region actually ran (--steps < k: one shorter launch)
                       "launches": len(sizes), "steps_per_launch": max(base),
                       "launch_sizes": sorted(set(sizes), reverse=True),
                       "parallelism": "lane-sharded x%d" % world, "block": a.block, "physics_overrides": phys},
            # per env step: kernel_ms = launch duration / k; achieved = the env step's algorithmic bytes over it
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_unit": "HBM bytes per env step of all lanes (PMC, profiles/pmc_traffic.json)",
                         "bytes_per_env_step": BYTES_PER_STEP_ALGO, "bytes_per_env_step_layout": BYTES_PER_STEP_LAYOUT,
                         "kernel_ms": kern_ms, "kernel_ms_per_launch": kern_ms * a.steps / len(sizes)},
            "error_flags": flags,
        }
        if flops:
            peak = FP32_PEAK_TFLOPS if a.precision == "fp32" else FP64_PEAK_TFLOPS
            tf = phys_steps_per_step * flops / (kern_ms * 1e-3) / 1e12
            out["roofline_valu"] = {"bound": "valu-%s" % a.precision, "achieved": tf, "peak": peak, "unit": "TFLOP/s",
                                    "frac": tf / peak, "flops_per_env_step": flops,
                                    "source": "profiles/r06_flops_per_env_step.json (tools/flop_count.py)"}
        if a.hier:
            out["unit"] = "env-steps/s"
            out["physics_env_steps_per_step"] = phys_steps_per_step
            out["agent_transitions_per_s"] = total / wall_max
        if a.dist and a.gather_every and not a.policy:
            out["gather"] = {"every": a.gather_every, "backend": a.backend, "to_rank": 0, "transport": a.transport,
                             "op": ("rank 0 pulls every launch's rows (one contiguous range of every rank's packed "
                                    "step-major fragment) with the SDMA copy engines (IPC-mapped buffers, "
                                    "parallel.DmaGather) while the next launch runs, double-buffered"
                                    if a.transport == "dma" else
                                    "dist.gather of one packed step-major fragment (RCCL point-to-point), "
                                    "asynchronous, double-buffered") + "; completed inside the timed region",
                             "drain_launch_steps": drain,
                             "host_seconds": gather_s, "bytes_per_rank_per_step": n * (70 * 4 + 17 * 4 + 4 + 1),
                             "fragments": -(-a.steps // a.gather_every)}
        if world == 1 and not a.no_secondary and not a.hier and not a.policy:
            from ilrl_amd.clips import CLIP_NAMES
            clips = tuple(CLIP_NAMES) if a.clip == "all" else (a.clip,)
            out["parity"] = parity_sample(env, clips)
            sec = {}
            other = "fp64" if a.precision == "fp32" else "fp32"
            runs = [(other, other, phys, a.k), ("k1", a.precision, phys, 1)]
            if "split_penetration" not in phys:
                # continuity with the bench lines measured before the split-impulse model:
                # the same kernel on the previous workload (every limit / contact violation corrected at ERP)
                runs.append(("previous_model_split_off", a.precision, dict(phys, split_penetration=-1e30), a.k))
            for name, prec, ph, kk in runs:
                st, wu = 200, 24
                e2, w2, k2, _, _, _, _ = run(a, 1, 0, dev, n, prec, st, wu, ph, k=kk)
                e2.close()
                sec[name] = {"value": n * st / w2, "ms_per_step": w2 / st * 1e3, "kernel_ms": k2, "steps": st,
                             "warmup": wu, "steps_per_launch": kk, "precision": prec}
            out["secondary"] = sec
        if world == 1 and a.cpu_seconds > 0 and not a.hier:
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.cpu_workers or host_cores())
        print(json.dumps(out), flush=True)
    env.close()
    if a.dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

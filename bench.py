#!/usr/bin/env python3
"""Benchmark: env steps/s of the HIP humanoid imitation env (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4096 lanes per GPU, low-level imitation on motion02_04, uniform
random actions in [-1,1] (pre-generated pool, device resident), auto-reset of done lanes inside the
step launch.  A "step" = one hum_step launch advancing every lane one env step (4 physics substeps +
observation + imitation reward + bookkeeping).  Multi-GPU: one process per GPU, lanes sharded by rank
(global lane ids -> identical per-lane streams regardless of N), no data-path collective -> weak scaling.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))

# algorithmic HBM bytes per env-step of the step kernel (DESIGN.md "Roofline"): what the kernel must read
# and write per env: physics state 47 x f32 (read + write), bookkeeping 23 x f64 + 8 x i32 (read + write),
# action 17 x f32, obs 70 x f32, reward f32, done u8, frame i32  = 1165 B (clip tables are cache resident).
BYTES_PER_STEP_FP32 = 2 * 47 * 4 + 2 * (23 * 8 + 8 * 4) + 17 * 4 + 70 * 4 + 4 + 1 + 4
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--lanes", type=int, default=4096, help="env lanes per GPU")
    ap.add_argument("--clip", default="motion02_04", help="clip name, or 'all' = the four CMU clips round-robin per "
                                                          "lane (BASELINE config 3)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--block", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="CPU baseline processes (0 = min(16, cpus))")
    ap.add_argument("--phys", action="append", default=[], help="physics override k=v (hum_config field), diagnostics")
    ap.add_argument("--hier", action="store_true",
                    help="config 5: HierarchicalHumanoidEnv two-level rollout (hum_hier_step), clip motion09_03")
    return ap.parse_args()


def _cpu_worker(args):
    """Oracle (CPU restatement, fp64 C physics + numpy env logic) stepping for ~`seconds`."""
    seconds, seed = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as O
    from ilrl_amd.clips import load_clip
    clip = load_clip("motion02_04")
    env = O.OracleLowLevelEnv(clip, seed=seed, lane=0)
    env.reset()
    rng = np.random.default_rng(seed)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, _, d, _ = env.step(rng.uniform(-1, 1, 17).astype(np.float32))
        n += 1
        if d:
            env.reset()
    return n, time.perf_counter() - t0


def cpu_baseline(seconds, workers):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(seconds, 1000 + w) for w in range(workers)])
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": workers, "kind": "port",
            "sample": "oracle/ (fp64 C physics restatement + numpy env logic; PyBullet absent) on motion02_04, "
                      "%d processes x %.0f s of uniform-random-action steps with resets (%d steps)" % (workers, seconds, steps)}


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from ilrl_amd.vec_env import HumanoidVecEnv

    n = a.lanes
    phys = {}
    for kv in a.phys:
        k, v = kv.split("=")
        phys[k] = float(v) if "." in v else int(v)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [(torch.rand(n, 17, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
    if a.hier:
        from ilrl_amd.hier_env import HIER_CLIP, HierVecEnv
        a.clip = HIER_CLIP
        env = HierVecEnv(n, seed=0, device=local, lane_offset=rank * n, precision=a.precision, block_size=a.block,
                         **phys)
        hpool = [(torch.rand(n, 2, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
        step = lambda s: env.step(hpool[s % 16], pool[s % 16], autoreset=True)
    else:
        from ilrl_amd.clips import CLIP_NAMES
        clips = tuple(CLIP_NAMES) if a.clip == "all" else (a.clip,)
        env = HumanoidVecEnv(n, clips=clips, seed=0, device=local, lane_offset=rank * n, precision=a.precision,
                             block_size=a.block, **phys)
        step = lambda s: env.step(pool[s % 16], autoreset=True)
    env.reset()
    for w in range(a.warmup):
        step(w)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for s in range(a.steps):
        step(s)
    ev1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / a.steps            # average launch duration on the launch stream
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())
    flags = env.error_flags()
    if rank == 0:
        total = n * world * a.steps
        value = total / wall_max
        bpl = BYTES_PER_STEP_FP32 if a.precision == "fp32" else BYTES_PER_STEP_FP32 + 2 * 47 * 4
        achieved = n * bpl / (kern_ms * 1e-3) / 1e9
        traffic = None
        tp = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(tp):
            try:
                tj = json.load(open(tp))
                key = "%s_%d_%s" % (a.clip, n, a.precision)
                if key in tj:
                    traffic = tj[key]["bytes_per_launch"]
            except Exception:
                traffic = None
        out = {
            "metric": "env steps/sec at N parallel humanoids, 1/2/4/8 MI355X; obs/reward max-abs-err vs PyBullet",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": wall_max / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.precision.replace("fp", "f"), "data": "synthetic",
            "config": {"workload": ("HumanoidBulletEnv-v0-Hier two-level rollout (high heading every 5 low steps), "
                                    if a.hier else "HumanoidBulletEnv-v0-Low step+reward, ") +
                                   "%s, %d envs/GPU, uniform random actions, auto-reset" % (a.clip, n),
                       "envs_per_gpu": n, "clip": a.clip,
                       "parallelism": "lane-sharded x%d" % world, "block": a.block, "physics_overrides": phys},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_env_step": bpl, "kernel_ms": kern_ms},
            "error_flags": flags,
        }
        if a.hier:
            out["metric"] = "agent transitions/sec at N parallel hierarchical humanoids (5 of 6 are physics env steps)"
            out["unit"] = "agent-steps/s"
        pp = os.path.join(REPO, "profiles", "parity_fp32_kernel1.json")   # written by tests/test_gpu_parity.py
        if a.precision == "fp32" and os.path.exists(pp) and not a.hier:
            out["parity"] = dict(json.load(open(pp)), source="profiles/parity_fp32_kernel1.json")
        if world == 1 and a.cpu_seconds > 0 and not a.hier:
            workers = a.cpu_workers or min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, workers)
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Does a transfer overlap the env kernel?  (each env wave holds a SIMD's whole register
file and four blocks fill a CU's LDS, so no other kernel's wave is resident while hum_step_k runs.)

On one GPU: a 32-step hum_step_k launch of 4096 lanes (~3.6 ms) on torch's stream, and beside it a 46.3 MB
device-to-device transfer (config 4's per-rank fragment: 4096 lanes x 32 steps x 353 B) by
  copy_     torch's copy_ on a second stream (hipMemcpyAsync device-to-device)
  peer      hipMemcpyPeerAsync on a second stream (same device)
  sdma      hsa_amd_memory_async_copy_on_engine forced onto an SDMA engine (tools/micro/dma.cpp)
  kernel    a small elementwise kernel on a second stream (what an RCCL send / recv kernel would need: CUs)
Each is timed alone and started together with the env launch; overlap = (alone_env + alone_x - together) / alone_x
(1 = fully hidden, 0 = serialised)."""
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

dev = torch.device("cuda", 0)
n, k = 4096, 32
env = HumanoidVecEnv(n, clips=("motion02_04",), seed=0)
env.reset()
acts = torch.rand(k, n, 17, device=dev) * 2 - 1
out = env.step_k_out(k)
NB = n * k * 353
src = torch.randint(0, 255, (NB,), dtype=torch.uint8, device=dev)
dst = torch.empty_like(src)
s2 = torch.cuda.Stream(dev)
hip = ctypes.CDLL("libamdhip64.so")
dma = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdma.so"))
dma.dma_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int]


def env_launch():
    env.step_k(acts, autoreset=True, out=out)


def xfer(kind):
    if kind == "copy_":
        with torch.cuda.stream(s2):
            dst.copy_(src)
    elif kind == "peer":
        r = hip.hipMemcpyPeerAsync(ctypes.c_void_p(dst.data_ptr()), 0, ctypes.c_void_p(src.data_ptr()), 0,
                                   ctypes.c_size_t(NB), ctypes.c_void_p(s2.cuda_stream))
        assert r == 0, r
    elif kind == "sdma":
        r = dma.dma_copy(dst.data_ptr(), src.data_ptr(), NB, 1, 1)
        assert r >= 0, "hsa copy failed: %d" % r
    elif kind == "kernel":
        with torch.cuda.stream(s2):
            dst.view(torch.int32)[: NB // 64].add_(1)


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def completion_offsets(kind, reps=5):
    """the transfer issued right AFTER the env launch was enqueued (its waves already own the CUs): when does it
    complete, measured from the launch's start?  ~alone_ms = it ran beside the launch; ~env_ms = it waited for it."""
    outs = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ex = torch.cuda.Event(enable_timing=True)
        e0.record()
        env_launch()
        e1.record()
        time.sleep(2e-4)   # the launch's waves are resident before the transfer is issued
        if kind == "sdma":
            t0 = time.perf_counter()
            xfer(kind)   # host-issued, host-waited
            host_done = (time.perf_counter() - t0) * 1e3 + 0.2
            torch.cuda.synchronize(dev)
            outs.append((host_done, e0.elapsed_time(e1)))
        else:
            s2.wait_event(e0)
            xfer(kind)
            ex.record(s2)
            torch.cuda.synchronize(dev)
            outs.append((e0.elapsed_time(ex), e0.elapsed_time(e1)))
    outs.sort()
    return outs[len(outs) // 2]


for _ in range(3):
    env_launch()
res = {"bytes": NB, "env_alone_ms": timed(env_launch)}
for kind in ("copy_", "peer", "kernel", "sdma"):
    xfer(kind)
    alone = timed(lambda: xfer(kind))

    def both():
        env_launch()
        xfer(kind)
    together = timed(both)
    res[kind] = {"alone_ms": alone, "with_env_ms": together,
                 "overlap": (res["env_alone_ms"] + alone - together) / alone}
    done_at, env_ms = completion_offsets(kind)
    res[kind]["completes_after_launch_start_ms"] = done_at
    res[kind]["env_launch_ms"] = env_ms
    print(kind, json.dumps(res[kind]), flush=True)
    assert torch.equal(dst, src) or kind == "kernel"
    dst.zero_()
print(json.dumps(res, indent=1))

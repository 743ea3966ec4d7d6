"""Diagnostic: which waves are the slow ones?  Per-block work log of the cooperative kernel (diag build,
-DHUM_PHASE_TIMING): duration vs PGS length, row rounds, narrow-phase rounds, contacts and in-kernel resets."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
import torch
from ilrl_amd import _native as N
from ilrl_amd.vec_env import HumanoidVecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1   # env steps per launch (hum_step_k); per-step figures divide by K
nb = n // 4
env = HumanoidVecEnv(n, clips=("motion02_04",), seed=0)
env.reset()
L = N.lib()
L.hum_debug_wave_log.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
g = torch.Generator(device="cuda").manual_seed(1)
pool = [(torch.rand(K, n, 17, device="cuda", generator=g) * 2 - 1).contiguous() for _ in range(8)]
# EARLY=1: the driver's bench shape instead of the steady state - every launch starts from a fresh reset of all lanes
# (a new seed each time), 5 warm-up env steps in one launch, then the logged launch of K steps (bench.py --steps K
# --warmup 5)
EARLY = os.environ.get("EARLY") == "1"
if not EARLY:
    for s in range(10):
        env.step_k(pool[s % 8], autoreset=True)
rows = []
buf = np.zeros((nb, 32), np.uint32)
for s in range(30):
    if EARLY:
        env.close()
        env = HumanoidVecEnv(n, clips=("motion02_04",), seed=100 + s)
        env.reset()
        env.step_k(pool[s % 8][:5].contiguous(), autoreset=True)
    L.hum_debug_wave_log(None, nb, 1)
    _, _, done, _ = env.step_k(pool[s % 8], autoreset=True)[:4]
    L.hum_debug_wave_log(buf.ctypes.data, nb, 0)
    d = done.cpu().numpy().reshape(K, nb, 4).sum((0, 2))
    rows.append(np.column_stack([buf[:, :5].astype(np.float64), d, np.full(nb, s), buf[:, 9:32].astype(np.float64)]))
    st = buf[:, 5].astype(np.int64)
    st = (st - st.min()) % (1 << 32)
    hw = buf[:, 6].astype(np.int64)
    xcc = buf[:, 7].astype(np.int64) & 0xF
    cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 0x7) << 5)   # cu | sh | se
    key = xcc * 1024 + cu
    _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    occ = cnt[inv]
    end = st + buf[:, 4]
    if s < 3 or s == 29:
        print("step %d: distinct CUs %d, blocks/CU histogram %s, start spread p50 %.0f max %.0f, end max %.0f, "
              "mean dur by occupancy %s" % (s, len(cnt), np.bincount(cnt).tolist(), np.median(st), st.max(), end.max(),
              {int(o): int(buf[occ == o, 0].mean()) for o in np.unique(occ)}))
        late = st > 0.3 * end.max()
        if late.any():
            print("   late-starting blocks: %d (ids %s)" % (late.sum(), np.nonzero(late)[0][:10].tolist()))
        for x in range(8):
            m = xcc == x
            sx = st[m]
            ex = sx + buf[m, 4]
            print("   xcc %d: start (10 ns ticks) min %d max %d, end max %d; dur real mean %d min %d max %d; cycles/tick %.1f" % (
                x, sx.min(), sx.max(), ex.max(), buf[m, 4].mean(), buf[m, 4].min(), buf[m, 4].max(),
                buf[m, 0].mean() / buf[m, 4].mean()))
        simd = (hw >> 4) & 3
        print("   xcc histogram %s; simd histogram %s" % (np.bincount(xcc).tolist(), np.bincount(simd).tolist()))
X = np.concatenate(rows)
print("env steps per launch K = %d (per-block-step figures below are per env step: launch totals / K)" % K)
X[:, [0, 1, 2, 3, 4, 5]] /= K
X[:, 7:30] /= K
dur = X[:, 0]
names = ["pgs_len(sum max nrows)", "row_rounds", "narrow_rounds", "resets"]
feat = X[:, [1, 2, 3, 5]]
print("mean duration %.0f; per launch max/mean median %.2f" % (dur.mean(), np.median([
    dur[X[:, 6] == s].max() / dur[X[:, 6] == s].mean() for s in range(30)])))
q = np.quantile(dur, [0.5, 0.9, 0.99, 0.999])
print("duration quantiles p50 %.0f p90 %.0f p99 %.0f p99.9 %.0f max %.0f" % (*q, dur.max()))
slow = dur >= np.quantile(dur, 0.99)
for k, nm in enumerate(names):
    print("  %-24s all %.2f  slowest1%% %.2f  corr %.2f" % (nm, feat[:, k].mean(), feat[slow, k].mean(),
                                                          np.corrcoef(feat[:, k], dur)[0, 1]))
A = np.column_stack([feat, np.ones(len(dur))])
coef, *_ = np.linalg.lstsq(A, dur, rcond=None)
print("linear fit cycles: " + ", ".join("%s %.0f" % (nm, c) for nm, c in zip(names + ["const"], coef)))
res = dur - A @ coef
print("fit residual std %.0f (duration std %.0f)" % (res.std(), dur.std()))
ph = X[:, 7:17]
pn = ["fk", "pass1", "pass2", "base+pass3", "geom/limits", "contacts", "rows", "pgs", "integrate", "post_step"]
top = dur >= np.quantile(dur, 0.99)
print("phase cycles per block-step: mean | slowest 1%% | corr with duration")
for k in range(10):
    print("  %-12s %8.0f | %8.0f | %.2f" % (pn[k], ph[:, k].mean(), ph[top, k].mean(), np.corrcoef(ph[:, k], dur)[0, 1]))
sub = X[:, 17:30]   # sub-phase markers 11-23 (HUM_SUBPHASE builds): time from the previous marker
subn = {11: "fk: sin/cos", 12: "fk: chain", 13: "pass1: parent vel", 14: "pass1: inertia+bias", 15: "pass3: base",
        17: "post: book load", 19: "post: calc_state", 20: "post: reward", 21: "post: target",
        22: "post: ref obs + done", 16: "post: obs row", 23: "post: rew/done/frame", 18: "post: return"}
if os.environ.get("PGS_SUB") == "1":   # HUM_SUBPHASE_PGS builds: the Delassus PGS's split instead of the post step's
    subn = {11: "fk: sin/cos", 12: "fk: chain", 13: "pass1: parent vel", 14: "pass1: inertia+bias", 15: "pass3: base",
            19: "pgs: A operands", 20: "pgs: A MFMA", 21: "pgs: A stores + rows", 22: "pgs: sweeps"}
if os.environ.get("ROWS_SUB") == "1":   # HUM_SUBPHASE_ROWS builds: the rows phase's split instead of the post step's
    subn = {11: "fk: sin/cos", 12: "fk: chain", 13: "pass1: parent vel", 14: "pass1: inertia+bias", 15: "pass3: base",
            19: "rows: setup + contact", 20: "rows: Jacobian", 21: "rows: M^-1 J^T solve", 22: "rows: jm + coupling"}
if sub.any():
    print("sub-phase cycles per block-step (each taken out of its phase above): mean | slowest 1%")
    for k, nm in subn.items():
        print("  %-22s %8.0f | %8.0f" % (nm, sub[:, k - 11].mean(), sub[top, k - 11].mean()))
pg = ph[:, 7] / np.maximum(X[:, 1], 1)
print("pgs cycles per unit pgs_len: mean %.0f (per row-iteration at 5 iters: %.0f)" % (pg.mean(), pg.mean() / 5))

#!/usr/bin/env python3
"""Summarise tools/gpu/r04_fused_l2.sh: per launch of the step kernel (fused closed loop vs env only), its average
duration and the L2 (TCC) / L1 (TCP) / HBM counters; L2 request bytes at 128 B per request, the L2 bandwidth they
imply over the kernel's duration, against the guide's ~34.5 TB/s aggregate L2 (MI355X_MICROARCH.md, L2 section)."""
import glob
import os
import sqlite3
import sys


def kernel_avgs(db):
    c = sqlite3.connect(db)
    return {n: (calls, avg) for n, calls, avg in c.execute("select name,total_calls,average from top_kernels")}


def counters(db):
    c = sqlite3.connect(db)
    out = {}
    for kn, cn, v in c.execute("select kernel_name,counter_name,value from counters_collection"):
        out.setdefault(kn, {}).setdefault(cn, []).append(v)
    return {k: {cn: sum(v) / len(v) for cn, v in d.items()} for k, d in out.items()}


def main():
    root = sys.argv[1]
    for mode in ("fused", "env"):
        kt = kernel_avgs(os.path.join(root, "kt_%s" % mode, "run_results.db"))
        step = max((n for n in kt if "step_group" in n), key=lambda n: kt[n][0] * kt[n][1])
        calls, avg_us = kt[step]
        ctr = {}
        for pas in ("hm", "rq", "tcp", "fetch"):
            for db in glob.glob(os.path.join(root, "%s_%s" % (pas, mode), "*.db")):
                for kn, d in counters(db).items():
                    if kn == step:
                        ctr.update(d)
        print("== %s: %s  %d launches, %.1f us avg" % (mode, step[:60], calls, avg_us))
        for k in sorted(ctr):
            print("   %-32s %.4g per launch" % (k, ctr[k]))
        if "TCC_REQ_sum" in ctr:
            b = ctr["TCC_REQ_sum"] * 128.0
            print("   L2 request bytes (x128 B)        %.4g per launch -> %.2f TB/s over the launch (guide: ~34.5 TB/s)" %
                  (b, b / (avg_us * 1e-6) / 1e12))
        if "TCC_HIT_sum" in ctr and "TCC_MISS_sum" in ctr:
            print("   L2 hit rate                      %.4f" % (ctr["TCC_HIT_sum"] / max(ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"], 1)))


if __name__ == "__main__":
    main()

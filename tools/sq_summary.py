#!/usr/bin/env python3
"""Summarise SQ PMC passes (tools/gpu/pmc_sq.sh) for the step kernel: per-launch totals and per-wave ratios.

usage: tools/sq_summary.py DIR [kernel_prefix=step_group]
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are quad-cycles (MI355X_MICROARCH.md 'cycle constants' row).
"""
import glob
import os
import sqlite3
import sys


def main():
    d = sys.argv[1]
    kp = sys.argv[2] if len(sys.argv) > 2 else "step_group"
    vals = {}
    for db in sorted(glob.glob(os.path.join(d, "p*", "run_results.db"))):
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
        kcol = "kernel_name" if "kernel_name" in cols else None
        for name, v, n in c.execute("select counter_name, avg(value), count(*) from counters_collection where %s like ? "
                                    "group by counter_name" % kcol, ("%" + kp + "%",)):
            vals[name] = (v, n)
    out = []
    for k in sorted(vals):
        out.append("%-24s %16.1f  (avg over %d launches)" % (k, vals[k][0], vals[k][1]))
    g = lambda k: vals.get(k, (float("nan"),))[0]
    waves = g("SQ_WAVES")
    if waves == waves:
        out.append("per wave: insts VALU %.0f  LDS %.0f  SALU %.0f  SMEM %.0f  VMEM rd %.0f wr %.0f" % (
            g("SQ_INSTS_VALU") / waves, g("SQ_INSTS_LDS") / waves, g("SQ_INSTS_SALU") / waves, g("SQ_INSTS_SMEM") / waves,
            g("SQ_INSTS_VMEM_RD") / waves, g("SQ_INSTS_VMEM_WR") / waves))
        wc = g("SQ_WAVE_CYCLES")
        out.append("per wave: cycles %.0f = active %.1f%% + wait_inst %.1f%% (lds %.1f%%) + wait(park) %.1f%%; "
                   "VALU active %.1f%%, LDS active %.1f%%, LDS bank-conflict cycles %.0f" % (
                       4 * wc / waves, 100 * g("SQ_ACTIVE_INST_ANY") / wc, 100 * g("SQ_WAIT_INST_ANY") / wc,
                       100 * g("SQ_WAIT_INST_LDS") / wc, 100 * g("SQ_WAIT_ANY") / wc, 100 * g("SQ_ACTIVE_INST_VALU") / wc,
                       100 * g("SQ_ACTIVE_INST_LDS") / wc, g("SQ_LDS_BANK_CONFLICT") / waves))
    print("\n".join(out))


if __name__ == "__main__":
    main()

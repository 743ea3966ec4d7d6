#!/usr/bin/env python3
"""Summarise the FETCH_SIZE / WRITE_SIZE calibration passes of tools/micro/fetch_calib (tools/gpu/fetch_calib.sh):
counter bytes per dispatch / the dispatch's known byte count, per access width.

usage: tools/fetch_calib_summary.py DIR   (DIR/fetch, DIR/write hold the rocprofv3 databases)
"""
import os
import sqlite3
import sys

BYTES = 64 << 20
KNOWN = {"wrrow": (BYTES // 280) * 280}


def main():
    root = sys.argv[1]
    print("# FETCH_SIZE / WRITE_SIZE calibration on gfx950 (tools/micro/fetch_calib.hip), counter / known bytes")
    for db, ctr, pre in (("fetch", "FETCH_SIZE", "rd"), ("write", "WRITE_SIZE", "wr")):
        con = sqlite3.connect(os.path.join(root, db, "run_results.db"))
        rows = {}
        for name, v in con.execute("select kernel_name, value from counters_collection where counter_name=?", (ctr,)):
            base = name.split("(")[0].strip()
            if base.startswith(pre):
                rows.setdefault(base, []).append(v * 1024.0)   # KB -> B
        for k in sorted(rows):
            vals = rows[k]
            known = KNOWN.get(k, BYTES)
            avg = sum(vals) / len(vals)
            print("%-6s %-10s %14.0f B/dispatch  known %12d B  ratio %.3f  (%d dispatches)"
                  % (k, ctr, avg, known, avg / known, len(vals)))


if __name__ == "__main__":
    main()

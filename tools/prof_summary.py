#!/usr/bin/env python3
"""Summarise rocprofv3 databases (kernel-trace/stats + FETCH_SIZE / WRITE_SIZE passes) into profiles/.

usage: tools/prof_summary.py TAG [prof_root=gpurun_out] [lanes=4096] [clip=motion02_04] [precision=fp32] [k=8]
                             [instantiation=step_group_kernelIfLi4ELb0ELi3E]
(k = env steps per launch of the profiled bench command; instantiation: the mangled name substring of the profiled
kernel, whose register / spill counts are read from the shipped code object's metadata note)
Writes profiles/<TAG>_kernel_stats.txt and updates profiles/pmc_traffic.json (bench.py reads it).
HBM bytes per launch follow MI355X_MICROARCH.md: FETCH_SIZE counts half the bytes of wide coalesced
streaming reads on gfx950 (reported both raw and x2); WRITE_SIZE is exact for 16-B stores.
"""
import json
import os
import sqlite3
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_object_meta(kname, inst=None):
    """The kernel's register / spill / segment sizes from the AMDGPU metadata note of the shipped library's code
    objects (tools/spill_map.py kernel_meta); the vgpr_count there includes the AGPRs (unified register file).
    rocprofv3's summary names every instantiation "step_group_kernel": `inst` is the mangled template-argument
    substring of the one profiled (the benchmarked low-level fp32 kernel, POLICY 3, by default)."""
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from spill_map import kernel_meta
    from test_cpu_isa import code_objects
    lib = os.path.join(REPO, "imitation-learning-rl_amd", "ilrl_amd", "_lib", "libhumenv.so")
    if not os.path.exists(lib):
        return None
    tmp = tempfile.mkdtemp()
    for j, co in enumerate(code_objects(lib)):
        p = os.path.join(tmp, "co_%d.o" % j)
        open(p, "wb").write(co)
        for name, m in kernel_meta(p).items():
            if (inst or "step_group_kernelIfLi4ELb0ELi3E") in name:
                return m
    return None


def main():
    tag = sys.argv[1]
    root = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out")
    lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    clip = sys.argv[4] if len(sys.argv) > 4 else "motion02_04"
    prec = sys.argv[5] if len(sys.argv) > 5 else "fp32"
    k = int(sys.argv[6]) if len(sys.argv) > 6 else 8
    out = []
    con = sqlite3.connect(os.path.join(root, "prof_kt", "run_results.db"))
    out.append("# rocprofv3 --kernel-trace --stats -T  (bench.py, %d lanes, %s, %s)" % (lanes, clip, prec))
    # rocpd's top_kernels view reports durations in microseconds
    out.append("%-48s %8s %14s %12s %8s" % ("kernel", "calls", "total_us", "avg_us", "pct"))
    step_avg, kname = None, None
    for r in con.execute("select name,total_calls,total_duration,average,percentage from top_kernels "
                         "order by total_duration desc"):
        out.append("%-48s %8d %14.1f %12.3f %8.3f" % r)
        if kname is None and r[0].startswith("step"):
            kname, step_avg = r[0], r[3]
    kname = kname or "step_group_kernel"
    row = con.execute("select vgpr_count, accum_vgpr_count, sgpr_count, scratch_size, lds_size, workgroup_x, grid_x "
                      "from kernels where name=? limit 1", (kname,)).fetchone()
    if row:
        out.append("%s rocprofv3 resources: vgpr=%s agpr=%s sgpr=%s scratch/lane=%s lds=%s wg=%s grid=%s "
                   "(rocprofv3 reports no AGPRs for this code object: the note below is authoritative)" % ((kname,) + row))
    meta = code_object_meta(kname, sys.argv[7] if len(sys.argv) > 7 else None)
    if meta:
        out.append("%s code object (AMDGPU metadata note of the shipped libhumenv.so): vgpr_count=%s agpr_count=%s "
                   "vgpr_spill_count=%s sgpr_spill_count=%s private_segment_fixed_size=%s B/lane "
                   "group_segment_fixed_size=%s B" % (kname, meta.get("vgpr_count"), meta.get("agpr_count", "0"),
                                                      meta.get("vgpr_spill_count"), meta.get("sgpr_spill_count"),
                                                      meta.get("private_segment_fixed_size"),
                                                      meta.get("group_segment_fixed_size")))
    pmc = {}
    for db, ctr in (("prof_fetch", "FETCH_SIZE"), ("prof_write", "WRITE_SIZE")):
        p = os.path.join(root, db, "run_results.db")
        if not os.path.exists(p):
            continue
        c = sqlite3.connect(p)
        vals = [v for (v,) in c.execute("select value from counters_collection where kernel_name=? and "
                                        "counter_name=?", (kname, ctr))]
        if vals:
            pmc[ctr] = sum(vals) / len(vals) * 1024.0   # KB -> bytes per launch
            out.append("%s %s: %.1f KB/launch avg over %d launches" % (ctr, kname, pmc[ctr] / 1024, len(vals)))
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        traffic = 2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]
        out.append("HBM traffic per launch of %d env steps (2*FETCH_SIZE + WRITE_SIZE, gfx950 correction): %.3e B = "
                   "%.1f B/env-step (uncorrected FETCH: %.1f B/env-step)" % (k, traffic, traffic / lanes / k,
                                                                             (pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) / lanes / k))
        tp = os.path.join(REPO, "profiles", "pmc_traffic.json")
        tj = json.load(open(tp)) if os.path.exists(tp) else {}
        tj["%s_%d_%s_k%d" % (clip, lanes, prec, k)] = {
            "bytes_per_launch": traffic, "steps_per_launch": k, "bytes_per_env_step": traffic / lanes / k,
            "fetch_size_bytes_raw": pmc["FETCH_SIZE"], "write_size_bytes": pmc["WRITE_SIZE"],
            "kernel": kname, "kernel_avg_us": step_avg, "source": "profiles/%s_kernel_stats.txt" % tag}
        json.dump(tj, open(tp, "w"), indent=1)
    txt = "\n".join(out) + "\n"
    open(os.path.join(REPO, "profiles", "%s_kernel_stats.txt" % tag), "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()

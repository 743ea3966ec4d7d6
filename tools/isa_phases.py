#!/usr/bin/env python3
"""Static per-phase instruction counts of the cooperative step kernel (diagnostic).

Compiles humanoid_env.hip for gfx950 with -DHUM_PHASE_MARK -DHUM_DIAG_F32_ONLY (asm comment markers at the
phase ends of group_substep / the kernel) and counts VALU / LDS / SALU / VMEM instructions between markers;
loops inside a phase are listed (backward branches) so dynamic counts can be estimated.
usage: [ISA_FLAGS="extra hipcc flags"] tools/isa_phases.py [out.s]
"""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "imitation-learning-rl_amd", "csrc", "humanoid_env.hip")
# HOT=1: the shipped benchmarked kernel's translation unit and flags (csrc/Makefile HOTFLAGS)
HOT = os.environ.get("HOT") == "1"
if HOT:
    SRC = os.path.join(REPO, "imitation-learning-rl_amd", "csrc", "group_f32_low.hip")
HOTFLAGS = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp", "-fno-slp-vectorize", "-mllvm", "-disable-machine-licm"]
NAMES = {1: "fk", 2: "pass1", 3: "pass2", 4: "base+pass3", 5: "geom/limits", 6: "contacts", 7: "rows", 8: "pgs",
         9: "integrate", 10: "post_step"}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa_phases.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                           "-S", "-DHUM_PHASE_MARK", "-DHUM_DIAG_F32_ONLY", "-o", out, SRC]
                          + (HOTFLAGS if HOT else [])
                          + os.environ.get("ISA_FLAGS", "").split())
    lines = open(out).read().split("\n")
    st = [i for i, l in enumerate(lines) if re.match(r"_ZN3hkk17step_group_kernelIfLi4ELb0ELi3EEEvNS_5KArgsE:", l)][0]
    en = [i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end")][0]
    cur = 0
    cnt = collections.defaultdict(collections.Counter)
    labels = {}
    for i in range(st, en):
        l = lines[i].strip()
        if l.startswith(".LBB"):
            labels[l.rstrip(":")] = (i, cur)
    loops = collections.defaultdict(list)
    for i in range(st, en):
        l = lines[i].strip()
        m = re.search(r"@phase (\d+)", l)
        if m:
            cur = int(m.group(1))
            continue
        if not l or l.startswith((";", ".")) or l.endswith(":"):
            continue
        op = l.split()[0]
        cls = ("valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else "salu" if op.startswith("s_")
               and not op.startswith(("s_load", "s_buffer")) else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_"))
               else "smem" if op.startswith(("s_load", "s_buffer")) else "other")
        cnt[cur + 1 if cur < 10 else 0][cls] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = l.split()[-1]
            if tgt in labels and labels[tgt][0] < i:
                loops[cur + 1].append((tgt, i - labels[tgt][0]))
    print("%-14s %7s %6s %6s %6s" % ("phase", "valu", "lds", "salu", "vmem"))
    for k in sorted(cnt):
        c = cnt[k]
        print("%-14s %7d %6d %6d %6d   loops(len): %s" % (NAMES.get(k, "pre/post"), c["valu"], c["lds"], c["salu"], c["vmem"],
                                                          ", ".join("%d" % n for _, n in loops.get(k, []))[:80]))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where does a shipped kernel touch scratch?  (the benchmarked POLICY-3 twin spills.)

Reads the gfx950 code objects out of libhumenv.so (tests/test_cpu_isa.py code_objects), disassembles the named
kernel, and lists every scratch load / store with the innermost loop (backward branch span) that contains it, plus
the kernel's register / spill metadata from the code object notes.
usage: tools/spill_map.py [kernel-substring=step_group_kernelIfLi4ELb0ELi3E] [lib]"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_cpu_isa import code_objects  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin/"


def kernel_meta(co_path):
    """{kernel name: {vgpr_count, agpr_count, vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size,
    group_segment_fixed_size}} from the code object's AMDGPU metadata note"""
    txt = subprocess.check_output([LLVM + "llvm-readelf", "--notes", co_path], text=True)
    out, cur = {}, None
    for line in txt.splitlines():
        if re.match(r"^  - \.", line):   # a kernel record starts (its argument records are indented deeper)
            if cur and "name" in cur:
                out[cur["name"]] = cur
            cur = {}
        m = re.match(r"^  (?:- |  )\.(\w+):\s+(\S+)", line)   # the kernel record's own keys only
        if m and cur is not None:
            cur[m.group(1)] = m.group(2)
    if cur and "name" in cur:
        out[cur["name"]] = cur
    return out


def main():
    sub = sys.argv[1] if len(sys.argv) > 1 else "step_group_kernelIfLi4ELb0ELi3E"
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "imitation-learning-rl_amd", "ilrl_amd", "_lib",
                                                             "libhumenv.so")
    tmp = tempfile.mkdtemp()
    for j, co in enumerate(code_objects(lib)):
        p = os.path.join(tmp, "co_%d.o" % j)
        open(p, "wb").write(co)
        meta = kernel_meta(p)
        names = [n for n in meta if sub in n]
        if not names:
            continue
        name = names[0]
        m = meta[name]
        print("%s: vgpr %s agpr %s vgpr_spill %s sgpr_spill %s scratch/lane %s B lds %s B" % (
            name, m.get("vgpr_count"), m.get("agpr_count"), m.get("vgpr_spill_count"), m.get("sgpr_spill_count"),
            m.get("private_segment_fixed_size"), m.get("group_segment_fixed_size")))
        dis = subprocess.check_output([LLVM + "llvm-objdump", "-d", p], text=True).splitlines()
        s = [i for i, l in enumerate(dis) if l.endswith(">:") and name in l][0]
        e = next((i for i in range(s + 1, len(dis)) if dis[i].endswith(">:")), len(dis))
        body = dis[s + 1:e]
        addr = []
        for l in body:
            a = re.search(r"//\s*([0-9A-F]{12}):", l)
            addr.append(int(a.group(1), 16) if a else None)
        loops = []   # (start addr, end addr) of every backward branch
        for l, a in zip(body, addr):
            mm = re.search(r"s_(?:cbranch_\w+|branch)\s.*<[^+>]+\+0x([0-9a-f]+)>", l)
            if mm and a is not None:
                base = addr[0] - int(re.search(r"\+0x([0-9a-f]+)>", body[0]).group(1), 16) if "+0x" in body[0] else None
                tgt = int(mm.group(1), 16) + (base or 0)
                if tgt < a:
                    loops.append((tgt, a))
        total = 0
        for l, a in zip(body, addr):
            op = l.split()[0] if l.strip() else ""
            if op.startswith("scratch_") and a is not None:
                inner = [lp for lp in loops if lp[0] <= a <= lp[1]]
                span = min((lp[1] - lp[0] for lp in inner), default=None)
                total += 1
                print("  %06X %-26s innermost loop %s" % (a, op, "%d bytes" % span if span else "-"))
        print("  %d scratch instructions; %d loops" % (total, len(loops)))
        # where the phases sit: the physics substep (DPP reductions = the PGS, ds_bpermute = row couplings, LDS
        # traffic) vs lane 0's float64 env logic (v_*_f64), per 4 KB of code, with the scratch instructions in each
        print("  per 4 KB of code: instructions, DPP, ds_bpermute, LDS, f64 VALU, scratch")
        bins = {}
        for l, a in zip(body, addr):
            if a is None:
                continue
            d = bins.setdefault(a // 0x1000, [0, 0, 0, 0, 0, 0])
            d[0] += 1
            d[1] += ("row_" in l or "quad_perm" in l)
            d[2] += "ds_bpermute" in l
            d[3] += bool(re.match(r"\s+ds_", l))
            d[4] += "_f64" in l
            d[5] += "scratch_" in l
        for b in sorted(bins):
            print("  %06X %5d %4d %4d %4d %4d %3d" % ((b * 0x1000,) + tuple(bins[b])))
        return


if __name__ == "__main__":
    main()

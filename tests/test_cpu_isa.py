"""CPU check of the built gfx950 code objects (no GPU needed): no kernel of libhumenv.so uses a flat (generic-pointer)
memory instruction.

Round 3's MachineLICM build faulted with HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in the fp64 cooperative kernel
(DESIGN.md section 4).  Its flat loads / stores - a value read from LDS or from global memory through ONE generic
pointer (the spilled-contact read in group_rows, the slow PGS path, the non-finite output row, the fused policy's
input row) - had their 64-bit addresses assembled inside divergent branches from registers the spill code had
reloaded, and an address beyond the legal range reached the memory system.  Every such access is now two
address-space-typed ones (HUM_LDS / HUM_GLOBAL); with no flat instruction left, the MachineLICM build passes the
faulting call and the fp64 tests (profiles/r04_licm_fault.txt).  This test keeps it that way."""
import os
import re
import struct
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "imitation-learning-rl_amd", "ilrl_amd", "_lib", "libhumenv.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path, target="gfx950"):
    """The device code objects of a HIP fat binary (clang offload bundles embedded in the shared library)."""
    data = open(path, "rb").read()
    out, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return out
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, idl = struct.unpack_from("<QQQ", data, p)
            ident = data[p + 24:p + 24 + idl].decode()
            p += 24 + idl
            if target in ident:
                out.append(data[i + off:i + off + size])
        pos = i + len(MAGIC)


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(OBJDUMP), reason="needs the built library")
def test_no_flat_memory_instructions(tmp_path):
    cos = code_objects(LIB)
    assert len(cos) >= 3   # humanoid_env.hip, group_f32.hip, group_f32_policy.hip (+ policy.hip)
    kernels, flat = 0, []
    for j, co in enumerate(cos):
        f = tmp_path / ("co_%d.o" % j)
        f.write_bytes(co)
        dis = subprocess.check_output([OBJDUMP, "-d", str(f)], text=True)
        fn = None
        for line in dis.splitlines():
            if line.endswith(">:"):
                fn = line.split("<")[-1][:-2]
                kernels += "step_group_kernel" in fn
            elif re.match(r"\s+flat_\w+", line):
                flat.append((fn, line.strip()[:80]))
    assert kernels >= 8
    assert not flat, "flat (generic-pointer) memory instructions: %s" % flat[:5]


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(OBJDUMP), reason="needs the built library")
def test_env_specialised_fp32_kernels_present(tmp_path):
    """The fp32, 4-envs-per-block plane kernels are env-specialised: POLICY 1 (hum_rollout_fused),
    2 (hum_hier_rollout_fused), 3 (hum_step_k, low-level env: the benchmarked kernel), 4 (hum_step_k, hierarchical
    env); the generic POLICY 0 instantiation of that shape is no longer built (its launch paths moved to the twins)."""
    names = set()
    for j, co in enumerate(code_objects(LIB)):
        f = tmp_path / ("co_%d.o" % j)
        f.write_bytes(co)
        dis = subprocess.check_output([OBJDUMP, "-d", str(f)], text=True)
        names |= {line.split("<")[-1][:-2] for line in dis.splitlines() if line.endswith(">:")}
    pre = "_ZN3hkk17step_group_kernelIfLi4ELb0EL"
    for pol in (1, 2, 3, 4):
        assert "%si%dEEEvNS_5KArgsE" % (pre, pol) in names, "POLICY %d fp32 kernel missing" % pol
    assert "%si0EEEvNS_5KArgsE" % pre not in names

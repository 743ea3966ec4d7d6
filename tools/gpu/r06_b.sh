#!/bin/bash
# Round 6: the heightfield ridge contacts (capsule bodies across convex terrain edges) on the GPU, and the plane
# kernels bitwise unchanged by the larger contact capacity (the round-5 library as the A build).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_terrain.py > $O/pytest_terrain.log 2>&1 || { tail -30 $O/pytest_terrain.log; exit 3; }
grep -E "passed|failed|ridge lanes|state max" $O/pytest_terrain.log | tail -12
L=imitation-learning-rl_amd/ilrl_amd/_lib
timeout -k 10 300 env ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_base.so python3 tools/diag_lib_bitwise.py dump $O/base.npz > $O/dump_base.log 2>&1 || { tail -5 $O/dump_base.log; exit 4; }
timeout -k 10 300 python3 tools/diag_lib_bitwise.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -5 $O/dump_new.log; exit 5; }
python3 tools/diag_lib_bitwise.py cmp $O/base.npz $O/new.npz | tail -5
rm -f $O/base.npz $O/new.npz
B="--cpu-seconds 0 --no-secondary"
timeout -k 10 300 python3 bench.py $B > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 6; }
echo "bench_c2: $(grep '^{' $O/bench_c2.log | tail -1 | cut -c1-120)"

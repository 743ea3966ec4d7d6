#!/bin/bash
# Round 6: terrain ridge tests (conditioned fp32 gate), plane kernels bitwise vs the round-5 library, the c2 line,
# the RLlib adapter lines (low, hier) before trimming, and the copy-engine overlap probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_terrain.py > $O/pytest_terrain.log 2>&1 || { grep -E "PASSED|FAILED|ridge|Error" $O/pytest_terrain.log | tail -30; exit 3; }
grep -E "passed|failed|ridge lanes" $O/pytest_terrain.log | tail -6
L=imitation-learning-rl_amd/ilrl_amd/_lib
timeout -k 10 300 env ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_base.so python3 tools/diag_lib_bitwise.py dump $O/base.npz > $O/dump_base.log 2>&1 || { tail -5 $O/dump_base.log; exit 4; }
timeout -k 10 300 python3 tools/diag_lib_bitwise.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -5 $O/dump_new.log; exit 5; }
python3 tools/diag_lib_bitwise.py cmp $O/base.npz $O/new.npz > $O/bitwise.txt 2>&1; tail -3 $O/bitwise.txt
rm -f $O/base.npz $O/new.npz
B="--cpu-seconds 0 --no-secondary"
timeout -k 10 300 python3 bench.py $B > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 6; }
echo "bench_c2: $(grep '^{' $O/bench_c2.log | tail -1 | cut -c1-100)"
timeout -k 10 300 python3 bench.py --adapter --steps 200 --warmup 20 > $O/adapter_low.log 2>&1 || { tail -5 $O/adapter_low.log; exit 7; }
timeout -k 10 300 python3 bench.py --adapter --hier --steps 200 --warmup 20 > $O/adapter_hier.log 2>&1 || { tail -5 $O/adapter_hier.log; exit 8; }
for f in adapter_low adapter_hier; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-200)"; done
timeout -k 10 200 python3 tools/micro/overlap.py > $O/overlap.json 2> $O/overlap.err || { tail -5 $O/overlap.err; exit 9; }
cat $O/overlap.json

#!/bin/bash
# Round 6: the SDMA fragment transport (DmaGather) through the multi-rank bench tests, the overlap probe with
# completion offsets, and the adapter lines after the GC pause.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 200 python3 tools/micro/overlap.py > $O/overlap.json 2> $O/overlap.err || { cat $O/overlap.json; tail -5 $O/overlap.err; exit 9; }
grep -v "^ " $O/overlap.json | head -5
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_bench_multirank.py -k dma > $O/pytest_dma.log 2>&1 || { grep -E "PASSED|FAILED|Error|bench line|assert" $O/pytest_dma.log | tail -30; exit 3; }
grep -E "passed|failed|bench line" $O/pytest_dma.log | tail -6
for r in 1; do
timeout -k 10 300 python3 bench.py --adapter --steps 200 --warmup 20 > $O/adapter_low_$r.log 2>&1 || { tail -5 $O/adapter_low_$r.log; exit 7; }
timeout -k 10 300 python3 bench.py --adapter --hier --steps 200 --warmup 20 > $O/adapter_hier_$r.log 2>&1 || { tail -5 $O/adapter_hier_$r.log; exit 8; }
done
for f in adapter_low_1 adapter_hier_1; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("%.3f M  %.3f ms/step" % (j["value"]/1e6, j["ms_per_step"]))')"; done
timeout -k 10 300 python3 bench.py --force-dist --gather-every 32 --transport dma --cpu-seconds 0 --no-secondary > $O/bench_dma1.log 2>&1 || { tail -5 $O/bench_dma1.log; exit 10; }
timeout -k 10 300 python3 bench.py --force-dist --gather-every 32 --transport collective --cpu-seconds 0 --no-secondary > $O/bench_coll1.log 2>&1 || { tail -5 $O/bench_coll1.log; exit 11; }
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --no-secondary > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 12; }
for f in bench_dma1 bench_coll1 bench_c2; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("%.3f M  %.4f ms/step" % (j["value"]/1e6, j["ms_per_step"]))')"; done

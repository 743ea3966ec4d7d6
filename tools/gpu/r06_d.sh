#!/bin/bash
# Round 6: the trimmed RLlib adapters (equality with the raw path, then their bench lines) and the overlap probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_adapter.py tests/test_gpu_hier.py tests/test_gpu_parity.py -k "adapter or base_env or vector or gym" > $O/pytest.log 2>&1 || { grep -E "PASSED|FAILED|Error|assert" $O/pytest.log | tail -30; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -3
for r in 1 2; do
timeout -k 10 300 python3 bench.py --adapter --steps 200 --warmup 20 > $O/adapter_low_$r.log 2>&1 || { tail -5 $O/adapter_low_$r.log; exit 7; }
timeout -k 10 300 python3 bench.py --adapter --hier --steps 200 --warmup 20 > $O/adapter_hier_$r.log 2>&1 || { tail -5 $O/adapter_hier_$r.log; exit 8; }
done
for f in adapter_low_1 adapter_low_2 adapter_hier_1 adapter_hier_2; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("%.3f M  %.3f ms/step" % (j["value"]/1e6, j["ms_per_step"]))')"; done
timeout -k 10 200 python3 tools/micro/overlap.py > $O/overlap.json 2> $O/overlap.err || { cat $O/overlap.json; tail -5 $O/overlap.err; exit 9; }
cat $O/overlap.json

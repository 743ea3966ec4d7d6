#!/bin/bash
# Round 6: per-launch chunked SDMA pulls + the drain launch - parity (multi-rank bitwise) and the driver-shape drain
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06tail2; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 700 python3 -u -m pytest tests/test_gpu_traj_pack.py tests/test_gpu_bench_multirank.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || grep -E "PASSED|FAILED|bench line" $O/pytest.log | cut -c1-260
B="--cpu-seconds 0 --no-secondary"
run() { n=$1; shift; timeout -k 10 200 python3 bench.py "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 5; }; echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M", round(d["ms_per_step"],4), "ms/step", d["config"]["launch_sizes"], (d.get("gather") or {}).get("transport"), (d.get("gather") or {}).get("drain_launch_steps"))')"; }
for r in 1 2; do
run s20_none_$r --steps 20 --warmup 5 $B
run s20_dma_$r --force-dist --gather-every 32 --transport dma --steps 20 --warmup 5 $B
done
run s1000_dma --force-dist --gather-every 32 --transport dma $B
run s1000_none $B

#!/bin/bash
# Round 6: the chunked SDMA gather - pack tests, hier gather run, driver-shape and long-run lines (x3)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06tail4; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_traj_pack.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-seconds 0 --no-secondary"
run() { n=$1; shift; timeout -k 10 200 python3 bench.py "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 5; }; grep '^{' $O/$n.log | tail -1 > $O/$n.jsonl; echo "$n: $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read()); print(round(d["value"]/1e6,3), "M", round(d["ms_per_step"],4), "ms/step", d["config"]["launch_sizes"], (d.get("gather") or {}).get("transport"), (d.get("gather") or {}).get("drain_launch_steps"))' $O/$n.jsonl)"; }
run hier_dma20 --hier --force-dist --gather-every 32 --transport dma --steps 20 --warmup 5 $B
for r in 1 2 3; do
run fd_none20_$r --force-dist --gather-every 0 --steps 20 --warmup 5 $B
run dma20_$r --force-dist --gather-every 32 --transport dma --steps 20 --warmup 5 $B
run coll20_$r --force-dist --gather-every 32 --transport collective --steps 20 --warmup 5 $B
done
run dma1000 --force-dist --gather-every 32 --transport dma $B
run fd_none1000 --force-dist --gather-every 0 $B

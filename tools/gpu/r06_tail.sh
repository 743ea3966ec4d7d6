#!/bin/bash
# Round 6: the gather's drain at the driver's shape (--steps 20 --warmup 5: one timed launch, its fragment's pull exposed)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06tail; mkdir -p $O
B="--cpu-seconds 0 --no-secondary"
run() { n=$1; shift; timeout -k 10 200 python3 bench.py "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 5; }; echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M", round(d["ms_per_step"],4), "ms/step", d["config"]["launch_sizes"], (d.get("gather") or {}).get("transport"))')"; }
for r in 1 2; do
run s20_none_$r --steps 20 --warmup 5 $B
run s20_dma_$r --force-dist --gather-every 32 --transport dma --steps 20 --warmup 5 $B
run s20_coll_$r --force-dist --gather-every 32 --transport collective --steps 20 --warmup 5 $B
done
run s1000_dma --force-dist --gather-every 32 --transport dma $B

#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05shape; mkdir -p $O
B="--cpu-seconds 0 --no-secondary"
run() { tag=$1; shift; timeout -k 10 200 env "$@" > $O/$tag.log 2>&1 || { tail -3 $O/$tag.log; exit 3; }; echo "$tag: $(grep '^{' $O/$tag.log | tail -1 | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("%.2f M  %.4f ms  kernel %.4f" % (j["value"]/1e6, j["ms_per_step"], j["roofline"]["kernel_ms"]))')"; }
for r in 1 2; do
run s20w5_$r python3 bench.py --steps 20 --warmup 5 $B
run s20w100_$r python3 bench.py --steps 20 --warmup 100 $B
run s32w5_$r python3 bench.py --steps 32 --warmup 5 $B
run s320w5_$r python3 bench.py --steps 320 --warmup 5 $B
run s20w5_k20_$r python3 bench.py --steps 20 --warmup 5 --k 20 $B
done

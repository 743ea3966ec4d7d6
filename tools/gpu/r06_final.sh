#!/bin/bash
# Round 6 measurement pass on the committed build: all GPU tests + parity summaries, rocprofv3 kernel trace and
# FETCH/WRITE passes (launches of 32 env steps only), SQ counters, the default bench line with the CPU baseline
# (tools/gpu/measure.sh), the other configs (tools/gpu/configs.sh), the terrain line, config 5's closed loops, the
# low-level closed loops, the driver's short shape (--steps 20 --warmup 5) three times, the gather on both
# transports (one RCCL rank), the adapter lines, smoke.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu/measure.sh || exit $?
bash tools/gpu/configs.sh || exit $?
B="--cpu-seconds 0 --no-secondary"
run() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 3; }; }
run bench_terrain $B --terrain random
run bench_hier_policy --hier --policy $B
run bench_hier_policy_fused --hier --policy --fused $B
run bench_policy --policy $B
run bench_fused --policy --fused $B
for r in 1 2 3; do run bench_driver_$r --steps 20 --warmup 5 $B; done
run bench_gather_dma --force-dist --gather-every 32 --transport dma $B
run bench_gather_coll --force-dist --gather-every 32 --transport collective $B
run bench_adapter_low --adapter --steps 200 --warmup 20
run bench_adapter_hier --adapter --hier --steps 200 --warmup 20
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 7; }
for f in bench_terrain bench_hier_policy bench_hier_policy_fused bench_policy bench_fused bench_driver_1 bench_driver_2 bench_driver_3 bench_gather_dma bench_gather_coll bench_adapter_low bench_adapter_hier; do
  echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-150)"; done
echo final done

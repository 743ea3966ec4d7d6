#!/bin/bash
# Round 5 measurement pass on the committed build: GPU tests + parity summaries, rocprofv3 kernel trace and
# FETCH/WRITE passes (launches of 32 env steps only), SQ counters, the default bench line with the CPU baseline
# (tools/gpu/measure.sh), the other configs (tools/gpu/configs.sh), config 5's closed loop unfused and fused, the
# low-level closed loops, the driver's short shape (--steps 20 --warmup 5) three times, the RCCL gather line, smoke.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu/measure.sh || exit $?
bash tools/gpu/configs.sh || exit $?
B="--cpu-seconds 0 --no-secondary"
timeout -k 10 300 python3 bench.py --hier --policy $B > $O/bench_hier_policy.log 2>&1 || { tail -5 $O/bench_hier_policy.log; exit 3; }
timeout -k 10 300 python3 bench.py --hier --policy --fused $B > $O/bench_hier_policy_fused.log 2>&1 || { tail -5 $O/bench_hier_policy_fused.log; exit 3; }
timeout -k 10 300 python3 bench.py --policy $B > $O/bench_policy.log 2>&1 || { tail -5 $O/bench_policy.log; exit 3; }
timeout -k 10 300 python3 bench.py --policy --fused $B > $O/bench_fused.log 2>&1 || { tail -5 $O/bench_fused.log; exit 4; }
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $B > $O/bench_driver_$r.log 2>&1 || { tail -5 $O/bench_driver_$r.log; exit 5; }
done
timeout -k 10 300 python3 bench.py --force-dist --gather-every 32 $B > $O/bench_gather.log 2>&1 || { tail -5 $O/bench_gather.log; exit 6; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 7; }
for f in bench_hier_policy bench_hier_policy_fused bench_policy bench_fused bench_driver_1 bench_driver_2 bench_driver_3 bench_gather; do
  echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-150)"; done
echo final done

#!/bin/bash
# Round 4 measurement pass on the committed build: GPU tests + parity summaries, rocprofv3 kernel trace and
# FETCH/WRITE passes (launches of 32 env steps only), SQ counters, the default bench line
# with the CPU baseline (tools/gpu/measure.sh), then the other configs' lines, the closed loops and the driver's
# short shape (--steps 20 --warmup 5).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu/measure.sh || exit $?
bash tools/gpu/configs.sh || exit $?
timeout -k 10 300 python3 bench.py --policy --cpu-seconds 0 --no-secondary > gpurun_out/bench_policy.log 2>&1 || { tail -5 gpurun_out/bench_policy.log; exit 3; }
timeout -k 10 300 python3 bench.py --policy --fused --cpu-seconds 0 --no-secondary > gpurun_out/bench_fused.log 2>&1 || { tail -5 gpurun_out/bench_fused.log; exit 4; }
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-secondary > gpurun_out/bench_driver_$r.log 2>&1 || { tail -5 gpurun_out/bench_driver_$r.log; exit 5; }
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 6; }
for f in bench_policy bench_fused bench_driver_1 bench_driver_2 bench_driver_3; do echo "$f: $(tail -1 gpurun_out/$f.log | cut -c1-160)"; done
echo final done

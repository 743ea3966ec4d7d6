#!/bin/bash
# bench lines of the other BASELINE configs on the current build: 4 clips round-robin (config 3), hierarchical
# two-level rollout (config 5); the default line (config 2) comes from measure.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --clip all --cpu-seconds 0 > gpurun_out/bench_clipall.log 2>&1 || { tail -5 gpurun_out/bench_clipall.log; exit 1; }
tail -1 gpurun_out/bench_clipall.log | cut -c1-200
timeout -k 10 300 python3 bench.py --hier --cpu-seconds 0 > gpurun_out/bench_hier.log 2>&1 || { tail -5 gpurun_out/bench_hier.log; exit 1; }
tail -1 gpurun_out/bench_hier.log | cut -c1-200

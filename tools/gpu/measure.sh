#!/bin/bash
# Round measurement pass: GPU tests (parity summary -> profiles/), rocprofv3 kernel trace + FETCH/WRITE PMC
# passes + SQ counters on the default bench workload, then the default bench line (with the CPU baseline).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ILRL_PARITY_OUT=gpurun_out/parity timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
./tools/profile_gpu.sh > gpurun_out/profile.log 2>&1 || { tail -20 gpurun_out/profile.log; exit 1; }
./tools/gpu/pmc_sq.sh gpurun_out/sq || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
echo measure done

#!/bin/bash
# scratch-fix build: bench, sweep, rocprof kernel stats + FETCH/WRITE, SQ counters.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
./tools/sweep_gpu.sh || exit $?
./tools/profile_gpu.sh > gpurun_out/profile.log 2>&1 || exit $?
./tools/gpu/pmc_sq.sh gpurun_out/sq || exit $?
echo all done

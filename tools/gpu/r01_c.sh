#!/bin/bash
# full GPU tests + bench lines for configs 2, 3, 5 (+ parity summary for bench.py)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ILRL_PARITY_OUT=profiles timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
timeout -k 10 300 python3 bench.py --clip all --cpu-seconds 0 > gpurun_out/bench_allclips.log 2>&1 || exit $?
tail -1 gpurun_out/bench_allclips.log
timeout -k 10 300 python3 bench.py --hier --cpu-seconds 0 > gpurun_out/bench_hier.log 2>&1 || exit $?
tail -1 gpurun_out/bench_hier.log

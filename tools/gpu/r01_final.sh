#!/bin/bash
# round-1 measurement pass: GPU parity tests (+ parity summary), default bench, rocprof kernel trace + PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ILRL_PARITY_OUT=gpurun_out/parity timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x -s \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
./tools/profile_gpu.sh || exit $?

#!/bin/bash
# GPU test pass: all gpu-marked tests (stop at first failure), log under gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
exit $rc

#!/bin/bash
# Round-3 call after the fp64 cooperative-kernel fault: the fp64 kernel's tests first (one pytest process, stop at
# the first failure), then every gpu test, a same-box library A/B (LIBS / KS), and the measurement script.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest ${CANARY:-tests/test_gpu_hier.py} -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/canary.log 2>&1 || { tail -30 gpurun_out/canary.log; exit 1; }
tail -2 gpurun_out/canary.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -rf -s > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
if [ "${LIBS:-}" != "" ]; then
  bash tools/gpu/libab.sh > gpurun_out/libab.txt 2>&1 || { cat gpurun_out/libab.txt; exit 3; }
  cat gpurun_out/libab.txt
fi
if [ "${WLOG:-0}" = "1" ]; then
  bash tools/gpu/wave_log.sh > gpurun_out/wave_log_out.txt 2>&1 || { tail -20 gpurun_out/wave_log_out.txt; exit 4; }
  tail -30 gpurun_out/wave_log_out.txt
fi
TESTS=skip bash tools/gpu/r03_full.sh

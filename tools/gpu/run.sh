#!/bin/bash
# One GPU call: the gpu-marked tests (stop at the first failure), then a bench line.  Logs under gpurun_out/.
#   TESTS=...   pytest selection (default: tests)
#   BENCH=...   extra bench.py arguments ("skip" = no bench)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-tests}" != "skip" ]; then
  timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread -rf -s > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-}" != "skip" ]; then
  timeout -k 10 300 python3 -u bench.py ${BENCH:-} > gpurun_out/bench.jsonl 2> gpurun_out/bench.err
  rc=$?
  cat gpurun_out/bench.jsonl
  exit $rc
fi

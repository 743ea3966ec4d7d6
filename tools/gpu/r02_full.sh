#!/bin/bash
# Round-2 measurement call: gpu tests, the bench lines (configs 2, 3, 5), rocprofv3 kernel stats + PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
if [ "${TESTS:-tests}" != "skip" ]; then
  timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread -rf -s > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_c2.jsonl 2> gpurun_out/bench_c2.err || { cat gpurun_out/bench_c2.err | tail; exit 2; }
cat gpurun_out/bench_c2.jsonl
timeout -k 10 300 python3 -u bench.py --clip all --no-secondary --cpu-seconds 0 > gpurun_out/bench_c3.jsonl 2>&1 || exit 3
timeout -k 10 300 python3 -u bench.py --hier --cpu-seconds 0 > gpurun_out/bench_c5.jsonl 2>&1 || exit 4
tail -1 gpurun_out/bench_c3.jsonl; tail -1 gpurun_out/bench_c5.jsonl
if [ "${PROF:-1}" = "1" ]; then
  ARGS="--steps 100 --warmup 10 --cpu-seconds 0 --no-secondary"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_kt -o run -- python3 bench.py $ARGS > gpurun_out/prof_kt.log 2>&1 || exit 5
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/prof_fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof_fetch.log 2>&1 || exit 6
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/prof_write -o run -- python3 bench.py $ARGS > gpurun_out/prof_write.log 2>&1 || exit 7
fi
echo ALLDONE

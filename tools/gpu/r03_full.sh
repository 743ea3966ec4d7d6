#!/bin/bash
# Round-3 measurement call: gpu tests, bench lines (configs 2, 3, 5 at the default K and K=1), rocprofv3
# kernel stats of config 2 (fp32 and fp64) + FETCH_SIZE / WRITE_SIZE PMC passes.  Every GPU step has its own
# time limit and the steps are chained: the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
if [ "${TESTS:-tests}" != "skip" ]; then
  timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread -rf -s > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
[ "${BENCH:-1}" = "1" ] || exit 0
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_c2.jsonl 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 2; }
cat gpurun_out/bench_c2.jsonl
timeout -k 10 300 python3 -u bench.py --clip all --no-secondary --cpu-seconds 0 > gpurun_out/bench_c3.jsonl 2>&1 || exit 3
timeout -k 10 300 python3 -u bench.py --hier --cpu-seconds 0 > gpurun_out/bench_c5.jsonl 2>&1 || exit 4
timeout -k 10 300 python3 -u bench.py --policy --no-secondary --cpu-seconds 0 > gpurun_out/bench_policy.jsonl 2>&1 || exit 5
tail -1 gpurun_out/bench_c3.jsonl; tail -1 gpurun_out/bench_c5.jsonl; tail -1 gpurun_out/bench_policy.jsonl
if [ "${PROF:-1}" = "1" ]; then
  ARGS="--steps 96 --warmup 16 --cpu-seconds 0 --no-secondary"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_kt -o run -- python3 bench.py $ARGS > gpurun_out/prof_kt.log 2>&1 || exit 6
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_kt64 -o run -- python3 bench.py $ARGS --precision fp64 > gpurun_out/prof_kt64.log 2>&1 || exit 7
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/prof_fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof_fetch.log 2>&1 || exit 8
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/prof_write -o run -- python3 bench.py $ARGS > gpurun_out/prof_write.log 2>&1 || exit 9
fi
[ "${CALIB:-1}" = "1" ] && { bash tools/gpu/fetch_calib.sh > gpurun_out/calib.log 2>&1 || exit 10; cat gpurun_out/calib.log; }
echo ALLDONE

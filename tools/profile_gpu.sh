#!/bin/bash
# rocprofv3 kernel-trace/stats pass + separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the bench workload.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
# only whole launches of k = 32 env steps (the bench default) and no secondary legs (their k = 1 launches would be
# averaged in): per-launch figures then divide by 32
ARGS="--steps ${STEPS:-64} --warmup ${WARMUP:-32} --cpu-seconds 0 --no-secondary ${EXTRA:-}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_kt -o run -- python3 bench.py $ARGS > gpurun_out/prof_kt.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/prof_fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/prof_write -o run -- python3 bench.py $ARGS > gpurun_out/prof_write.log 2>&1 || exit $?
find gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write -type f | head -50
echo done

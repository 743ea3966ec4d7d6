#!/bin/bash
# envs-per-block sweep of the cooperative kernel (+ GPU parity tests on the default).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
run() { timeout -k 10 120 python3 bench.py --steps ${STEPS:-100} --warmup 10 --cpu-seconds 0 "$@" 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-60s %10.0f steps/s %8.3f ms' % (' '.join(sys.argv[1:]), d['value'], d['ms_per_step']))" "$@" ; }
{
for e in 4 2 1; do
run --phys envs_per_block=$e
run --phys envs_per_block=$e --lanes 16384
done
} > gpurun_out/epb_sweep.log 2>&1
cat gpurun_out/epb_sweep.log

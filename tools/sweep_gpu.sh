#!/bin/bash
# quick timing sweep of bench variants (diagnostics); $@ = extra variants file lines ignored
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() { timeout -k 10 120 python3 bench.py --steps ${STEPS:-30} --warmup 3 --cpu-seconds 0 "$@" 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-60s %10.0f steps/s %8.3f ms' % (' '.join(sys.argv[1:]), d['value'], d['ms_per_step']))" "$@" ; }
{
run
run --phys kernel=0
run --phys self_collision=0
run --phys max_contacts=0
run --phys solver_iters=0
run --precision fp64
run --lanes 16384
run --lanes 65536
} > gpurun_out/sweep.log 2>&1
cat gpurun_out/sweep.log

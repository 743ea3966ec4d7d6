#!/bin/bash
# experiment loop: phase breakdown (diag lib) + bench of the fast lib (fp32 cooperative kernel only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for f in $L/libhumenv_diag*.so; do
  echo "== $(basename $f)"
  ILRL_AMD_LIB=$f timeout -k 10 120 python3 tools/phase_timing.py 4096 > gpurun_out/phase.log 2>&1 || { cat gpurun_out/phase.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/phase.log
done
ILRL_AMD_LIB=$L/libhumenv_fast.so timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_fast.log 2>&1 || { tail -5 gpurun_out/bench_fast.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_fast.log').read().strip().splitlines()[-1]); print('bench fast: %.0f steps/s %.4f ms' % (d['value'], d['ms_per_step']))"

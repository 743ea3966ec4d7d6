#!/bin/bash
# A/B throughput of experiment libraries: bench each libhumenv_{fast,v*}.so, two alternating passes
cd "$GRAFT_REPO_ROOT" || exit 1
shopt -s nullglob
mkdir -p gpurun_out
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for pass in 1 2; do
  for f in $L/libhumenv_fast.so $L/libhumenv_v*.so; do
    ILRL_AMD_LIB=$f timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('%-24s %.0f steps/s %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" $(basename $f)
  done
done

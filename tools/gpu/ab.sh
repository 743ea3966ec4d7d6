#!/bin/bash
# A/B bench of experiment libraries (fp32 cooperative kernel only): LIBS="name1 name2 ..." -> _lib/libhumenv_<name>.so;
# EXTRA = bench args for every library, EXTRA_<name> = extra args for one (e.g. EXTRA_e2w2="--phys envs_per_block=2")
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for rep in 1 2; do
for n in ${LIBS}; do
  v="EXTRA_$n"
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_$n.so timeout -k 10 120 python3 bench.py --steps ${STEPS:-1000} --warmup 100 --cpu-seconds 0 --no-secondary ${EXTRA:-} ${!v:-} > gpurun_out/ab_$n.log 2>&1 || { tail -5 gpurun_out/ab_$n.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$n.log').read().strip().splitlines()[-1]); print('%-10s %.3fM env-steps/s  kernel %.4f ms  flags %d' % ('$n', d['value']/1e6, d['roofline']['kernel_ms'], d['error_flags']))"
done
done

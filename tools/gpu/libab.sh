#!/bin/bash
# A/B of kernel libraries x env steps per launch on one box: LIBS="default old ..." (default = libhumenv.so,
# NAME = _lib/libhumenv_NAME.so), KS="1 8"; one short bench line each (1000 env steps after 100 warm-up)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for rep in $(seq ${REPS:-1}); do
for n in ${LIBS:-default}; do
  for k in ${KS:-1 8}; do
    lib=$L/libhumenv_$n.so; [ "$n" = default ] && lib=$L/libhumenv.so
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --k $k --steps ${STEPS:-1024} --warmup 96 --cpu-seconds 0 --no-secondary ${EXTRA:-} > gpurun_out/ab_${n}_k$k.log 2>&1 || { tail -5 gpurun_out/ab_${n}_k$k.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_${n}_k$k.log').read().strip().splitlines()[-1]); print('%-8s k=%-3d %.3fM env-steps/s  kernel/step %.4f ms  flags %d' % ('$n', $k, d['value']/1e6, d['roofline']['kernel_ms'], d['error_flags']))"
  done
done
done

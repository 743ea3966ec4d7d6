#!/bin/bash
# policy GPU tests, then closed-loop bench (bench.py --policy) for each library in LIBS ("main" = the shipped one)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_policy.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_policy.log 2>&1 || { tail -30 gpurun_out/pytest_policy.log; exit 1; }
tail -2 gpurun_out/pytest_policy.log
for n in ${LIBS:-main}; do
  lib=$L/libhumenv_$n.so; [ "$n" = main ] && lib=$L/libhumenv.so
  ILRL_AMD_LIB=$lib timeout -k 10 180 python3 bench.py --policy --steps ${STEPS:-1000} --warmup 100 --cpu-seconds 0 --no-secondary > gpurun_out/pab_$n.log 2>&1 || { tail -5 gpurun_out/pab_$n.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/pab_$n.log').read().strip().splitlines()[-1]); print('%-8s %.3fM env-steps/s  %.4f ms/step' % ('$n', d['value']/1e6, d['ms_per_step']))"
done

#!/bin/bash
# per-block wave log of the cooperative kernel (diagnostic build libhumenv_wlog.so, tools/wave_log.py) for each K in
# $KS (env steps per launch, default "1 8")
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for k in ${KS:-1 8}; do
  echo "=== K = $k"
  ILRL_AMD_LIB=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib/libhumenv_wlog.so timeout -k 10 120 python3 tools/wave_log.py 4096 $k > gpurun_out/wave_log_k$k.log 2>&1 || { tail -5 gpurun_out/wave_log_k$k.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/wave_log_k$k.log | sed -n '/^mean duration/,$p'
done

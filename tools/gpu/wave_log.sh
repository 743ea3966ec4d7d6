#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ILRL_AMD_LIB=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib/libhumenv_wlog.so timeout -k 10 120 python3 tools/wave_log.py 4096 > gpurun_out/wave_log.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/wave_log.log; exit $rc

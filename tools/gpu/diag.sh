#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ILRL_AMD_LIB=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib/libhumenv_diag.so timeout -k 10 300 python tools/phase_timing.py 4096 > gpurun_out/phase.log 2>&1
echo rc=$?
cat gpurun_out/phase.log

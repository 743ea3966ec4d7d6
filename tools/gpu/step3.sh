#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
./tools/sweep_gpu.sh || exit $?
ILRL_AMD_LIB=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib/libhumenv_diag.so timeout -k 10 300 python tools/phase_timing.py 4096 > gpurun_out/phase.log 2>&1 || exit $?
cat gpurun_out/phase.log

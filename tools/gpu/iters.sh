#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for f in ${LIBS:-libhumenv_fast.so libhumenv_vold.so}; do
  ILRL_AMD_LIB=$L/$f timeout -k 10 120 python3 tools/iters_sweep.py 2>&1 | grep -v amdgpu.ids || exit 1
done

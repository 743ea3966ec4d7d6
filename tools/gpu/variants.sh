#!/bin/bash
# run tools/diag_phys2.py against each variant library in _lib/ (name pattern libhumenv_v*.so) + fast
cd "$GRAFT_REPO_ROOT" || exit 1
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for f in $L/libhumenv_fast.so $L/libhumenv_v*.so; do
  ILRL_AMD_LIB=$f timeout -k 10 120 python3 tools/diag_phys2.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done

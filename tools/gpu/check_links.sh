#!/bin/bash
# the wave_log workload on the fast library, then on the link-check library
cd "$GRAFT_REPO_ROOT" || exit 1
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for f in libhumenv_chk.so libhumenv_fast.so; do
  echo "== $f"
  ILRL_AMD_LIB=$L/$f timeout -k 10 120 python3 tools/check_links.py 4096 40 2>&1 | grep -v amdgpu.ids || exit 1
done

#!/bin/bash
# Round 5: wave logs (per-phase cycles per block-step, tools/wave_log.py) of two diagnostic builds at K env steps per
# launch: libhumenv_wlog.so (this source) and libhumenv_${B:-wlogvel}.so.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05w}
mkdir -p $O
for v in wlog ${B:-wlogvel}; do
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib/libhumenv_$v.so timeout -k 10 150 python3 tools/wave_log.py 4096 ${K:-32} > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  echo "=== $v"; grep -v amdgpu.ids $O/$v.log | sed -n '/^mean duration/,$p' | head -40
done

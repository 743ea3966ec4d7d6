#!/bin/bash
# Round 4: wave-log A/B (tools/wave_log.py, diagnostic builds -DHUM_WAVE_LOG) of the libraries in WLIBS
# (ilrl_amd/_lib/libhumenv_<name>.so), K = 32 env steps per launch, then the bench A/B of LIBS (tools/gpu/r04_ab.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04wl}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
for v in ${WLIBS:-wlogbase wlog}; do
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_$v.so timeout -k 10 120 python3 tools/wave_log.py 4096 32 > $O/wave_log_$v.log 2>&1 || { tail -5 $O/wave_log_$v.log; exit 1; }
  echo "=== $v"; grep -v amdgpu.ids $O/wave_log_$v.log | sed -n '/^mean duration/,$p'
  if [ -n "$EARLY_TOO" ]; then
    EARLY=1 ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_$v.so timeout -k 10 200 python3 tools/wave_log.py 4096 20 > $O/wave_log_early_$v.log 2>&1 || { tail -5 $O/wave_log_early_$v.log; exit 1; }
    echo "=== $v early (fresh reset, 5 warm-up steps, one 20-step launch)"; grep -v amdgpu.ids $O/wave_log_early_$v.log | sed -n '/^mean duration/,$p'
  fi
done
[ -n "$NO_BENCH" ] || SKIP_TESTS=1 TAG=${TAG:-r04wl} bash tools/gpu/r04_ab.sh

#!/bin/bash
# Round 4 iteration: GPU tests with the default library, same-box bench A/B (tools/gpu/r04_ab.sh), then the
# wave logs (steady and early) of the diagnostic builds in WLIBS.
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04it}
TAG=$T bash tools/gpu/r04_ab.sh || exit $?
[ -n "$WLIBS" ] && { NO_BENCH=1 EARLY_TOO=${EARLY_TOO:-1} TAG=$T bash tools/gpu/r04_wlog_ab.sh || exit $?; }
if [ -n "$FP32AB" ]; then
  LIBS="$FP32AB" timeout -k 10 900 python3 tools/diag_fp32_ab.py > gpurun_out/$T/fp32ab.log 2>&1 || { tail -5 gpurun_out/$T/fp32ab.log; exit 8; }
  grep -v amdgpu.ids gpurun_out/$T/fp32ab.log
fi
exit 0

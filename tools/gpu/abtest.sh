#!/bin/bash
# One call: a same-box A/B of kernel libraries (tools/gpu/libab.sh: LIBS, KS, REPS), then the gpu tests and the
# round's measurement script (tools/gpu/r03_full.sh, BENCH=0 to skip) on the default library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${LIBS:-}" != "" ]; then
  bash tools/gpu/libab.sh > gpurun_out/libab.txt 2>&1 || { cat gpurun_out/libab.txt; exit 1; }
  cat gpurun_out/libab.txt
fi
bash tools/gpu/r03_full.sh

#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_gpu.py motion08_03_l0 > gpurun_out/diag.log 2>&1
echo rc=$?

#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the step kernel's access widths (tools/micro/fetch_calib.hip); one
# counter per rocprofv3 pass; summary by tools/fetch_calib_summary.py
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/fetch -o run -- ./tools/micro/fetch_calib > gpurun_out/calib/fetch.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib/write -o run -- ./tools/micro/fetch_calib > gpurun_out/calib/write.log 2>&1 || exit 2
python3 tools/fetch_calib_summary.py gpurun_out/calib

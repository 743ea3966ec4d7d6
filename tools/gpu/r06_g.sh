#!/bin/bash
# Round 6: the DMA transport with its probe / agreement step (multi-rank bench tests, both transports).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_bench_multirank.py tests/test_gpu_traj_pack.py > $O/pytest.log 2>&1 || { grep -E "PASSED|FAILED|Error|assert" $O/pytest.log | tail -30; exit 3; }
grep -E "passed|failed|bench line" $O/pytest.log | cut -c1-220 | tail -8

#!/bin/bash
# Round 6: chunked SDMA gather (batched control receives, spin-then-block waits) - multi-rank bitwise + the drain
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06tail3; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_bench_multirank.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -k dma > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED|bench line" $O/pytest.log | cut -c1-200
bash tools/gpu/r06_trace.sh

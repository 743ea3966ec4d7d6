#!/bin/bash
# Round 4, parity pass: the fp32-yardstick scale tests, the fused-rollout / check-finite regressions, config 4's
# 8 x 4096 shape, then one default bench line.  Logs and per-config parity JSON under gpurun_out/r04/.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp ILRL_PARITY_OUT=$O
( while sleep 50; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python3 -u -m pytest ${TESTS:-tests/test_gpu_scale.py tests/test_gpu_policy.py tests/test_gpu_boundary.py tests/test_gpu_bench_multirank.py} \
    -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread -rf -s > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -40
# 0 = all passed, 1 = some failed (assertions): the GPU is fine, go on; anything else (crash, timeout): stop
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python3 -u bench.py ${BENCH:-} > $O/bench.jsonl 2> $O/bench.err || exit 3
cat $O/bench.jsonl
# config 5's closed loop: both levels' policies on the device (hum_hier_rollout)
timeout -k 10 300 python3 -u bench.py --hier --policy --steps 320 --warmup 32 > $O/bench_c5_policy.jsonl 2> $O/bench_c5_policy.err || exit 4
cat $O/bench_c5_policy.jsonl
exit $rc

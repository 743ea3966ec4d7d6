#!/bin/bash
# env steps per launch sweep (hum_step_k): bench lines for each K in $KS (default "1 4 8 16 32") after the gpu tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-tests}" != "skip" ]; then
  timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
[ "${KS:-}" = skip ] && exit 0
for k in ${KS:-1 4 8 16 32}; do
  timeout -k 10 200 python3 -u bench.py --k $k --no-secondary --cpu-seconds 0 ${EXTRA:-} > gpurun_out/k$k.jsonl 2> gpurun_out/k$k.err || { tail -5 gpurun_out/k$k.err; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/k$k.jsonl').read().strip().splitlines()[-1]); print('k=%-3d %.3fM env-steps/s  kernel/step %.4f ms  wall/step %.4f ms flags %d' % ($k, d['value']/1e6, d['roofline']['kernel_ms'], d['ms_per_step'], d['error_flags']))"
done

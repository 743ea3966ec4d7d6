#!/bin/bash
# Round 5: the fused two-level rollout (hum_hier_rollout_fused) - policy tests, then config 5 closed-loop bench lines,
# unfused vs fused interleaved (REPS rounds), and the default config-2 line as a control.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05hf}
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_policy.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_policy.log 2>&1
  rc=$?; tail -25 $O/pytest_policy.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python3 bench.py --hier --policy --k 32 --cpu-seconds 0 --no-secondary > $O/hier_unfused_$r.jsonl 2>>$O/bench.err || { tail -5 $O/bench.err; exit 7; }
  timeout -k 10 300 python3 bench.py --hier --policy --fused --k 32 --cpu-seconds 0 --no-secondary > $O/hier_fused_$r.jsonl 2>>$O/bench.err || { tail -5 $O/bench.err; exit 7; }
done
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --no-secondary > $O/default.jsonl 2>>$O/bench.err || { tail -5 $O/bench.err; exit 7; }
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/*.jsonl')):
    j = json.loads([x for x in open(f) if x.startswith('{')][-1])
    print('%-22s %.2f M/s  ms/step %.4f  kernel_ms %.4f' % (f.split('/')[-1], j['value'] / 1e6, j['ms_per_step'], j['roofline']['kernel_ms']))
" | tee $O/summary.txt

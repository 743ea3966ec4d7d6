#!/bin/bash
# Round 5: the trajectory gather on the RCCL code path (one rank, --force-dist: RCCL refuses two ranks on one device)
# against the same run without it, REPS rounds interleaved; then the multi-rank bench tests.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05g}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 ${REPS:-3}); do
  for g in 0 32; do
    timeout -k 10 200 python3 bench.py --force-dist --gather-every $g --cpu-seconds 0 --no-secondary > $O/gather_${g}_$r.jsonl 2>>$O/gather.err || { tail -5 $O/gather.err; exit 7; }
  done
done
python3 -c "
import json,glob,collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('$O/gather_*_*.jsonl')):
    g = f.split('/')[-1].split('_')[1]; j = json.loads([x for x in open(f) if x.startswith('{')][-1]); d[g].append(j['value'] / 1e6)
for g, x in sorted(d.items()): print('gather-every %-3s %s  mean %.2f M env-steps/s' % (g, ' '.join('%.2f' % y for y in x), sum(x) / len(x)))
" | tee $O/gather_summary.txt
grep '^{' $O/gather_32_1.jsonl | tail -1 > $O/gather_line.json
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bench_multirank.py tests/test_gpu_multiproc.py -m gpu -q -p no:cacheprovider --timeout 580 --timeout-method thread -rf > $O/pytest_multirank.log 2>&1
  rc=$?
  tail -5 $O/pytest_multirank.log
  exit $rc
fi

#!/bin/bash
# Round 5: where the trajectory gather's cost goes (one rank, RCCL code path): none / pack only / gather only / both.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05gd}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 ${REPS:-2}); do
  for m in none pack comm full; do
    g=32; [ $m = none ] && g=0
    d=$m; [ $m = full ] && d=""
    ILRL_GATHER_DIAG=$d timeout -k 10 200 python3 bench.py --force-dist --gather-every $g --cpu-seconds 0 --no-secondary > $O/gd_${m}_$r.jsonl 2>>$O/gd.err || { tail -5 $O/gd.err; exit 7; }
  done
done
python3 -c "
import json,glob,collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('$O/gd_*_*.jsonl')):
    m = f.split('/')[-1].split('_')[1]; j = json.loads([x for x in open(f) if x.startswith('{')][-1]); d[m].append(j['value'] / 1e6)
for m, x in d.items(): print('%-5s %s  mean %.2f M env-steps/s' % (m, ' '.join('%.2f' % y for y in x), sum(x) / len(x)))
" | tee $O/gd_summary.txt

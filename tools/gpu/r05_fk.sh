#!/bin/bash
# Round 5: chain-parallel FK - bitwise A/B against the serial-FK build (both translation units), then same-box bench
# A/B (REPS interleaved), then the wave log of the new build if present.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05fk}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/diag_lib_bitwise.py dump $O/new.npz > $O/bit.log 2>&1 || { tail -5 $O/bit.log; exit 3; }
ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_${BASE:-fkser}.so timeout -k 10 200 python3 tools/diag_lib_bitwise.py dump $O/base.npz >> $O/bit.log 2>&1 || { tail -5 $O/bit.log; exit 4; }
python3 tools/diag_lib_bitwise.py cmp $O/base.npz $O/new.npz | tee $O/bitwise.txt | tail -8
rm -f $O/new.npz $O/base.npz
for r in $(seq 1 ${REPS:-3}); do
  for v in ${BASE:-fkser} new; do
    lib=$L/libhumenv.so; [ $v != new ] && lib=$L/libhumenv_$v.so
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-seconds 0 --no-secondary > $O/ab_${v}_$r.jsonl 2>>$O/ab.err || { tail -5 $O/ab.err; exit 7; }
  done
done
python3 -c "
import json,glob,collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('$O/ab_*_*.jsonl')):
    v = f.split('/')[-1][3:].rsplit('_', 1)[0]; j = json.loads([x for x in open(f) if x.startswith('{')][-1]); d[v].append(j['value'] / 1e6)
for v, x in sorted(d.items()): print('%-10s %s  mean %.2f M env-steps/s' % (v, ' '.join('%.2f' % y for y in x), sum(x) / len(x)))
" | tee $O/ab_summary.txt

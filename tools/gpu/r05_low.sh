#!/bin/bash
# Round 5: the low-level-only twin of the hot kernel (FK publish) - bitwise dumps of each build against HEAD's, then
# same-box bench A/B (REPS interleaved), then the kernel-level GPU tests with the default build
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05low}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
VARS=${VARS:-head new lowrt lownopub}
mkdir -p $O
export TMPDIR=/tmp
for v in $VARS; do
  lib=$L/libhumenv_$v.so; [ $v = new ] && lib=$L/libhumenv.so
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 tools/diag_lib_bitwise.py dump $O/$v.npz >> $O/bit.log 2>&1 || { tail -5 $O/bit.log; exit 3; }
done
BV=${VARS%% *}   # the first build is the bitwise reference
for v in $VARS; do echo "== $BV vs $v"; python3 tools/diag_lib_bitwise.py cmp $O/$BV.npz $O/$v.npz > $O/cmp_$v.txt; tail -1 $O/cmp_$v.txt; done
rm -f $O/*.npz
for r in $(seq 1 ${REPS:-3}); do
  for v in $VARS; do
    lib=$L/libhumenv_$v.so; [ $v = new ] && lib=$L/libhumenv.so
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
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hier.py tests/test_gpu_step_k.py tests/test_gpu_policy.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1
tail -4 $O/pytest.log

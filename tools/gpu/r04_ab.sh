#!/bin/bash
# Round 4 iteration: every GPU test with the default library, then a same-box A/B of bench.py (default config 2
# line, no secondary legs) over the libraries named in LIBS (ilrl_amd/_lib/libhumenv_<name>.so; "new" = the default
# libhumenv.so), REPS rounds interleaved.  TAG names the output directory.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ab}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp ILRL_PARITY_OUT=$O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread -rf \
      > $O/pytest_gpu.log 2>&1
  rc=$?
  tail -6 $O/pytest_gpu.log
  [ $rc -ne 0 ] && { echo "tests failed rc=$rc"; exit $rc; }
fi
export ILRL_AMD_AB=1
for r in $(seq 1 ${REPS:-2}); do
  for v in ${LIBS:-base new}; do
    lib=$L/libhumenv_$v.so; [ $v = new ] && lib=$L/libhumenv.so
    ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-seconds 0 --no-secondary ${BENCH:-} > $O/ab_${v}_$r.jsonl 2>>$O/ab.err || { tail -3 $O/ab.err; exit 7; }
  done
done
python3 -c "
import json,glob,collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('$O/ab_*_*.jsonl')):
    v = f.split('/')[-1][3:].rsplit('_', 1)[0]; d[v].append(json.load(open(f))['value'] / 1e6)
for v, x in d.items(): print('%-12s %s  mean %.2f M env-steps/s' % (v, ' '.join('%.2f' % y for y in x), sum(x) / len(x)))
" | tee $O/ab_summary.txt

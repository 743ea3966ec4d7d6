#!/bin/bash
# Round 5 iteration on one box: the GPU tests (every failure listed, parity summaries under $O), the fp32 per-lane
# accuracy A/B from identical states (tools/diag_fp32_ab.py over LIBS, 512 lanes) and a same-box bench A/B of the
# default config-2 line over LIBS (ilrl_amd/_lib/libhumenv_<name>.so; "new" = libhumenv.so), REPS rounds interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05a}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp ILRL_PARITY_OUT=$O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
      > $O/pytest_gpu.log 2>&1
  rc=$?
  tail -12 $O/pytest_gpu.log
  [ $rc -ne 0 ] && [ -z "$CONTINUE" ] && { echo "tests failed rc=$rc"; exit $rc; }
fi
export ILRL_AMD_AB=1
if [ -z "$SKIP_FP32AB" ]; then
  LIBS="${LIBS:-base new}" N=512 timeout -k 10 300 python3 tools/diag_fp32_ab.py > $O/fp32ab.txt 2>&1 || { tail -5 $O/fp32ab.txt; exit 8; }
  cp gpurun_out/fp32ab/fp32ab.json $O/ 2>/dev/null
  grep -E "==|ratio" $O/fp32ab.txt
fi
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
echo iter done

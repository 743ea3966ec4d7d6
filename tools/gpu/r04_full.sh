#!/bin/bash
# Round 4 validation: every GPU test, then same-box A/Bs (default vs round-3 library: bench default, --steps 20, the
# fused closed loop; MachineLICM on/off for the fp64 kernel), then a rocprofv3 kernel-stats pass of the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04d}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp ILRL_PARITY_OUT=$O
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread -rf \
    > $O/pytest_gpu.log 2>&1
rc=$?
tail -4 $O/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ -n "$SKIP_TESTS" ] || { timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 8; }; }
tail -1 $O/smoke.log
export ILRL_AMD_AB=1
# accuracy study: the same fp32 scale comparisons with correctly rounded rcp / sqrt / rsqrt
mkdir -p $O/exact
[ -n "$SKIP_TESTS" ] || ILRL_PARITY_OUT=$O/exact ILRL_AMD_LIB=$L/libhumenv_exact.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py \
    -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf -k "fp32" > $O/exact/pytest.log 2>&1
rc4=$?
tail -2 $O/exact/pytest.log
[ $rc4 -ne 0 ] && [ $rc4 -ne 1 ] && exit $rc4
for r in 1 2; do
  for v in prev new; do
    lib=$L/libhumenv.so; [ $v = prev ] && lib=$L/libhumenv_prev.so
    ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-seconds 0 --no-secondary > $O/ab_${v}_$r.jsonl 2>>$O/ab.err || exit 7
    ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --policy --fused --cpu-seconds 0 --no-secondary > $O/abpf_${v}_$r.jsonl 2>>$O/ab.err || exit 7
  done
  for v in licm nolicm; do
    lib=$L/libhumenv.so; [ $v = licm ] && lib=$L/libhumenv_licm.so
    ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --precision fp64 --steps 320 --warmup 32 --cpu-seconds 0 --no-secondary > $O/ab64_${v}_$r.jsonl 2>>$O/ab.err || exit 7
  done
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/ab*_*.jsonl')): print(f.split('/')[-1], '%.2f M' % (json.load(open(f))['value']/1e6))"
unset ILRL_AMD_AB
timeout -k 10 300 python3 -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit 9
cat $O/bench.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-seconds 0 --no-secondary > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 10; }
find $GRAFT_REPO_ROOT/$O/prof -name "*stats*" | head
exit $rc

#!/bin/bash
# Round 5: the hierarchical env's high-level transitions take the kernel's precomputed hinge sin / cos (no serial
# sin / cos on lane 0): bitwise dumps against the previous build, the hier / policy GPU tests, same-box A/B of the
# config-5 lines (REPS interleaved)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05hsc}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp
for v in prevhs new; do
  lib=$L/libhumenv_$v.so; [ $v = new ] && lib=$L/libhumenv.so
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 tools/diag_lib_bitwise.py dump $O/$v.npz >> $O/bit.log 2>&1 || { tail -5 $O/bit.log; exit 3; }
done
echo "bitwise prevhs vs new: $(python3 tools/diag_lib_bitwise.py cmp $O/prevhs.npz $O/new.npz | tee $O/cmp.txt | tail -1)"
rm -f $O/*.npz
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_policy.py tests/test_gpu_hier.py tests/test_gpu_scale.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head -5
grep -q " failed\| error" $O/pytest.log && exit 5
B="--cpu-seconds 0 --no-secondary"
for r in $(seq 1 ${REPS:-3}); do
  for v in prevhs new; do
    lib=$L/libhumenv_$v.so; [ $v = new ] && lib=$L/libhumenv.so
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --hier $B > $O/h_${v}_$r.jsonl 2>>$O/ab.err || { tail -5 $O/ab.err; exit 7; }
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --hier --policy --fused $B > $O/hpf_${v}_$r.jsonl 2>>$O/ab.err || { tail -5 $O/ab.err; exit 7; }
  done
done
python3 -c "
import json,glob,collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('$O/*_*_*.jsonl')):
    v = f.split('/')[-1].rsplit('_', 1)[0]; j = json.loads([x for x in open(f) if x.startswith('{')][-1]); d[v].append(j['value'] / 1e6)
for v, x in sorted(d.items()): print('%-12s %s  mean %.2f M env-steps/s' % (v, ' '.join('%.2f' % y for y in x), sum(x) / len(x)))
" | tee $O/ab_summary.txt

#!/bin/bash
# Round 5: env-specialised twins of the other hot kernels - the fused low-level policy kernel with the hierarchical code
# compiled out (p1low), the hierarchical env's kernel with the low-level-only branches compiled out (hieronly):
# bitwise dumps + the policy tests with each, then same-box A/B of the closed loops they serve
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05twins}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp
lib_of() { if [ $1 = new ]; then echo $L/libhumenv.so; else echo $L/libhumenv_$1.so; fi; }
for v in new p1low hieronly; do
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/diag_lib_bitwise.py dump $O/$v.npz >> $O/bit.log 2>&1 || { tail -5 $O/bit.log; exit 3; }
done
for v in p1low hieronly; do echo "== new vs $v: $(python3 tools/diag_lib_bitwise.py cmp $O/new.npz $O/$v.npz | tail -1)"; done
rm -f $O/*.npz
for v in p1low hieronly; do
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$(lib_of $v) timeout -k 10 300 python3 -u -m pytest tests/test_gpu_policy.py tests/test_gpu_hier.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/pytest_$v.log 2>&1; echo "tests $v: $(tail -1 $O/pytest_$v.log)"
done
B="--cpu-seconds 0 --no-secondary"
for r in $(seq 1 ${REPS:-3}); do
  for v in new p1low; do
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$(lib_of $v) timeout -k 10 200 python3 bench.py --policy --fused $B > $O/fused_${v}_$r.jsonl 2>>$O/ab.err || { tail -5 $O/ab.err; exit 7; }
  done
  for v in new hieronly; do
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$(lib_of $v) timeout -k 10 200 python3 bench.py --hier $B > $O/hier_${v}_$r.jsonl 2>>$O/ab.err || { tail -5 $O/ab.err; exit 8; }
  done
done
python3 -c "
import json,glob,collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('$O/*_*_*.jsonl')):
    v = f.split('/')[-1].rsplit('_', 1)[0]; j = json.loads([x for x in open(f) if x.startswith('{')][-1]); d[v].append(j['value'] / 1e6)
for v, x in sorted(d.items()): print('%-16s %s  mean %.2f M env-steps/s' % (v, ' '.join('%.2f' % y for y in x), sum(x) / len(x)))
" | tee $O/ab_summary.txt

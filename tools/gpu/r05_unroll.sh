#!/bin/bash
# Round 5: the policy networks' 256 x 256 layer unroll (HUM_PH2_UNROLL 8 / 16 shipped / 32): same-box A/B of the two
# fused closed loops, then the policy tests with the best variant named by BEST (optional)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05unr}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp
B="--cpu-seconds 0 --no-secondary"
for r in $(seq 1 ${REPS:-3}); do
  for v in new u8 u32; do
    lib=$L/libhumenv_$v.so; [ $v = new ] && lib=$L/libhumenv.so
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --policy --fused $B > $O/pf_${v}_$r.jsonl 2>>$O/ab.err || { tail -5 $O/ab.err; exit 7; }
    ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --hier --policy --fused $B > $O/hpf_${v}_$r.jsonl 2>>$O/ab.err || { tail -5 $O/ab.err; exit 7; }
  done
done
python3 -c "
import json,glob,collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('$O/*_*_*.jsonl')):
    v = f.split('/')[-1].rsplit('_', 1)[0]; j = json.loads([x for x in open(f) if x.startswith('{')][-1]); d[v].append(j['value'] / 1e6)
for v, x in sorted(d.items()): print('%-10s %s  mean %.2f M env-steps/s' % (v, ' '.join('%.2f' % y for y in x), sum(x) / len(x)))
" | tee $O/ab_summary.txt
for v in u8 u32; do
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_policy.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1; echo "policy tests $v: $(tail -1 $O/pytest_$v.log)"
done

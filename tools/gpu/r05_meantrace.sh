#!/bin/bash
# Round 5: the fused loops' policy-mean traces (ABI 13) - the GPU suite, then the SampleBatch closed-loop lines
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05mt}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head -5
grep -q " failed\| error" $O/pytest.log && exit 5
B="--cpu-seconds 0 --no-secondary"
for f in "--policy --fused" "--policy --fused --sample-batch" "--hier --policy --fused" "--hier --policy --fused --sample-batch"; do
  t=$(echo $f | tr -d ' -'); timeout -k 10 300 python3 bench.py $f $B > $O/$t.log 2>&1 || { tail -5 $O/$t.log; exit 6; }
  echo "$f: $(grep '^{' $O/$t.log | tail -1 | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("%.2f M  %.4f ms/step" % (j["value"]/1e6, j["ms_per_step"]))')"
done

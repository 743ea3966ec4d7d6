#!/bin/bash
# Round 5: the SampleBatch policy columns (action_dist_inputs, action_logp, vf_preds) - policy tests, then the fused
# closed loops with and without forming them per launch.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05m}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_policy.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for f in "--policy --fused" "--policy --fused --sample-batch" "--hier --policy --fused" "--hier --policy --fused --sample-batch"; do
  i=$((i+1))
  timeout -k 10 200 python3 bench.py $f --cpu-seconds 0 --no-secondary > $O/b$i.jsonl 2>>$O/bench.err || { tail -5 $O/bench.err; exit 9; }
  echo "$f: $(grep '^{' $O/b$i.jsonl | tail -1 | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(round(j['value']/1e6,2), 'M', round(j['ms_per_step'],4), 'ms/step')")"
done | tee $O/summary.txt

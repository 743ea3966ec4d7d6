#!/bin/bash
# Round 4: where does the driver's short run (--steps 20 --warmup 5: one 20-step launch from fresh resets) lose
# against the steady state?  Wave log (diagnostic build libhumenv_wlogbase.so) steady + early, then bench.py in
# both shapes with the shipped library.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04early}
mkdir -p $O
export TMPDIR=/tmp
NO_BENCH=1 WLIBS=${WLIBS:-wlogbase} EARLY_TOO=1 TAG=${TAG:-r04early} bash tools/gpu/r04_wlog_ab.sh || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-secondary > $O/bench_driver_$r.jsonl 2>>$O/bench.err || exit 7
  timeout -k 10 200 python3 bench.py --cpu-seconds 0 --no-secondary > $O/bench_default_$r.jsonl 2>>$O/bench.err || exit 7
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/bench_*.jsonl')):
    d = json.load(open(f)); print(f.split('/')[-1], '%.2f M' % (d['value'] / 1e6), d['config'].get('steps_per_launch'), d['steps'], d['warmup'])
"

#!/bin/bash
# Workload A/B on the current build: the default (Bullet split-impulse limits/contacts) vs every violation corrected
# at ERP (the round-2 model before the split-impulse change), plus the closed-loop policy line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A="--cpu-seconds 0 --no-secondary"
timeout -k 10 300 python3 -u bench.py $A > gpurun_out/ab_split.jsonl 2>gpurun_out/ab.err || exit 1
timeout -k 10 300 python3 -u bench.py $A --phys split_penetration=-1.0e30 > gpurun_out/ab_nosplit.jsonl 2>>gpurun_out/ab.err || exit 2
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --policy > gpurun_out/ab_policy.jsonl 2>>gpurun_out/ab.err || exit 3
for f in ab_split ab_nosplit ab_policy; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/$f.jsonl').read().strip().split('\n')[-1]); print('$f', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), 'ms', d['config']['physics_overrides'])"; done

#!/bin/bash
# Round 4, verdict item 6: is the fused closed loop (hum_rollout_fused) L2-bound on re-streaming the policy weights?
# rocprofv3 kernel trace + L2 / L1 counter passes (one counter group per pass) for the fused closed loop and for
# the env-only bench (same lanes, same k), summarised by tools/l2_summary.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04l2}
mkdir -p $O
A="--steps 64 --warmup 8 --cpu-seconds 0 --no-secondary"
for mode in fused env; do
  X=""; [ $mode = fused ] && X="--policy --fused"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$mode -o run -- python3 bench.py $A $X > $O/kt_$mode.log 2>&1 || { tail -5 $O/kt_$mode.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/hm_$mode -o run -- python3 bench.py $A $X > $O/hm_$mode.log 2>&1 || { tail -5 $O/hm_$mode.log; exit 2; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$mode -o run -- python3 bench.py $A $X > $O/fetch_$mode.log 2>&1 || { tail -5 $O/fetch_$mode.log; exit 5; }
  timeout -s KILL 200 rocprofv3 --pmc TCC_REQ_sum TCC_READ_sum -d $O/rq_$mode -o run -- python3 bench.py $A $X > $O/rq_$mode.log 2>&1 || { tail -5 $O/rq_$mode.log; exit 3; }
  timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $O/tcp_$mode -o run -- python3 bench.py $A $X > $O/tcp_$mode.log 2>&1 || { tail -5 $O/tcp_$mode.log; exit 4; }
done
python3 tools/l2_summary.py $O | tee $O/l2_summary.txt

#!/bin/bash
# Round 6 first pass: the re-gated full-size parity tests (config 3 at 1024 lanes, config 5 over its physics
# transitions), the trajectory-pack tests, and the driver-shape bench line twice plus the default line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
export ILRL_PARITY_OUT=$O/parity
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_traj_pack.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
B="--cpu-seconds 0 --no-secondary"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 $B > $O/bench_driver_$r.log 2>&1 || { tail -5 $O/bench_driver_$r.log; exit 4; }
done
timeout -k 10 300 python3 bench.py $B > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 5; }
for f in bench_driver_1 bench_driver_2 bench_c2; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-160)"; done

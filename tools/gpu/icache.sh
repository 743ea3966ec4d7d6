#!/bin/bash
# Instruction-cache counters (SQC) for experiment libraries: LIBS="a b" -> _lib/libhumenv_<name>.so
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ic
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for n in ${LIBS}; do
  ILRL_AMD_LIB=$L/libhumenv_$n.so timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
     -d gpurun_out/ic/$n -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-secondary > gpurun_out/ic/$n.log 2>&1 || { tail -5 gpurun_out/ic/$n.log; exit 1; }
  python3 - "$n" <<'PY'
import sqlite3, sys, glob
n = sys.argv[1]
db = glob.glob("gpurun_out/ic/%s/**/*.db" % n, recursive=True) or glob.glob("gpurun_out/ic/%s/*.db" % n)
c = sqlite3.connect(db[0])
rows = c.execute("select counter_name, avg(value), count(*) from counters_collection where kernel_name like 'step_group%' group by counter_name").fetchall()
print(n, {r[0]: round(r[1]) for r in rows})
PY
done

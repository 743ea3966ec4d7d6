#!/bin/bash
# SQ instruction/stall counters for the step kernel (each pass its own rocprofv3 run; no trace domains).
# usage: tools/gpu/pmc_sq.sh OUTDIR [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/sq}; shift
ARGS="--steps 64 --warmup 32 --cpu-seconds 0 --no-secondary $*"   # whole launches of k = 32 only
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
    -d "$OUT/p1" -o run -- python3 bench.py $ARGS > "$OUT/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -d "$OUT/p2" -o run -- python3 bench.py $ARGS > "$OUT/p2.log" 2>&1 || exit $?
echo pmc_sq done

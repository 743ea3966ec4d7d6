#!/bin/bash
# Round 5: per-phase VALU lane utilisation (tools/lane_util.py): counter calibration on the micro-benchmark, the saved
# benchmark state, then one SQ pass per stop-after-phase variant (each its own rocprofv3 run).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05lu}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES"
timeout -s KILL 60 rocprofv3 --pmc $C -d $O/calib -o run -- ./tools/micro/lane_util > $O/calib.log 2>&1 || { tail -5 $O/calib.log; exit 3; }
timeout -k 10 200 python3 tools/lane_util.py save $O/state.npz > $O/save.log 2>&1 || { tail -5 $O/save.log; exit 4; }
for v in ${VARIANTS:-lu0 lu1 lu2 lu3 lu4 lu5 lu6 lu7 lu8 lu9 luall}; do
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_$v.so timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$v -o run -- python3 tools/lane_util.py run $O/state.npz > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 5; }
  tail -1 $O/$v.log
done
rm -f $O/state.npz
python3 tools/lane_util.py dump $O && python3 tools/lane_util.py summary $O | tee $O/summary.txt

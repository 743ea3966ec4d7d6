#!/bin/bash
# Round 5: wave log with the rows phase split (HUM_SUBPHASE_ROWS build libhumenv_wlogrows.so)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05wr}
mkdir -p $O
ROWS_SUB=1 ILRL_AMD_AB=1 ILRL_AMD_LIB=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib/libhumenv_wlogrows.so timeout -k 10 150 python3 tools/wave_log.py 4096 ${K:-32} > $O/wlog.log 2>&1 || { tail -5 $O/wlog.log; exit 1; }
sed -n '/^mean duration/,$p' $O/wlog.log

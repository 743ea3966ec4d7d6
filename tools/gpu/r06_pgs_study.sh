#!/bin/bash
# Round 6: PGS stall attribution.  Wave logs (tools/wave_log.py, 4096 lanes, k = 32 steady
# state) of four timing-only builds: base; the 16-lane DPP reduction replaced by four dependent plain adds (nodpp);
# the row-ahead LDS loads replaced by register copies (noload); both.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06pgs; mkdir -p $O
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for v in base nodpp noload both base; do
  ILRL_AMD_LIB=$L/libhumenv_wlog_$v.so timeout -k 10 200 python3 tools/wave_log.py 4096 32 > $O/wlog_$v.log 2>&1 || { tail -5 $O/wlog_$v.log; exit 3; }
  echo "== $v"; grep -E "^mean duration|pgs cycles per unit|^  pgs |^  rows " $O/wlog_$v.log
done

#!/bin/bash
# Round 5: -ffp-contract=on for the hot translation units (con), and the FK publish on top (conpub): bitwise dumps
# against con, same-box A/B against the shipped build, the whole GPU suite with each variant
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05con}
mkdir -p $O
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
TAG=${TAG:-r05con} VARS="con new conpub" REPS=${REPS:-3} bash tools/gpu/r05_low.sh || exit $?
for v in con conpub; do
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_$v.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/suite_$v.log 2>&1
  echo "suite $v: $(tail -1 $O/suite_$v.log)"
  grep FAILED $O/suite_$v.log | head -5
done

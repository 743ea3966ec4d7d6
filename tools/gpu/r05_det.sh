#!/bin/bash
# Round 5: determinism check of two builds (each dumped twice) + the hier / step_k GPU tests with the default build
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r05det}
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 tools/diag_lib_bitwise.py dump $O/new$r.npz > $O/bit.log 2>&1 || { tail -5 $O/bit.log; exit 3; }
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_${BASE:-prevfk}.so timeout -k 10 200 python3 tools/diag_lib_bitwise.py dump $O/base$r.npz >> $O/bit.log 2>&1 || { tail -5 $O/bit.log; exit 4; }
done
echo "== new vs new"; python3 tools/diag_lib_bitwise.py cmp $O/new1.npz $O/new2.npz | tail -3
echo "== base vs base"; python3 tools/diag_lib_bitwise.py cmp $O/base1.npz $O/base2.npz | tail -3
echo "== base vs new"; python3 tools/diag_lib_bitwise.py cmp $O/base1.npz $O/new1.npz | tail -3
rm -f $O/*.npz
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hier.py tests/test_gpu_step_k.py tests/test_gpu_policy.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1
tail -5 $O/pytest.log

# Fused closed loop A/B on one box (profiles/r03f_policy_fused_ab.txt): parity of the fused rollout for the current
# build and a hand-built variant (libhumenv_pk.so: group_f32_policy.hip with the packed hidden layers), then
# bench --policy --fused for the current build, the variant and the previous build (libhumenv_prev.so), alternating.
mkdir -p gpurun_out/pf
L=imitation-learning-rl_amd/ilrl_amd/_lib
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_policy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pf/pytest.log 2>&1 && tail -1 gpurun_out/pf/pytest.log &&
ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_pk.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_policy.py -x -q --timeout 120 --timeout-method thread -k fused > gpurun_out/pf/pytest_pk.log 2>&1 && tail -1 gpurun_out/pf/pytest_pk.log || exit 4
for r in 1 2; do
 for v in new pk prev; do
  lib=$L/libhumenv.so; [ $v = pk ] && lib=$L/libhumenv_pk.so; [ $v = prev ] && lib=$L/libhumenv_prev.so
  ILRL_AMD_AB=1 ILRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --policy --fused --cpu-seconds 0 --no-secondary > gpurun_out/pf/${v}_fused_$r.jsonl 2>>gpurun_out/pf/err || exit 5
 done
done
timeout -k 10 200 python3 bench.py --cpu-seconds 0 --no-secondary > gpurun_out/pf/new_c2.jsonl 2>>gpurun_out/pf/err && echo PFDONE

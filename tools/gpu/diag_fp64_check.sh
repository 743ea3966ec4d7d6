mkdir -p gpurun_out
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
run() { timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -s -k "fp32-c2" > gpurun_out/scale_$1.log 2>&1; echo "== $1 rc=$?"; grep -E "^c[0-9]_" gpurun_out/scale_$1.log | python3 -c "import sys,json; [print({k: v for k, v in json.loads(l.split(' ',1)[1]).items() if k in ('fp64_kernel_same_state','fp64_worst_lanes')}) for l in sys.stdin]"; }
ILRL_FP64_CHECK_KERNEL=1 run default_k1 && ILRL_FP64_CHECK_KERNEL=0 run default_k0 && ILRL_AMD_AB=1 ILRL_AMD_LIB=$L/libhumenv_prev.so ILRL_FP64_CHECK_KERNEL=1 run prev_k1

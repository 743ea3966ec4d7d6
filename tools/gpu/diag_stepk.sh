# step_k per-lane kernel case under three builds: base (HEAD, MachineLICM on), prev (HEAD sources, LICM off), default
mkdir -p gpurun_out
L=$PWD/imitation-learning-rl_amd/ilrl_amd/_lib
for lib in base prev default; do
  f=$L/libhumenv_$lib.so; [ $lib = default ] && f=$L/libhumenv.so
  ILRL_AMD_LIB=$f timeout -k 10 120 python3 -u -m pytest "tests/test_gpu_step_k.py::test_step_k_equals_k_steps[kernel=0-precision=fp32]" -m gpu -q -p no:cacheprovider --timeout 100 --timeout-method thread > gpurun_out/stepk_$lib.log 2>&1
  echo "$lib rc=$? $(tail -1 gpurun_out/stepk_$lib.log)"
done

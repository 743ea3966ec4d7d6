#!/bin/bash
# Wave-log diagnostic library with extra flags (tools/wave_log.py with ILRL_AMD_LIB=...): the fp32 cooperative kernel
# of humanoid_env.hip with -DHUM_WAVE_LOG -DHUM_SUBPHASE, plus the given flags (e.g. the PGS stall-study switches).
# usage: tools/build_wlog_variant.sh NAME "hipcc flags" -> ilrl_amd/_lib/libhumenv_wlog_NAME.so
set -e
NAME=$1; shift
FLAGS="$*"
C=$(cd "$(dirname "$0")/../imitation-learning-rl_amd/csrc" && pwd)
make -s -C "$C" all >/dev/null
B=$C/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -disable-machine-licm \
    -ffp-contract=on -DHUM_WAVE_LOG -DHUM_SUBPHASE -DHUM_DIAG_F32_ONLY -DHUM_MAXR_LDS=29 $FLAGS -c -o $B/wlog_$NAME.o $C/humanoid_env.hip
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $C/../ilrl_amd/_lib/libhumenv_wlog_$NAME.so \
    $B/wlog_$NAME.o $B/clip_csv.o $B/policy.o $B/traj_pack.o $B/frag_dma.o -L/opt/rocm/lib -lhsa-runtime64
echo built libhumenv_wlog_$NAME.so

#!/bin/bash
# Experiment library: the shipped objects with the benchmarked kernel (group_f32_low.hip) recompiled with extra
# flags (after the Makefile's HOTFLAGS; HOTFLAGS= to drop them).  usage: tools/build_variant.sh NAME "hipcc flags" -> ilrl_amd/_lib/libhumenv_NAME.so (tools/gpu/ab.sh)
set -e
NAME=$1; shift
FLAGS="$*"
C=$(cd "$(dirname "$0")/../imitation-learning-rl_amd/csrc" && pwd)
make -s -C "$C" all >/dev/null
B=$C/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function ${HOTFLAGS--mllvm -amdgpu-sched-strategy=iterative-ilp -fno-slp-vectorize -mllvm -disable-machine-licm} $FLAGS -c -o $B/gf32_$NAME.o $C/group_f32_low.hip
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $C/../ilrl_amd/_lib/libhumenv_$NAME.so \
    $B/humanoid_env.o $B/group_f32.o $B/gf32_$NAME.o $B/group_f32_policy.o $B/group_f32_hier_policy.o $B/clip_csv.o $B/policy.o $B/traj_pack.o $B/frag_dma.o -L/opt/rocm/lib -lhsa-runtime64
echo built libhumenv_$NAME.so

#!/bin/bash
# Round 6: the chunked SDMA gather's timeline at the driver's shape (ILRL_DMA_TRACE=1), engine split variants
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06trace; mkdir -p $O
B="--steps 20 --warmup 5 --cpu-seconds 0 --no-secondary"
for r in 1 2; do
timeout -k 10 200 python3 bench.py --force-dist --gather-every 0 $B > $O/fd_none_$r.log 2>&1 || { tail -5 $O/fd_none_$r.log; exit 4; }
echo "fd_none_$r: $(grep '^{' $O/fd_none_$r.log | cut -c100-190)"
for sp in 1; do
ILRL_AMD_DMA_SPLIT=$sp ILRL_DMA_TRACE=1 timeout -k 10 200 python3 bench.py --force-dist --gather-every 32 --transport dma $B > $O/s20_sp${sp}_$r.log 2>&1 || { tail -5 $O/s20_sp${sp}_$r.log; exit 5; }
echo "split $sp: $(grep dma-trace $O/s20_sp${sp}_$r.log | cut -c1-600)"; echo "  $(grep '^{' $O/s20_sp${sp}_$r.log | cut -c100-190)"
done
done

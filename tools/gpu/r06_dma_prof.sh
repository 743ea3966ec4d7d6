#!/bin/bash
# Round 6: rocprofv3 kernel + memory-copy trace of the chunked SDMA gather (one rank, --force-dist, 96 steps)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06dmaprof; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --force-dist --gather-every 32 --transport dma --steps 96 --warmup 8 --cpu-seconds 0 --no-secondary > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log | cut -c1-200
find $O/trace -name "*.csv" | head -20

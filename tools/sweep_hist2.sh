#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out
for m in 0 1 2; do
  r=$(HUFF_HIST_EXPERIMENT=$m timeout -k 10 120 python tools/kbench.py --phase hist --workload uniform --iters 20); echo "m=$m $r"
done > gpurun_out/hist_sweep2.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof/hist1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --phase hist --workload uniform --iters 10 > /dev/null 2>&1

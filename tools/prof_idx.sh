#!/usr/bin/env bash
set -euo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/prof/idx -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload zipf --iters 3 > $root/gpurun_out/prof/idx.log 2>&1

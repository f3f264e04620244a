#!/usr/bin/env bash
# Kernel profile of the wide-letter path (tools/wbench.py) on the GPU box.
#   tools/prof_wide.sh <width> <tag>
set -euo pipefail
w=${1:-2}; tag=${2:-wide_w$w}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
wb="$root/tools/wbench.py --width $w --iters 5"
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d "$out/$name" -o run --output-format csv -- python3 $wb > "$out/$name.log" 2>&1
}
run trace --kernel-trace --stats
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo "profile $tag done"

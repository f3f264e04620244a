#!/usr/bin/env bash
# Kernel profile of one phase of the hot path on the GPU box (run under gpurun).
#   tools/profile.sh <phase> <workload> <tag>
# Writes gpurun_out/prof/<tag>/... : a --kernel-trace --stats pass and separate
# --pmc passes (TCC FETCH_SIZE and WRITE_SIZE cannot share a pass; counters
# are never combined with the sys/runtime trace domains).
set -euo pipefail
phase=${1:-all}; wl=${2:-uniform}; tag=${3:-${phase}_${wl}}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
kb="$root/tools/kbench.py --phase $phase --workload $wl --iters 10"
run() { # name, extra rocprofv3 args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d "$out/$name" -o run --output-format csv -- python3 $kb > "$out/$name.log" 2>&1
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
echo "profile $tag done"

#!/usr/bin/env bash
# Decode-kernel profile (run under gpurun): kernel trace + two SQ PMC passes of
# tools/kbench.py --phase decode for one workload and decode variant.
#   tools/prof_dec.sh <workload> <variant> <tag>
set -euo pipefail
wl=${1:-zipf}; v=${2:-9}; tag=${3:-dec_${wl}_$v}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
export HUFF_DEC_VARIANT=$v
kb="$root/tools/kbench.py --phase decode --workload $wl --iters 10"
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d "$out/$name" -o run --output-format csv -- python3 $kb > "$out/$name.log" 2>&1
}
run trace --kernel-trace --stats
run sqa --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sqb --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo "prof_dec $tag done"

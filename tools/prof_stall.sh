#!/usr/bin/env bash
# Stall-attribution PMC passes (TA/TD/TCP/LDS) for one phase and workload.
#   tools/prof_stall.sh <phase> <workload> <tag>
set -euo pipefail
phase=$1; wl=$2; tag=$3
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
kb="$root/tools/kbench.py --phase $phase --workload $wl --iters 10 --no-verify"
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 "$@" -d "$out/$name" -o run --output-format csv -- python3 $kb > "$out/$name.log" 2>&1
}
run trace --kernel-trace --stats
run p1 --pmc TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
run p2 --pmc SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY
run p3 --pmc TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
run p4 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVES
python3 $root/tools/summarize_prof.py "$out" > "$root/gpurun_out/prof_${tag}.json"
echo "prof_stall $tag done"

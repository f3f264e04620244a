#!/usr/bin/env bash
# Round 6: LDS and TA counters of the indexed decode, linear stage
# (HUFF_COL_STAGE=0) against the column stage, 1 GiB Zipf and text.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/colpmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for wl in zipf text; do
  for c in 0 1; do
    HUFF_COL_STAGE=$c timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD \
      -d $out/sq_${wl}_c$c -o run --output-format csv -- python3 $root/tools/kbench.py --phase decode --workload $wl --iters 3 > $out/sq_${wl}_c$c.log 2>&1 || exit 1
    HUFF_COL_STAGE=$c timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
      -d $out/ta_${wl}_c$c -o run --output-format csv -- python3 $root/tools/kbench.py --phase decode --workload $wl --iters 3 > $out/ta_${wl}_c$c.log 2>&1 || echo "ta pass failed"
  done
done
echo colpmc done

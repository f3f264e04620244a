#!/usr/bin/env bash
# Round 6: LDS counters of the general decoder on 1 GiB uniform through the
# general kernels (HUFF_DISABLE_FIXED8=1) with 4 lookups per refill (auto)
# and with 2 (HUFF_DEC_REFILL=2): LDS instructions, LDS-array and
# bank-conflict cycles beside the GPU cycles (profiles/r06/refill/pmc_*).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/refill_pmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
export HUFF_DISABLE_FIXED8=1
for r in auto 2; do
  if [ $r = auto ]; then unset HUFF_DEC_REFILL; else export HUFF_DEC_REFILL=$r; fi
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    -d $out/pmc_r$r -o run --output-format csv -- \
    python3 $root/tools/kbench.py --phase decode --workload uniform --iters 5 > $out/pmc_r$r.log 2>&1 || exit 1
done
echo pmc done

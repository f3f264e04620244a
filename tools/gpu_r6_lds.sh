#!/usr/bin/env bash
# Round 6: is the decoders' LDS array the bound? GPU clock cycles
# (GRBM_GUI_ACTIVE) beside the LDS-array cycles (SQ_LDS_IDX_ACTIVE, summed
# over the CUs) and the bank-conflict cycles, for the indexed decode and the
# index-free pipeline on 1 GiB Zipf. One PMC pass per phase.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/lds; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for ph in decode indexless; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace_$ph -o run --output-format csv -- \
    python3 $root/tools/kbench.py --phase $ph --workload zipf --iters 5 > $out/trace_$ph.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    -d $out/pmc_$ph -o run --output-format csv -- \
    python3 $root/tools/kbench.py --phase $ph --workload zipf --iters 5 > $out/pmc_$ph.log 2>&1 || exit 1
done
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $out/trace_w2 -o run --output-format csv -- \
  python3 $root/tools/wbench.py --width 2 --iters 5 > $out/trace_w2.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS \
  -d $out/pmc_w2 -o run --output-format csv -- python3 $root/tools/wbench.py --width 2 --iters 5 > $out/pmc_w2.log 2>&1 || exit 1
echo lds done

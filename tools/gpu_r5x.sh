#!/usr/bin/env bash
# Round 5, pass x: PMC passes of the wide-letter bench at W = 2 (the task
# decoder's instruction mix, LDS activity and conflicts, wait cycles).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5x}
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
wb="$root/tools/wbench.py --width 2 --iters 3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $wb > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/sq1 -o run --output-format csv -- python3 $wb > $out/sq1.log 2>&1 || { tail -5 $out/sq1.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $out/sq2 -o run --output-format csv -- python3 $wb > $out/sq2.log 2>&1 || { tail -5 $out/sq2.log; exit 1; }
echo done

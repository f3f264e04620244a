#!/usr/bin/env bash
# PMC of the wide task decoder, W = 2/4/8 (one SQ pass each, kernel trace first)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3ad}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for w in 2 4 8; do
  wb="$root/tools/wbench.py --width $w --iters 2"
  timeout -s KILL 120 rocprofv3 --kernel-trace -d $out/w${w}_trace -o run --output-format csv -- python3 $wb > $out/w${w}_trace.log 2>&1 || { tail -5 $out/w${w}_trace.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/w${w}_sq -o run --output-format csv -- python3 $wb > $out/w${w}_sq.log 2>&1 || { tail -5 $out/w${w}_sq.log; exit 1; }
done
echo done

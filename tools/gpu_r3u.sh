#!/usr/bin/env bash
# PMC of the index-free pipeline (Zipf) and of the restart-index decode/pack
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3u}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for ph in indexless all; do
  kb="$root/tools/kbench.py --phase $ph --workload zipf --iters 3"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/${ph}_trace -o run --output-format csv -- python3 $kb > $out/${ph}_trace.log 2>&1 || { tail -5 $out/${ph}_trace.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/${ph}_sq1 -o run --output-format csv -- python3 $kb > $out/${ph}_sq1.log 2>&1 || { tail -5 $out/${ph}_sq1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $out/${ph}_sq2 -o run --output-format csv -- python3 $kb > $out/${ph}_sq2.log 2>&1 || { tail -5 $out/${ph}_sq2.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/${ph}_fetch -o run --output-format csv -- python3 $kb > $out/${ph}_fetch.log 2>&1 || { tail -5 $out/${ph}_fetch.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/${ph}_write -o run --output-format csv -- python3 $kb > $out/${ph}_write.log 2>&1 || { tail -5 $out/${ph}_write.log; exit 1; }
done
echo done

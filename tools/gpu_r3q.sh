#!/usr/bin/env bash
# profile the wide task decoder (W=2) : kernel trace + SQ/TA PMC passes
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3q}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
wb="$root/tools/wbench.py --width 2 --iters 3"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $wb > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/sq1 -o run --output-format csv -- python3 $wb > $out/sq1.log 2>&1 || { tail -5 $out/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $out/sq2 -o run --output-format csv -- python3 $wb > $out/sq2.log 2>&1 || { tail -5 $out/sq2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_DATA_STALLED_BY_TC_sum -d $out/ta -o run --output-format csv -- python3 $wb > $out/ta.log 2>&1 || { tail -5 $out/ta.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 $wb > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 $wb > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
echo done

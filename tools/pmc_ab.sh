#!/usr/bin/env bash
# PMC A/B of one env knob for one kbench phase: per value, a kernel-trace
# pass and two SQ counter passes (LDS/VALU occupancy counters), summarised
# by tools/summarize_prof.py into gpurun_out/<tag>/<workload>_<value>.json.
#   tools/pmc_ab.sh <tag> <phase> <workload> <VAR> <values...>
set -euo pipefail
tag=$1; phase=$2; wl=$3; var=$4; shift 4
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  d=$out/prof_${wl}_$v
  mkdir -p "$d"
  kb="$root/tools/kbench.py --phase $phase --workload $wl --iters 10 --no-verify"
  export "$var=$v"
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$d/trace" -o run --output-format csv -- python3 $kb > "$d/trace.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    -d "$d/p1" -o run --output-format csv -- python3 $kb > "$d/p1.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -d "$d/p2" -o run --output-format csv -- python3 $kb > "$d/p2.log" 2>&1
  python3 $root/tools/summarize_prof.py "$d" > "$out/${wl}_$v.json"
  unset "$var"
done
echo "pmc_ab $tag done"

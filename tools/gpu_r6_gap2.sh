#!/usr/bin/env bash
# Round 6: idle time inside the headline step with the library's kernel
# timing on and off (tools/timing_ab.py under a kernel trace; blocks split by
# tools/step_gaps.py), plus the host phase times with timing off.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6gap2}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
HUFF_HOST_TRACE=1 timeout -k 10 200 python -u tools/timing_ab.py --steps 20 --reps 1 > $out/ab.txt 2> $out/host_trace.err || { tail -5 $out/host_trace.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python3 $root/tools/timing_ab.py --steps 20 --reps 2 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
python3 $root/tools/step_gaps.py $out/trace/run_kernel_trace.csv --split 500 > $out/gaps.txt && cat $out/gaps.txt

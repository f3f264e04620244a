#!/usr/bin/env bash
# Round 6: where the headline step's host gap goes: a kernel trace of the
# default workload's timed steps and the host-side phase times of compress
# (HUFF_HOST_TRACE=1).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6gap}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
HUFF_HOST_TRACE=1 timeout -k 10 200 python -u bench.py --side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3 > $out/bench.json 2> $out/host_trace.err || { tail -5 $out/host_trace.err; exit 1; }
tail -5 $out/host_trace.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python3 $root/bench.py --side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
echo trace done

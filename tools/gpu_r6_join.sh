#!/usr/bin/env bash
# Round 6: the pass 1 -> pass 2 idle of the headline step, host stamps joined
# with a kernel trace (tools/host_join.py), library kernel timing off.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6join}
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
HUFF_HOST_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python3 $root/tools/timing_ab.py --steps 20 --reps 1 > $out/trace.log 2> $out/host_trace.err || { tail -5 $out/host_trace.err; exit 1; }
python3 $root/tools/host_join.py $out/host_trace.err $out/trace/run_kernel_trace.csv | tee $out/join.txt
python3 $root/tools/step_gaps.py $out/trace/run_kernel_trace.csv --split 500 | tee $out/gaps.txt
cd $root && timeout -k 10 200 python -u bench.py --side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['kernels'])"

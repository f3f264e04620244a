#!/usr/bin/env bash
# Round 6: the N=1 software pipeline (next pass 1 queued ahead of the decode)
# against serial steps: bench lines, and a kernel trace of the pipelined bench
# with its idle gaps; HUFF_LIB_AB=rows0: pass 1 without the fused
# rows-sum + publish kernel.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6pipe}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
B="--side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py $B > $out/pipe_$r.json 2> $out/pipe_$r.err || { tail -5 $out/pipe_$r.err; exit 1; }
  timeout -k 10 200 python -u bench.py $B --no-pipeline > $out/serial_$r.json 2> $out/serial_$r.err || { tail -5 $out/serial_$r.err; exit 1; }
done
for f in $out/pipe_*.json $out/serial_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})" $f; done
timeout -k 10 200 python -u bench.py --workload zipf --side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3 > $out/zipf_pipe.json 2> $out/zipf_pipe.err || { tail -5 $out/zipf_pipe.err; exit 1; }
timeout -k 10 200 python -u bench.py --workload zipf --side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3 --no-pipeline > $out/zipf_serial.json 2> $out/zipf_serial.err || { tail -5 $out/zipf_serial.err; exit 1; }
for r in 1 2; do
  HUFF_LIB_AB=rows0 timeout -k 10 200 python -u bench.py $B > $out/rows0_$r.json 2> $out/rows0_$r.err || { tail -5 $out/rows0_$r.err; exit 1; }
done
for f in $out/rows0_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})" $f; done
for f in $out/zipf_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], 'indexfree_ms', d['e2e']['indexfree_decode_ms'])" $f; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python3 $root/bench.py $B --time-every 1000 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
python3 $root/tools/step_gaps.py $out/trace/run_kernel_trace.csv --split 500 | tee $out/gaps.txt

#!/usr/bin/env bash
# Round 6: pass 1's fused rows-sum + publish kernel (k_rows_publish) at 64 /
# 128 / 256 workgroups against the two-kernel tail (HUFF_LIB_AB=rows0), on the
# pipelined headline bench, with a kernel trace of the default build.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6rp}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
B="--side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3"
for r in 1 2; do
  for v in default rows0 rp64 rp256; do
    if [ $v = default ]; then env=""; else env="HUFF_LIB_AB=$v"; fi
    env $env timeout -k 10 200 python -u bench.py $B > $out/${v}_$r.json 2> $out/${v}_$r.err || { tail -5 $out/${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})" $out/${v}_$r.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $root/bench.py $B --time-every 1000 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
head -12 $out/trace/run_kernel_stats.csv | cut -c1-160

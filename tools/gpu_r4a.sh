#!/usr/bin/env bash
# Round-4 baseline: index-free decode kernel trace (Zipf, text) of the round-3 build.
#   tools/gpu_r4a.sh <tag>
set -euo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r4a}
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for wl in zipf text; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/idx_$wl -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_$wl.json 2> $out/idx_$wl.err
  echo "idx $wl done"
done
cd $root
timeout -k 10 300 python bench.py --no-cpu-baseline --workload zipf --file-path none > $out/bench_zipf.json 2> $out/bench_zipf.err
echo "bench done"

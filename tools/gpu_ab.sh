#!/usr/bin/env bash
# A/B of one env knob on the GPU box: GPU parity tests, then kbench of a
# phase per workload with the knob's values, then the bench lines.
#   tools/gpu_ab.sh <tag> <phase> <VAR> <values...>
set -euo pipefail
tag=$1; phase=$2; var=$3; shift 3
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
for w in uniform zipf text; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 120 python tools/kbench.py --phase $phase --workload $w --iters 20 > "$out/${phase}_${w}_$v.json" 2> "$out/${phase}_${w}_$v.err"
  done
done
for w in uniform zipf text; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > "$out/bench_$w.json" 2> "$out/bench_$w.err"
done
echo "gpu_ab $tag done"

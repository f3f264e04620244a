#!/usr/bin/env bash
# GPU parity tests then the three N=1 bench lines (no CPU baseline).
#   tools/gpu_tests_bench.sh <tag>
set -euo pipefail
out=gpurun_out/${1:-tb}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1
for w in uniform zipf text; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > "$out/bench_$w.json" 2> "$out/bench_$w.err"
done
echo "tests+bench done"

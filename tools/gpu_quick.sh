#!/usr/bin/env bash
# GPU parity tests, per-phase kernel timings (uniform), C-only step bench,
# and the Python bench line (uniform). Outputs under gpurun_out/quick/.
set -euo pipefail
out=gpurun_out/quick
mkdir -p $out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $out/tests.log 2>&1
(for k in 0 1 2; do timeout -k 10 60 tools/stepbench $k 20; done) > $out/stepbench.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench_uniform.json 2> $out/bench_uniform.err
for w in zipf text; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > $out/bench_$w.json 2> $out/bench_$w.err
done

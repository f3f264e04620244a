#!/usr/bin/env bash
# Wide-letter GPU tests first (new code), then the whole GPU suite, then one
# bench line with the cpu_baseline (cpu-fast leg included).
set -euo pipefail
out=gpurun_out/wide
mkdir -p $out
timeout -k 10 600 python -m pytest tests/test_gpu_wide.py -x -q -p no:cacheprovider > $out/wide_tests.log 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $out/tests.log 2>&1
timeout -k 10 300 python bench.py > $out/bench_uniform.json 2> $out/bench_uniform.err

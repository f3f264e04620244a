#!/usr/bin/env bash
# Round 5, pass aa: the index-free tests with the sample-overflow stress case
# (a 1-bit code beside codes up to 30 bits), with fix-up statistics.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5aa}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_wide.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log

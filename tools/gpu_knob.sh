#!/usr/bin/env bash
# Parity tests with an env knob set, then kbench of a phase for each value
# of the knob on zipf and text (interleaved twice).
#   tools/gpu_knob.sh <tag> <phase> <VAR> <test-value> <values...>
set -euo pipefail
tag=$1; phase=$2; var=$3; tv=$4; shift 4
out=gpurun_out/$tag
mkdir -p "$out"
env "$var=$tv" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_check.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
tail -2 "$out/tests.log"
for rep in 1 2; do
  for w in zipf text; do
    for v in "$@"; do
      env "$var=$v" timeout -k 10 120 python tools/kbench.py --phase $phase --workload $w --iters 20 >> "$out/${phase}_${w}_$v.json" 2>> "$out/${phase}_${w}_$v.err"
    done
  done
done
echo "gpu_knob $tag done"

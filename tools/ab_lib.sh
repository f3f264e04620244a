#!/usr/bin/env bash
# Same-box A/B of two builds: lib/libhuffgpu.so (new) vs lib/ab/libhuffgpu.so
# (old), interleaved, for one phase over the workloads given.
#   tools/ab_lib.sh <phase> <workloads...>
set -euo pipefail
phase=$1; shift
out=gpurun_out/ablib; mkdir -p $out
for rep in 1 2; do
  for w in "$@"; do
    HUFF_LIB_AB=ab timeout -k 10 120 python tools/kbench.py --phase $phase --workload $w --iters 20 > $out/${w}_old_$rep.json 2>/dev/null
    timeout -k 10 120 python tools/kbench.py --phase $phase --workload $w --iters 20 > $out/${w}_new_$rep.json 2>/dev/null
  done
done
echo "ab done"

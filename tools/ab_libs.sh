#!/usr/bin/env bash
# Same-box A/B/C of builds: lib/libhuffgpu.so ("new") and lib/<name>/libhuffgpu.so
# for each name given in LIBS, interleaved, for one phase over the workloads.
#   LIBS="ab c32" tools/ab_libs.sh <phase> <workloads...>
set -euo pipefail
phase=$1; shift
out=gpurun_out/ablibs; mkdir -p $out
for rep in 1 2; do
  for w in "$@"; do
    for l in new $LIBS; do
      if [ "$l" = new ]; then
        timeout -k 10 120 python tools/kbench.py --phase $phase --workload $w --iters 20 > $out/${w}_${l}_$rep.json 2>/dev/null
      else
        HUFF_LIB_AB=$l timeout -k 10 120 python tools/kbench.py --phase $phase --workload $w --iters 20 > $out/${w}_${l}_$rep.json 2>/dev/null
      fi
    done
  done
done
echo "ab done"

#!/usr/bin/env bash
# Round 6: timing experiments of the one-pass index-free decoder: variant
# libraries (lib/<name>, tools/build_variant.sh) through kbench --phase
# indexless, Zipf, --no-verify (the experiments skip work).
#   tools/gpu_r6_sdab.sh <tag> <variant>...
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for rep in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then lib=""; else lib=$v; fi
    HUFF_LIB_AB=$lib timeout -k 10 120 python tools/kbench.py --phase indexless --workload ${WL:-zipf} --iters 20 --no-verify > $out/${v}_$rep.json 2> $out/${v}_$rep.err || { tail -5 $out/${v}_$rep.err; exit 1; }
    echo "$v $(cat $out/${v}_$rep.json)"
  done
done

#!/usr/bin/env bash
# Round 5: phase stamps of the index-free pipeline and the indexed decoder
# (timing build lib/stamps), then the byte map's pieces-per-lane A/B inside
# the bench step.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5b}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for wl in zipf text; do
  HUFF_LIB_AB=stamps timeout -k 10 200 python -u tools/stamps.py --workload $wl > $out/stamps_$wl.json 2> $out/stamps_$wl.err || { tail -20 $out/stamps_$wl.err; exit 1; }
  echo "stamps $wl done"
done
LIBS="bm8 bm2" REPS=3 bash tools/gpu_benchab.sh $tag/benchab

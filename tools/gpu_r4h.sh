#!/usr/bin/env bash
# Round 4: split index-free decode (HUFF_SPLIT=1) timing (kernel trace) of
# the default build and the LIBS variants on Zipf and text; KB_ARGS is passed
# to kbench (e.g. --no-verify for timing-only experiment builds).
#   LIBS="a b" KB_ARGS="--no-verify" tools/gpu_r4h.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r4h}
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
export HUFF_SPLIT=1
for l in new ${LIBS:-}; do
  for wl in ${WLS:-zipf text}; do
    if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/${l}_$wl -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 ${KB_ARGS:-} > $out/${l}_$wl.json 2> $out/${l}_$wl.err || { echo "kbench $l $wl failed"; tail -5 $out/${l}_$wl.err; exit 1; }
    echo -n "$l $wl: "; grep phase $out/${l}_$wl.json
  done
done
echo "r4h done"

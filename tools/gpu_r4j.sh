#!/usr/bin/env bash
# Round 4: index-free decode (default path) of the default build and the LIBS
# variants, kernel trace per run, Zipf and text.
#   LIBS="a b" tools/gpu_r4j.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r4j}
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for l in new ${LIBS:-}; do
  for wl in zipf text; do
    if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/${l}_${wl}_$rep -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/${l}_${wl}_$rep.json 2> $out/${l}_${wl}_$rep.err || { echo "kbench $l $wl failed"; tail -5 $out/${l}_${wl}_$rep.err; exit 1; }
    echo -n "$l $wl $rep: "; python3 -c "import json; d=json.loads(open('$out/${l}_${wl}_$rep.json').read().strip().splitlines()[-1]); print(round(d['wall_ms_per_iter'],4))"
  done
done
done
echo "r4j done"

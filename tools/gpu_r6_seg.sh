#!/usr/bin/env bash
# Round 6: the index-free decode's segment length (HUFF_SEG_TARGET, variant
# libraries seg736 / seg608: 5 staged workgroups per CU instead of 4) against
# the default 992 bits: index-free parity under each, then kbench --phase
# indexless on Zipf and text, alternated.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6seg}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for v in seg736 seg608; do
  HUFF_LIB_AB=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_indexfree.py -x -q --timeout 120 --timeout-method thread > $out/pytest_$v.log 2>&1; tail -1 $out/pytest_$v.log
done
for r in 1 2; do
  for v in default seg736 seg608; do
    if [ $v = default ]; then env=""; else env="HUFF_LIB_AB=$v"; fi
    for wl in zipf text; do
      env $env timeout -k 10 120 python -u tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_${v}_${wl}_$r.json 2> $out/idx_${v}_${wl}_$r.err || { tail -5 $out/idx_${v}_${wl}_$r.err; exit 1; }
    done
  done
done
for f in $out/idx_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], round(d['wall_ms_per_iter'], 4))" $f; done

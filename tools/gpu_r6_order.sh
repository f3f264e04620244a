#!/usr/bin/env bash
# Round 6: byte-map cache-order knobs inside the bench's step (HUFF_BYTEMAP_ORDER:
# pr/dr = pass 2 / decode walk blocks from the end, ps/ds = default-policy
# stores), alternated same-box runs of the headline workload.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-order}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for rep in 1 2 3; do
  for k in ${KNOBS:-none dr ps ps,dr ds}; do
    HUFF_BYTEMAP_ORDER=$k timeout -k 10 200 python -u bench.py --no-cpu-baseline --file-path none --side none --no-general --no-other-scaling --steps 40 > $out/bench_${k}_$rep.json 2> $out/bench_${k}_$rep.err || { echo "bench $k failed"; tail -5 $out/bench_${k}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/bench_${k}_$rep.json').read().strip().splitlines()[-1]); print('$k $rep', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
echo order done

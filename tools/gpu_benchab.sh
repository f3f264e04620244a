#!/usr/bin/env bash
# Same-box A/B of variant libraries inside the bench's own step (kernels timed
# in context, not alone): the default build ("new") and each LIBS variant,
# alternated REPS times, the headline workload only.
#   LIBS="a b" REPS=3 tools/gpu_benchab.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-benchab}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for rep in $(seq 1 ${REPS:-3}); do
  for l in new ${LIBS:-}; do
    if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --file-path none --side none --no-general --no-other-scaling --steps 40 ${BENCH_ARGS:-} > $out/bench_${l}_$rep.json 2> $out/bench_${l}_$rep.err || { echo "bench $l failed"; tail -5 $out/bench_${l}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/bench_${l}_$rep.json').read().strip().splitlines()[-1]); print('$l $rep', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
echo "benchab done"

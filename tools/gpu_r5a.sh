#!/usr/bin/env bash
# Round 5, first GPU pass: GPU suite, smoke, the default bench (with its new
# general / scaling_other records), and the uniform kernel profile (trace +
# PMC) for the byte map's staging fix.
#   tools/gpu_r5a.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5a}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
echo "bench done"
bash tools/profile.sh all uniform ${tag}_all_uniform > /dev/null 2>&1 || { echo "profile uniform failed"; exit 1; }
echo "profile done"

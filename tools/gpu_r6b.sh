#!/usr/bin/env bash
# Round 6 pass: GPU suite, smoke, the default bench and the strong-scaling
# per-rank sizes (tools/gpu_r6_scale.sh).   tools/gpu_r6b.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6b}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
echo "bench done"
[ "${SCALE:-1}" = 0 ] && exit 0
bash tools/gpu_r6_scale.sh ${tag}_scale

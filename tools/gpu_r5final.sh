#!/usr/bin/env bash
# Round-5 closing GPU pass: full GPU suite, smoke, the default bench, a
# kernel trace of the bench, per-workload kernel profiles (trace + PMC
# passes, tools/profile.sh) for the traffic summaries and the index-free
# decode, the wide-letter and batch benches. PROFILES=0 stops after the
# bench trace; PART=profiles runs only what follows it.
#   tools/gpu_r5final.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5f}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
if [ "${PART:-all}" != profiles ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
echo "bench done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/bench_trace -o run --output-format csv -- python3 $root/bench.py --steps 5 --warmup 2 --no-cpu-baseline --file-path none > $out/bench_trace.log 2>&1 || { tail -20 $out/bench_trace.log; exit 1; }
echo "bench trace done"
fi
cd $root
[ "${PROFILES:-1}" = 0 ] && exit 0
for wl in uniform zipf text; do
  bash tools/profile.sh all $wl ${tag}_all_$wl > /dev/null 2>&1 || { echo "profile $wl failed"; exit 1; }
  echo "profile $wl done"
done
for wl in zipf text; do
  bash tools/profile.sh indexless $wl ${tag}_idx_$wl > /dev/null 2>&1 || { echo "profile idx $wl failed"; exit 1; }
done
echo "profiles done"
for w in 2 4 8; do
  timeout -k 10 180 python tools/wbench.py --width $w --iters 5 --indexless > $out/wbench_w$w.json 2>>$out/wbench.err || { echo "wbench $w failed"; exit 1; }
done
timeout -k 10 180 python tools/batchbench.py > $out/batchbench.json 2>>$out/batch.err || { echo "batchbench failed"; exit 1; }
echo "wide + batch done"

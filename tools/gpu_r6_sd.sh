#!/usr/bin/env bash
# Round 6: the one-pass index-free decoder (syncdec.hip): index-free parity
# tests, then kbench of the index-free decode with it and with the pipeline
# (HUFF_SYNC_DECODE=0), Zipf and text, and a kernel trace.
#   tools/gpu_r6_sd.sh <tag> [tests...]
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6sd}; shift || true
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
tests=${TESTS:-tests/test_gpu_indexfree.py}
timeout -k 10 300 python -u -m pytest $tests -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for wl in zipf text; do
  HUFF_FIX_STATS=1 timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 1 > /dev/null 2> $out/stats_$wl.err || { tail -20 $out/stats_$wl.err; exit 1; }
  grep "sync decode" $out/stats_$wl.err | tail -1
  for sd in 1 0; do
    HUFF_SYNC_DECODE=$sd timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/kb_${wl}_sd$sd.json 2> $out/kb_${wl}_sd$sd.err || { tail -20 $out/kb_${wl}_sd$sd.err; exit 1; }
    cat $out/kb_${wl}_sd$sd.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload zipf --iters 10 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
echo trace done

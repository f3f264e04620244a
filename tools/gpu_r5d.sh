#!/usr/bin/env bash
# Round 5: index-free pipeline, second form (one walk per thread; the chunk
# that reaches the segment end cut back to its window; workgroup counts
# scanned instead of segment counts, k_mark_lite scanning inside a
# workgroup; total published to pinned memory; walk-table skip codes read
# from global memory): GPU suite, stamps,
# index-free timing A/B against the round-4 library (lib/r04), without the
# walk table, and with 8-wave skip workgroups, and a kernel trace.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5d}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for wl in zipf text; do
  HUFF_LIB_AB=stamps timeout -k 10 200 python -u tools/stamps.py --workload $wl > $out/stamps_$wl.json 2> $out/stamps_$wl.err || { tail -20 $out/stamps_$wl.err; exit 1; }
  for rep in 1 2 3; do
    timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_new_$rep.json 2> $out/idx_$wl.err || { tail -20 $out/idx_$wl.err; exit 1; }
    HUFF_SKIP_WALK=0 timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_nowalk_$rep.json 2> $out/idx_$wl.err || { tail -20 $out/idx_$wl.err; exit 1; }
    for v in r04 wlds; do HUFF_LIB_AB=$v timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_${v}_$rep.json 2> $out/idx_$wl.err || { tail -20 $out/idx_$wl.err; exit 1; }; done
  done
  for f in $out/idx_${wl}_*.json; do echo "$(basename $f) $(grep -o '"wall_ms_per_iter": [0-9.]*' $f)"; done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/idx_trace -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload zipf --iters 5 > $out/idx_trace.log 2>&1 || { tail -20 $out/idx_trace.log; exit 1; }
echo "trace done"

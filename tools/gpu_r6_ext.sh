#!/usr/bin/env bash
# Round 6: kernel timing carried on the dispatch packets (launch_k) against
# two hipEventRecord markers per timed region (HUFF_TIME_MARKERS=1): step
# time with timing on/off, the bench's per-kernel averages, and a kernel
# trace of the same bench to check those averages against; events with
# and without the system-scope fence (HUFF_TIME_FENCE).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6ext}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
B="--side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3"
timeout -k 10 200 python -u tools/timing_ab.py --steps 20 --reps 3 > $out/ab_ext.txt 2>&1 || { tail -5 $out/ab_ext.txt; exit 1; }
HUFF_TIME_MARKERS=1 timeout -k 10 200 python -u tools/timing_ab.py --steps 20 --reps 3 > $out/ab_markers.txt 2>&1 || { tail -5 $out/ab_markers.txt; exit 1; }
for f in device none; do
  HUFF_TIME_FENCE=$f timeout -k 10 200 python -u tools/timing_ab.py --steps 20 --reps 3 > $out/ab_fence_$f.txt 2>&1 || { tail -5 $out/ab_fence_$f.txt; exit 1; }
done
HUFF_TIME_MARKERS=1 timeout -k 10 200 python -u tools/timing_ab.py --steps 20 --reps 3 > $out/ab_markers_b.txt 2>&1 || { tail -5 $out/ab_markers_b.txt; exit 1; }
grep -H '{' $out/ab_*.txt
timeout -k 10 200 python -u bench.py $B > $out/bench_ext.json 2> $out/bench_ext.err || { tail -5 $out/bench_ext.err; exit 1; }
HUFF_TIME_MARKERS=1 timeout -k 10 200 python -u bench.py $B > $out/bench_markers.json 2> $out/bench_markers.err || { tail -5 $out/bench_markers.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $root/bench.py $B > $out/prof.log 2>&1 || { tail -5 $out/prof.log; exit 1; }
echo done

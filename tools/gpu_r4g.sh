#!/usr/bin/env bash
# Round 4: the split decoder's GPU tests, then index-free timing of the split
# path (kernel trace) and the older path (HUFF_SPLIT=0) on the same box.
#   tools/gpu_r4g.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r4g}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/split_tests.log 2>&1
rc=$?; tail -2 $out/split_tests.log; [ $rc = 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
for wl in zipf text; do
  HUFF_SPLIT=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/idx_$wl -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_$wl.json 2> $out/idx_$wl.err || { echo "kbench $wl failed"; tail -5 $out/idx_$wl.err; exit 1; }
  grep phase $out/idx_$wl.json
  HUFF_SPLIT=0 timeout -k 10 240 python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_old_$wl.json 2> $out/idx_old_$wl.err || { echo "old $wl failed"; exit 1; }
  echo -n "old: "; grep phase $out/idx_old_$wl.json
done
echo "r4g done"

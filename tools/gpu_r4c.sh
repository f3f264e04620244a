#!/usr/bin/env bash
# Round 4: the index-free / fixture / batch / wide tests touched this round,
# then kernel traces of 1 GiB Zipf / text index-free decodes (split path).
#   tools/gpu_r4c.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r4c}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_derived_fixtures.py tests/test_gpu_batch.py tests/test_gpu_wide.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "foreign or past_table or file_path or indexfree or world1 or quirks or cli_gpu or synthetic or limits or growth or alignment or index_free" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
for wl in zipf text; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/idx_$wl -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_$wl.json 2> $out/idx_$wl.err || { echo "kbench $wl failed"; tail -5 $out/idx_$wl.err; exit 1; }
  echo "idx $wl done"; grep phase $out/idx_$wl.json
done

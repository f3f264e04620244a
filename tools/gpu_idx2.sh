#!/usr/bin/env bash
# index-free decode: GPU tests touching it, then a kernel-trace profile
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-idx2}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "foreign or indexless or file_path or wide or dev_decompress or smoke" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
cd /tmp && export TMPDIR=/tmp
for w in zipf text; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_$w -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $w --iters 3 > $out/kb_$w.log 2>&1 || exit 1
done
echo "idx2 done"

#!/usr/bin/env bash
# Round 5, pass oo: the calibration's read and copy shapes, per kernel
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5oo}
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $root/tools/calib_shapes.py > $out/calib.log 2>&1 || { tail -20 $out/calib.log; exit 1; }
tail -1 $out/calib.log

#!/usr/bin/env bash
# Round 5, pass h: pass 1 with the totals folded by k_hist1's last workgroup
# (no k_rows_sum / k_hist_publish launches): GPU suite, then the bench-step
# A/B against the previous build (lib/prev).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r5h; mkdir -p $out
cd $root
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -3 $out/gpu_tests.txt
LIBS=prev REPS=3 tools/gpu_benchab.sh r5h/benchab

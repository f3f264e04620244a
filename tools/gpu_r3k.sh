#!/usr/bin/env bash
# wide encoder v2 + batched trees: tests, wbench, PMC of the wide kernels
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3k}; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_batch.py -q -x -p no:cacheprovider --timeout 180 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error|assert" $out/tests.log | head -30; exit 1; }
for w in 2 4 8; do
  timeout -k 10 200 python -u tools/wbench.py --width $w --iters 10 > $out/wbench_w$w.json 2> $out/wbench_w$w.err || { tail -20 $out/wbench_w$w.err; exit 1; }
  cat $out/wbench_w$w.json
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/prof_w2 -o run -- python3 $root/tools/wbench.py --width 2 --iters 5 > $out/prof_w2.log 2>&1 || { tail -5 $out/prof_w2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/pmc_w2_sq -o run -- python3 $root/tools/wbench.py --width 2 --iters 2 > $out/pmc_w2_sq.log 2>&1 || { tail -5 $out/pmc_w2_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_w2_fetch -o run -- python3 $root/tools/wbench.py --width 2 --iters 2 > $out/pmc_w2_fetch.log 2>&1 || { tail -5 $out/pmc_w2_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_w2_write -o run -- python3 $root/tools/wbench.py --width 2 --iters 2 > $out/pmc_w2_write.log 2>&1 || { tail -5 $out/pmc_w2_write.log; exit 1; }
echo pmc done

#!/usr/bin/env bash
# ifd iteration: tests, timing (forced single pass vs multi-kernel), and the
# stats build's path counters.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3f}; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_gpu_ifd.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/ifd_tests.log 2>&1 || { tail -30 $out/ifd_tests.log; exit 1; }
tail -1 $out/ifd_tests.log
for w in zipf text; do for f in 2 0; do
  HUFF_IFD=$f timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 10 > $out/idx_${w}_ifd${f}.json 2>>$out/err.log || exit 1
done
  HUFF_LIB_AB=ifdstats HUFF_IFD=2 HUFF_IFD_TRACE=1 timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 2 > $out/stats_${w}.json 2> $out/stats_${w}.err || exit 1
done
for f in $out/idx_*.json; do echo "$(basename $f) $(python3 -c "import json;d=json.load(open('$f'));print(round(d['wall_ms_per_iter'],4), round(d.get('ifd_kernel_ms',-1),4))")"; done
grep -h "ifd:" $out/stats_*.err | sort | uniq -c | head

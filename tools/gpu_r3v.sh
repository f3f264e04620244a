#!/usr/bin/env bash
# k_ifd after the ticket/look-back change: its GPU tests, then the single pass
# against the multi-kernel path on 1 GiB Zipf and text (same box).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3v}; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_ifd.py -x -q --timeout 120 --timeout-method thread > $out/ifd_tests.log 2>&1 || { tail -30 $out/ifd_tests.log; exit 1; }
tail -2 $out/ifd_tests.log
for w in zipf text; do
  HUFF_IFD=2 HUFF_IFD_TRACE=1 timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 10 > $out/${w}_ifd.json 2>$out/${w}_ifd.err || exit 1
  HUFF_IFD=0 timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 10 > $out/${w}_multi.json 2>$out/${w}_multi.err || exit 1
done
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json;d=json.load(open('$f'));print(round(d['wall_ms_per_iter'],4), round(d.get('ifd_kernel_ms',-1),4))")"; done
tail -2 $out/zipf_ifd.err $out/text_ifd.err

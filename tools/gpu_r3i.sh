#!/usr/bin/env bash
# full GPU suite + smoke + default bench (closing-style check of the tree)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3i}; mkdir -p $out
cd $root
timeout -k 10 800 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error" $out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['e2e'])"

#!/usr/bin/env bash
# Round 6 closing pass: the GPU suite and smoke, the default bench line, and
# a rocprofv3 kernel-trace summary of the same bench command (profiles/r06/final/).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-final}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['kernels'].items()}); print('zipf', d['side']['zipf']['value'], d['side']['zipf']['e2e']['indexfree_decode_ms'], {k: v['avg_ms'] for k, v in d['side']['zipf']['kernels'].items()}); print('general', d['general']['value'], {k: v['avg_ms'] for k, v in d['general']['kernels'].items()})" $out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- python3 $root/bench.py > $out/prof_bench.json 2> $out/prof_bench.err || { tail -5 $out/prof_bench.err; exit 1; }
echo final done

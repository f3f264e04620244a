#!/usr/bin/env bash
# Round 6: per-phase wave budgets (s_memtime stamps, tools/stamps.py) of the
# index-free pipeline's two walks on 1 GiB Zipf and text, from the timing
# build (tools/build_variant.sh stamps "-DHUFF_STAMPS" ...), plus a kernel
# trace of the same decode with the product library (profiles/r06/budget/)
set -euo pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/budget
mkdir -p $O
for w in zipf text; do
  HUFF_LIB_AB=stamps timeout -k 10 180 python tools/stamps.py --workload $w > $O/stamps_$w.json
  tail -c 300 $O/stamps_$w.json; echo
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/kbench.py --phase indexless --workload zipf > $GRAFT_REPO_ROOT/$O/kbench_zipf.json
echo done

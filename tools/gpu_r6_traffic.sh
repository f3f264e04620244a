#!/usr/bin/env bash
# Round 6: PMC traffic of the general kernels on the headline workload
# (HUFF_DISABLE_FIXED8=1: k_pack / k_decode_fixed and the index-free
# pipeline on 1 GiB uniform), for bench.py's general.roofline.traffic and
# general.e2e.indexfree_roofline.traffic.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd $root
export HUFF_DISABLE_FIXED8=1
bash tools/profile.sh all uniform r6_all_uniform_general > /dev/null 2>&1 || { echo "profile all failed"; exit 1; }
echo "all done"
bash tools/profile.sh indexless uniform r6_idx_uniform_general > /dev/null 2>&1 || { echo "profile idx failed"; exit 1; }
echo "indexless done"

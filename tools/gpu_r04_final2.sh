#!/bin/bash
# Round 4 closing measurements, part 2: the K=30 10M-link PMC record (copied to profiles/ on the
# box), then the BASELINE config lines (k10_b8, k20_b8 and k30_10m carry their stamped traffic).
# usage: bash tools/gpu_r04_final2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_r04_prof.sh $TAG/prof30 $OUT/pmc_r04_K30.json 30 4 --K 30 --P 50000 --E 10000000 --test-frac 0 > $OUT/prof30.txt 2>&1 || { tail -20 $OUT/prof30.txt; exit 1; }
cp $OUT/pmc_r04_K30.json profiles/pmc_r04_K30.json
bash tools/gpu_r04_configs.sh $TAG/cfg || exit 1

#!/bin/bash
# Per-wave phases of the large-K pass (stamp build) at K=30 on 10M links and K=20 x 8: prologue
# (V tables), chunk loop, tail.  usage: bash tools/gpu_r04_stamp30.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-stamp30}
bash tools/gpu_r03_stamp.sh $TAG/k30 --K 30 --P 50000 --E 10000000 --test-frac 0 --steps 3 --warmup 1 || exit 1
bash tools/gpu_r03_stamp.sh $TAG/k20 --K 20 --samples 8 || exit 1

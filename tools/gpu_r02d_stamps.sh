#!/bin/bash
# Phase stamps (stamp build) at K=20 x 8 and K=30 on 10M links.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r02_stamp.sh stamp20 --K 20 --samples 8 && bash tools/gpu_r02_stamp.sh stamp30 --K 30 --P 50000 --E 10000000 --steps 3 --warmup 1

#!/bin/bash
# SK_Y (the stream-0 small-K E-step with Y entries) against SK_U (three streams) on one box: the
# default bench at several unit counts, then the stamp build's per-wave phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sky}
bash tools/gpu_r03_ab.sh $TAG/ab "sku|-|MMSBM_SK_Y=0" "sky3840|-|MMSBM_SK_Y=1" "sky2560|-|MMSBM_UNITS=2560,2560" \
    "sky1920|-|MMSBM_UNITS=1920,1920" "sky1280|-|MMSBM_UNITS=1280,1280" "sky5120|-|MMSBM_UNITS=5120,5120" \
    "sku2|-|MMSBM_SK_Y=0" || exit 1
bash tools/gpu_r03_stamp.sh $TAG/stamp_sky || exit 1
MMSBM_SK_Y=0 bash tools/gpu_r03_stamp.sh $TAG/stamp_sku || exit 1

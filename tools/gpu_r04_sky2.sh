#!/bin/bash
# SK_Y (gathers hoisted into the prologue) vs SK_U, and SK_U with its first block's gathers
# hoisted before the V tables (tools/_build/libmmsbm_ghoist.so, -DMMSBM_SK_GHOIST=1), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sky2}
bash tools/gpu_r03_ab.sh $TAG/ab "sku|-|MMSBM_SK_Y=0" "sku_ghoist|tools/_build/libmmsbm_ghoist.so|MMSBM_SK_Y=0" \
    "sky1920|-|MMSBM_UNITS=1920,1920" "sky2560|-|MMSBM_UNITS=2560,2560" "sky3840|-|MMSBM_SK_Y=1" \
    "sku_ghoist2|tools/_build/libmmsbm_ghoist.so|MMSBM_SK_Y=0" "sku2|-|MMSBM_SK_Y=0" || exit 1
MMSBM_UNITS=1920,1920 bash tools/gpu_r03_stamp.sh $TAG/stamp_sky || exit 1

#!/bin/bash
# SK_Y with the X0 rows as Y entries vs SK_U: fold0 K=10 at B=1 (headline) and B=8 (config 4's
# per-GPU share), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sky3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_r03_ab.sh $TAG/ab "sku|-|MMSBM_SK_Y=0" "sky1920|-|MMSBM_SK_Y=1 MMSBM_UNITS=1920,1920" \
    "sky3840|-|MMSBM_SK_Y=1" "sku2|-|MMSBM_SK_Y=0" || exit 1
for spec in "sku|MMSBM_SK_Y=0" "sky3840|MMSBM_SK_Y=1" "sky1920|MMSBM_SK_Y=1 MMSBM_UNITS=1920,1920" "sky7680|MMSBM_SK_Y=1 MMSBM_UNITS=7680,7680"; do
  IFS='|' read -r label envs <<< "$spec"
  env $envs timeout -k 10 200 python -u bench.py --K 10 --samples 8 --steps 200 --warmup 10 --no-cpu-baseline > $OUT/b8_$label.json 2> $OUT/b8_$label.err || { tail -5 $OUT/b8_$label.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b8_$label.json'))
print('B=8 %-10s %.0f sample-iter/s  iter %.1f us' % ('$label', d['value'], d['iteration']['us']), {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
done

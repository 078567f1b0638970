#!/bin/bash
# Run one pytest selection under several env variants on the GPU box.
# usage: bash tools/gpu_variants.sh TAG "-k expr" "label|ENV=a ENV2=b" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; SEL=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "$@"; do
  IFS='|' read -r label envs <<< "$v"
  env $envs timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu $SEL > $OUT/pytest_$label.log 2>&1
  rc=$?
  echo "$label rc=$rc $(tail -1 $OUT/pytest_$label.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

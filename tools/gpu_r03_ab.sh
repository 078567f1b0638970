#!/bin/bash
# A/B of library builds and env settings on the default bench, in one box session.
# usage: bash tools/gpu_r03_ab.sh TAG "label|lib|ENV=V ENV2=V" ...   (lib "-" = in-tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab}; shift
mkdir -p $OUT
for spec in "$@"; do
  IFS='|' read -r label lib envs <<< "$spec"
  if [ "$lib" = "-" ]; then unset MMSBM_LIB; else export MMSBM_LIB=$PWD/$lib; fi
  env $envs timeout -k 10 120 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline > $OUT/$label.json 2> $OUT/$label.err || { tail -5 $OUT/$label.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$label.json'))
print('%-14s value %.0f it/s  iter %.2f us  L %.13g' % ('$label', d['value'], d['iteration']['us'], d['final_loglik']),
      {k: round(v['back_to_back'],2) for k, v in d['kernel_us'].items()}, d['plan'].get('wg_stream0'), d['plan'].get('wg_stream12'))"
done

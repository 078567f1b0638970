#!/bin/bash
# Large-K A/B of run-time switches on one box (K=30 on 10M links, K=20 x 8): each variant is
# "name|VAR=value VAR2=value" (or "name|-" for the defaults), run in the order given.
# usage: bash tools/gpu_r04_envab.sh TAG "full|-" "ysp0|MMSBM_YSPLIT=0" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for cfg in "k30|--K 30 --P 50000 --E 10000000 --test-frac 0 --steps 4 --warmup 1 --roofline-launches 5" "k20|--K 20 --samples 8 --steps 60 --warmup 5 --roofline-launches 50"; do
  IFS='|' read -r name args <<< "$cfg"
  for spec in "$@"; do
    IFS='|' read -r v envs <<< "$spec"
    [ "$envs" = "-" ] && envs=""
    timeout -k 10 400 env $envs python -u bench.py --no-cpu-baseline $args > $OUT/${name}_$v.json 2> $OUT/${name}_$v.err || { tail -5 $OUT/${name}_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${name}_$v.json')); print('$name $v', '%.1f it/s' % d['value'], {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
  done
done

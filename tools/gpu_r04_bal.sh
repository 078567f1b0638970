#!/bin/bash
# Large-K A/B on one box, K=30 on 10M links and K=20 x 8: the default build against
# MMSBM_BALANCE=0 (whole runs per unit), twice each.  usage: bash tools/gpu_r04_bal.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab2}
mkdir -p $OUT
for cfg in "k30|--K 30 --P 50000 --E 10000000 --test-frac 0 --steps 4 --warmup 1 --roofline-launches 5" "k20|--K 20 --samples 8 --steps 60 --warmup 5 --roofline-launches 50"; do
  IFS='|' read -r name args <<< "$cfg"
  for v in full bal0 full2 bal02; do
    unset MMSBM_LIB MMSBM_BALANCE
    if [ ${v%2} = bal0 ]; then export MMSBM_BALANCE=0; elif [ $v != full ] && [ $v != full2 ]; then export MMSBM_LIB=$PWD/tools/_build/libmmsbm_$v.so; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > $OUT/${name}_$v.json 2> $OUT/${name}_$v.err || { tail -5 $OUT/${name}_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${name}_$v.json')); print('$name $v', '%.1f it/s' % d['value'], {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
  done
done
unset MMSBM_LIB MMSBM_BALANCE

#!/bin/bash
# The gene kernel's parts (tools/_build/libmmsbm_g{1,2,4}.so: x0, S, Y workgroups only; timings
# only) with balanced units (default) and whole runs per unit (MMSBM_BALANCE=0), K=30 on 10M links
# and K=20 x 8.  usage: bash tools/gpu_r04_gene2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-gene2}
mkdir -p $OUT
for cfg in "k30|--K 30 --P 50000 --E 10000000 --test-frac 0 --steps 4 --warmup 1 --roofline-launches 5" "k20|--K 20 --samples 8 --steps 30 --warmup 3 --roofline-launches 50"; do
  IFS='|' read -r name args <<< "$cfg"
  for bal in 1 0; do
    for v in full 1 2 4; do
      unset MMSBM_LIB
      [ $v != full ] && export MMSBM_LIB=$PWD/tools/_build/libmmsbm_g$v.so
      MMSBM_BALANCE=$bal timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > $OUT/${name}_b${bal}_$v.json 2> $OUT/${name}_b${bal}_$v.err || { tail -5 $OUT/${name}_b${bal}_$v.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$OUT/${name}_b${bal}_$v.json')); print('$name balance=$bal gene-only=$v', {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
    done
  done
done
unset MMSBM_LIB

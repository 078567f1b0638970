#!/bin/bash
# Where pass A's time goes at K=30 on 10M links (and K=20 x 8): the default build against the
# ablation builds (tools/_build/libmmsbm_abl{1,2,3,4}.so, -DMMSBM_ABL: 1 = no Y stores, 2 = theta
# gathers from 64 hot rows, 3 = both, 4 = no partial-row stores; timings only, results invalid),
# the gene kernel with its workgroup kinds in blockIdx order (libmmsbm_mix0.so), and the round-3
# whole-run unit packing (MMSBM_BALANCE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-abl}
mkdir -p $OUT
for cfg in "k30|--K 30 --P 50000 --E 10000000 --test-frac 0 --steps 4 --warmup 1 --roofline-launches 5" "k20|--K 20 --samples 8 --steps 30 --warmup 3 --roofline-launches 50"; do
  IFS='|' read -r name args <<< "$cfg"
  for v in full bal0 abl1 abl2 abl3 abl4 mix0; do
    unset MMSBM_LIB MMSBM_BALANCE
    if [ $v = bal0 ]; then export MMSBM_BALANCE=0; elif [ $v != full ]; then export MMSBM_LIB=$PWD/tools/_build/libmmsbm_$v.so; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > $OUT/${name}_$v.json 2> $OUT/${name}_$v.err || { tail -5 $OUT/${name}_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${name}_$v.json')); print('$name $v', {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
  done
done
unset MMSBM_LIB MMSBM_BALANCE

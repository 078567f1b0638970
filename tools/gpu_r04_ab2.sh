#!/bin/bash
# Large-K A/B on one box, K=30 on 10M links and K=20 x 8: the default build (balanced units, pass
# kernel capped at 128 VGPRs, Y stride padded to 64 B, gene kinds in blockIdx order) against
# MMSBM_BALANCE=0 and the variant builds tools/_build/libmmsbm_{mix1,wpe1,yal1,yal16,wt0}.so
# (-DMMSBM_GENE_MIX=1: gene-kernel kinds interleaved; -DMMSBM_PASS_WPE=1: no VGPR cap; -DMMSBM_YALIGN=1 / 16: Y stride K / 128 B; -DMMSBM_WT=0: plain
# partial-row stores).  usage: bash tools/gpu_r04_ab2.sh TAG [variants...] (default: the list below;
# "full*" = the default build, "bal0*" = MMSBM_BALANCE=0, else tools/_build/libmmsbm_<name>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab2}
shift
VARS="${*:-full mix1 bal0 wpe1 yal1 yal16 wt0 full2}"
mkdir -p $OUT
for cfg in "k30|--K 30 --P 50000 --E 10000000 --test-frac 0 --steps 4 --warmup 1 --roofline-launches 5" "k20|--K 20 --samples 8 --steps 60 --warmup 5 --roofline-launches 50"; do
  IFS='|' read -r name args <<< "$cfg"
  for v in $VARS; do
    unset MMSBM_LIB MMSBM_BALANCE
    case $v in full*) ;; bal0*) export MMSBM_BALANCE=0;; *) export MMSBM_LIB=$PWD/tools/_build/libmmsbm_$v.so;; esac
    timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > $OUT/${name}_$v.json 2> $OUT/${name}_$v.err || { tail -5 $OUT/${name}_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${name}_$v.json')); print('$name $v', '%.1f it/s' % d['value'], {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
  done
done
unset MMSBM_LIB MMSBM_BALANCE

#!/bin/bash
# Where the large-K gene kernel's time goes: the kernel with one workgroup kind only
# (tools/_build/libmmsbm_g{1,2,4}.so, -DMMSBM_GENE_ONLY: 1 = X0 gene workgroups, 2 = S partials,
# 4 = Y sums; timings only, results not valid), at K=20 x 8 and K=30 on 10M links; then the
# launch-overhead probe of the default bench configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-gene}
mkdir -p $OUT
for cfg in "k20|--K 20 --samples 8 --steps 30 --warmup 3 --roofline-launches 50" "k30|--K 30 --P 50000 --E 10000000 --test-frac 0 --steps 4 --warmup 1 --roofline-launches 5"; do
  IFS='|' read -r name args <<< "$cfg"
  for v in full 1 2 4; do
    if [ $v = full ]; then unset MMSBM_LIB; else export MMSBM_LIB=$PWD/tools/_build/libmmsbm_g$v.so; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > $OUT/${name}_$v.json 2> $OUT/${name}_$v.err || { tail -5 $OUT/${name}_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${name}_$v.json')); print('$name gene-only=$v', {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
  done
done
unset MMSBM_LIB
timeout -k 10 200 python -u tools/overhead_probe.py > $OUT/overhead.json 2> $OUT/overhead.err || { tail -5 $OUT/overhead.err; exit 1; }
cat $OUT/overhead.json

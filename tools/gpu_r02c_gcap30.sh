#!/bin/bash
# K=30 on 10M links: pass-A gene cap sweep (MMSBM_GCAP: smaller V tables, more workgroups per CU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-gcap30}
mkdir -p $OUT
for g in 13 8 6 4; do
  MMSBM_GCAP=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 30 --P 50000 --E 10000000 --steps 10 --warmup 2 --roofline-launches 5 \
      > $OUT/k30_g$g.json 2> $OUT/k30_g$g.err || { tail -20 $OUT/k30_g$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/k30_g$g.json')); print('gcap $g', round(d['value'],1), {k: round(v['back_to_back'],1) for k,v in d['kernel_us'].items()})"
done

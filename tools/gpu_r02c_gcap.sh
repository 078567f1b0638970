#!/bin/bash
# Pass-A gene cap sweep (MMSBM_GCAP) at K=20 x 8 samples and K=30 on 10M links, with the library
# named by MMSBM_LIB (default: the in-tree build).  A smaller cap shrinks the V tables in LDS so
# more pass-A workgroups share a CU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-gcap}
mkdir -p $OUT
line() { python3 -c "import json; d=json.load(open('$1')); print('$1', round(d['value'],1), {k: round(v['back_to_back'],1) for k,v in d['kernel_us'].items()})"; }
for g in 0 9 5 4; do
  MMSBM_GCAP=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 20 --samples 8 --steps 100 --warmup 5 --roofline-launches 100 \
      > $OUT/k20_g$g.json 2> $OUT/k20_g$g.err || { tail -20 $OUT/k20_g$g.err; exit 1; }
  line $OUT/k20_g$g.json
done
for g in 0 4; do
  MMSBM_GCAP=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 30 --P 50000 --E 10000000 --steps 10 --warmup 2 --roofline-launches 5 \
      > $OUT/k30_g$g.json 2> $OUT/k30_g$g.err || { tail -20 $OUT/k30_g$g.err; exit 1; }
  line $OUT/k30_g$g.json
done

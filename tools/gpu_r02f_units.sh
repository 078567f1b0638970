#!/bin/bash
# fold0 K=10 work-plan unit sweep (MMSBM_UNITS = stream-0 units, stream-1/2 units) on the current
# kernels, 2000-step bench lines, the default measured first and last.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-units}
mkdir -p $OUT
for u in 1536,3072 1280,3072 1792,3072 1536,2560 1536,3584 1280,2560 1536,3072; do
  MMSBM_UNITS=$u timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2000 --warmup 50 > $OUT/u_$u.json 2> $OUT/u_$u.err || { tail -20 $OUT/u_$u.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/u_$u.json')); print('$u', round(d['value']), {k: round(v['back_to_back'],2) for k,v in d['kernel_us'].items()})"
done

#!/bin/bash
# Unit-count sweep of the small-K plan (MMSBM_UNITS=a,b) at the default bench config.
# usage: bash tools/gpu_r03_units.sh TAG "a1,b1 a2,b2 ..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-units}; shift
LIST=$1; shift
mkdir -p $OUT
for u in $LIST; do
  MMSBM_UNITS=$u timeout -k 10 120 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline --roofline-launches 300 "$@" > $OUT/u_$u.json 2> $OUT/u_$u.err || { echo "units $u failed"; tail -5 $OUT/u_$u.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/u_$u.json'))
print('units %-10s %7.0f it/s  %6.2f us' % ('$u', d['value'], d['iteration']['us']), {k: round(v['back_to_back'],2) for k,v in d['kernel_us'].items()}, 'wg', d['plan']['wg_stream0'], d['plan']['wg_stream12'], 'units', d['plan']['units'])"
done

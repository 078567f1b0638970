#!/bin/bash
# Unit-count sweep (MMSBM_UNITS="stream0,stream12") of the default bench configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-units}; shift
mkdir -p $OUT
for u in "$@"; do
  MMSBM_UNITS=$u timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline \
      > $OUT/bench_${u/,/_}.json 2> $OUT/bench_${u/,/_}.err || { tail -5 $OUT/bench_${u/,/_}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_${u/,/_}.json'))
print('$u', 'value %.0f it/s  iter %.1f us' % (d['value'], d['iteration']['us']),
      {k: round(v['back_to_back'],2) for k, v in d['kernel_us'].items()})"
done

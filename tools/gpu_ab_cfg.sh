#!/bin/bash
# A/B of library builds on one bench configuration: BENCH_ARGS="--K 20 --samples 8 ..." and
# each argument a library path ("-" = in-tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-abcfg}; shift
mkdir -p $OUT
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset MMSBM_LIB; else export MMSBM_LIB=$PWD/$lib; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1])
print('$lib', 'value %.1f  iter %.1f us' % (d['value'], d['iteration']['us']),
      {k: round(v['back_to_back'],2) for k, v in d['kernel_us'].items()})"
done

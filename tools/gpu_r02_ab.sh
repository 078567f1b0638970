#!/bin/bash
# A/B of library builds on the default bench: each argument is a library path ("-" = in-tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab}; shift
mkdir -p $OUT
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset MMSBM_LIB; else export MMSBM_LIB=$PWD/$lib; fi
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b$i.json'))
print('$lib', 'value %.0f it/s  iter %.1f us' % (d['value'], d['iteration']['us']),
      {k: round(v['back_to_back'],2) for k, v in d['kernel_us'].items()})"
done

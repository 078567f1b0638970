#!/bin/bash
# hipGraph A/B: the graph test, then bench lines with MMSBM_GRAPH = 0 / 4 / 16 / 64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-graph}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k graph --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for g in 0 4 16 64 0 16; do
  MMSBM_GRAPH=$g timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline \
      > $OUT/bench_g$g.json 2> $OUT/bench_g$g.err || { tail -20 $OUT/bench_g$g.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_g$g.json')); print('G=$g', round(d['value']), d['ms_per_step'])"
done
for g in 0 16; do
  MMSBM_GRAPH=$g timeout -k 10 200 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline --K 20 --samples 8 \
      > $OUT/bench20_g$g.json 2> $OUT/bench20_g$g.err || { tail -20 $OUT/bench20_g$g.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench20_g$g.json')); print('K20x8 G=$g', round(d['value']), d['ms_per_step'])"
done

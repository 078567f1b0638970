#!/bin/bash
# A/B of a candidate build (tools/_build/libmmsbm_pipe.so) against the in-tree build: parity and
# config tests on the candidate, then K=20x8 and K=30 10M bench lines for both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pipe}
mkdir -p $OUT
CAND=$PWD/tools/_build/libmmsbm_pipe.so
MMSBM_LIB=$CAND timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { python3 -c "import json; d=json.load(open('$1')); print('$1', round(d['value'],1), {k: round(v['back_to_back'],1) for k,v in d['kernel_us'].items()})"; }
for lib in base cand; do
  if [ $lib = cand ]; then export MMSBM_LIB=$CAND; else unset MMSBM_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 20 --samples 8 --steps 100 --warmup 5 --roofline-launches 100 \
      > $OUT/k20_$lib.json 2> $OUT/k20_$lib.err || { tail -20 $OUT/k20_$lib.err; exit 1; }
  line $OUT/k20_$lib.json
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --K 30 --P 50000 --E 10000000 --steps 10 --warmup 2 --roofline-launches 5 \
      > $OUT/k30_$lib.json 2> $OUT/k30_$lib.err || { tail -20 $OUT/k30_$lib.err; exit 1; }
  line $OUT/k30_$lib.json
done

#!/bin/bash
# K=10 A/B of tools/_build/libmmsbm_pipe.so against the in-tree build: parity tests on the
# candidate, then alternating bench lines (2000 steps each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab10}
mkdir -p $OUT
CAND=$PWD/tools/_build/libmmsbm_pipe.so
MMSBM_LIB=$CAND timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_joint.py -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { python3 -c "import json; d=json.load(open('$1')); print('$1', round(d['value'],1), {k: round(v['back_to_back'],2) for k,v in d['kernel_us'].items()})"; }
for i in 1 2 3; do
  for lib in base cand; do
    if [ $lib = cand ]; then export MMSBM_LIB=$CAND; else unset MMSBM_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2000 --warmup 50 > $OUT/${lib}_$i.json 2> $OUT/${lib}_$i.err || { tail -20 $OUT/${lib}_$i.err; exit 1; }
    line $OUT/${lib}_$i.json
  done
done

#!/bin/bash
# Big-fin occupancy change at K=20: parity/config tests, then K=20 bench lines (x8 and x1, twice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-fin20}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_joint.py -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { python3 -c "import json; d=json.load(open('$1')); print('$1', round(d['value'],1), {k: round(v['back_to_back'],1) for k,v in d['kernel_us'].items()})"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 20 --samples 8 --steps 100 --warmup 5 --roofline-launches 100 \
      > $OUT/k20_b8_$i.json 2> $OUT/k20_b8_$i.err || { tail -20 $OUT/k20_b8_$i.err; exit 1; }
  line $OUT/k20_b8_$i.json
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 20 --steps 400 --warmup 20 > $OUT/k20_b1.json 2> $OUT/k20_b1.err || { tail -20 $OUT/k20_b1.err; exit 1; }
line $OUT/k20_b1.json

#!/bin/bash
# V-table kernel check: parity + config + joint GPU tests, then the config bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-vtab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_joint.py tests/test_gpu_linkshard.py -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { python3 -c "import json; d=json.load(open('$1')); print('$1', round(d['value'],1), {k: round(v['back_to_back'],1) for k,v in d['kernel_us'].items()})"; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 20 --samples 8 --steps 100 --warmup 5 --roofline-launches 100 \
    > $OUT/k20_b8.json 2> $OUT/k20_b8.err || { tail -20 $OUT/k20_b8.err; exit 1; }
line $OUT/k20_b8.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --K 30 --P 50000 --E 10000000 --steps 10 --warmup 2 --roofline-launches 5 \
    > $OUT/k30_10m.json 2> $OUT/k30_10m.err || { tail -20 $OUT/k30_10m.err; exit 1; }
line $OUT/k30_10m.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --K 20 --steps 400 --warmup 20 > $OUT/k20_b1.json 2> $OUT/k20_b1.err || { tail -20 $OUT/k20_b1.err; exit 1; }
line $OUT/k20_b1.json

#!/bin/bash
# Round-2b iteration check: parity + config + joint GPU tests, then the config bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-iter}; shift
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_joint.py -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/gpu_r02_configs.sh ${OUT#gpurun_out/}
timeout -k 10 300 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json

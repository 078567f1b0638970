#!/bin/bash
# Round-2 joint model check: joint GPU tests, smoke, joint bench, rocprofv3 kernel stats of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/joint
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_joint.py -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python -u tools/bench_joint.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/tools/bench_joint.py "$@" > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | head -20

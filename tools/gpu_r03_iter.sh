#!/bin/bash
# Round 3 kernel iteration: parity tests (default build), the default bench line, stamps.
# usage: bash tools/gpu_r03_iter.sh TAG [TESTS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-iter}; shift
TESTS=${1:-tests/test_gpu_parity.py}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_short.json 2> $OUT/bench_short.err || { tail -20 $OUT/bench_short.err; exit 1; }
for f in bench bench_short; do python3 - $OUT/$f.json $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("%-12s value %.0f it/s  iter %.2f us  L %.13g  frac %.3f" % (sys.argv[2], d["value"], d["iteration"]["us"], d["final_loglik"], d["roofline"]["frac"]),
      {k: (round(v["back_to_back"], 2), round(v["in_loop"], 2)) for k, v in d["kernel_us"].items()})
PY
done
bash tools/gpu_r03_stamp.sh $TAG/stamp > /dev/null || exit 1
cat $OUT/stamp/analysis.txt

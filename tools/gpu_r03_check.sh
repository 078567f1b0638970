#!/bin/bash
# Round 3: all GPU tests, then one default bench line (N=1) and a driver-like short one.
# usage: bash tools/gpu_r03_check.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-check}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/bench_short.json 2> $OUT/bench_short.err || { tail -20 $OUT/bench_short.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
for f in ("bench.json", "bench_short.json"):
    d = json.load(open(sys.argv[1] + "/" + f))
    r = d["roofline"]
    print(f, "value %.0f it/s  iter %.2f us  8d frac %.3f  exec frac %.4f  digest %s" % (
        d["value"], d["iteration"]["us"], r["frac"], r["executed"]["frac"], d["samples"]["digest"]))
    print({k: (round(v["back_to_back"], 2), round(v["in_loop"], 2)) for k, v in d["kernel_us"].items()})
PY

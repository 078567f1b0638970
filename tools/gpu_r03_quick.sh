#!/bin/bash
# Quick GPU iteration: one test file (default the parity tests), then a default bench line.
# usage: bash tools/gpu_r03_quick.sh TAG [TESTS] [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-quick}; shift
TESTS=${1:-tests/test_gpu_parity.py}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench.json"))
r = d["roofline"]
print("value %.0f it/s  iter %.2f us  8d frac %.3f  exec frac %.4f  digest %s" % (
    d["value"], d["iteration"]["us"], r["frac"], r["executed"]["frac"], d["samples"]["digest"]))
print({k: (round(v["back_to_back"], 2), round(v["in_loop"], 2)) for k, v in d["kernel_us"].items()})
print(d["plan"])
PY

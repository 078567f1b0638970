#!/bin/bash
# Round 4: the GPU suite (or a subset: PYTEST_ARGS), smoke(), and a short bench line, each under
# its own time limit; stops at the first failure.
# usage: bash tools/gpu_r04_check.sh TAG [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-check}; shift
SEL=${*:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
grep -E "passed|failed" $OUT/pytest.log | tail -1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || { tail -20 $OUT/bench_short.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
for f in bench_short bench; do python3 - $OUT/$f.json $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("%-12s value %.0f it/s  iter %.2f us  frac %.3f (%s)  traffic %s  cpu %s" % (sys.argv[2], d["value"], d["iteration"]["us"], r["frac"], r.get("frac_basis"), r["traffic"], (d.get("cpu_baseline") or {}).get("value")),
      {k: v and (round(v["back_to_back"], 2), round(v["in_loop"], 2)) for k, v in d["kernel_us"].items()})
PY
done

#!/bin/bash
# Round 3 closing measurements of one build: the whole GPU suite, the rocprofv3 trace + PMC passes
# and the build-stamped traffic record (copied to profiles/ so the bench lines that follow carry
# it), the default and the driver-like bench lines, stamps, and the BASELINE configs 3-5 shares.
# usage: bash tools/gpu_r03_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
bash tools/gpu_r03_prof.sh $TAG/prof $OUT/pmc_r03_K10.json > $OUT/prof.txt 2>&1 || { tail -20 $OUT/prof.txt; exit 1; }
cp $OUT/pmc_r03_K10.json profiles/pmc_r03_K10.json
tail -12 $OUT/prof.txt
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || { tail -20 $OUT/bench_short.err; exit 1; }
for f in bench bench_short; do python3 - $OUT/$f.json $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("%-12s value %.0f it/s  iter %.2f us  frac %.3f  traffic %s  cpu %s" % (sys.argv[2], d["value"], d["iteration"]["us"], r["frac"], r["traffic"], (d.get("cpu_baseline") or {}).get("value")),
      {k: (round(v["back_to_back"], 2), round(v["in_loop"], 2)) for k, v in d["kernel_us"].items()})
PY
done
bash tools/gpu_r03_stamp.sh $TAG/stamp > /dev/null || exit 1
bash tools/gpu_r02_configs.sh $TAG/cfg > $OUT/cfg.txt 2>&1 || { tail -20 $OUT/cfg.txt; exit 1; }
for f in k10_b8 k20_b8 k30_10m; do python3 -c "
import json; d=json.load(open('$OUT/cfg/$f.json')); print('$f', round(d['value'], 1), d['unit'], round(d['iteration']['us'], 1), {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"; done

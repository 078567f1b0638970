#!/bin/bash
# Round 4 closing measurements of one build, part 1: the GPU suite, smoke(), the PMC traffic
# records of the headline (K=10, 1 sample) and of K=10 x 8 / K=20 x 8 (copied to profiles/ on the
# box so the bench lines that follow carry them), the bench lines and the per-wave stamps.
# usage: bash tools/gpu_r04_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
bash tools/gpu_r04_prof.sh $TAG/prof10 $OUT/pmc_r04_K10.json 400 20 > $OUT/prof10.txt 2>&1 || { tail -20 $OUT/prof10.txt; exit 1; }
cp $OUT/pmc_r04_K10.json profiles/pmc_r04_K10.json
bash tools/gpu_r04_prof.sh $TAG/prof10b8 $OUT/pmc_r04_K10_B8.json 100 10 --K 10 --samples 8 > $OUT/prof10b8.txt 2>&1 || { tail -20 $OUT/prof10b8.txt; exit 1; }
cp $OUT/pmc_r04_K10_B8.json profiles/pmc_r04_K10_B8.json
bash tools/gpu_r04_prof.sh $TAG/prof20 $OUT/pmc_r04_K20.json 100 10 --K 20 --samples 8 > $OUT/prof20.txt 2>&1 || { tail -20 $OUT/prof20.txt; exit 1; }
cp $OUT/pmc_r04_K20.json profiles/pmc_r04_K20.json
tail -12 $OUT/prof10.txt
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || { tail -20 $OUT/bench_short.err; exit 1; }
for f in bench bench_short; do python3 - $OUT/$f.json $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("%-12s value %.0f it/s  iter %.2f us  frac %.3f (%s)  traffic %s  cpu %s" % (sys.argv[2], d["value"], d["iteration"]["us"], r["frac"], r.get("frac_basis"), r["traffic"], (d.get("cpu_baseline") or {}).get("value")),
      {k: (round(v["back_to_back"], 2), round(v["in_loop"], 2)) for k, v in d["kernel_us"].items()})
PY
done
bash tools/gpu_r04_configs.sh $TAG/cfg0 > /dev/null 2>&1 || true   # (config lines without the K30 record)
timeout -k 10 300 python -u tools/overhead_probe.py > $OUT/overhead.json 2> $OUT/overhead.err || { tail -5 $OUT/overhead.err; exit 1; }
cat $OUT/overhead.json

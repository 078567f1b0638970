#!/bin/bash
# rocprofv3 kernel trace (stats) of a short bench run; prints the per-kernel summary.
# usage: bash tools/gpu_r03_trace.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${1:-trace}; shift
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 400 --warmup 20 --no-cpu-baseline --roofline-launches 200 "$@" > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    n = row["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    print("%-40s calls %6s  avg %9.0f ns  min %7s  max %7s" % (n[:40], row["Calls"], float(row["AverageNs"]), row["MinNs"], row["MaxNs"]))
PY
python3 -c "
import json; d=json.load(open('$OUT/trace.json'))
print('bench (under trace): %.0f it/s, %.2f us' % (d['value'], d['iteration']['us']), {k: round(v['back_to_back'],2) for k,v in d['kernel_us'].items()})"

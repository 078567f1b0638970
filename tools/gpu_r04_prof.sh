#!/bin/bash
# rocprofv3 kernel-trace stats, then PMC passes (one counter group per pass, each under its own
# time limit) and the build-stamped traffic record, for one bench configuration.
# usage: bash tools/gpu_r04_prof.sh TAG OUT_JSON TRACE_STEPS PMC_STEPS [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
TAG=${1:-prof}; REC=${2:-gpurun_out/pmc.json}; TS=${3:-400}; PS=${4:-20}; shift 4
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps $TS --warmup 5 --no-cpu-baseline --no-events "$@" > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE FETCH_SIZE" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $R/bench.py --steps $PS --warmup 2 --no-cpu-baseline --no-events --roofline-launches 3 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt 2>&1
E_OBS=$(python3 -c "import json; print(json.load(open('$OUT/trace.json'))['config']['E_obs'])")
K=$(python3 -c "import json; print(json.load(open('$OUT/trace.json'))['config']['K'])")
B=$(python3 -c "import json; print(json.load(open('$OUT/trace.json'))['config']['samples_per_gpu'])")
python3 tools/pmc_to_traffic.py $OUT $K $E_OBS $B $REC
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    n = row["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    print("%-40s calls %6s  avg %9.0f ns" % (n[:40], row["Calls"], float(row["AverageNs"])))
PY

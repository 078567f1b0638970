#!/bin/bash
# One parameterised runner for every measurement on the GPU box (replaces the per-round one-shot
# scripts; their outputs under profiles/ stay the provenance of past numbers).
#
#   bash tools/gpu.sh TAG STEP [args] [:: STEP [args] ...]
#
# Outputs go to gpurun_out/TAG/.  Every GPU step runs under its own time limit and the chain
# stops at the first failure (no step is retried).  Steps:
#   tests [pytest args]            the GPU suite (pytest -m gpu), e.g. `tests -k pool`
#   smoke                          __graft_entry__.smoke()
#   bench NAME [bench.py args]     one bench line -> NAME.json (prints a summary)
#   configs                        the headline (2,000 and 20 steps) and the BASELINE config lines
#   prof NAME TRACE_STEPS PMC_STEPS [bench.py args]
#                                  rocprofv3 kernel-trace stats, the PMC passes (one counter
#                                  group per pass) and the build-stamped traffic record NAME.pmc.json
#   ab NAME "bench args" VARIANT...
#                                  A/B on one box, each VARIANT a library path ("-" = in-tree),
#                                  "env:VAR=v,VAR2=v" (in-tree library) or "LIB+env:VAR=v"
#   py NAME SCRIPT [args]          a tools/ script (GPU measurement aid) -> NAME.txt
#   stamp NAME LIB [bench args]    per-wave phase stamps of a stamp build (tools/build_variant.py
#                                  LIB -DMMSBM_STAMP=1), analysed by tools/stamp_analyze.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

summ() {  # one-line summary of a bench JSON line
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-28s %10.1f %s  iter %8.2f us  frac %.3f (credited %.3f, executed %.3f)  %s" % (
    sys.argv[1].split("/")[-1], d["value"], d["unit"], d["iteration"]["us"], r["frac"],
    r["frac_credited"], r["frac_executed"],
    {k: round(v["back_to_back"], 2) for k, v in d["kernel_us"].items()}))
PY
}

bench() {
  local name=$1; shift
  timeout -k 10 500 python -u bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "bench $name failed"; tail -20 "$OUT/$name.err"; return 1; }
  summ "$OUT/$name.json"
}

step() {
  local cmd=$1; shift
  case "$cmd" in
  tests)
    timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread "$@" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; return 1; }
    tail -3 "$OUT/pytest.log" ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; return 1; }
    tail -2 "$OUT/smoke.log" ;;
  bench)
    bench "$@" ;;
  configs)
    bench headline --steps 2000 --warmup 20 --no-cpu-baseline &&
    bench headline_short --no-cpu-baseline &&
    bench k10_b8 --K 10 --samples 8 --steps 200 --warmup 10 --no-cpu-baseline &&
    bench k20_b8 --K 20 --samples 8 --steps 100 --warmup 5 --roofline-launches 100 --no-cpu-baseline &&
    bench k30_10m --K 30 --P 50000 --E 10000000 --test-frac 0 --steps 10 --warmup 2 --roofline-launches 5 --no-cpu-baseline ;;
  prof)
    local name=$1 ts=$2 ps=$3; shift 3
    local P=$OUT/$name
    mkdir -p "$P"
    ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps "$ts" --warmup 5 --no-cpu-baseline --no-events "$@" > "$P/trace.json" 2> "$P/trace.err" ) || { echo "trace failed"; tail -20 "$P/trace.err"; return 1; }
    local i=0
    for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS" \
               "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE FETCH_SIZE" \
               "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      ( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d "$P/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps "$ps" --warmup 2 --no-cpu-baseline --no-events --roofline-launches 3 "$@" > "$P/p$i.log" 2>&1 ) || { echo "pmc pass $i failed"; tail -5 "$P/p$i.log"; return 1; }
    done
    python3 tools/pmc_summary.py "$P" > "$P/pmc_summary.txt" 2>&1
    read -r K E_OBS B < <(python3 -c "import json; c=json.load(open('$P/trace.json'))['config']; print(c['K'], c['E_obs'], c['samples_per_gpu'])")
    python3 tools/pmc_to_traffic.py "$P" "$K" "$E_OBS" "$B" "$OUT/$name.pmc.json"
    cp "$(find "$P/trace" -name "*kernel_stats.csv" | head -1)" "$P/kernel_stats.csv"
    python3 - "$P/kernel_stats.csv" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    n = row["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    print("%-40s calls %6s  avg %9.0f ns" % (n[:40], row["Calls"], float(row["AverageNs"])))
PY
    ;;
  ab)
    local name=$1 args=$2; shift 2
    local i=0
    for v in "$@"; do
      i=$((i+1))
      local envs="" lib="$v"
      unset MMSBM_LIB
      if [ "${v#*+env:}" != "$v" ]; then lib="${v%%+env:*}"; envs=$(echo "${v#*+env:}" | tr ',' ' ');
      elif [ "${v#env:}" != "$v" ]; then lib="-"; envs=$(echo "${v#env:}" | tr ',' ' '); fi
      if [ "$lib" != "-" ]; then export MMSBM_LIB=$R/$lib; fi
      timeout -k 10 500 env $envs python -u bench.py --no-cpu-baseline $args > "$OUT/${name}_$i.json" 2> "$OUT/${name}_$i.err" || { echo "ab $name variant $v failed"; tail -10 "$OUT/${name}_$i.err"; return 1; }
      echo -n "[$v] "; summ "$OUT/${name}_$i.json"
    done
    unset MMSBM_LIB ;;
  stamp)
    local name=$1 lib=$2; shift 2
    MMSBM_STAMP=1 MMSBM_STAMP_DUMP="$OUT/$name.bin" MMSBM_LIB="$R/$lib" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --roofline-launches 5 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "stamp $name failed"; tail -5 "$OUT/$name.err"; return 1; }
    python3 tools/stamp_analyze.py "$OUT/$name.bin" "$OUT/$name.json" > "$OUT/$name.txt" && rm -f "$OUT/$name.bin"
    head -60 "$OUT/$name.txt" ;;
  py)
    local name=$1 script=$2; shift 2
    timeout -k 10 600 python -u "$script" "$@" > "$OUT/$name.txt" 2> "$OUT/$name.err" || { echo "py $name failed"; tail -20 "$OUT/$name.err"; return 1; }
    tail -5 "$OUT/$name.txt" ;;
  *)
    echo "unknown step $cmd"; return 2 ;;
  esac
}

args=()
for a in "$@" "::"; do
  if [ "$a" = "::" ]; then
    if [ ${#args[@]} -gt 0 ]; then
      echo "== ${args[*]}"
      step "${args[@]}" || exit 1
    fi
    args=()
  else
    args+=("$a")
  fi
done
echo "all steps done"

#!/bin/bash
# Headline (fold0 K=10, 1 sample) A/B of the default build against a variant build
# tools/_build/libmmsbm_<VAR>.so (default pvs0: the K^2 P^s stride),
# bench lines and one PMC pass of the LDS counters each.  usage: bash tools/gpu_r04_k10ab.sh TAG [VAR]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${1:-pvs}
mkdir -p $OUT
export TMPDIR=/tmp
VAR=${2:-pvs0}
for v in full $VAR full2 ${VAR}2; do
  unset MMSBM_LIB
  case $v in full*) ;; *) export MMSBM_LIB=$R/tools/_build/libmmsbm_${VAR}.so;; esac
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2000 --warmup 20 > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-trace -d $OUT/pmc_$v/p1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-events --steps 50 --warmup 2 --roofline-launches 3 > $OUT/pmc_$v.log 2>&1) || { echo "pmc $v failed"; tail -5 $OUT/pmc_$v.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/pmc_$v > $OUT/pmc_$v.txt 2>&1
  python3 - $OUT/$v.json $OUT/pmc_$v.txt "$v" <<'PY'
import json, re, sys
d = json.load(open(sys.argv[1]))
txt = open(sys.argv[2]).read()
conf = {}
for blk in txt.split("== ")[1:]:
    head = blk.split("\n")[0]
    if "sk_" not in head:
        continue
    vals = dict(re.findall(r"(SQ_\w+)\s+([\d.]+)", blk))
    conf[head.split("(")[0].strip()] = round(float(vals.get("SQ_LDS_BANK_CONFLICT", 0)) / max(float(vals.get("SQ_LDS_IDX_ACTIVE", 1)), 1), 3)
print(sys.argv[3], "%.0f it/s" % d["value"], "iter %.2f us" % d["iteration"]["us"],
      {k: round(v["back_to_back"], 2) for k, v in d["kernel_us"].items()}, "LDS conflict", conf)
PY
done
unset MMSBM_LIB

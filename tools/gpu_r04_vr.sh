#!/bin/bash
# A/B of pass A's V / theta row strides (MMSBM_VR_ODD=1, the default build, against
# tools/_build/libmmsbm_vr0.so = the round-3 even strides): K=20 x 8 and K=30 on 10M links, bench
# lines plus one PMC pass of the LDS counters per build.  usage: bash tools/gpu_r04_vr.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${1:-vr}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "k20|--K 20 --samples 8 --steps 60 --warmup 5 --roofline-launches 50" "k30|--K 30 --P 50000 --E 10000000 --test-frac 0 --steps 6 --warmup 1 --roofline-launches 5"; do
  IFS='|' read -r name args <<< "$cfg"
  for v in odd vr0; do
    if [ $v = odd ]; then unset MMSBM_LIB; else export MMSBM_LIB=$R/tools/_build/libmmsbm_vr0.so; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > $OUT/${name}_$v.json 2> $OUT/${name}_$v.err || { tail -5 $OUT/${name}_$v.err; exit 1; }
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-trace -d $OUT/pmc_${name}_$v/p1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-events $args > $OUT/pmc_${name}_$v.log 2>&1) || { echo "pmc $name $v failed"; tail -5 $OUT/pmc_${name}_$v.log; exit 1; }
    python3 tools/pmc_summary.py $OUT/pmc_${name}_$v > $OUT/pmc_${name}_$v.txt 2>&1
    python3 - $OUT/${name}_$v.json $OUT/pmc_${name}_$v.txt "$name $v" <<'PY'
import json, re, sys
d = json.load(open(sys.argv[1]))
txt = open(sys.argv[2]).read()
conf = {}
for blk in txt.split("== ")[1:]:
    head = blk.split("\n")[0]
    if "pass_kernel" not in head and "gene_kernel" not in head:
        continue
    vals = dict(re.findall(r"(SQ_\w+)\s+([\d.]+)", blk))
    c, a = float(vals.get("SQ_LDS_BANK_CONFLICT", 0)), float(vals.get("SQ_LDS_IDX_ACTIVE", 1))
    conf[head.split("<")[0][-11:]] = "%.3f" % (c / max(a, 1))
print(sys.argv[3], "%.1f it/s" % d["value"], "iter %.1f us" % d["iteration"]["us"],
      {k: round(v["back_to_back"], 1) for k, v in d["kernel_us"].items()}, "lds conflict", conf)
PY
  done
done
unset MMSBM_LIB

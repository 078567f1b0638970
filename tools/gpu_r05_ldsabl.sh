#!/bin/bash
# Where the fused small-K kernel's LDS bank conflicts come from: builds of a scratch copy of the
# sources (tools/_build/libmmsbm_lds<bit>.so, -DLDSABL=bit; timings and counters only, results
# invalid) that point one kind of LDS read at conflict-free addresses: 1 = V-table formation's
# P^s reads, 2 = the V operand loads, 4 = the Z-operand transpose reads, 8 = the X contraction's
# M and P^s reads, 16 = the S scoop's theta and M reads.  One PMC pass each, fold0 K=10.
# usage: bash tools/gpu_r05_ldsabl.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${1:-ldsabl}
mkdir -p $OUT
export TMPDIR=/tmp
for v in full lds1 lds2 lds4 lds8 lds16; do
  unset MMSBM_LIB
  [ $v != full ] && export MMSBM_LIB=$R/tools/_build/libmmsbm_$v.so
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-trace -d $OUT/pmc_$v/p1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-events --steps 50 --warmup 2 --roofline-launches 3 > $OUT/pmc_$v.log 2>&1) || { echo "pmc $v failed"; tail -5 $OUT/pmc_$v.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/pmc_$v > $OUT/pmc_$v.txt 2>&1
  python3 - $OUT/pmc_$v.txt "$v" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for blk in txt.split("== ")[1:]:
    head = blk.split("\n")[0]
    if "sk_pass_kernel<10, 3>" not in head:
        continue
    vals = dict(re.findall(r"(SQ_\w+)\s+([\d.]+)", blk))
    c, a = float(vals["SQ_LDS_BANK_CONFLICT"]), float(vals["SQ_LDS_IDX_ACTIVE"])
    print("%-6s fused: conflict cycles %.0f of %.0f LDS cycles (%.3f), %s" % (sys.argv[2], c, a, c / a, head.split("(")[1].strip(") ")))
PY
done
unset MMSBM_LIB

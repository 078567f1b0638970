#!/bin/bash
# Round 3: the small-K kernels with grouped chunk chains, pass A + pass B vs the fused E-step
# (MMSBM_SK_FUSED=1): parity tests of both, default bench lines, stamps of both.
# usage: bash tools/gpu_r03_fused.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-fused}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for F in 0 1; do
  MMSBM_SK_FUSED=$F timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $OUT/pytest_f$F.log 2>&1 || { tail -60 $OUT/pytest_f$F.log; exit 1; }
  echo "fused=$F: $(tail -1 $OUT/pytest_f$F.log)"
done
for FU in 0:- 1:- 1:1536,3072; do
  F=${FU%%:*}; U=${FU##*:}
  if [ "$U" = - ]; then unset MMSBM_UNITS; else export MMSBM_UNITS=$U; fi
  MMSBM_SK_FUSED=$F timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline "$@" > $OUT/bench_f${F}_$U.json 2> $OUT/bench_f${F}_$U.err || { tail -20 $OUT/bench_f${F}_$U.err; exit 1; }
  python3 - $OUT/bench_f${F}_$U.json $F $U <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("fused=%s units %s value %.0f it/s  iter %.2f us  L %.12g" % (sys.argv[2], sys.argv[3], d["value"], d["iteration"]["us"], d["final_loglik"]),
      {k: (round(v["back_to_back"], 2), round(v["in_loop"], 2)) for k, v in d["kernel_us"].items()}, d["plan"]["wg_stream0"], d["plan"]["wg_stream12"])
PY
done
for F in 0 1; do
  unset MMSBM_UNITS
  MMSBM_SK_FUSED=$F bash tools/gpu_r03_stamp.sh $TAG/stamp_f$F > /dev/null || exit 1
  echo "== stamps fused=$F"; cat $OUT/stamp_f$F/analysis.txt
done

#!/bin/bash
# Stamp build (tools/_build/libmmsbm_stamp.so, -DMMSBM_STAMP=1): per-wave phase cycles of one bench
# configuration, analysed on the box.  usage: bash tools/gpu_r03_stamp.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-stamp}; shift
mkdir -p $OUT
MMSBM_STAMP=1 MMSBM_STAMP_DUMP=$PWD/$OUT/stamp.bin MMSBM_LIB=$PWD/tools/_build/libmmsbm_stamp.so \
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --roofline-launches 5 "$@" \
    > $OUT/stamp.json 2> $OUT/stamp.err || { tail -5 $OUT/stamp.err; exit 1; }
python3 tools/stamp_analyze.py $OUT/stamp.bin > $OUT/analysis.txt && rm -f $OUT/stamp.bin
cat $OUT/analysis.txt

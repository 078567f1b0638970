#!/bin/bash
# Quick GPU iteration: parity tests, one bench line, then the stamp build's phase cycles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-quick}; shift
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value %.0f it/s  iter %.1f us' % (d['value'], d['iteration']['us']))
print({k: (round(v['back_to_back'],2), round(v['in_loop'],2)) for k, v in d['kernel_us'].items()})"
MMSBM_STAMP=1 MMSBM_LIB=$PWD/tools/_build/libmmsbm_stamp.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --roofline-launches 5 "$@" > $OUT/stamp.json 2> $OUT/stamp.err || { tail -5 $OUT/stamp.err; exit 1; }
grep "mmsbm stamp" $OUT/stamp.err | tail -4

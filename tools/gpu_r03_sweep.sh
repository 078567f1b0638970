#!/bin/bash
# Round 3: the whole GPU suite, then the default bench at E +-6.25 / 12.5 / 18.75 / 25 % and on hub-heavy folds
# (no cliff across E, skewed within 15 % of uniform).
# usage: bash tools/gpu_r03_sweep.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
for spec in 67500: 73125: 78750: 84375: 90000: 95625: 101250: 106875: 112500: 90000:0.02,0.3 90000:0.01,0.6 90000:0.05,0.5; do
  E=${spec%%:*}; H=${spec##*:}
  tag=e${E}_h${H}
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline --roofline-launches 200 --E $E ${H:+--hub $H} > $OUT/$tag.json 2> $OUT/$tag.err || { tail -10 $OUT/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$tag.json'))
p=d['plan']
print('E %6d hub %-9s %7.0f it/s  %6.2f us  E_obs %6d  units %5d  wg %4d' % ($E, '$H' or '-', d['value'], d['iteration']['us'], d['config']['E_obs'], p['units'], p['wg_stream0'] + p['wg_stream12']),
      {k: round(v['back_to_back'],2) for k, v in d['kernel_us'].items()})"
done

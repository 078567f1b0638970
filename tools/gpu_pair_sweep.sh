#!/bin/bash
# Joint model: parts-per-workgroup sweep of the pair launch (MMSBM_PAIR_PARTS), bench_joint lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pairsweep}; shift
mkdir -p $OUT
for n in "$@"; do
  MMSBM_PAIR_PARTS=$n timeout -k 10 200 python -u tools/bench_joint.py > $OUT/p$n.json 2> $OUT/p$n.err || { tail -5 $OUT/p$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/p$n.json'))
print('parts $n', 'value %.0f  iter %.1f us' % (d['value'], d['ms_per_step'] * 1e3), d['split_us'], d['pair_plan']['pair_em_wgs'])"
done

#!/bin/bash
# Environment sweep of the default bench: each argument is "VAR=value[;VAR2=value2]" ("-" = none).
# usage: bash tools/gpu_r02_env.sh TAG [--bench-args ...] -- SETTING ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-env}; shift
BA=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do BA+=("$1"); shift; done
shift
mkdir -p $OUT
i=0
for setting in "$@"; do
  i=$((i+1))
  envs=()
  if [ "$setting" != "-" ]; then IFS=';' read -ra envs <<< "$setting"; fi
  env "${envs[@]}" timeout -k 10 200 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline "${BA[@]}" \
      > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b$i.json'))
print('$setting', 'value %.1f  iter %.1f us' % (d['value'], d['iteration']['us']),
      {k: round(v['back_to_back'],2) for k, v in d['kernel_us'].items()}, 'wg_a', d['plan']['wg_stream0'])"
done

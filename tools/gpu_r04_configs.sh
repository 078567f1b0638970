#!/bin/bash
# BASELINE configs 3-5 per-GPU shares on one MI355X: bench lines into gpurun_out/$TAG
# (config 5: 10M TRAIN links, --test-frac 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }; python3 -c "
import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']
print('$name', round(d['value'], 1), d['unit'], 'iter %.1f us' % d['iteration']['us'], 'frac %.3f (%s)' % (r['frac'], r['frac_basis']), {k: round(v['back_to_back'], 1) for k, v in d['kernel_us'].items()})"; }
run k10_b8 --K 10 --samples 8 --steps 200 --warmup 10
run k20_b8 --K 20 --samples 8 --steps 100 --warmup 5 --roofline-launches 100
run k30_10m --K 30 --P 50000 --E 10000000 --test-frac 0 --steps 10 --warmup 2 --roofline-launches 5
echo done

# Bench lines for the other BASELINE configs (measurement): K=20 x 8 samples, K=30 on a larger fold.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline --K 20 --samples 8 --steps 20 --warmup 3 --roofline-launches 20 > $OUT/k20_b8.json 2> $OUT/k20_b8.err || { echo "k20 failed"; tail -5 $OUT/k20_b8.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/k20_b8.json'));print('k20_b8', round(d['value']), d['ms_per_step'], d['kernel_us'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --K 10 --samples 8 --steps 50 --warmup 5 --roofline-launches 50 > $OUT/k10_b8.json 2> $OUT/k10_b8.err || { echo "k10b8 failed"; tail -5 $OUT/k10_b8.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/k10_b8.json'));print('k10_b8', round(d['value']), d['ms_per_step'], d['kernel_us'], d['roofline']['frac'])"
timeout -k 10 600 python bench.py --no-cpu-baseline --K 30 --samples 1 --P 50000 --E 1000000 --steps 3 --warmup 1 --roofline-launches 3 > $OUT/k30_1m.json 2> $OUT/k30_1m.err || { echo "k30 failed"; tail -5 $OUT/k30_1m.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/k30_1m.json'));print('k30_1m', d['value'], d['ms_per_step'], d['kernel_us'], d['roofline']['frac'])"

# A/B of the S-accumulation kernel: product build vs build/libmmsbm_occ2.so (-DMX_OCC4=0),
# K=20 x 8 samples and K=30 on 1M links.  usage: bash tools/gpu_m1x_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-m1xab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
show() { python -c "import json;d=json.load(open('$1'));print('$2', round(d['value'],1), d['ms_per_step'], {k: round(v,1) for k,v in d['kernel_us'].items()}, round(d['roofline']['frac'],3))"; }
for v in prod occ2; do
  if [ $v = occ2 ]; then export MMSBM_LIB=$GRAFT_REPO_ROOT/build/libmmsbm_occ2.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --K 20 --samples 8 --steps 20 --warmup 3 --roofline-launches 20 > $OUT/k20_b8_$v.json 2> $OUT/k20_$v.err || { echo "k20 $v failed"; tail -5 $OUT/k20_$v.err; exit 1; }
  show $OUT/k20_b8_$v.json k20_b8_$v
  timeout -k 10 300 python bench.py --no-cpu-baseline --K 30 --samples 1 --P 50000 --E 1000000 --steps 3 --warmup 1 --roofline-launches 3 > $OUT/k30_1m_$v.json 2> $OUT/k30_$v.err || { echo "k30 $v failed"; tail -5 $OUT/k30_$v.err; exit 1; }
  show $OUT/k30_1m_$v.json k30_1m_$v
done

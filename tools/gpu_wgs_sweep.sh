# Workgroups-per-sample sweep (MMSBM_SACC_WGS) on batched configs.  usage: bash tools/gpu_wgs_sweep.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-wgs}
mkdir -p $OUT
run() {  # label, env, args
  env $2 timeout -k 10 300 python bench.py --no-cpu-baseline $3 > $OUT/$1.json 2> $OUT/$1.err || { echo "$1 failed"; tail -5 $OUT/$1.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1', round(d['value'],1), {k: round(x,1) for k,x in d['kernel_us'].items()}, round(d['roofline']['frac'],3), round(d['final_loglik'],6))"
}
for g in 256 128 64 32; do
  run k10b8_g$g MMSBM_SACC_WGS=$g "--K 10 --samples 8 --steps 50 --warmup 5 --roofline-launches 50"
done
for g in 256 128 64 32; do
  run k20b8_g$g MMSBM_SACC_WGS=$g "--K 20 --samples 8 --steps 20 --warmup 3 --roofline-launches 20"
done

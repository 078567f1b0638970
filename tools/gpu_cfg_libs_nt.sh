# One bench config across measurement builds, no tests (product + build/<lib>.so ...), twice.
# usage: bash tools/gpu_cfg_libs_nt.sh TAG "bench args" lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for v in prod "$@"; do
    if [ $v = prod ]; then unset MMSBM_LIB; else export MMSBM_LIB=$GRAFT_REPO_ROOT/build/$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err || { echo "$v failed"; tail -5 $OUT/$v.$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v.$rep.json'));print('$v', round(d['value'],1), {k: round(x,1) for k,x in d['kernel_us'].items()}, round(d['roofline']['frac'],3), round(d['final_loglik'],6))"
  done
done

# A/B of measurement builds on the default bench: product build, then each build/<lib>.so
# given (MMSBM_LIB), twice in alternation.  usage: bash tools/gpu_libs_ab.sh TAG lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for v in prod "$@"; do
    if [ $v = prod ]; then unset MMSBM_LIB; else export MMSBM_LIB=$GRAFT_REPO_ROOT/build/$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err || { echo "$v failed"; tail -5 $OUT/$v.$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v.$rep.json'));print('$v', round(d['value']), {k: round(x,2) for k,x in d['kernel_us'].items()}, round(d['final_loglik'],9))"
  done
done

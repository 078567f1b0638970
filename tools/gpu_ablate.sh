# E-step ablation builds (measurement): bench each libmmsbm_ab*.so, report E back-to-back time.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ablate}
mkdir -p $OUT
for lib in trigenicinteractionpredictor_amd/_build/libmmsbm.so trigenicinteractionpredictor_amd/_build/libmmsbm_ab*.so; do
  tag=$(basename $lib .so)
  MMSBM_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
  echo "$tag $(python -c "import json;d=json.load(open('$OUT/$tag.json'));print(round(d['value']), d['kernel_us'])")"
done

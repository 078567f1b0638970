# A/B of runtime switches on the default bench.  usage: bash tools/gpu_env_ab.sh TAG "label|ENV=v ..." ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "base|" "$@"; do
  IFS='|' read -r label envs <<< "$v"
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > $OUT/$label.json 2> $OUT/$label.err || { echo "$label failed"; tail -5 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));print('$label', round(d['value']), {k: round(x,2) for k,x in d['kernel_us'].items()}, round(d['final_loglik'],9))"
done

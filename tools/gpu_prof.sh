# rocprofv3 kernel-trace stats for bench variants: bash tools/gpu_prof.sh TAG "label|ENV|args" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-prof}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  IFS='|' read -r label envs args <<< "$v"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$label -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-events $args > $OUT/$label.json 2>$OUT/$label.err || exit 1
done
echo done

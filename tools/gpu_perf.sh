# Perf probe on the GPU box: parity tests, bench variants, optional rocprofv3 kernel stats.
# usage: bash tools/gpu_perf.sh TAG "label|ENV=a ENV2=b|--bench-args" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
fi
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 2
for v in "$@"; do
  IFS='|' read -r label envs args <<< "$v"
  env $envs timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline $args > $OUT/bench_$label.json 2>$OUT/bench_$label.err || exit 3
done
if [ -n "$PROFILE" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_bench.json 2>&1 || exit 4
fi
echo done

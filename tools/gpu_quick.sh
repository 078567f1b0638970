# Quick GPU check: parity tests, bench, traced bench (needs the measurement build
# trigenicinteractionpredictor_amd/_build/libmmsbm_trace.so: build.command(out, ['-DEMX_TRACE=1'])),
# optional variant benches.
# usage: bash tools/gpu_quick.sh TAG ["label|ENV=a|--bench-args" ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
MMSBM_LIB=trigenicinteractionpredictor_amd/_build/libmmsbm_trace.so MMSBM_TRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 2 > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -20 $OUT/trace.err; exit 3; }
grep "mmsbm trace" $OUT/trace.err | tail -2
for v in "$@"; do
  IFS='|' read -r label envs args <<< "$v"
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline $args > $OUT/bench_$label.json 2>$OUT/bench_$label.err || { echo "variant $label failed"; tail -5 $OUT/bench_$label.err; exit 4; }
  echo "$label: $(python -c "import json;d=json.load(open('$OUT/bench_$label.json'));print(round(d['value']), d['kernel_us'])")"
done
echo done

# GPU tests, default bench, rocprofv3 kernel trace of the same bench with in-loop medians.
# usage: bash tools/gpu_bench_prof.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-bp}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 2; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', round(d['value']), d['ms_per_step'], d['kernel_us'], d['roofline']['frac'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "rocprof failed"; tail -20 $OUT/prof_bench.err; exit 3; }
python $GRAFT_REPO_ROOT/tools/trace_loop.py $OUT/prof/run_kernel_trace.csv

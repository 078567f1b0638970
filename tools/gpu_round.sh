# Round check on the GPU box: gpu parity tests, smoke, default bench (with cpu_baseline),
# rocprofv3 kernel-trace stats of the same bench command.  usage: bash tools/gpu_round.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-round}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rocminfo > $OUT/rocminfo.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 2; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 3; }
cat $OUT/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "rocprof failed"; tail -20 $OUT/prof_bench.err; exit 4; }
cat $OUT/prof_bench.json
echo done

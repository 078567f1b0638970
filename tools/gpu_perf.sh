# Perf probe on the GPU box: parity tests, bench, ablations, rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 2
for ab in 1 2 3; do
  MMSBM_ABLATE=$ab timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/$TAG/bench_ablate$ab.json 2>/dev/null || exit 3
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.json 2>&1 || exit 4
echo done

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "Marketing Name|gfx950" > gpurun_out/r1_info.txt || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 && \
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/r1_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 10 > gpurun_out/r1_bench.log 2>&1
echo "exit $?"

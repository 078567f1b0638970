#!/bin/bash
# Round-2 GPU check: every -m gpu test (one process, per-test time limit), then one bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?
tail -c 3000 gpurun_out/bench.json
exit $(( rc > rc2 ? rc : rc2 ))

#!/bin/bash
# smoke() and the 2-rank (gloo, both ranks on one GPU) restart-sharded bench with its replay digest, on one build.
# usage: bash tools/gpu_r03_smoke2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-smoke2}; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo --no-cpu-baseline > $OUT/ranks2.json 2> $OUT/ranks2.err || { tail -20 $OUT/ranks2.err; exit 1; }
tail -c 400 $OUT/ranks2.json

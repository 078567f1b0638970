# Rehearse the N-rank bench path on one GPU: 2 ranks share cuda:0, collectives over gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ranks}
mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo --roofline-launches 20 > $OUT/bench2.json 2> $OUT/bench2.err || { echo "2-rank bench failed"; tail -20 $OUT/bench2.err; exit 1; }
cat $OUT/bench2.json

# Rehearse the N-rank bench path on one GPU: 2 ranks share cuda:0, collectives over gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ranks}
mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo --roofline-launches 20 > $OUT/bench2.json 2> $OUT/bench2.err || { echo "2-rank bench failed"; tail -20 $OUT/bench2.err; exit 1; }
cat $OUT/bench2.json
# link-sharded single sample: 1 rank, then 2 ranks sharing the GPU (all-reduce over gloo)
timeout -k 10 300 python bench.py --shard links --steps 50 --warmup 5 --no-cpu-baseline --roofline-launches 20 > $OUT/links1.json 2> $OUT/links1.err || { echo "links x1 failed"; tail -20 $OUT/links1.err; exit 2; }
cat $OUT/links1.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --shard links --steps 50 --warmup 5 --backend gloo --roofline-launches 20 > $OUT/links2.json 2> $OUT/links2.err || { echo "links x2 failed"; tail -20 $OUT/links2.err; exit 3; }
cat $OUT/links2.json

# The multi-GPU launch path (torch.distributed.run, RCCL process group, max-over-ranks timing)
# at N=1 on the one-GPU box; the driver runs N=2..8 on a full node.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dist}
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 > $O/bench_dist1.json 2> $O/bench_dist1.err
echo "exit $?"

# kernel trace of the default bench (GPU busy union) + HW-queue A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-trace}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_q8.json 2> $O/bench_q8.err && \
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_q16.json 2> $O/bench_q16.err
echo "exit $?"

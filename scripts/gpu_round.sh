set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r1
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/r1/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --ref-len 100000000 --pairs 200000 --cpu-pairs 50000 --steps 2 > gpurun_out/r1/bench_small.json 2> gpurun_out/r1/bench_small.err && \
timeout -k 10 900 python bench.py --stats-out gpurun_out/r1/stats_full.json > gpurun_out/r1/bench_full.json 2> gpurun_out/r1/bench_full.err
echo "exit $?"

# Site-check pre-pass check: all GPU tests, then two benches (sites on).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-st}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err && \
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err
echo "exit $?"

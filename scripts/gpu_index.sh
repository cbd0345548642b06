# GPU index-build check: index parity tests + one bench (index phases in the log).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ix}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_index_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_index.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "exit $?"

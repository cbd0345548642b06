# Parity tests + isolated kernel timings (kab.py) + a default bench.  Usage: bash scripts/gpu_quick.sh TAG [kab variants...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-q}
shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python scripts/kab.py "$@" > $O/kab.jsonl 2> $O/kab.err && \
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "exit $?"

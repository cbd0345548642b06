# Parity tests + isolated kernel timings (kab.py) + default bench (+ extra host thread counts in $THREADS).
# Usage: [THREADS="24 32"] bash scripts/gpu_quick.sh TAG [kab variants...]
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
rc=$?
echo "exit $rc"
[ $rc -ne 0 ] && exit $rc
for T in $THREADS; do
  timeout -k 10 400 python bench.py --threads $T --no-cpu-baseline > $O/bench_t$T.json 2> $O/bench_t$T.err || exit $?
done
echo "all ok"

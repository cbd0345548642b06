# GPU round: parity tests, smoke, bench.  Usage: bash scripts/gpu_round.sh TAG [extra bench thread counts...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --stats-out $O/stats_full.json > $O/bench_full.json 2> $O/bench_full.err
rc=$?
echo "exit $rc"
[ $rc -ne 0 ] && exit $rc
for T in "$@"; do
  timeout -k 10 400 python bench.py --threads $T --no-cpu-baseline > $O/bench_t$T.json 2> $O/bench_t$T.err || exit $?
done
echo "all ok"

# Every BASELINE.json config through bench.py (with the CPU baseline leg and SAM parity on its sample).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-configs}
mkdir -p $O
for W in pe150_3g pe250_3g pe150_250m se100_5m; do
  timeout -k 10 400 python3 bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || exit $?
done
echo "exit 0"

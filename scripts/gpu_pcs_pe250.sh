# Host PC samples of the default bench (NO_PCS=1: skipped), then a kernel trace of the PE 2x250 workload
# (trace + stats only; summary with the GPU busy union via scripts/prof_summary.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pcs_pe250}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$NO_PCS" ]; then
  RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --no-multi-device --steps 5 > $O/bench.json 2> $O/bench.err || exit $?
  echo "pcs done"
fi
P=$O/prof_pe250
mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/trace -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --no-multi-device --steps 4 --warmup 2 > $P/bench_trace.json 2> $P/bench_trace.err || exit $?
python3 scripts/prof_summary.py $P $P/sum > /dev/null || exit $?
find $P -name "*.db" -delete
find $P -name "*.csv" -size +1M -delete
echo "trace done"

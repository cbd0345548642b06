# rocprofv3 passes over the default bench command (kernel trace + stats, then
# one PMC pass per TCC counter, as MI355X_MICROARCH.md prescribes), summarised
# on the box (scripts/prof_summary.py) and the databases dropped, so what comes
# back stays under gpurun's 64 MiB.
# Usage: bash scripts/gpu_prof.sh TAG   (BENCH_ARGS overrides the bench flags;
# the environment passes through, e.g. RSA_BUCKET_LINES=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 6 --warmup 2"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/bench_trace.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/bench_write.json 2> $OUT/bench_write.err
rc=$?
echo "profile exit $rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/prof_summary.py $OUT $OUT/sum || exit $?
find $OUT -name "*.db" -delete
find $OUT -name "*.csv" -size +1M -delete
ls $OUT

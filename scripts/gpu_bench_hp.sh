# bench (no CPU leg) + host-only replay scaling, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-bhp}
mkdir -p $O
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err && \
timeout -k 10 500 ./oracle/_ref/host_prof 3000000000 24 1000000 2 1 16 > $O/hp.txt 2>&1
echo "exit $?"

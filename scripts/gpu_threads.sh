# Host-thread sweep of the default bench (is the mapping host- or GPU-bound?).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-thr}
mkdir -p $O
for t in 16 8 12 16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --threads $t > $O/b_$t.json 2> $O/b_$t.err || exit $?
done
echo "exit 0"

# Repeated default benches (no CPU baseline), to read the per-step spread.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rep}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$i.json 2> $O/b_$i.err || exit $?
done
echo "exit 0"

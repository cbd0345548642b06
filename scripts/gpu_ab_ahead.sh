# A/B of the record/result prefetch distance (RSA_PREFETCH_AHEAD 4 default vs 8 vs 2), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abahead}
mkdir -p $O
for i in 1 2; do
  for v in 4 8 2; do
    RSA_PREFETCH_AHEAD=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
  done
done
echo "exit 0"

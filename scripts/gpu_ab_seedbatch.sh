# A/B of chunks per seeding call (RSA_SEED_BATCH 1 default vs 2), alternating, default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-absb}
mkdir -p $O
for i in 1 2 3; do
  for v in 1 2; do
    RSA_SEED_BATCH=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
  done
done
echo "exit 0"

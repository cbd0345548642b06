# A/B of extra waiting workers (RSA_WAIT_WORKERS 8 default vs 4 vs 12), alternating, default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abww4}
mkdir -p $O
for i in 1 2; do
  for v in ${WW_LIST:-8 4 12}; do
    RSA_WAIT_WORKERS=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
  done
done
echo "exit 0"

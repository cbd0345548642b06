# Extra wait workers under callback waits: 8 (default) vs 24 vs 16, alternating, 5 timed steps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abww3}
mkdir -p $O
for i in 1 2; do
  for w in 8 24 16; do
    RSA_WAIT_WORKERS=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/b_w${w}_$i.json 2> $O/b_w${w}_$i.err || exit $?
  done
done
echo "exit 0"

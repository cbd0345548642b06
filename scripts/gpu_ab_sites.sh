# A/B of the site-check pre-pass (RSA_SITES=0 off), alternating, 8 timed steps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-absites}
mkdir -p $O
for i in 1 2; do
  for v in 1 0; do
    RSA_SITES=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 > $O/b${v}_$i.json 2> $O/b${v}_$i.err || exit $?
  done
done
echo "exit 0"

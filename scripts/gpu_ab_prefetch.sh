# A/B of the prefetches in the store phase (RSA_PREFETCH=1 default vs 0),
# alternating, 10 timed steps each; then host PC samples of the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abpf}
mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    RSA_PREFETCH=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
  done
done
RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/pcs_bench.json 2> $O/pcs_bench.err || exit $?
echo "exit 0"

# Extra wait workers A/B under callback waits (RSA_WAIT_WORKERS), plus a host PC profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abww2}
mkdir -p $O
rm -f $O/pcs.txt
RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/pcs_bench.json 2> $O/pcs_bench.err || exit $?
for w in 8 16 24 4; do
  RSA_WAIT_WORKERS=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/b_w$w.json 2> $O/b_w$w.err || exit $?
done
echo "exit 0"

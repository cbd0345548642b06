# Host PC samples of the mapping under the GPU engine (RSA_PC_SAMPLE), 16 threads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pcs}
mkdir -p $O
rm -f $O/pcs.txt
RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/bench.json 2> $O/bench.err
echo "exit $?"

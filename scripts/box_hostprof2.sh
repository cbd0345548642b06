# PC-sampled host profile of the replayed pipeline on the GPU box's cores.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-hostprof2}
mkdir -p $O
HP_SAMPLE=$O/pcs16.txt timeout -k 10 500 ./oracle/_ref/host_prof 3000000000 24 1000000 6 16 > $O/hp16.txt 2>&1 && \
HP_SAMPLE=$O/pcs1.txt timeout -k 10 500 ./oracle/_ref/host_prof 3000000000 24 500000 3 1 > $O/hp1.txt 2>&1
echo "exit $?"

# Host-only pipeline scaling on the GPU box's cores (record/replay, no GPU work).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-hostprof}
mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled > $O/thp.txt 2>&1
lscpu > $O/lscpu.txt 2>&1
timeout -k 10 500 ./oracle/_ref/host_prof 3000000000 24 1000000 2 1 8 16 24 > $O/hp.txt 2>&1
echo "exit $?"

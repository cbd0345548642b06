# Wait-worker / HW-queue variants of the host pipeline on the headline workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ww}
mkdir -p $O
nproc > $O/host.txt; cat /sys/fs/cgroup/cpu.max >> $O/host.txt 2>&1; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/host.txt; free -g >> $O/host.txt
V="RSA_WAIT_WORKERS=0 RSA_WAIT_WORKERS=8 RSA_WAIT_WORKERS=16 RSA_WAIT_WORKERS=0 RSA_WAIT_WORKERS=16 RSA_WAIT_WORKERS=24"
timeout -k 10 300 python3 scripts/kab.py --pairs 1000000 --threads 16 $V > $O/hwq4.jsonl 2> $O/hwq4.err && \
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 scripts/kab.py --pairs 1000000 --threads 16 $V > $O/hwq16.jsonl 2> $O/hwq16.err
echo "exit $?"

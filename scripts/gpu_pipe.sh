# Host pipeline variants on the default bench.  Usage: bash scripts/gpu_pipe.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pipe}
mkdir -p $O
B="python bench.py --no-cpu-baseline --pairs 500000"
RSA_SPIN_WAIT=1 RSA_PREFETCH=0 timeout -k 10 300 $B > $O/spin_nopf.json 2> $O/spin_nopf.err && \
RSA_SPIN_WAIT=1 timeout -k 10 300 $B > $O/spin_pf.json 2> $O/spin_pf.err && \
RSA_PREFETCH=0 timeout -k 10 300 $B > $O/block_nopf.json 2> $O/block_nopf.err && \
timeout -k 10 300 $B > $O/block_pf.json 2> $O/block_pf.err && \
timeout -k 10 300 $B --threads 24 > $O/block_pf_t24.json 2> $O/block_pf_t24.err && \
RSA_PREFETCH=0 timeout -k 10 300 $B --threads 24 > $O/block_nopf_t24.json 2> $O/block_nopf_t24.err
echo "exit $?"

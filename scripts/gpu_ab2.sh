# bench + host pipeline A/B (prefetch of reference windows, wait workers).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab2}
mkdir -p $O
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python3 scripts/kab.py --pairs 1000000 --threads 16 RSA_PREFETCH_REF=0 RSA_PREFETCH_REF=1 RSA_WAIT_WORKERS=0 RSA_WAIT_WORKERS=8 RSA_PREFETCH_REF=0 RSA_PREFETCH_REF=1 RSA_WAIT_WORKERS=0 RSA_WAIT_WORKERS=8 > $O/kab.jsonl 2> $O/kab.err
echo "exit $?"

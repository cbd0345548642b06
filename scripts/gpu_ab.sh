# Isolated per-kernel timings (one host thread, so no concurrent kernels) for
# kernel variants selected by environment switches.  Usage: bash scripts/gpu_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}
O=gpurun_out/$TAG
mkdir -p $O
B="python bench.py --threads 1 --pairs 100000 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 $B > $O/wave.json 2> $O/wave.err && \
RSA_RS_LANE=1 RSA_FN_LANE=1 timeout -k 10 300 $B > $O/lane.json 2> $O/lane.err
echo "exit $?"

# Kernel + memory-copy trace of a bench workload (no counters): the GPU's kernel and
# DMA activity over the mapping span (scripts/busy_copies.py).  Usage: bash scripts/gpu_copies.sh TAG [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-copies}
shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-multi-device --steps 4 --warmup 2 "$@" > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/busy_copies.py $(find $O/trace -name "*.db" | head -1) > $O/busy.txt 2>&1 || { cat $O/busy.txt; exit 1; }
cat $O/busy.txt
find $O -name "*.db" -delete

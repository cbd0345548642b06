# Kernel-variant A/B (scripts/kab.py) on the GPU box.  Usage: bash scripts/gpu_ab.sh TAG VARIANT...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python scripts/kab.py "$@" > gpurun_out/$TAG/kab.jsonl 2> gpurun_out/$TAG/kab.err
echo "exit $?"

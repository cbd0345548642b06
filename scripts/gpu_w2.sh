# Extension parity first (pair scan, two-layout scan, forced rescans), then the round.
# Usage: bash scripts/gpu_w2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-w2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_extend_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_ext.log 2>&1
rc=$?; tail -3 $O/pytest_ext.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_round.sh $TAG

# GPU tests with the stream-callback waits, then an A/B of the wait mechanism
# (RSA_WAIT=callback default vs event), alternating, 5 timed steps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abwait}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for i in 1 2; do
  for v in callback event; do
    RSA_WAIT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
  done
done
echo "exit 0"

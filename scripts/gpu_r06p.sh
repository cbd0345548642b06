# Round 6: every GPU test, twice (separate processes, no -x), to catch a rare SAM difference
# (test_multi_device_gpu reports the differing lines now).  An assertion failure lets the
# second pass run; a fault, abort or time limit ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06p}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu_$i.log 2>&1
  rc=$?
  tail -3 $O/pytest_gpu_$i.log
  grep -A30 "^E " $O/pytest_gpu_$i.log | head -60
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stop"; exit $rc; fi
done
echo "all ok"

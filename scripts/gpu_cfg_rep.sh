# Config SAM parity (tests/test_configs_gpu.py, all four configs in one process), run twice
# in one call; a mismatch leaves its first differing records in gpurun_out/samdiff_*.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cfgrep}
mkdir -p $O
for pass in 1 2; do
  timeout -k 10 540 python -u -m pytest tests/test_configs_gpu.py -q --timeout 500 --timeout-method thread > $O/pass$pass.log 2>&1
  rc=$?
  echo "pass $pass: exit $rc $(tail -1 $O/pass$pass.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done

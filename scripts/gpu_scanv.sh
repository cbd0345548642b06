# k_ext_scan_v check: extension parity tests, then isolated A/B of the scan kernels
# (RSA_SCAN_V=0: k_ext_scan_g) at chunk and combined-call sizes.  Usage: bash scripts/gpu_scanv.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-scanv}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_extend_gpu.py tests/test_host_cases_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_ext.log 2>&1 || { tail -30 $O/pytest_ext.log; exit 1; }
tail -3 $O/pytest_ext.log
for V in 0 1; do
  RSA_SCAN_V=$V RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 7300 22000 65536 > $O/scan_v$V.txt 2>&1 || exit $?
  echo "RSA_SCAN_V=$V"; cat $O/scan_v$V.txt
done

# Extension parity (oracle + GPU e2e SAM), then the isolated scan timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-extiter}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_extend_gpu.py tests/test_e2e_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_ext.log 2>&1
rc=$?; tail -3 $O/pytest_ext.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/micro/scan_bench.py 1 7300 65536 > $O/scan_bench.txt 2>&1 || exit $?
cat $O/scan_bench.txt

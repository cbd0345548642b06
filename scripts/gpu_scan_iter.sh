# Extension parity tests + isolated scan timing vs batch size (scripts/micro/scan_bench.py) + kab.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_extend_gpu.py tests/test_e2e_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/micro/scan_bench.py > $O/scan_bench.txt 2>&1 || exit $?
grep "n=" $O/scan_bench.txt
timeout -k 10 300 python scripts/kab.py --threads 1 --pairs 60000 > $O/kab.jsonl 2> $O/kab.err || exit $?
cat $O/kab.jsonl

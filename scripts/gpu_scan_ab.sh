# GPU parity tests (all, or PYTEST_ARGS), then the isolated extension-kernel timing
# (scripts/micro/scan_bench.py) of this tree vs ab/librsa_gpu_old.so, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/scanab
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
SCAN_BENCH_LIB=$GRAFT_REPO_ROOT/ab/librsa_gpu_old.so timeout -k 10 120 python scripts/micro/scan_bench.py 7300 22000 65536 > $O/old_$r.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/micro/scan_bench.py 7300 22000 65536 > $O/new_$r.txt 2>&1 || exit 1
echo old; grep n= $O/old_$r.txt; echo new; grep n= $O/new_$r.txt
done

# Round 6: the scan's shared code-4 profile row -- extension parity tests, then isolated
# A/B against abtmp/librsa_gpu_base.so (round-5 kernel) at 150 and 250 bp.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06e}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_extend_gpu.py tests/test_host_cases_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_ext.log 2>&1 || { tail -30 $O/pytest_ext.log; exit 1; }
tail -2 $O/pytest_ext.log
for rep in 1 2; do
  for L in 150 250; do
    SCAN_BENCH_L=$L RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 4000 12700 22000 > $O/scan_new_${L}_$rep.txt 2>&1 || exit 1
    SCAN_BENCH_L=$L SCAN_BENCH_LIB=abtmp/librsa_gpu_base.so RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 4000 12700 22000 > $O/scan_base_${L}_$rep.txt 2>&1 || exit 1
    echo "== L=$L new $rep"; grep -v amdgpu.ids $O/scan_new_${L}_$rep.txt; echo "== L=$L base $rep"; grep -v amdgpu.ids $O/scan_base_${L}_$rep.txt
  done
done
echo "all ok"

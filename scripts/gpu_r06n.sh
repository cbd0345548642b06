# Round 6: redo after the panel pass -- determinism of repeated mappings (the buggy build
# abtmp/base6 against this one), the multi-device test, the extension tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06n}
mkdir -p $O
for b in base6 fix; do
  cp abtmp/$b/librsa_gpu.so abtmp/$b/librsalign.so rabbitsalign_amd/lib/ || exit 1
  echo "== $b"
  timeout -k 10 300 python3 scripts/micro/det_check.py > $O/det_$b.txt 2>&1 || { tail -20 $O/det_$b.txt; exit 1; }
  grep -v amdgpu.ids $O/det_$b.txt
done
timeout -k 10 600 python -u -m pytest tests/test_multi_device_gpu.py tests/test_extend_gpu.py tests/test_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo "all ok"

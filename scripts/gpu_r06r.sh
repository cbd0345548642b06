# Round 6: the index tests then the multi-device test (the order of the one failing
# suite run), repeated in fresh processes; the multi-device test reports differing lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06r}
mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python -u -m pytest tests/test_index_gpu.py tests/test_multi_device_gpu.py -v --timeout 200 --timeout-method thread > $O/pt_$i.log 2>&1
  rc=$?
  echo "rep $i rc $rc: $(tail -1 $O/pt_$i.log)"
  grep -A12 "^E " $O/pt_$i.log | head -30
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop"; exit $rc; fi
done
echo "all ok"

# Round 6: every GPU test with RSA_POISON=2 (every lane buffer refilled with 0xA5 at the start of
# each call: a kernel that reads what an earlier call left behind fails), then the multi-device
# SAM diff under the same mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06x2}
mkdir -p $O
RSA_POISON=2 timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_poison2.log 2>&1
rc=$?
tail -3 $O/pytest_poison2.log
grep -E "^FAILED|^E " $O/pytest_poison2.log | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stop"; exit $rc; fi
RSA_POISON=2 timeout -k 10 400 python3 scripts/micro/multi_dev_diff.py 6 /tmp/mdd > $O/mdd_poison2.txt 2>&1 || { tail -30 $O/mdd_poison2.txt; exit 1; }
grep -v amdgpu.ids $O/mdd_poison2.txt | tail -20
echo "all ok"

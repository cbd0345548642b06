# Round 6: reference tail padding and the entry past the last randstrobe initialised in both
# open paths -- every GPU test, smoke, and repeated two-context mappings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06aa}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 scripts/micro/multi_dev_diff.py 10 /tmp/mdd > $O/mdd.txt 2>&1 || { tail -30 $O/mdd.txt; exit 1; }
grep -v amdgpu.ids $O/mdd.txt | tail -3
echo "all ok"

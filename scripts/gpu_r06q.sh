# Round 6: multi-device SAM vs one context with the added context on the .sti table layout
# (RSA_BUCKET_LINES=0) while the first keeps its bucket lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06q}
mkdir -p $O
MDD_LINES2=0 timeout -k 10 500 python3 scripts/micro/multi_dev_diff.py 6 /tmp/mdd > $O/mdd_lines2.txt 2>&1 || { tail -30 $O/mdd_lines2.txt; exit 1; }
grep -v amdgpu.ids $O/mdd_lines2.txt | tail -60
echo "all ok"

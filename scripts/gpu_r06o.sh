# Round 6: the multi-device SAM against the one-context SAM, repeated, with the differing lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06o}
mkdir -p $O
timeout -k 10 500 python3 scripts/micro/multi_dev_diff.py ${REPS:-12} /tmp/mdd > $O/mdd.txt 2>&1 || { tail -30 $O/mdd.txt; exit 1; }
grep -v amdgpu.ids $O/mdd.txt | tail -60
echo "all ok"

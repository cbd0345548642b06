# Round 6, first call: fresh SQ counters of the round-5 score scan (isolated launches),
# then the round-5 exit-time abort's command once more with the process's mappings
# dumped at exit (RSA_MAPS_OUT), so a native stack trace can be attributed.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06a}
mkdir -p $O
bash scripts/gpu_ext_pmc.sh ${1:-r06a}/extpmc > $O/extpmc.log 2>&1 || { tail -20 $O/extpmc.log; exit 1; }
cat $O/extpmc/pmc_summary.txt
RSA_MAPS_OUT=$O/maps.txt timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/tl -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --steps 3 --warmup 1 > $O/tl.json 2> $O/tl.err
rc=$?
echo "tl exit $rc"
tail -25 $O/tl.err
find $O/tl -name "*.db" -delete
exit 0

# Round 5: device timeline of PE 2x250 (kernel trace only) and isolated seeding
# kernels at 250 bp.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/tl -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --steps 3 --warmup 1 > $O/tl.json 2> $O/tl.err || { tail -20 $O/tl.err; exit 1; }
python3 scripts/timeline.py $(find $O/tl -name "*.db" | head -1) > $O/timeline.txt; cat $O/timeline.txt
python3 scripts/prof_summary.py $O $O/sum > /dev/null
find $O/tl -name "*.db" -delete
RSA_KTIMER_EVERY=1 timeout -k 10 300 python3 scripts/micro/seed_bench.py --read-len 250 --calls 20 > $O/seed250.txt 2>&1 || exit 1
tail -30 $O/seed250.txt
echo "all ok"

# Round 5: GPU tests after the adaptive seeding download; PE 2x250 bench with
# stats; device timeline of PE 2x250 (kernel + memory-copy trace, no counters);
# isolated seeding kernels at 250 bp.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05e}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python bench.py --workload pe250_3g --no-cpu-baseline --steps 8 --warmup 3 --stats-out $O/stats_pe250.json > $O/bench_pe250.json 2> $O/bench_pe250.err || { tail -20 $O/bench_pe250.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/stats_pe250.json'))['kernel_stats'];print('second trips', d['seed_second_trips'], 'seed calls', d['seed_calls'], d['calls_ms'])"
grep -E "step [0-9]:" $O/bench_pe250.err | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/tl -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --steps 3 --warmup 1 > $O/tl.json 2> $O/tl.err || { tail -20 $O/tl.err; exit 1; }
python3 scripts/timeline.py $(find $O/tl -name "*.db" | head -1) > $O/timeline.txt; cat $O/timeline.txt
find $O/tl -name "*.db" -delete
RSA_KTIMER_EVERY=1 timeout -k 10 300 python3 scripts/micro/seed_bench.py --read-len 250 --calls 20 > $O/seed250.txt 2>&1 || exit 1
tail -30 $O/seed250.txt
echo "all ok"

# Round 6 final tree: every BASELINE config through bench.py (CPU leg + SAM parity on its sample), then
# the PE 2x250 device timeline (kernel trace, torch-free process) for its kernel shares.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06u}
mkdir -p $O
for W in pe150_3g pe250_3g pe150_250m se100_5m; do
  timeout -k 10 500 python3 bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail -20 $O/bench_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$W.json'));print('$W','value',d['value'],'inmem',d['in_memory']['value'],'cpu',d['cpu_baseline']['value'],'parity',d['parity'].get('sam_identical'))"
done
RSA_BENCH_NO_TORCH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --steps 4 --warmup 2 > $O/kt.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
python3 scripts/timeline.py $(find $O/kt -name "*.db" | head -1) > $O/pe250_timeline.txt
mkdir -p $O/pe250prof && mv $O/kt $O/pe250prof/trace && python3 scripts/prof_summary.py $O/pe250prof $O/pe250 > /dev/null
find $O -name "*.db" -delete
head -25 $O/pe250_rocprof.md
echo "all ok"

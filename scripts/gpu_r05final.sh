# Round 5 record: every GPU test, the smoke test, the default bench, PE 2x250.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], 'mem', d['in_memory']['value'], 'core_us', d['host_cpu']['core_us_per_read'], 'cpu', d['cpu_baseline']['value'], 'roofline', d['roofline']['kernel'], d['roofline']['frac'])"
timeout -k 10 500 python bench.py --workload pe250_3g --no-cpu-baseline --steps 8 --warmup 3 > $O/bench_pe250.json 2> $O/bench_pe250.err || { tail -20 $O/bench_pe250.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_pe250.json'));print('pe250', d['value'], 'mem', d['in_memory']['value'])"
echo "all ok"

# Round 6 final tree (test switches added): every GPU test + smoke, the default bench (with the CPU leg),
# fresh SQ counters of the scan, and the kernel trace + FETCH/WRITE passes of the default
# bench (torch-free process: one ROCm runtime, the profiler's).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06z}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],'inmem',d['in_memory']['value'],'cpu',d['cpu_baseline']['value'],'parity',d['parity'].get('sam_identical'))"
bash scripts/gpu_ext_pmc.sh ${1:-r06z}/extpmc > $O/extpmc.log 2>&1 || { tail -20 $O/extpmc.log; exit 1; }
grep scan_v $O/extpmc/pmc_summary.txt
RSA_BENCH_NO_TORCH=1 bash scripts/gpu_prof.sh ${1:-r06z} > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -3 $O/prof.log
echo "all ok"

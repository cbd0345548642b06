# Round 5 checkpoint: every GPU test, the seeding-kernel A/B (old vs new, kernel trace),
# the default bench (with the CPU leg), then the rocprofv3 trace + FETCH/WRITE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05b}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash scripts/gpu_sites_ab.sh ${TAG}_seed old n5 2>&1 | grep -E "^old|^n5" || exit 1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('value',d['value'],'mem',d['in_memory']['value'],'core_us',d['host_cpu']['core_us_per_read'],'cpu',(d['cpu_baseline'] or {}).get('value'),'parity',(d['parity'] or {}).get('sam_identical'),'head',r.get('kernel'),r.get('avg_launch_us'),r.get('frac'),[ (k['kernel'],k['avg_launch_us']) for k in r['top_kernels']])"
bash scripts/gpu_prof.sh $TAG > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -E "k_sites|k_seed_query|k_find_nams_w2|k_ext_scan_v|k_seed_scan|k_seed_count|k_compact|GPU busy" gpurun_out/prof_$TAG/sum_rocprof.md | head -20
echo "all ok"

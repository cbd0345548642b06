# Final-tree record for a round: every GPU test, smoke, the default bench (with the CPU
# leg), then the rocprofv3 kernel trace + FETCH/WRITE PMC passes.  Usage: bash scripts/gpu_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],'mem',d['in_memory']['value'],'core_us',d['host_cpu']['core_us_per_read'],'cpu',(d['cpu_baseline'] or {}).get('value'),'parity',(d['parity'] or {}).get('sam_identical'),'scan',d['roofline']['achieved'])"
bash scripts/gpu_prof.sh $TAG || exit $?
echo "all ok"

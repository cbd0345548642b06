# Round-4 GPU check: parity tests, smoke, bench (N=1), the bench's launcher with
# more GPUs than visible (must fail cleanly), and the product's multi-device leg
# rehearsed as two engines on GPU 0.  Usage: bash scripts/gpu_r04.sh TAG [notests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "notests" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
  tail -3 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
timeout -k 10 600 python bench.py --stats-out $O/stats_full.json > $O/bench_full.json 2> $O/bench_full.err || exit $?
python -c "import json;d=json.load(open('$O/bench_full.json'));print('value',d['value'],'mem',d['in_memory']['value'],'core_us',d['host_cpu']['core_us_per_read'],'cpu',(d['cpu_baseline'] or {}).get('value'),'parity',(d['parity'] or {}).get('sam_identical'))"
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_g2.json 2> $O/bench_g2.err
echo "bench --gpus 2 on one GPU: exit $? (2 expected)"; tail -2 $O/bench_g2.err
RSA_BENCH_DEVICES=0,0 timeout -k 10 400 python bench.py --multi-device-leg --gpus 2 --steps 3 > $O/bench_md00.json 2> $O/bench_md00.err || exit $?
cat $O/bench_md00.json
echo "all ok"

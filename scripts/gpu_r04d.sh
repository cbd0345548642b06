# Round-4 batch: extension parity tests, the N-rank rehearsal, PE250 with the wider band64
# grid, and an A/B of the combined-extension leaders.  Usage: bash scripts/gpu_r04d.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04d}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_extend_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_ext.log 2>&1 || { tail -20 $O/pytest_ext.log; exit 1; }
tail -1 $O/pytest_ext.log
bash scripts/gpu_rehearse.sh $TAG/rehearse || exit $?
timeout -k 10 300 python3 bench.py --workload pe250_3g --steps 6 --warmup 3 --no-cpu-baseline > $O/pe250.json 2> $O/pe250.err || exit $?
python3 -c "import json;d=json.load(open('$O/pe250.json'));print('pe250',d['value'],d['in_memory']['value'],{k:v['avg_us'] for k,v in d['kernels'].items() if 'ext' in k})"
REPS=2 STEPS=8 bash scripts/gpu_ab_env.sh $TAG/ab "" "RSA_EXT_LEADERS=1" || exit $?
echo "all ok"

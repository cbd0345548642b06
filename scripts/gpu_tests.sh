# GPU parity tests (+ optional short bench). Usage: bash scripts/gpu_tests.sh TAG [bench]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-t}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
if [ "$2" = "bench" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline --stats-out $O/stats.json > $O/bench.json 2> $O/bench.err || exit $?
  python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d['roofline'].get('kernel'), d['roofline'].get('avg_launch_us'))"
fi
echo "all ok"

# GPU parity tests, then isolated kernel times (scripts/kab.py, one host thread) and a short bench.
# Usage: bash scripts/gpu_tests_kab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kab.py --threads 1 --pairs 60000 RSA_EXT_GROUP=1 RSA_EXT_GROUP=6 > $O/kab.jsonl 2> $O/kab.err || exit $?
cat $O/kab.jsonl
timeout -k 10 400 python bench.py --no-cpu-baseline --stats-out $O/stats.json > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['achieved'], r['frac'])"

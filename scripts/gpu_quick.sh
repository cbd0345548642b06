# Quick GPU check after a change: the given test files (default: every GPU test), smoke,
# and a short bench.  Usage: bash scripts/gpu_quick.sh TAG [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-quick}
shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest ${@:-tests -m gpu} -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 6 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],'mem',d['in_memory']['value'],'core_us',d['host_cpu']['core_us_per_read'],'cpu',(d['cpu_baseline'] or {}).get('value'),'parity',(d['parity'] or {}).get('sam_identical'),'scan',d['roofline']['achieved'])"

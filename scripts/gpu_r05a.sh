# Round 5: every GPU test (incl. the rank/world part mode and exact .sti ties), then the
# N=2 rehearsal of bench.py's shared-input rank mode (both ranks on GPU 0, gloo).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
RSA_BENCH_REHEARSE=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 4 --warmup 3 --no-cpu-baseline --no-multi-device > $O/bench_g2.json 2> $O/bench_g2.err
rc=$?
echo "rehearsal exit $rc"
tail -8 $O/bench_g2.err
python3 -c "import json;d=json.load(open('$O/bench_g2.json'));print({k:d.get(k) for k in ('value','n_gpus','ms_per_step')}, d.get('parity'), d.get('shared_input'))"
exit $rc

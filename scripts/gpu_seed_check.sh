set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/seedscan
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_seed_gpu.py tests/test_e2e_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || exit 1
python3 scripts/prof_summary.py $O $O/sum > /dev/null && grep -E "k_seed_scan|k_compact|k_sites|GPU busy" $O/sum_rocprof.md
find $O -name "*.db" -delete
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['in_memory']['value'], d['device_counters']['calls_ms'])"

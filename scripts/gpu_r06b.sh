# Round 6: scan staging rework -- extension parity tests, isolated A/B of the scan
# (this tree vs abtmp/librsa_gpu_base.so = the round-5 kernel), SQ counters, short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_extend_gpu.py tests/test_host_cases_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_ext.log 2>&1 || { tail -30 $O/pytest_ext.log; exit 1; }
tail -2 $O/pytest_ext.log
for rep in 1 2; do
  RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 7300 12700 22000 > $O/scan_new_$rep.txt 2>&1 || exit 1
  SCAN_BENCH_LIB=abtmp/librsa_gpu_base.so RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 7300 12700 22000 > $O/scan_base_$rep.txt 2>&1 || exit 1
  echo "== new $rep"; cat $O/scan_new_$rep.txt; echo "== base $rep"; cat $O/scan_base_$rep.txt
done
bash scripts/gpu_ext_pmc.sh ${1:-r06b}/extpmc > $O/extpmc.log 2>&1 || { tail -20 $O/extpmc.log; exit 1; }
grep scan_v $O/extpmc/pmc_summary.txt
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 6 --warmup 2 --stats-out $O/stats.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],'inmem',d['in_memory'].get('value'));r=d['roofline'];print(json.dumps(r.get('ext_scan',r))[:600])"
echo "all ok"

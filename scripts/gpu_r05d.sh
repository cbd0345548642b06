# Round 5: every GPU test (wave-cooperative rescue, scan query in LDS); scan A/B
# (lib_ab/n5 = previous scan); PE 2x250 and PE 2x150 benches with kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in old new; do
  if [ $v = old ]; then export SCAN_BENCH_LIB=rabbitsalign_amd/lib_ab/n5/librsa_gpu.so; else unset SCAN_BENCH_LIB; fi
  RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 7300 12700 22000 > $O/scan_$v.txt 2>&1 || exit 1
  echo "scan $v"; grep "^n=" $O/scan_$v.txt
done
unset SCAN_BENCH_LIB
for wl in pe250_3g pe150_3g; do
  timeout -k 10 500 python bench.py --workload $wl --no-cpu-baseline --steps 8 --warmup 3 --stats-out $O/stats_$wl.json > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));k=d['kernels'];print('$wl', d['value'], 'mem', d['in_memory']['value'], 'core_us', d['host_cpu']['core_us_per_read'], {n:k[n]['avg_us'] for n in k})"
done
echo "all ok"

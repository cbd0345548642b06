# Round 5: PE 2x150 and PE 2x250 benches with kernel stats (after the seeding rework).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g}
mkdir -p $O
for wl in ${WLS:-pe150_3g pe250_3g}; do
  timeout -k 10 500 python bench.py --workload $wl --no-cpu-baseline --steps 8 --warmup 3 --stats-out $O/stats_$wl.json > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));k=d['kernels'];print('$wl', d['value'], 'mem', d['in_memory']['value'], 'core_us', d['host_cpu']['core_us_per_read'], {n:k[n]['avg_us'] for n in k})"
  grep -E "step [0-9]:" $O/bench_$wl.err | tail -1
done

if [ -n "$PCS" ]; then
  RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --no-multi-device --steps 5 > $O/pcs_bench.json 2> $O/pcs_bench.err || exit 1
  echo "pcs ok"
fi
echo "all ok"

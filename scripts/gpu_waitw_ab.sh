# RSA_WAIT_WORKERS A/B (extra workers parked in device waits: default 3/4 of the threads = 12,
# then 6 and 0), two rounds; the figures are host core-us a read and the streamed rate.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-waitab}
mkdir -p $O
for r in 1 2; do
  for w in ${WS:-12 6 0}; do
    RSA_WAIT_WORKERS=$w timeout -k 10 400 python bench.py --no-cpu-baseline --no-multi-device --steps 8 --warmup 3 > $O/bench_w${w}_$r.json 2> $O/bench_w${w}_$r.err || { tail -20 $O/bench_w${w}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_w${w}_$r.json'));print('RSA_WAIT_WORKERS=$w round $r', d['value'], 'mem', d['in_memory']['value'], 'core_us', d['host_cpu']['core_us_per_read'], 'sys', d['host_cpu'].get('sys_fraction'))"
  done
done

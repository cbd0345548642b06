# RSA_WAIT_WORKERS 12 vs 6 on PE 2x250 (device-bound), two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-wait250}
mkdir -p $O
for r in 1 2; do
  for w in 12 6; do
    RSA_WAIT_WORKERS=$w timeout -k 10 400 python bench.py --workload pe250_3g --no-cpu-baseline --no-multi-device --steps 6 --warmup 3 > $O/b_w${w}_$r.json 2> $O/b_w${w}_$r.err || { tail -20 $O/b_w${w}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_w${w}_$r.json'));print('pe250 RSA_WAIT_WORKERS=$w round $r', d['value'], 'mem', d['in_memory']['value'], 'core_us', d['host_cpu']['core_us_per_read'])"
  done
done

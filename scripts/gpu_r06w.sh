# Round 6: k_seed_query's 256-bp LDS class (21 KB a block) at 6 / 7 waves a SIMD against the
# 512-bp class at 5 -- seeding parity tests, isolated launches at 150 / 250 bp on a 3 Gb
# index (settings alternated in one process), then the headline and PE 2x250 benches A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06w}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_seed_gpu.py tests/test_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for L in 150 250; do
  timeout -k 10 400 python3 scripts/micro/seed_bench.py --read-len $L --calls 12 --rounds 3 \
    --ab "RSA_SEED_SHORT=0|RSA_SEED_SHORT=1|RSA_SEED_SHORT=7" > $O/seed_ab_$L.txt 2>&1 || { tail -20 $O/seed_ab_$L.txt; exit 1; }
  grep '"env"' $O/seed_ab_$L.txt
done
summ() {
python3 - $1 <<'EOF2'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for v in d["ab"]:
    k = v["kern"]
    print(v["env"], "median", v["median"], "mean", v["mean"], {n: k[n].get("us_per_launch") for n in k if isinstance(k[n], dict)})
EOF2
}
timeout -k 10 600 python bench.py --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 4 --ab-steps 4 \
  --ab "RSA_SEED_SHORT=0|RSA_SEED_SHORT=1|RSA_SEED_SHORT=7" > $O/ab150.json 2> $O/ab150.err || { tail -20 $O/ab150.err; exit 1; }
summ $O/ab150.json
timeout -k 10 600 python bench.py --workload pe250_3g --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 3 --ab-steps 4 \
  --ab "RSA_SEED_SHORT=0|RSA_SEED_SHORT=1" > $O/ab250.json 2> $O/ab250.err || { tail -20 $O/ab250.err; exit 1; }
summ $O/ab250.json
echo "all ok"

# Round 6: host PC samples of the headline bench (fresh breakdown of the workers' CPU),
# then PE 2x250 k_ext_band16 capacity 8192 vs 16384 (nibble cells), alternating in one process.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06l}
mkdir -p $O
echo "root $GRAFT_REPO_ROOT"
RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 > $O/bench_pcs.json 2> $O/bench_pcs.err || { tail -20 $O/bench_pcs.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_pcs.json'));print('pcs bench value',d['value'],'inmem',d['in_memory']['value'],'core_us',d['host_cpu']['core_us_per_read'])"
timeout -k 10 700 python bench.py --workload pe250_3g --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 5 --ab-steps 4 \
  --ab "RSA_BAND16_DIRCAP=8192|RSA_BAND16_DIRCAP=16384" > $O/ab250.json 2> $O/ab250.err || { tail -20 $O/ab250.err; exit 1; }
python3 - $O/ab250.json <<'EOF2'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for v in d["ab"]:
    k = v["kern"]
    print(v["env"], "median", v["median"], "mean", v["mean"], "rates", v.get("rates"), {n: k[n].get("us_per_launch") for n in k if isinstance(k[n], dict)})
EOF2
echo "all ok"

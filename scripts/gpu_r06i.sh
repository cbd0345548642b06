# Round 6: in-stream redo pass -- extension parity tests (all three redo paths), then
# RSA_REDO_DEV=0 (host path) vs the default, alternating in one process, PE 2x150 and 2x250.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06i}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_extend_gpu.py tests/test_host_cases_gpu.py tests/test_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_ext.log 2>&1 || { tail -30 $O/pytest_ext.log; exit 1; }
tail -2 $O/pytest_ext.log
summ() {
python3 - $1 <<'EOF2'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for v in d["ab"]:
    k = v["kern"]
    fe = sorted(b - a for a, b in v["first_ext_ms"])
    print(v["env"], "median", v["median"], "mean", v["mean"], "first ext ms med", round(fe[len(fe)//2], 2), {n: k[n].get("us_per_launch") for n in k if isinstance(k[n], dict)}, "scan Gcells/s", k.get("scan_gcells_s"))
EOF2
}
timeout -k 10 600 python bench.py --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 4 --ab-steps 4 \
  --ab "RSA_REDO_DEV=0|RSA_REDO_DEV=128" > $O/ab150.json 2> $O/ab150.err || { tail -20 $O/ab150.err; exit 1; }
summ $O/ab150.json
timeout -k 10 600 python bench.py --workload pe250_3g --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 3 --ab-steps 4 \
  --ab "RSA_REDO_DEV=0|RSA_REDO_DEV=128" > $O/ab250.json 2> $O/ab250.err || { tail -20 $O/ab250.err; exit 1; }
summ $O/ab250.json
echo "all ok"

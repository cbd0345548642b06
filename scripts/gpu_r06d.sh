# Round 6: seeding + e2e parity (k_sites 8 lanes a NAM); wave priority of the extension
# kernels (s_setprio, RSA_EXT_SETPRIO) and k_sites lanes (RSA_SITES_G) A/B on the
# headline and on PE 2x250, alternating in one process; then the memory-copy-trace profile
# of PE 2x250 without torch (one ROCm runtime in the process).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_seed_gpu.py tests/test_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_seed.log 2>&1 || { tail -30 $O/pytest_seed.log; exit 1; }
tail -2 $O/pytest_seed.log
summ() {
python3 - $1 <<'EOF2'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for v in d["ab"]:
    k = v["kern"]
    print(v["env"], "median", v["median"], "mean", v["mean"], {n: k[n].get("us_per_launch") for n in k if isinstance(k[n], dict)}, "scan Gcells/s", k.get("scan_gcells_s"))
EOF2
}
timeout -k 10 600 python bench.py --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 4 --ab-steps 4 \
  --ab "RSA_EXT_SETPRIO=0,RSA_SITES_G=16|RSA_EXT_SETPRIO=1,RSA_SITES_G=16|RSA_EXT_SETPRIO=1,RSA_SITES_G=8" > $O/ab150.json 2> $O/ab150.err || { tail -20 $O/ab150.err; exit 1; }
summ $O/ab150.json
timeout -k 10 600 python bench.py --workload pe250_3g --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 3 --ab-steps 4 \
  --ab "RSA_EXT_SETPRIO=0,RSA_SITES_G=16|RSA_EXT_SETPRIO=1,RSA_SITES_G=16|RSA_EXT_SETPRIO=1,RSA_SITES_G=8" > $O/ab250.json 2> $O/ab250.err || { tail -20 $O/ab250.err; exit 1; }
summ $O/ab250.json
RSA_BENCH_NO_TORCH=1 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/tl -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --steps 3 --warmup 1 > $O/tl.json 2> $O/tl.err
echo "memory-copy-trace profile (no torch) exit $?"; grep -E "tool finalization|SIGSEGV|Aborted" $O/tl.err | head -5
find $O/tl -name "*.db" -delete
echo "all ok"

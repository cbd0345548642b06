# Round 6: nibble-packed direction matrix in k_ext_band16 (5-6 waves a SIMD instead of
# 3-5) -- extension parity tests, isolated band timing at 150 / 250 bp (this build vs
# abtmp/base6 = the previous commit), PE 2x250 capacity A/B (8192 vs 16384) in one process,
# then the PE 2x250 and default benches alternating the two builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06k}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_extend_gpu.py tests/test_host_cases_gpu.py tests/test_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_ext.log 2>&1 || { tail -30 $O/pytest_ext.log; exit 1; }
tail -2 $O/pytest_ext.log
for L in 150 250; do
  for b in nib base6; do
    SCAN_BENCH_L=$L SCAN_BENCH_LIB=abtmp/$b/librsa_gpu.so RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 7300 22000 > $O/micro_${b}_$L.txt 2>&1 || exit 1
    echo "== $b L=$L"; grep -v amdgpu.ids $O/micro_${b}_$L.txt
  done
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
timeout -k 10 600 python bench.py --workload pe250_3g --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 3 --ab-steps 4 \
  --ab "RSA_BAND16_DIRCAP=8192|RSA_BAND16_DIRCAP=16384" > $O/ab250.json 2> $O/ab250.err || { tail -20 $O/ab250.err; exit 1; }
summ $O/ab250.json
for i in 1 2; do
  for b in base6 nib; do
    cp abtmp/$b/librsa_gpu.so abtmp/$b/librsalign.so rabbitsalign_amd/lib/ || exit 1
    timeout -k 10 400 python bench.py --workload pe250_3g --no-cpu-baseline --warmup 3 --steps 8 > $O/pe250_${b}_$i.json 2> $O/pe250_${b}_$i.err || { tail -20 $O/pe250_${b}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/pe250_${b}_$i.json'));k=d['kernels'];print('pe250 $b $i value',d['value'],'inmem',d['in_memory']['value'],'band16 us',k.get('ext_band',{}).get('avg_us'),'band64 us',k.get('ext_band_wide',{}).get('avg_us'),'parity',d.get('parity',{}).get('sam_identical'))"
  done
done
for b in base6 nib; do
  cp abtmp/$b/librsa_gpu.so abtmp/$b/librsalign.so rabbitsalign_amd/lib/ || exit 1
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/pe150_$b.json 2> $O/pe150_$b.err || { tail -20 $O/pe150_$b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pe150_$b.json'));k=d['kernels'];print('pe150 $b value',d['value'],'inmem',d['in_memory']['value'],'band16 us',k.get('ext_band',{}).get('avg_us'),'parity',d.get('parity',{}).get('sam_identical'))"
done
echo "all ok"

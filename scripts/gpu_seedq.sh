# Seeding GPU tests, then per-phase cycles (RSA_SEED_PROF build) and the product
# kernels' isolated times at 150 and 250 bp.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-seedq}
mkdir -p $O
if [ "${TESTS}" != none ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_seed_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_seed.log 2>&1 || { tail -30 $O/pytest_seed.log; exit 1; }
tail -1 $O/pytest_seed.log
fi
for L in 150 250; do
  RSA_GPU_LIB=rabbitsalign_amd/lib_ab/prof/librsa_gpu.so timeout -k 10 300 python3 scripts/micro/seed_bench.py --read-len $L --calls 20 > $O/prof$L.txt 2>&1 || { tail $O/prof$L.txt; exit 1; }
  timeout -k 10 300 python3 scripts/micro/seed_bench.py --read-len $L --calls 20 > $O/seed$L.txt 2>&1 || { tail $O/seed$L.txt; exit 1; }
  echo "== $L"; grep seedprof $O/prof$L.txt | tail -2
  python3 -c "import json,sys;t=open('$O/seed$L.txt').read();d=json.loads(t[t.index('{'):]);print({k:v['avg_us'] for k,v in d['kernels'].items()}, d['wall_ms_per_call'])"
done

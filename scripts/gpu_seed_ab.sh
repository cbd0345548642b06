# Isolated seeding calls (profiling builds) for the given lib_ab variants, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-seedab}
shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    RSA_GPU_LIB=rabbitsalign_amd/lib_ab/$v/librsa_gpu.so timeout -k 10 300 python3 scripts/micro/seed_bench.py --calls 20 > $O/$v.$rep.txt 2>&1 || { tail $O/$v.$rep.txt; exit 1; }
    echo "== $v $rep"; grep "query/wave" $O/$v.$rep.txt | tail -1 | sed 's/.*lookup: //'
    python3 -c "import json;t=open('$O/$v.$rep.txt').read();d=json.loads(t[t.index('{'):]);print({k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done

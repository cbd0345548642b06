# Isolated seeding calls at three reference sizes (bucket-line tables of 2, 8 and 32 GB):
# does the fused kernel's load issue stall follow the table size?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-seedref}
mkdir -p $O
for R in 3e8 1e9 3e9; do
  RSA_GPU_LIB=rabbitsalign_amd/lib_ab/prof/librsa_gpu.so timeout -k 10 300 python3 scripts/micro/seed_bench.py --ref-len $R --calls 20 > $O/r$R.txt 2>&1 || { tail $O/r$R.txt; exit 1; }
  echo "== ref $R"; grep "^index" $O/r$R.txt; grep "query/wave" $O/r$R.txt | tail -1 | sed 's/.*lookup: //'
  python3 -c "import json;t=open('$O/r$R.txt').read();d=json.loads(t[t.index('{'):]);print({k:v['avg_us'] for k,v in d['kernels'].items()})"
done

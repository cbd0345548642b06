# Per-phase cycles of the fused query kernel and k_find_nams_w2 (RSA_SEED_PROF build
# in lib_ab/prof) on isolated seeding calls at 150 and 250 bp.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-seedprof}
mkdir -p $O
export RSA_GPU_LIB=rabbitsalign_amd/lib_ab/prof/librsa_gpu.so
for L in 150 250; do
  timeout -k 10 300 python3 scripts/micro/seed_bench.py --read-len $L --calls 20 > $O/seed$L.txt 2>&1 || { tail $O/seed$L.txt; exit 1; }
  echo "== $L"; grep seedprof $O/seed$L.txt | tail -1; grep -A3 '"lookup"\|"find_nams"' $O/seed$L.txt | grep avg
done

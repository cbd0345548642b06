# Isolated A/B of scan-kernel builds: each argument names a directory holding a
# librsa_gpu.so; scan_bench.py times it at chunk / combined-call sizes for 150 bp
# (window 257) and 250 bp (window 357) queries.  Usage: bash scripts/gpu_ab_scan.sh TAG DIR...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abscan}
shift
mkdir -p $O
for rep in 1 2; do
  for d in "$@"; do
    k=$(basename "$d")
    for L in 150 250; do
      SCAN_BENCH_L=$L SCAN_BENCH_LIB=$d/librsa_gpu.so RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 7300 12700 22000 65536 > $O/${k}_L${L}_$rep.txt 2>&1 || exit $?
      echo "== $k L=$L rep $rep"; grep "n=" $O/${k}_L${L}_$rep.txt
    done
  done
done
echo "exit 0"

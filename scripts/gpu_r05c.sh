# Round 5: every GPU test; the scan A/B (lib_ab/n5 = previous k_ext_scan_v vs the current
# build: query staged in LDS, best row found as the best grows); the SAM sink hand-off A/B
# (RSA_SINK_DIRECT 1/0/1, sink traces summarised by scripts/sink_report.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in old new; do
  if [ $v = old ]; then export SCAN_BENCH_LIB=rabbitsalign_amd/lib_ab/n5/librsa_gpu.so; else unset SCAN_BENCH_LIB; fi
  RSA_KTIMER_EVERY=1 timeout -k 10 200 python3 scripts/micro/scan_bench.py 7300 12700 22000 65536 > $O/scan_$v.txt 2>&1 || exit 1
  echo "scan $v"; cat $O/scan_$v.txt
done
unset SCAN_BENCH_LIB
for d in 1 0 1; do
  rm -f $O/sink_d$d.txt
  RSA_SINK_DIRECT=$d RSA_SINK_TRACE=$O/sink_d$d.txt timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_d$d.json 2> $O/bench_d$d.err || { tail -20 $O/bench_d$d.err; exit 1; }
  echo "RSA_SINK_DIRECT=$d"; python3 scripts/sink_report.py $O/sink_d$d.txt $O/bench_d$d.json | tail -12
done
echo "all ok"

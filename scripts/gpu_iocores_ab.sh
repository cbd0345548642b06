# RSA_IO_CORES A/B (1 = default, 2 = a second core kept from the workers for the writer and
# readers), alternating, two rounds, with sink traces (writer rate and step end as the figures).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ioab}
mkdir -p $O
for r in 1 2; do
  for c in 2 1; do
    rm -f $O/sink_c${c}_$r.txt
    RSA_IO_CORES=$c RSA_SINK_TRACE=$O/sink_c${c}_$r.txt timeout -k 10 400 python bench.py --no-cpu-baseline --no-multi-device --steps 8 --warmup 3 > $O/bench_c${c}_$r.json 2> $O/bench_c${c}_$r.err || { tail -20 $O/bench_c${c}_$r.err; exit 1; }
    echo "== RSA_IO_CORES=$c round $r"; python3 scripts/sink_report.py $O/sink_c${c}_$r.txt $O/bench_c${c}_$r.json | tail -4
  done
done

# RSA_EARLY_SEEDS A/B (chunks seeded alongside chunk 0: 2 = default, 5), alternating, two rounds,
# with sink traces: the figures are the writer's idle time at chunks 1-4 and the step end.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-earlyab}
mkdir -p $O
for r in 1 2; do
  for e in 5 2; do
    rm -f $O/sink_e${e}_$r.txt
    RSA_EARLY_SEEDS=$e RSA_SINK_TRACE=$O/sink_e${e}_$r.txt timeout -k 10 400 python bench.py --no-cpu-baseline --no-multi-device --steps 8 --warmup 3 > $O/bench_e${e}_$r.json 2> $O/bench_e${e}_$r.err || { tail -20 $O/bench_e${e}_$r.err; exit 1; }
    echo "== RSA_EARLY_SEEDS=$e round $r"; python3 scripts/sink_report.py $O/sink_e${e}_$r.txt $O/bench_e${e}_$r.json | tail -2
  done
done

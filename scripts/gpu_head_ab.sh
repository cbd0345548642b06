# Head-first gate A/B (RSA_HEAD_FIRST 1/0, alternating, two rounds) on the default bench, with
# sink traces: the acceptance figures are the writer's first write, idle time and step end.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-headab}
mkdir -p $O
for r in 1 2; do
  for h in 1 0; do
    rm -f $O/sink_h${h}_$r.txt
    RSA_HEAD_FIRST=$h RSA_SINK_TRACE=$O/sink_h${h}_$r.txt timeout -k 10 400 python bench.py --no-cpu-baseline --no-multi-device --steps 8 --warmup 3 > $O/bench_h${h}_$r.json 2> $O/bench_h${h}_$r.err || { tail -20 $O/bench_h${h}_$r.err; exit 1; }
    echo "== RSA_HEAD_FIRST=$h round $r"; python3 scripts/sink_report.py $O/sink_h${h}_$r.txt $O/bench_h${h}_$r.json | tail -2
  done
done

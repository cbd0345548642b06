# When does the writer get chunk 0?  Sink traces of the default bench under three prefetch
# settings (RSA_PREFETCH, RSA_EARLY_SEEDS); scripts/sink_report.py prints the first write,
# idle and busy time of each step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sinkfirst}
mkdir -p $O
for cfg in "default" "RSA_PREFETCH=12" "RSA_EARLY_SEEDS=0"; do
  tag=$(echo $cfg | tr '=' '_')
  rm -f $O/sink_$tag.txt
  if [ "$cfg" = default ]; then envs=""; else envs="$cfg"; fi
  env $envs RSA_SINK_TRACE=$O/sink_$tag.txt timeout -k 10 400 python bench.py --no-cpu-baseline --no-multi-device --steps 8 --warmup 3 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  echo "== $cfg"; python3 scripts/sink_report.py $O/sink_$tag.txt $O/bench_$tag.json | tail -3
done

# Default bench (5 timed steps) under several settings, each with the SAM writer
# traced (RSA_SINK_TRACE): per step the first write, the writer's idle and busy time
# and its rate (scripts/sink_report.py).  Settings alternate over ROUNDS rounds.
# Usage: bash scripts/gpu_sink_ab.sh TAG "VAR=val ..." ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sinkab}
shift
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-1}); do
  k=0
  for setting in "$@"; do
    k=$((k + 1))
    T0=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | awk '{print $2}' | tr '\n' ' ')
    env $setting RSA_SINK_TRACE=$O/sink_${k}_$r.txt timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 > $O/b_${k}_$r.json 2> $O/b_${k}_$r.err || exit $?
    T1=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | awk '{print $2}' | tr '\n' ' ')
    echo "== [$k/$r] ${setting}   cgroup cpu.stat nr_throttled/throttled_usec before: $T0 after: $T1"
    python3 scripts/sink_report.py $O/sink_${k}_$r.txt $O/b_${k}_$r.json
  done
done
echo "exit 0"

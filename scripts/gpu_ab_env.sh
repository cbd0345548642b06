# A/B of host tuning switches on the default bench, alternating settings, REPS rounds.
# Usage: [REPS=2] [STEPS=10] bash scripts/gpu_ab_env.sh TAG "RSA_PREFETCH=1" "RSA_PREFETCH=0" ...
# BENCH_ARGS adds bench flags (e.g. "--workload pe250_3g").
# (each argument is one setting: space-separated VAR=value pairs, "" for the defaults)
# e.g. gpu_ab_env.sh abw "RSA_WAIT_WORKERS=12" "RSA_WAIT_WORKERS=4"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abenv}
shift
mkdir -p $O
for i in $(seq 1 ${REPS:-2}); do
  k=0
  for setting in "$@"; do
    k=$((k + 1))
    env $setting timeout -k 10 300 python bench.py --no-cpu-baseline --no-multi-device ${BENCH_ARGS} --steps ${STEPS:-10} > $O/b_${k}_$i.json 2> $O/b_${k}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/b_${k}_$i.json'));print(json.dumps({'setting':'$setting','rep':$i,'value':d['value'],'in_memory':d.get('in_memory',{}).get('value'),'ms_per_step':d['ms_per_step'],'scan_Gcells':d['roofline'].get('achieved'),'scan_us':d['roofline'].get('avg_launch_us'),'core_us':d.get('host_cpu',{}).get('core_us_per_read')}))" | tee -a $O/ab.jsonl
  done
done
echo "exit 0"

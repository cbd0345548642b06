# A/B of library builds on the default bench, alternating: each argument names a
# directory holding librsa_gpu.so + librsalign.so (built from another commit);
# they are copied over rabbitsalign_amd/lib before each run, the last one stays.
# Usage: [REPS=2] bash scripts/gpu_ab_libs.sh TAG DIR...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ablibs}
shift
mkdir -p $O
for i in $(seq 1 ${REPS:-2}); do
  for d in "$@"; do
    cp "$d"/librsa_gpu.so "$d"/librsalign.so rabbitsalign_amd/lib/ || exit 1
    k=$(basename "$d")
    timeout -k 10 300 python bench.py --no-cpu-baseline  > $O/b_${k}_$i.json 2> $O/b_${k}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/b_${k}_$i.json'));print(json.dumps({'build':'$k','rep':$i,'value':d['value'],'in_memory':d.get('in_memory',{}).get('value'),'ms_per_step':d['ms_per_step'],'scan_us':d['kernels']['ext_scan']['avg_us'],'core_us_per_read':d.get('host_cpu',{}).get('core_us_per_read')}))" | tee -a $O/ab.jsonl
  done
done
echo "exit 0"

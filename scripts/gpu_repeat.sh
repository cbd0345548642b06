# The default bench repeated (20 timed steps each, no CPU leg) for a median on one box.
# Usage: bash scripts/gpu_repeat.sh TAG N
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-repeat}
mkdir -p $O
for i in $(seq 1 ${2:-4}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-multi-device > $O/b_$i.json 2> $O/b_$i.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b_$i.json'));print(json.dumps({'run':$i,'value':d['value'],'in_memory':d['in_memory']['value'],'ms_per_step':d['ms_per_step'],'core_us':d['host_cpu']['core_us_per_read'],'scan':d['roofline']['achieved'],'frac':d['roofline']['frac']}))" | tee -a $O/runs.jsonl
done
echo "exit 0"

# Round 6: SE 1x100 twice (its round-6 figures moved 20.6 -> 18.4 between two runs) and the
# default bench once more, on the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06ab}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --workload se100_5m --no-cpu-baseline > $O/se100_$i.json 2> $O/se100_$i.err || { tail -20 $O/se100_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/se100_$i.json'));print('se100 $i',d['value'],d['in_memory']['value'],d['host_cpu']['core_us_per_read'])"
done
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('pe150',d['value'],d['in_memory']['value'],d['cpu_baseline']['value'],d['parity'].get('sam_identical'))"
echo "all ok"

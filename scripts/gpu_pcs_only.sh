# Host PC samples of the default bench (5 steps, no CPU leg, no multi-device leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pcs}
mkdir -p $O
RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --no-multi-device --steps 5 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],'mem',d['in_memory']['value'],'core_us',d['host_cpu']['core_us_per_read'])"

# A/B of chunks per extend call (RSA_EXT_GROUP) on the default bench. Usage: bash scripts/gpu_ab_group.sh TAG "1 2 4"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2; do
  for G in $2; do
    RSA_EXT_GROUP=$G timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 --warmup 3 > $O/g${G}_$rep.json 2> $O/g${G}_$rep.err || exit $?
    python -c "import json;d=json.load(open('$O/g${G}_$rep.json'));k=d['kernels'];print('G=$G rep=$rep', d['value'], 'scan_us', k['ext_scan']['avg_us'], 'launches', k['ext_scan']['launches'], 'frac', d['roofline']['frac'], d['roofline']['kernel'])"
  done
done

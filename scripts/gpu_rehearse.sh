# The N-rank bench path rehearsed on a 1-GPU box: `bench.py --gpus 2` self-launches two
# ranks under torch.distributed.run, both on GPU 0 with a gloo process group
# (RSA_BENCH_REHEARSE=1), each pinned to half of the CPUs, with per-rank FASTQ/SAM files and
# the max-over-ranks timing; then the product's multi-device leg (two engines on GPU 0).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rehearse}
mkdir -p $O
RSA_BENCH_REHEARSE=1 timeout -k 10 500 python3 bench.py --gpus 2 --steps 4 --warmup 3 --no-cpu-baseline --md-steps 2 > $O/bench_g2.json 2> $O/bench_g2.err
rc=$?
echo "rehearsal exit $rc"
tail -5 $O/bench_g2.err
python3 -c "import json;d=json.load(open('$O/bench_g2.json'));print({k:d.get(k) for k in ('value','n_gpus','ms_per_step','rehearsal')}, d['config']['host_cpus_pinned'], (d.get('multi_device') or {}).get('value'))"
exit $rc

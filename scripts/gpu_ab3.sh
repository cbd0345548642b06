# seed batching A/B on the bench, with the engine-call wall breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab3}
mkdir -p $O
for i in 1 2; do
RSA_SEED_BATCH=1 timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/b1_$i.json 2> $O/b1_$i.err || exit $?
RSA_SEED_BATCH=4 timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/b4_$i.json 2> $O/b4_$i.err || exit $?
done
echo "exit 0"

# parity (extend + e2e + seed) then bench twice.  Usage: bash scripts/gpu_iter.sh TAG [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-iter}
shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_extend_gpu.py tests/test_e2e_gpu.py tests/test_seed_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 400 python3 bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python3 bench.py --no-cpu-baseline "$@" > $O/bench2.json 2> $O/bench2.err
echo "exit $?"

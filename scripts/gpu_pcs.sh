# GPU tests, then host PC samples (with the word at the stack pointer, for
# callers of leaf functions) of the mapping under the GPU engine, 16 threads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pcs}
mkdir -p $O
rm -f $O/pcs.txt
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
fi
RSA_PC_SAMPLE=$O/pcs.txt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/bench.json 2> $O/bench.err
echo "exit $?"

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r8
mkdir -p $O
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
RSA_SCAN_V=2 RSA_BAND_V=1 timeout -k 10 500 python -m pytest tests/test_extend_gpu.py tests/test_e2e_gpu.py -m gpu -x -q > $O/pytest_v2.log 2>&1 && \
timeout -k 10 400 python scripts/kab.py "" RSA_SCAN_V=1 RSA_SCAN_V=2 RSA_BAND_V=1 RSA_SCAN_V=2,RSA_BAND_V=1 RSA_RS_SCRATCH=1 > $O/kab.jsonl 2> $O/kab.err && \
bash scripts/gpu_pipe.sh r8/pipe
echo "exit $?"

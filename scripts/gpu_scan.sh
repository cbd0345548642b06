# Grouped-scan parity + A/B.  Usage: bash scripts/gpu_scan.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-scan}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_extend_gpu.py tests/test_e2e_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python3 scripts/kab.py --pairs 200000 --threads 1 RSA_SCAN_G=0 RSA_SCAN_G=1 > $O/kab.jsonl 2> $O/kab.err && \
timeout -k 10 300 python3 scripts/kab.py --pairs 1000000 --threads 16 RSA_SCAN_G=0 RSA_SCAN_G=1 RSA_SCAN_G=0 RSA_SCAN_G=1 > $O/kab16.jsonl 2> $O/kab16.err
echo "exit $?"

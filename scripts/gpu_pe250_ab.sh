# PE250 SAM parity (test_configs_gpu pe250_3g) under settings: default, positions-only site
# checks (RSA_SITE_ALIGN=0), the round-3 band64 grid (RSA_BAND64_GRID=512)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pe250ab}
mkdir -p $O
for setting in "X=1" "RSA_SITE_ALIGN=0" "RSA_BAND64_GRID=512" "RSA_SCAN_V=0"; do
  env $setting timeout -k 10 300 python -u -m pytest "tests/test_configs_gpu.py::test_baseline_config_sam_identical[pe250_3g]" -x -q --timeout 280 --timeout-method thread > $O/$setting.log 2>&1
  echo "$setting: exit $? $(tail -1 $O/$setting.log)"
done

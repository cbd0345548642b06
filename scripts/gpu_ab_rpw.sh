# A/B of reads per wave for k_randstrobes / k_find_nams (lane kernels), 5 timed steps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abrpw}
mkdir -p $O
for cfg in "64 16" "16 16" "32 16" "8 16" "64 16"; do
  set -- $cfg
  RSA_RPW_RS=$1 RSA_RPW_FN=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit $?
done
echo "exit 0"

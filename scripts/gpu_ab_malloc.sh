# A/B of glibc malloc tunables (arena trimming / mmap threshold / THP) on the
# mapping under the GPU engine, alternating, 5 timed steps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abmalloc}
mkdir -p $O
T1=glibc.malloc.trim_threshold=4294967296:glibc.malloc.mmap_threshold=33554432:glibc.malloc.top_pad=67108864
T2=$T1:glibc.malloc.hugetlb=1
for i in 1 2; do
  for v in base t1 t2; do
    case $v in base) T=;; t1) T=$T1;; t2) T=$T2;; esac
    GLIBC_TUNABLES=$T timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
  done
done
echo "exit 0"

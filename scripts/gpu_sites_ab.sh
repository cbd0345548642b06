# k_sites / seeding-call kernels: parity tests on the product build, then the isolated
# seeding kernels (scripts/micro/seed_bench.py, 1 Gb reference) under a kernel trace for
# the given librsa_gpu.so variants (rabbitsalign_amd/lib_ab/<v>).  Usage: TAG v...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sites_ab}
shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_seed_gpu.py tests/test_host_cases_gpu.py tests/test_e2e_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "$@"; do
  mkdir -p $O/$v
  RSA_GPU_LIB=rabbitsalign_amd/lib_ab/$v/librsa_gpu.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v/trace -o run -- python3 scripts/micro/seed_bench.py --ref-len 1e9 --calls 30 > $O/$v/trace.txt 2>&1 || exit 1
  python3 - $O/$v $v <<'EOF2'
import glob, os, sqlite3, sys
o, v = sys.argv[1], sys.argv[2]
tot = 0
row = []
for db in glob.glob(os.path.join(o, "trace", "**", "*.db"), recursive=True):
    for n, c, a in sqlite3.connect(db).execute("select name, count(*), avg(duration) from kernels group by name order by name"):
        n = n.split("(")[0].replace("void ", "")
        if n.startswith("k_") and "bucket" not in n and "index" not in n and not n.startswith("k_seg") and not n.startswith("k_ref"):
            row.append(f"{n}={a / 1e3:.1f}")
            tot += a / 1e3
print(v, f"sum_us={tot:.1f}", " ".join(row))
EOF2
  find $O/$v -name "*.db" -delete
done

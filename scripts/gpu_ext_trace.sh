# Kernel trace of the isolated extension launches (scripts/micro/scan_bench.py): each
# extension kernel's own duration, including the speculative scan and its redo pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-exttrace}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 scripts/micro/scan_bench.py ${SIZES:-7300 22000} > $O/bench.txt 2>&1 || exit $?
python3 - $O <<'PY'
import glob, os, sqlite3, sys, collections
o = sys.argv[1]
for db in glob.glob(os.path.join(o, "trace", "**", "*.db"), recursive=True):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration) from kernels group by name").fetchall()
    for n, k, a, mi, ma in sorted(rows, key=lambda r: -r[1] * r[2]):
        if "k_ext" in n or "k_cig" in n:
            print(f"{n.split('(')[0][:60]:60s} {k:5d} avg {a/1e3:8.1f} us  min {mi/1e3:8.1f}  max {ma/1e3:8.1f}")
PY
find $O -name "*.db" -delete
cat $O/bench.txt | grep n=

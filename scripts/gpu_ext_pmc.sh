# SQ counters of the extension kernels on isolated launches (scripts/micro/scan_bench.py,
# 22000 jobs: three chunks, the size of a combined call), one rocprofv3 pass per set.
# Usage: bash scripts/gpu_ext_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-extpmc}
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 scripts/micro/scan_bench.py 22000 > $O/trace.txt 2>&1 || exit $?
python3 - $O <<'EOF2'
import glob, os, sqlite3, sys
for db in glob.glob(os.path.join(sys.argv[1], "trace", "**", "*.db"), recursive=True):
    for n, k, a in sqlite3.connect(db).execute("select name, count(*), avg(duration) from kernels group by name"):
        if "k_ext" in n:
            print(f"trace {n.split('(')[0][:70]:70s} {k:4d} avg {a / 1e3:8.1f} us")
EOF2
timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/p1 -o run -- python3 scripts/micro/scan_bench.py 22000 > $O/p1.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/p2 -o run -- python3 scripts/micro/scan_bench.py 22000 > $O/p2.txt 2>&1 || exit $?
python3 - $O <<'EOF'
import glob, os, sqlite3, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p1", "p2"):
    for db in glob.glob(os.path.join(o, p, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        for k, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
            k = k.split("(")[0].replace("void ", "")
            acc[k][cn].append(v)
with open(os.path.join(o, "pmc_summary.txt"), "w") as f:
    for k, d in sorted(acc.items()):
        if not any(x in k for x in ("k_ext_scan_g", "k_ext_scan_v", "k_ext_scan<", "k_ext_band16", "k_ext_band64")):
            continue
        line = k + ": " + ", ".join(f"{cn} {sum(v) / len(v):.4g}" for cn, v in sorted(d.items()))
        print(line)
        f.write(line + "\n")
EOF
find $O -name "*.db" -delete
echo "exit 0"

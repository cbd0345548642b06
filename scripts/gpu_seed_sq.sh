# SQ counters of the seeding kernels (product build, isolated calls, 150 bp, 3 Gb reference):
# wait_any / wave cycles and friends, one PMC pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-seedsq}
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
timeout -s KILL 300 rocprofv3 --pmc $P1 -d $O/p1 -o run -- python3 scripts/micro/seed_bench.py --calls 10 > $O/p1.txt 2>&1 || { tail -5 $O/p1.txt; exit 1; }
python3 - $O <<'EOF2'
import glob, os, sqlite3, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for db in glob.glob(os.path.join(o, "p1", "**", "*.db"), recursive=True):
    for k, cn, v in sqlite3.connect(db).execute("select kernel_name, counter_name, value from counters_collection"):
        acc[k.split("(")[0].replace("void ", "")][cn].append(v)
for k, d in sorted(acc.items()):
    if not any(x in k for x in ("k_sites", "k_compact", "k_seed_query", "k_find_nams_w2", "k_rescue_w")):
        continue
    r = {cn: sum(v) / len(v) for cn, v in d.items()}
    w = max(1, r.get("SQ_WAVES", 1)); wc = max(1, r.get("SQ_WAVE_CYCLES", 1))
    print(f"{k[:24]:24s} waves {r.get('SQ_WAVES', 0):8.0f} valu/wave {r.get('SQ_INSTS_VALU', 0)/w:7.0f} "
          f"vmem_rd/wave {r.get('SQ_INSTS_VMEM_RD', 0)/w:6.1f} wave_cyc/wave {wc/w:8.0f} "
          f"wait_any {r.get('SQ_WAIT_ANY', 0)/wc:.2f} wait_inst {r.get('SQ_WAIT_INST_ANY', 0)/wc:.2f} "
          f"active {r.get('SQ_ACTIVE_INST_ANY', 0)/wc:.2f}")
EOF2
find $O -name "*.db" -delete

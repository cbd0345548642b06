# Address-translation and memory-pipeline counters of the seeding kernels
# (scripts/micro/seed_bench.py, 150 bp, 3 Gb reference), one PMC pass each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-seedtlb}
mkdir -p $O
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum"
P2="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P -d $O/p$i -o run -- python3 scripts/micro/seed_bench.py --calls 6 > $O/p$i.txt 2>&1 || { tail -5 $O/p$i.txt; exit 1; }
done
python3 - $O <<'EOF2'
import glob, os, sqlite3, sys, collections
o = sys.argv[1]
for i in (1, 2):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for db in glob.glob(os.path.join(o, f"p{i}", "**", "*.db"), recursive=True):
        for k, cn, v in sqlite3.connect(db).execute("select kernel_name, counter_name, value from counters_collection"):
            acc[k.split("(")[0].replace("void ", "")][cn].append(v)
    for k, d in sorted(acc.items()):
        if not any(x in k for x in ("k_sites", "k_seed_query", "k_find_nams_w2", "k_compact")):
            continue
        print(f"p{i} {k[:28]:28s} " + " ".join(f"{cn.replace('TCP_','').replace('_sum','')}={sum(v)/len(v):.4g}" for cn, v in sorted(d.items())))
EOF2
find $O -name "*.db" -delete

# The random line-fetch probe under the same translation counters as gpu_seed_tlb.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-probetlb}
mkdir -p $O
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum"
P2="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run -- scripts/micro/line_probe 32 > $O/p$i.txt 2>&1 || { tail -5 $O/p$i.txt; exit 1; }
done
python3 - $O <<'EOF2'
import glob, os, sqlite3, sys, collections
o = sys.argv[1]
for i in (1, 2):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for db in glob.glob(os.path.join(o, f"p{i}", "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        for k, disp, cn, v in c.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection"):
            rows[(k.split("(")[0], disp)][cn].append(v)
    for (k, disp), d in sorted(rows.items(), key=lambda x: x[0][1])[-40:]:
        print(f"p{i} {k[:26]:26s} d{disp:4d} " + " ".join(f"{cn.replace('TCP_','').replace('_sum','')}={sum(v):.4g}" for cn, v in sorted(d.items())))
EOF2
find $O -name "*.db" -delete

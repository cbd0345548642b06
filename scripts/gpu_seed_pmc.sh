# SQ counters of the seeding and site kernels in the bench (2 timed steps), one rocprofv3
# pass per counter set; per-kernel averages per launch.  Usage: bash scripts/gpu_seed_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-seedpmc}
mkdir -p $O
ARGS="--no-cpu-baseline --no-multi-device --steps 2 --warmup 1"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
timeout -s KILL 300 rocprofv3 --pmc $P1 -d $O/p1 -o run -- python3 bench.py $ARGS > $O/p1.txt 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc $P2 -d $O/p2 -o run -- python3 bench.py $ARGS > $O/p2.txt 2>&1 || exit $?
python3 - $O <<'EOF2'
import glob, os, sqlite3, sys, collections, json
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p1", "p2"):
    for db in glob.glob(os.path.join(o, p, "**", "*.db"), recursive=True):
        for k, cn, v in sqlite3.connect(db).execute("select kernel_name, counter_name, value from counters_collection"):
            k = k.split("(")[0].replace("void ", "")
            acc[k][cn].append(v)
keep = ("k_seed_query", "k_find_nams_w2", "k_sites", "k_rescue_w", "k_seed_scan", "k_compact", "k_ext_scan_v",
        "k_ext_band16", "k_shared_check")
out = {}
for k, d in sorted(acc.items()):
    if not any(k.startswith(x) for x in keep):
        continue
    out[k] = {cn: sum(v) / len(v) for cn, v in d.items()}
    r = out[k]
    print(f"{k[:40]:40s} waves {r.get('SQ_WAVES', 0):9.0f} valu/wave {r.get('SQ_INSTS_VALU', 0) / max(1, r.get('SQ_WAVES', 1)):8.0f} "
          f"lds/wave {r.get('SQ_INSTS_LDS', 0) / max(1, r.get('SQ_WAVES', 1)):7.0f} vmem_rd/wave {r.get('SQ_INSTS_VMEM_RD', 0) / max(1, r.get('SQ_WAVES', 1)):6.0f} "
          f"wait_any/busy {r.get('SQ_WAIT_ANY', 0) / max(1, r.get('SQ_WAVE_CYCLES', 1)):.2f}")
json.dump(out, open(os.path.join(o, "seed_pmc.json"), "w"), indent=1)
EOF2
find $O -name "*.db" -delete
find $O -name "*.csv" -size +1M -delete
echo "exit 0"

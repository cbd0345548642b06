# Isolated seeding kernels (scripts/micro/seed_bench.py, 1 Gb reference): kernel trace,
# then two SQ counter passes, for the given librsa_gpu.so builds.  Usage: TAG lib_dir...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-seedmicro}
shift
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
for v in "$@"; do
  export RSA_GPU_LIB=rabbitsalign_amd/lib_ab/$v/librsa_gpu.so
  mkdir -p $O/$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v/trace -o run -- python3 scripts/micro/seed_bench.py --ref-len 1e9 --calls 20 > $O/$v/trace.txt 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc $P1 -d $O/$v/p1 -o run -- python3 scripts/micro/seed_bench.py --ref-len 1e9 --calls 10 > $O/$v/p1.txt 2>&1 || exit 1
  python3 - $O/$v <<'EOF2'
import glob, os, sqlite3, sys, collections, csv
o = sys.argv[1]
for db in glob.glob(os.path.join(o, "trace", "**", "*.db"), recursive=True):
    for n, c, a in sqlite3.connect(db).execute("select name, count(*), avg(duration) from kernels group by name"):
        if any(k in n for k in ("k_sites", "k_compact", "k_seed_query", "k_find_nams_w2", "k_rescue_w", "k_seed_scan")):
            print(f"trace {n.split('(')[0][:40]:40s} calls {c:6d} avg_us {a / 1e3:9.2f}")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for db in glob.glob(os.path.join(o, "p1", "**", "*.db"), recursive=True):
    for k, cn, v in sqlite3.connect(db).execute("select kernel_name, counter_name, value from counters_collection"):
        acc[k.split("(")[0].replace("void ", "")][cn].append(v)
for k, d in sorted(acc.items()):
    if not any(x in k for x in ("k_sites", "k_compact", "k_seed_query", "k_find_nams_w2")):
        continue
    r = {cn: sum(v) / len(v) for cn, v in d.items()}
    w = max(1, r.get("SQ_WAVES", 1))
    print(f"pmc {k[:40]:40s} waves {r.get('SQ_WAVES', 0):8.0f} valu/wave {r.get('SQ_INSTS_VALU', 0)/w:7.0f} "
          f"vmem_rd/wave {r.get('SQ_INSTS_VMEM_RD', 0)/w:6.1f} wave_cyc/wave {r.get('SQ_WAVE_CYCLES', 0)/w:8.0f} "
          f"wait_any {r.get('SQ_WAIT_ANY', 0)/max(1, r.get('SQ_WAVE_CYCLES', 1)):.2f} "
          f"wait_inst {r.get('SQ_WAIT_INST_ANY', 0)/max(1, r.get('SQ_WAVE_CYCLES', 1)):.2f} "
          f"active {r.get('SQ_ACTIVE_INST_ANY', 0)/max(1, r.get('SQ_WAVE_CYCLES', 1)):.2f}")
EOF2
  find $O/$v -name "*.db" -delete
done

# Exact HBM read bytes per kernel from the request-size counters (one PMC pass over a short
# default bench): 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B, beside RDREQ itself.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rdreq}
mkdir -p $O
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $O/p -o run -- python3 bench.py --no-cpu-baseline --no-multi-device --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - $O <<'EOF2'
import glob, os, sqlite3, sys, collections, json
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for db in glob.glob(os.path.join(o, "p", "**", "*.db"), recursive=True):
    for k, cn, v in sqlite3.connect(db).execute("select kernel_name, counter_name, value from counters_collection"):
        acc[k.split("(")[0].replace("void ", "").strip()][cn].append(v)
out = {}
for k, d in acc.items():
    r = {cn: sum(v) / len(v) for cn, v in d.items()}
    n, n32, n64, n128 = (r.get(c, 0) for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"))
    out[k] = {"rdreq": n, "n32": n32, "n64": n64, "n128": n128, "read_bytes": 32 * n32 + 64 * n64 + 128 * n128,
              "launches": len(next(iter(d.values())))}
json.dump(out, open(os.path.join(o, "rdreq.json"), "w"), indent=1)
for k, v in sorted(out.items(), key=lambda kv: -kv[1]["read_bytes"] * kv[1]["launches"])[:14]:
    print(f"{k[:34]:34s} launches {v['launches']:5d} rdreq {v['rdreq']:12.0f} 32B {v['n32']:10.0f} 64B {v['n64']:10.0f} 128B {v['n128']:10.0f} bytes {v['read_bytes']/1e6:9.2f} MB")
EOF2
find $O -name "*.db" -delete

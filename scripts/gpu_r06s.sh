# Round 6: SAM pieces for the first chunk only (the writer's first bytes) -- A/B in one
# process on the headline, settings alternated.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06s}
mkdir -p $O
timeout -k 10 900 python bench.py --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 8 --ab-steps 4 \
  --ab "RSA_SAM_PIECE_FIRST=0|RSA_SAM_PIECE_FIRST=1000|RSA_SAM_PIECE_FIRST=2500" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 - $O/ab.json <<'EOF2'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for v in d["ab"]:
    fo = sorted(v["first_out_ms"])
    print(v["env"], "median", v["median"], "mean", v["mean"], "first_out med", fo[len(fo)//2], "core_us", sorted(v["core_us_per_read"])[len(fo)//2])
EOF2
echo "all ok"

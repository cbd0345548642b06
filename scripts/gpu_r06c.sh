# Round 6: host-pipeline A/B (SAM pieces, early prefetch window) on the headline
# workload, alternating in one process; then the round-5 exit-abort command once
# more (kernel + memory-copy trace of PE 2x250, mappings dumped at exit); then a
# kernel-trace-only profile of PE 2x250 (kernel shares on this tree).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06c}
mkdir -p $O
timeout -k 10 600 python bench.py --no-cpu-baseline --warmup 3 --steps 4 --ab-rounds 4 --ab-steps 4 \
  --ab "RSA_SAM_PIECE=0,RSA_EARLY_WINDOW=0|RSA_SAM_PIECE=2000,RSA_EARLY_WINDOW=0|RSA_SAM_PIECE=2000,RSA_EARLY_WINDOW=6|RSA_SAM_PIECE=0,RSA_EARLY_WINDOW=6" \
  > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 - $O/ab.json <<'EOF2'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for v in d["ab"]:
    fo = sorted(v["first_out_ms"]); fe = sorted(b - a for a, b in v["first_ext_ms"]); cu = sorted(v["core_us_per_read"])
    print(v["env"], "median", v["median"], "mean", v["mean"], "first_out med", fo[len(fo)//2], "first ext dur med", round(fe[len(fe)//2], 1), "core-us med", cu[len(cu)//2])
EOF2
RSA_MAPS_OUT=$O/maps.txt timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/tl -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --steps 3 --warmup 1 > $O/tl.json 2> $O/tl.err
echo "memory-copy-trace profile exit $?"; grep -E "tool finalization|SIGSEGV|Aborted" $O/tl.err | head -5
find $O/tl -name "*.db" -delete
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 bench.py --workload pe250_3g --no-cpu-baseline --steps 4 --warmup 2 > $O/kt.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
python3 scripts/timeline.py $(find $O/kt -name "*.db" | head -1) > $O/timeline.txt; cat $O/timeline.txt | head -40
find $O/kt -name "*.db" -delete
echo "all ok"

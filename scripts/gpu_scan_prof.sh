# Isolated kernel times (one host thread) + SQ counters of the DP scan. Usage: bash scripts/gpu_scan_prof.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python scripts/kab.py --threads 1 --pairs 60000 RSA_EXT_GROUP=1 RSA_EXT_GROUP=6 > $O/kab.jsonl 2> $O/kab.err || exit $?
cat $O/kab.jsonl
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_ext_scan_g|k_rs_wave|k_lookup|k_find_nams_w2|k_ext_band16|k_sites" --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU -d $O/sq -o run -- python3 scripts/kab.py --threads 1 --pairs 60000 RSA_EXT_GROUP=6 > $O/sq.log 2>&1 || exit $?
python3 - <<PY
import sqlite3, glob
db = glob.glob("$O/sq/**/run_results.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select kernel_name, counter_name, count(*), avg(value) from counters_collection group by kernel_name, counter_name").fetchall()
for r in rows: print(r[0].split("(")[0][:40], r[1], r[2], round(r[3], 1))
PY

# SQ counters per kernel (one host thread, isolated launches): instruction mix and wait states.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sq
mkdir -p $O
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc -o run -- python3 scripts/kab.py --pairs 30000 > $O/kab.jsonl 2> $O/kab.err
echo "exit $?"

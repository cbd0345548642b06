# Round-4 measurements on one box: SQ counters of the extension kernels (isolated
# launches), the rocprofv3 kernel trace + FETCH/WRITE PMC passes over the default
# bench, and the SAM sink bandwidth probes (O_DIRECT and buffered pwrite, 1-16 threads).
# Usage: bash scripts/gpu_r04_prof.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04}
mkdir -p gpurun_out/$TAG
timeout -k 10 100 scripts/micro/sam_sink_bw --direct /tmp > gpurun_out/$TAG/sink_direct.txt 2>&1; echo "sink probe exit $?"
cat gpurun_out/$TAG/sink_direct.txt
bash scripts/gpu_ext_pmc.sh ${TAG}_extpmc || exit $?
bash scripts/gpu_prof.sh $TAG || exit $?
echo "all ok"

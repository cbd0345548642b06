# Per-step timeline marks (chunk 0 seeded, last chunk's finish started, step end)
# of the default bench under several settings, one process each.
# Usage: bash scripts/gpu_tail.sh TAG "VAR=val ..." ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tail}
shift
mkdir -p $O
k=0
for setting in "$@"; do
  k=$((k + 1))
  env $setting timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 > $O/b_$k.json 2> $O/b_$k.err || exit $?
  echo "== ${setting:-default}"
  grep -E "step [0-9]+:|in-memory" $O/b_$k.err | sed 's/.*step/step/; s/thread-s.*sequential/seq/'
done
echo "exit 0"

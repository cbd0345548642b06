# Round 6: the GPU index build's tie path at 3 Gb -- a synthetic 3 Gb FASTA with a
# 10 Mb PAR-like region (chr1[1 Mb, 11 Mb) copied onto chr2 at the same coordinates),
# indexed on the GPU (ties replayed on the host) and on the host (--cpu-index); the two
# .sti streams are hashed (no 12 GB files on disk) and must be identical.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06g}
mkdir -p $O
FA=/tmp/rsa_tie_$$.fa
df -h /tmp | tail -1
timeout -k 10 300 python3 scripts/micro/tie_ref.py $FA 10000000 || exit 1
ls -la $FA
( time timeout -k 10 900 rabbitsalign_amd/bin/rsalign index -v -r 150 -t 16 -o /dev/stdout $FA | sha256sum > $O/gpu.sha ) 2> $O/gpu.err || { cat $O/gpu.err; rm -f $FA; exit 1; }
cat $O/gpu.err; cat $O/gpu.sha
( time timeout -k 10 900 rabbitsalign_amd/bin/rsalign index --cpu-index -v -r 150 -t 16 -o /dev/stdout $FA | sha256sum > $O/host.sha ) 2> $O/host.err || { cat $O/host.err; rm -f $FA; exit 1; }
cat $O/host.err; cat $O/host.sha
rm -f $FA
if [ "$(cut -d' ' -f1 $O/gpu.sha)" = "$(cut -d' ' -f1 $O/host.sha)" ]; then echo "sti identical"; else echo "sti DIFFER"; fi
echo "all ok"

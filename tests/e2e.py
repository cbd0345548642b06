"""End-to-end helpers: synthetic data + running the CLIs."""
import os
import subprocess

from helpers import ROOT

GEN = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsa_gen")
RSALIGN = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsalign")
CPU_PORT = os.path.join(ROOT, "oracle", "_build", "rsalign_cpu")
CPU_REF = os.path.join(ROOT, "oracle", "_ref", "rsalign_ref")


def run(*args, **kw):
    return subprocess.run([str(a) for a in args], check=True, capture_output=True, text=True, **kw)


def make_dataset(d, name="ds", ref_len=300_000, contigs=3, pairs=4000, L=150, mu=300, sigma=30, seed=1,
                 repeat_frac=0.03, n_runs=3, n_rate=0.001, se=False, cpu_index=False):
    """FASTA + FASTQ + the .sti next to the FASTA; the index is built on the GPU
    (rsalign's default) unless cpu_index asks for the host build."""
    fa = os.path.join(d, f"{name}.fa")
    run(GEN, "ref", seed, ref_len, contigs, fa, repeat_frac, n_runs)
    if se:
        fq = os.path.join(d, f"{name}.fq")
        run(GEN, "se", seed + 1, fa, pairs, L, fq, n_rate)
        reads = [fq]
    else:
        f1, f2 = os.path.join(d, f"{name}_1.fq"), os.path.join(d, f"{name}_2.fq")
        run(GEN, "reads", seed + 1, fa, pairs, L, mu, sigma, f1, f2, n_rate)
        reads = [f1, f2]
    run(RSALIGN, "index", "-r", L, "-t", 4, *(["--cpu-index"] if cpu_index else []), fa)
    return fa, reads


def sam_body(path):
    with open(path) as f:
        return [l for l in f if not l.startswith("@PG")]


def map_reads(binary, fa, reads, out, *opts):
    r = run(binary, "--use-index", *opts, "-o", out, fa, *reads)
    return r.stderr

"""Random reference + SW jobs shaped like the reference's extension and rescue
jobs (src/aln.cpp:446-456, pc.cpp:333-368), plus adversarial ones."""
import numpy as np

JOB_DTYPE = np.dtype([("query_offset", "<u8"), ("query_len", "<u4"), ("ref_id", "<i4"),
                      ("ref_start", "<u4"), ("ref_len", "<u4")])
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def random_reference(rng, n_contigs=3, length=200_000, n_runs=5):
    seqs = []
    for _ in range(n_contigs):
        s = ACGT[rng.integers(0, 4, length)].copy()
        for _ in range(n_runs):
            a = int(rng.integers(0, length - 100))
            s[a:a + int(rng.integers(1, 60))] = ord("N")
        # a low-complexity stretch
        a = int(rng.integers(0, length - 3000))
        s[a:a + 2000] = ACGT[rng.integers(0, 2, 2000)]
        seqs.append(s)
    offs = np.zeros(n_contigs + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(s) for s in seqs])
    return np.concatenate(seqs), offs


def mutate(rng, s: np.ndarray, sub=0.02, ind=0.01, n_rate=0.0):
    out = []
    i = 0
    while i < len(s):
        u = rng.random()
        if u < sub:
            out.append(int(ACGT[rng.integers(0, 4)]))
        elif u < sub + ind / 2:
            pass
        elif u < sub + ind:
            out.append(int(s[i]))
            out.append(int(ACGT[rng.integers(0, 4)]))
        else:
            out.append(int(s[i]))
        if rng.random() < 0.01:   # occasional longer indel
            gl = int(rng.integers(1, 15))
            if rng.random() < 0.5:
                i += gl
            else:
                out.extend(int(x) for x in ACGT[rng.integers(0, 4, gl)])
        i += 1
    a = np.array(out, dtype=np.uint8)
    if n_rate > 0:
        a[rng.random(len(a)) < n_rate] = ord("N")
    return a


def make_jobs(rng, ref, offs, n, qlen_choices=(150,)):
    """Returns (queries_blob, jobs, list of (query bytes, ref window bytes))."""
    queries = bytearray()
    jobs = np.zeros(n, dtype=JOB_DTYPE)
    pairs = []
    nc = len(offs) - 1
    for i in range(n):
        kind = rng.integers(0, 12)
        c = int(rng.integers(0, nc))
        clen = int(offs[c + 1] - offs[c])
        L = int(rng.choice(qlen_choices)) if kind < 8 else int(rng.integers(1, 400))
        rl = L + int(rng.integers(0, 120)) if kind < 6 else int(rng.integers(1, 700))
        if kind == 11:
            rl = int(rng.integers(2001, 2300))   # the >2000 sentinel
        rl = min(rl, clen)
        rs = int(rng.integers(0, clen - rl + 1))
        win = ref[int(offs[c]) + rs:int(offs[c]) + rs + rl]
        if kind < 9 and rl > 5:
            a = int(rng.integers(0, max(1, rl // 4)))
            q = mutate(rng, win[a:], sub=rng.choice([0.0, 0.01, 0.04, 0.1]), ind=rng.choice([0.0, 0.01, 0.03]),
                       n_rate=0.01 if kind == 3 else 0.0)
            if len(q) < L:
                q = np.concatenate([q, ACGT[rng.integers(0, 4, L - len(q))]])
            q = q[:L]
        else:
            q = ACGT[rng.integers(0, 4, L)]
        if kind == 10:
            q = np.full(L, ord("A"), dtype=np.uint8)
        qb = bytes(q)
        jobs[i] = (len(queries), len(qb), c, rs, rl)
        queries += qb
        pairs.append((qb, bytes(win)))
    return bytes(queries), jobs, pairs

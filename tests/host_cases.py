"""Hand-derived cases for the host pipeline's per-job arithmetic, the part of
the path both engines share (so no SAM comparison between them can catch an
error in it):

- the extension window, part2_extend_seed_get_str (src/pc.cpp:214-242);
- the mate-rescue window, part2_rescue_mate_get_str (src/pc.cpp:333-368), with
  the insert-size estimate before (mu 300, sigma 100) and after the freeze;
- the stored Alignment, part2_extend_seed_store_res (src/pc.cpp:177-212) and
  part2_rescue_mate_store_res (src/pc.cpp:291-331).

Each expectation is worked out from those lines in the comment beside it.  NAMs
are (query_start, query_end, ref_start, ref_end, is_rc).  The rescue window
keeps the reference's mixed arithmetic: `int - float` and `size_t + float` are
evaluated in float (24-bit mantissa), then truncated to int.  Above 2^26 floats
are 8 apart, which moves the window of a contig past 67 Mb by up to 7 bases.

tests/test_host_cases_cpu.py runs every case through bin/rsa_host_cases (the
product's host functions); tests/test_host_cases_gpu.py aligns the sequence cases
with rsa_extend and stores the results through the same host functions.
"""

# (name, nam, read_len, contig_len, expected (window_start, window_len))
EXTENSION_WINDOWS = [
    # projected_ref_start = max(0, 1010 - 10) = 1000; diff = |130 - 130| = 0;
    # ext_left = min(50, 1000) = 50 -> start 950; ext_right = min(50, 10000 - 1140) = 50;
    # size = 150 + 0 + 50 + 50 = 250
    ("interior", (10, 140, 1010, 1140, 0), 150, 10000, (950, 250)),
    # projected 30 - 10 = 20 < 50: ext_left = 20 -> start 0; size = 150 + 0 + 20 + 50 = 220
    ("near_start", (10, 150, 30, 170, 0), 150, 10000, (0, 220)),
    # projected max(0, 20 - 30) = 0: ext_left = 0, start 0; size = 150 + 0 + 0 + 50 = 200
    ("projected_before_contig", (30, 100, 20, 90, 0), 150, 10000, (0, 200)),
    # projected 850, start 800; ext_right = min(50, 1000 - 990) = 10; size = 150 + 50 + 10 = 210,
    # substr(800, 210) of a 1000-base contig keeps 200
    ("near_end", (50, 140, 900, 990, 0), 150, 1000, (800, 200)),
    # NAM ending at the contig end: ext_right = min(50, 1000 - 1000) = 0; size 150 + 50 = 200
    ("nam_at_end", (30, 150, 880, 1000, 0), 150, 1000, (800, 200)),
    # ref span 120, query span 100: diff 20; projected 500, start 450; size 150 + 20 + 50 + 50 = 270
    ("ref_longer", (0, 100, 500, 620, 0), 150, 10000, (450, 270)),
    # query span 120, ref span 100: |100 - 120| = 20, the same window
    ("query_longer", (0, 120, 500, 600, 0), 150, 10000, (450, 270)),
    # a reverse-complement NAM: the same arithmetic on its (rc) coordinates
    ("rc", (20, 150, 5020, 5150, 1), 150, 10000, (4950, 250)),
]

# (name, nam, read_len, contig_len, mu, sigma, expected (window_start, window_len))
RESCUE_WINDOWS = [
    # before the freeze (InsertSizeDistribution: mu 300, sigma 100, aln.hpp:79-90):
    # rc anchor: a = 5020 - 20 - (300 + 500) = 4200; b = 5020 - 20 + 150 / 2 = 5075
    ("rc_unfrozen", (20, 150, 5020, 5150, 1), 150, 10000, "300", "100", (4200, 875)),
    # forward anchor: a = 5130 + (150 - 130) - 75 = 5075; b = 5130 + 20 + 800.0 = 5950
    ("fwd_unfrozen", (0, 130, 5000, 5130, 0), 150, 10000, "300", "100", (5075, 875)),
    # after the freeze, mu 301.25 sigma 29.5 (mu + 5 sigma = 448.75, exact in float):
    # rc: a = 1000 - 448.75 = 551.25 -> 551 (truncation); b = 1000 + 75 = 1075
    ("rc_frozen", (0, 150, 1000, 1150, 1), 150, 10000, "301.25", "29.5", (551, 524)),
    # a = 100 - 448.75 = -348.75 -> -348, clamped by max(0, min(a, len)) to 0; b = 175
    ("rc_clamped_start", (0, 150, 100, 250, 1), 150, 10000, "301.25", "29.5", (0, 175)),
    # forward: a = 9950 + 0 - 75 = 9875; b = 9950 + 448.75 = 10398.75 -> 10398, clamped to 10000
    ("fwd_clamped_end", (0, 150, 9800, 9950, 0), 150, 10000, "301.25", "29.5", (9875, 125)),
    # NAM ending at the contig end, query_end 140: a = 10000 + 10 - 75 = 9935; b -> 10000
    ("fwd_at_end", (0, 140, 9860, 10000, 0), 150, 10000, "301.25", "29.5", (9935, 65)),
    # an odd read length: 151 / 2 = 75 (integer division); a = 2000 - 448.75 = 1551.25 -> 1551,
    # b = 2000 + 75 = 2075
    ("rc_odd_length", (0, 151, 2000, 2151, 1), 151, 10000, "301.25", "29.5", (1551, 524)),
    # float rounding above 2^26 (mu 301.5, sigma 30.25: 301.5 + 151.25 = 452.75, exact):
    # forward: a = 100000153 + 0 - 75 = 100000078 (integers); b = float(100000153) + 452.75:
    # float(100000153) = 100000152 (nearest multiple of 8), 100000152 + 452.75 = 100000604.75
    # -> nearest float 100000608 (100000600 is 4.75 away, 100000608 3.25) -> b = 100000608,
    # length 530 (exact arithmetic would give 527)
    ("fwd_float_rounding", (0, 150, 100000003, 100000153, 0), 150, 200000000, "301.5", "30.25",
     (100000078, 530)),
    # rc: a = float(100000013 - 10) - 452.75: float(100000003) = 100000000 (3 away; 100000008
    # is 5 away), 100000000 - 452.75 = 99999547.25 -> nearest float 99999544 (3.25 away;
    # 99999552 is 4.75) -> a = 99999544; b = 100000003 + 75 = 100000078; length 534
    ("rc_float_rounding", (10, 150, 100000013, 100000153, 1), 150, 200000000, "301.5", "30.25",
     (99999544, 534)),
]

EQ, X, S, I, D = 7, 8, 4, 1, 2


def op(n, o):
    return (n << 4) | o


# (name, kind, nam, read_len, contig_len, mu, sigma, info, expected alignment)
# info = (ref_start, ref_end, query_start, query_end, edit_distance, sw_score, ops) as the
# aligner returns it; expected = (ref_start, length, edit_distance, global_ed, score, is_rc,
# is_unaligned, gapped, ops)
STORES = [
    # extension: window start 950 (EXTENSION_WINDOWS "interior"); ref_start = 950 + 50 = 1000;
    # global_ed = 2 + 0 + (150 - 150) = 2; length = ref_end - ref_start = 150; gapped
    ("ext_plain", "ext", (10, 140, 1010, 1140, 0), 150, None, None, None,
     (50, 200, 0, 150, 2, 280, [op(70, EQ), op(1, X), op(30, EQ), op(1, X), op(48, EQ)]),
     (1000, 150, 2, 2, 280, 0, 0, 1, [op(70, EQ), op(1, X), op(30, EQ), op(1, X), op(48, EQ)])),
    # soft clips on both sides of an rc job: softclipped = 3 + (150 - 145) = 8, global_ed = 1 + 8;
    # window start 4950 ("rc"), ref_start = 4950 + 53 = 5003, length 192 - 53 = 139
    ("ext_rc_clipped", "ext", (20, 150, 5020, 5150, 1), 150, None, None, None,
     (53, 192, 3, 145, 1, 250, [op(3, S), op(60, EQ), op(1, D), op(81, EQ), op(5, S)]),
     (5003, 139, 1, 9, 250, 1, 0, 1, [op(3, S), op(60, EQ), op(1, D), op(81, EQ), op(5, S)])),
    # projected start 20 < 50: window start 0, ref_start = 0 + 20 = 20
    ("ext_near_start", "ext", (10, 150, 30, 170, 0), 150, None, None, None,
     (20, 170, 0, 150, 0, 320, [op(150, EQ)]),
     (20, 150, 0, 0, 320, 0, 0, 1, [op(150, EQ)])),
    # rescue of the mate of an rc anchor (window 4200, "rc_unfrozen"): ref_start = 4200 + 437;
    # the mate lands on the forward strand (is_rc = !nam.is_rc); global_ed / gapped stay as
    # part() left them (a fresh Alignment: 0 / false)
    ("rescue_rc_anchor", "rescue", (20, 150, 5020, 5150, 1), 150, 10000, "300", "100",
     (437, 587, 0, 150, 0, 320, [op(150, EQ)]),
     (4637, 150, 0, 0, 320, 0, 0, 0, [op(150, EQ)])),
    # forward anchor (window 5075): ref_start = 5075 + 225 = 5300, is_rc = 1
    ("rescue_fwd_anchor", "rescue", (0, 130, 5000, 5130, 0), 150, 10000, "300", "100",
     (225, 375, 0, 150, 1, 310, [op(100, EQ), op(1, X), op(49, EQ)]),
     (5300, 150, 1, 0, 310, 1, 0, 0, [op(100, EQ), op(1, X), op(49, EQ)])),
    # an empty CIGAR (the aligner's sentinel for a window over 2000, aligner.cpp:119-125):
    # is_unaligned = cigar.empty(); ref_start = window start + 0; length 0
    ("rescue_empty_cigar", "rescue", (0, 150, 1000, 1150, 1), 150, 10000, "301.25", "29.5",
     (0, 0, 0, 0, 100000, -1000000, []),
     (551, 0, 100000, 0, -1000000, 0, 1, 0, [])),
]

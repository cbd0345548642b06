"""Hand-derived Aligner::align cases (src/aligner.cpp:114-210, ext/ssw/ssw_cpp.cpp:54-210)
with the default scoring A=2 B=8 O=12 E=1, end bonus 10.  Each expectation is worked
out from the source text in the comment next to it; test_oracle_golden checks the
oracle's restatement against them and test_extend_gpu the GPU path."""
import random

EQ, X, S, I, D = 7, 8, 4, 1, 2


def op(n, o):
    return (n << 4) | o


def _ref(seed=17, n=200):
    rnd = random.Random(seed)
    return bytearray(rnd.choice(b"ACGT") for _ in range(n))


def _flip(b):
    return ord("A") if b != ord("A") else ord("C")


def _other(*avoid):
    """A base equal to none of `avoid`."""
    return next(c for c in b"ACGT" if c not in avoid)


def cigar_m(*ops):
    """SSW's own CIGAR words (ssw.c to_cigar_int: len << 4 | index in "MIDNSHP=X")."""
    code = {"M": 0, "I": 1, "D": 2}
    return [(n << 4) | code[o] for n, o in ops]


def cases():
    R = _ref()
    out = []
    # 1. exact 50-mer at ref 10: local 100, both ends reached -> +10 +10 (the extension
    #    loops run zero times, score + bonus > sw), 50=
    q = bytes(R[10:60])
    out.append(("exact", q, bytes(R), dict(sw_score=120, edit_distance=0, ref_start=10, ref_end=60, query_start=0,
                                           query_end=50, cigar=[op(50, EQ)])))
    # 2. mismatch at query 2: SSW clips 3 bases (94 > 90); the front extension X,=,= gives
    #    94 - 8 + 4 = 90, 90 + 10 > 94 -> 2=1X47=, then +10 at the end
    q2 = bytearray(R[10:60]); q2[2] = _flip(q2[2])
    out.append(("front_ext", bytes(q2), bytes(R), dict(sw_score=110, edit_distance=1, ref_start=10, ref_end=60,
                                                      query_start=0, query_end=50,
                                                      cigar=[op(2, EQ), op(1, X), op(47, EQ)])))
    # 3. tail X X = = = (-16 + 6 = -10): SSW ends at query 44 (45=5S, 90); front +10 -> 100;
    #    back extension 100 - 10 = 90, 90 + 10 == 100 is not > 100 -> the soft clip stays
    q3 = bytearray(R[10:60]); q3[45] = _flip(q3[45]); q3[46] = _flip(q3[46])
    out.append(("tail_tie", bytes(q3), bytes(R), dict(sw_score=100, edit_distance=0, ref_start=10, ref_end=55,
                                                     query_start=0, query_end=45, cigar=[op(45, EQ), op(5, S)])))
    # 4. tail X = = = = (-8 + 8 = 0): the forward pass keeps its first maximum (query 44);
    #    back extension 100 + 0 + 10 > 100 -> 45=1X4=
    q4 = bytearray(R[10:60]); q4[45] = _flip(q4[45])
    out.append(("tail_ext", bytes(q4), bytes(R), dict(sw_score=110, edit_distance=1, ref_start=10, ref_end=60,
                                                     query_start=0, query_end=50,
                                                     cigar=[op(45, EQ), op(1, X), op(4, EQ)])))
    # 5. N in query and reference at the same place: SSW scores it -8 (row/column 4 of the
    #    matrix), the =/X split compares translated codes, so N == N is '=' and no edit:
    #    49 * 2 - 8 = 90, +20 -> 110, 50=
    rn = bytearray(R); rn[30] = ord("N")
    q5 = bytes(rn[10:60])
    out.append(("n_eq_n", q5, bytes(rn), dict(sw_score=110, edit_distance=0, ref_start=10, ref_end=60, query_start=0,
                                              query_end=50, cigar=[op(50, EQ)])))
    # 6. three extra bases before a read that starts at reference 0: the front loop cannot
    #    run (rstart == 0), qstart stays 3 -> 3S47=, 94, then +10 at the end
    q6 = b"TTT" + bytes(R[0:47])
    q6 = bytearray(q6)
    for i in range(3):
        if q6[i] == R[i]:
            q6[i] = _flip(q6[i])
    out.append(("ref_start_clip", bytes(q6), bytes(R), dict(sw_score=104, edit_distance=0, ref_start=0, ref_end=47,
                                                           query_start=3, query_end=50, cigar=[op(3, S), op(47, EQ)])))
    # 7. both ends clipped: five flipped bases on each side of an exact 40-mer.  SSW's local
    #    maximum is the 40-mer (80; a flank base costs 8, a gap to reach a match 12 > the 10
    #    five matches could bring); the front extension scores 80 - 5 * 8 = 40 and 40 + 10 is
    #    not > 80, the back extension likewise: 5S40=5S, no edits (S is not counted)
    q7 = bytearray(R[10:60])
    for i in list(range(0, 5)) + list(range(45, 50)):
        q7[i] = _flip(q7[i])
    out.append(("both_clipped", bytes(q7), bytes(R), dict(sw_score=80, edit_distance=0, ref_start=15, ref_end=55,
                                                         query_start=5, query_end=45,
                                                         cigar=[op(5, S), op(40, EQ), op(5, S)])))
    # 8. one reference base (R[40] = 'C', between 'T' and 'A': no equal neighbour, so the
    #    gap has one place) missing from the query: 59 matches - gap_open 12 = 106; both
    #    ends reached -> +10 +10 = 126; D counts as an edit (ssw_cpp.cpp:126-210)
    q8 = bytes(R[10:40] + R[41:70])
    out.append(("deletion", q8, bytes(R), dict(sw_score=126, edit_distance=1, ref_start=10, ref_end=70,
                                               query_start=0, query_end=59,
                                               cigar=[op(30, EQ), op(1, D), op(29, EQ)])))
    # 9. a 'G' inserted between R[39] = 'T' and R[40] = 'C' (equal to neither): 60 matches -
    #    12 = 108, +20 -> 128, one I edit, the query end is 61
    q9 = bytes(R[10:40] + b"G" + R[40:70])
    out.append(("insertion", q9, bytes(R), dict(sw_score=128, edit_distance=1, ref_start=10, ref_end=70,
                                                query_start=0, query_end=61,
                                                cigar=[op(30, EQ), op(1, I), op(30, EQ)])))
    # 10. window longer than 2000: the sentinel (aligner.cpp:119-125)
    out.append(("ref_gt_2000", bytes(R[10:60]), bytes(_ref(3, 2001)), dict(sw_score=-1000000, edit_distance=100000,
                                                                           ref_start=0)))
    out += cases_r04(R)
    return out


def cases_r04(R):
    """Round-4 cases (VERDICT r03 "next" item 8).  SSW's part of each derivation (score1,
    begins/ends, the M/I/D CIGAR) is also checked against the reference's own ssw.c run
    here (ssw_core(), tests/test_oracle_golden.py::test_wrapper_cases_ssw_core_live)."""
    out = []
    # 11. a gap seven bases after a clip that the front extension replaces.  banded_sw's
    #     traceback appends a final M after its last move (ssw.c:756-770), so the CIGAR of
    #     an SSW alignment always begins with M: a clip cannot be followed by I or D
    #     directly; the closest case is a short = run, then the gap.
    #     query = R[18] (=), flip(R[19]) (X), R[20:27] (7 bases), b, R[27:67] (40 bases), with
    #     b equal to neither R[26] nor R[27] (the insertion has one place; asserted).
    #     SSW: 7 x 2 - 12 + 40 x 2 = 82 beats the 40-base run alone (80); the two leading
    #     bases add -8 + 2 < 0, so read_begin1 = 2, ref_begin1 = 20, read_end1 = 49, ref_end1 =
    #     66; banded_sw (refLen 47, readLen 48, band 2) keeps 82 and traces 7M1I40M.
    #     ConvertAlignment/CalculateNumberMismatch: 2S7=1I40=, mismatches 1 (the I).
    #     Aligner::align: front loop q1 vs R19 X (74), q0 vs R18 = (76); q reaches 0 and 76 + 10 >
    #     82: the 2S goes, front_cigar reversed (= X) is followed by 7=1I40= (no merge: X then
    #     =) -> 1=1X7=1I40=, ref_start 18, score 86, edits 2; back: query end reached, 86 + 10
    #     > 86 -> 96
    assert R[26] != R[27]
    b = _other(R[26], R[27])
    q11 = bytes([R[18], _flip(R[19])]) + bytes(R[20:27]) + bytes([b]) + bytes(R[27:67])
    out.append(("front_ext_then_ins", q11, bytes(R),
                dict(sw_score=96, edit_distance=2, ref_start=18, ref_end=67, query_start=0, query_end=50,
                     cigar=[op(1, EQ), op(1, X), op(7, EQ), op(1, I), op(40, EQ)])))
    # 12. the same with a deletion: R[27] is skipped (R[27] differs from R[26] and R[28], so
    #     the deletion has one place; asserted).  SSW 82 (7M1D40M, refLen 48, readLen 47);
    #     front extension as in 11 -> 1=1X7=1D40=, ref_start 18, ref_end 68, 86 + 10 = 96
    assert R[27] != R[26] and R[27] != R[28]
    q12 = bytes([R[18], _flip(R[19])]) + bytes(R[20:27]) + bytes(R[28:68])
    out.append(("front_ext_then_del", q12, bytes(R),
                dict(sw_score=96, edit_distance=2, ref_start=18, ref_end=68, query_start=0, query_end=49,
                     cigar=[op(1, EQ), op(1, X), op(7, EQ), op(1, D), op(40, EQ)])))
    # 13. end-bonus ties at both ends: query = R[10:60] with q3, q4, q45, q46 flipped.  Read
    #     outward from the 40-base core (q5..q44 = R15..R54, SSW 80, 40M), each flank is
    #     X X = = = (-16 + 6 = -10, every partial flank negative, so SSW clips both).  Front
    #     extension 80 - 10 = 70, 70 + 10 > 80 fails (equal); the back likewise: 5S40=5S, 80
    q13 = bytearray(R[10:60])
    for i in (3, 4, 45, 46):
        q13[i] = _flip(q13[i])
    out.append(("both_ends_tie", bytes(q13), bytes(R),
                dict(sw_score=80, edit_distance=0, ref_start=15, ref_end=55, query_start=5, query_end=45,
                     cigar=[op(5, S), op(40, EQ), op(5, S)])))
    # 14. N on both sides of a mismatch: ref N at 28 and 30, query = that ref[10:60] with q19
    #     (ref 29) changed to a base that matches neither its own nor a neighbouring ref base
    #     (no shifted diagonal scores; asserted).  SSW scores N-N -8: 47 matches - 3 x 8 = 70
    #     beats the right part alone (29 x 2 = 58) and any gap pair around the three bases
    #     (I3 + D3 costs 2 x (12 + 2) = 28 > 24), so the whole 50 bases align, 50M
    #     (refLen = readLen: band 1).  (With four bases N X X N a 4I4D pair, 30, beats four
    #     mismatches, 32: the live ssw.c check caught that in a first draft of this case.)
    #     The =/X split compares translated codes, N (4) == N (4): 19= (q0..q18) 1X 30=
    #     (q20..q49), mismatches 1.  Both ends reached: 70 + 10 + 10 = 90
    rn = bytearray(R)
    rn[28] = rn[30] = ord("N")
    q14 = bytearray(rn[10:60])
    q14[19] = _other(R[29], R[28], R[30])
    out.append(("n_around_mismatch", bytes(q14), bytes(rn),
                dict(sw_score=90, edit_distance=1, ref_start=10, ref_end=60, query_start=0, query_end=50,
                     cigar=[op(19, EQ), op(1, X), op(30, EQ)])))
    # 15. N inside the front extension: ref N at 12, query = that ref[10:60] with q3 flipped
    #     (q2 = N).  SSW: the prefix q0..q3 scores 2 + 2 - 8 - 8 < 0 (N-N is -8), every part
    #     of it too, so 4S46M (92, core q4..q49 = ref 14..59).  The front loop compares raw
    #     bytes (aligner.cpp:152-163): q3 X (84), q2 N == N '=' (86), q1, q0 = (90); 90 + 10 >
    #     92 -> X = = = reversed -> 3=1X, then 46= -> 3=1X46=, ref_start 10, 100, edits 1;
    #     back +10 -> 110
    rn2 = bytearray(R)
    rn2[12] = ord("N")
    q15 = bytearray(rn2[10:60])
    q15[3] = _flip(q15[3])
    out.append(("n_in_front_extension", bytes(q15), bytes(rn2),
                dict(sw_score=110, edit_distance=1, ref_start=10, ref_end=60, query_start=0, query_end=50,
                     cigar=[op(3, EQ), op(1, X), op(46, EQ)])))
    # 16. a window of exactly 2000 bases is aligned (the sentinel is for > 2000,
    #     aligner.cpp:119): an exact 50-mer at 1000 -> 100 + 10 + 10, 50=
    W = _ref(5, 2000)
    out.append(("ref_eq_2000", bytes(W[1000:1050]), bytes(W),
                dict(sw_score=120, edit_distance=0, ref_start=1000, ref_end=1050, query_start=0, query_end=50,
                     cigar=[op(50, EQ)])))
    # 17. one base more, the same exact 50-mer: the sentinel, no CIGAR
    W1 = _ref(5, 2001)
    out.append(("ref_eq_2001", bytes(W1[1000:1050]), bytes(W1),
                dict(sw_score=-1000000, edit_distance=100000, ref_start=0, cigar=[])))
    return out


def ssw_core():
    """SSW's own results for the cases whose derivation above states them:
    (score1, ref_begin1, ref_end1, read_begin1, read_end1, SSW CIGAR words)."""
    return {
        "exact": (100, 10, 59, 0, 49, cigar_m((50, "M"))),
        "deletion": (106, 10, 69, 0, 58, cigar_m((30, "M"), (1, "D"), (29, "M"))),
        "insertion": (108, 10, 69, 0, 60, cigar_m((30, "M"), (1, "I"), (30, "M"))),
        "both_clipped": (80, 15, 54, 5, 44, cigar_m((40, "M"))),
        "front_ext_then_ins": (82, 20, 66, 2, 49, cigar_m((7, "M"), (1, "I"), (40, "M"))),
        "front_ext_then_del": (82, 20, 67, 2, 48, cigar_m((7, "M"), (1, "D"), (40, "M"))),
        "both_ends_tie": (80, 15, 54, 5, 44, cigar_m((40, "M"))),
        "n_around_mismatch": (70, 10, 59, 0, 49, cigar_m((50, "M"))),
        "n_in_front_extension": (92, 14, 59, 4, 49, cigar_m((46, "M"))),
        "ref_eq_2000": (100, 1000, 1049, 0, 49, cigar_m((50, "M"))),
    }

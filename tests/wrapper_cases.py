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
    return out

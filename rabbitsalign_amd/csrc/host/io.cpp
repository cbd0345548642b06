// io.cpp -- CIGAR text, SAM records, FASTA, .sti read/write/build, FASTQ input.
// Restated from src/cigar.cpp, src/sam.cpp, src/refs.cpp, src/index.cpp,
// src/indexparameters.cpp and the kseq++ record semantics used by src/fastq.cpp.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <exception>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <thread>

#include "rsa_host.hpp"
#include "sti_order.hpp"

namespace rsa {

// ----------------------------------------------------------------- CIGAR --
Cigar Cigar::to_m() const {                        // cigar.cpp:6-18
    Cigar c;
    for (uint32_t x : ops) {
        uint32_t op = x & 0xf, len = x >> 4;
        if (op == C_EQ || op == C_X) c.push(C_M, len);
        else c.push(op, len);
    }
    return c;
}

// raw writers for the SAM record: the caller sizes the buffer first, so the
// fields go in without a capacity check per character
static const char kDigitPairs[201] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";

// digits written in place from the end backwards, two at a time (no staging buffer,
// so no variable-length memcpy call per number)
static inline char* put_uint(char* p, uint64_t v) {
    int n = 1;
    for (uint64_t t = 10; n < 20 && v >= t; t *= 10) ++n;
    char* const e = p + n;
    char* q = e;
    while (v >= 100) {
        const unsigned r = (unsigned)(v % 100);
        v /= 100;
        q -= 2;
        memcpy(q, kDigitPairs + 2 * r, 2);
    }
    if (v >= 10) { q -= 2; memcpy(q, kDigitPairs + 2 * v, 2); }
    else *--q = (char)('0' + v);
    return e;
}

static inline char* put_int(char* p, int64_t v) {
    if (v < 0) { *p++ = '-'; return put_uint(p, (uint64_t)(-v)); }
    return put_uint(p, (uint64_t)v);
}

// short fields (names, contig names, tags) by overlapping fixed-size moves that
// stay inside [0, n) of the source; SEQ / QUAL and longer go through memcpy
static inline char* put_str(char* p, std::string_view s) {
    const char* src = s.data();
    const size_t n = s.size();
    if (n >= 16 && n <= 32) {
        memcpy(p, src, 16);
        memcpy(p + n - 16, src + n - 16, 16);
    } else if (n >= 8 && n < 16) {
        memcpy(p, src, 8);
        memcpy(p + n - 8, src + n - 8, 8);
    } else if (n >= 4 && n < 8) {
        memcpy(p, src, 4);
        memcpy(p + n - 4, src + n - 4, 4);
    } else if (n < 4) {
        for (size_t i = 0; i < n; ++i) p[i] = src[i];
    } else {
        memcpy(p, src, n);
    }
    return p + n;
}

static inline void append_uint(std::string& out, uint64_t v) {
    char buf[24];
    int n = 0;
    do { buf[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (n) out.push_back(buf[--n]);
}

static inline void append_int(std::string& out, int64_t v) {
    if (v < 0) { out.push_back('-'); append_uint(out, (uint64_t)(-v)); }
    else append_uint(out, (uint64_t)v);
}

void Cigar::to_string(std::string& out) const {    // cigar.cpp:45-51
    for (uint32_t x : ops) {
        append_uint(out, x >> 4);
        out.push_back("MIDNSHP=X"[x & 0xf]);
    }
}

// to_m() (=/X -> M, merged by Cigar::push) printed directly
void Cigar::to_m_string(std::string& out) const {
    uint32_t cur = 0xff, len = 0;
    for (uint32_t x : ops) {
        uint32_t op = x & 0xf;
        if (op == C_EQ || op == C_X) op = C_M;
        if (op == cur) { len += x >> 4; continue; }
        if (cur != 0xff) { append_uint(out, len); out.push_back("MIDNSHP=X"[cur]); }
        cur = op;
        len = x >> 4;
    }
    if (cur != 0xff) { append_uint(out, len); out.push_back("MIDNSHP=X"[cur]); }
}

// ------------------------------------------------------------------- SAM --
static std::string_view strip_suffix(std::string_view name) {   // sam.cpp:29-40
    size_t len = name.size();
    if (len >= 2 && name[len - 2] == '/' && (name[len - 1] == '1' || name[len - 1] == '2'))
        return name.substr(0, len - 2);
    return name;
}

Sam::Sam(SamText& out, const References& refs, bool eqx, const std::string& rg_id, bool output_unmapped,
         bool details)
    : out_(out), refs_(refs), eqx_(eqx), output_unmapped_(output_unmapped), details_(details) {
    tail_ = rg_id.empty() ? "\n" : "\tRG:Z:" + rg_id + "\n";
}

// room for `bound` more bytes at the end of o (uninitialised); returns where they start
static inline char* sam_room(SamText& o, size_t bound, size_t& at) {
    at = o.size();
    o.resize(at + bound);
    return o.data() + at;
}
static inline void sam_trim(SamText& o, size_t at, const char* p0, const char* p) { o.resize(at + (size_t)(p - p0)); }

static char* put_details(char* p, const Details& d, bool paired) {   // sam.cpp:46-60
    p = put_str(p, "\tna:i:"); p = put_uint(p, d.nams);
    p = put_str(p, "\tnr:i:"); p = put_uint(p, d.nam_rescue ? 1 : 0);
    p = put_str(p, "\tal:i:"); p = put_uint(p, d.tried_alignment);
    p = put_str(p, "\tga:i:"); p = put_uint(p, d.gapped);
    if (paired) { p = put_str(p, "\tmr:i:"); p = put_uint(p, d.mate_rescue); }
    return p;
}
static const size_t kDetailsBound = 5 * (6 + 20);

void Sam::add_unmapped(const RecView& r, uint16_t flags) {   // sam.cpp:77-92
    if (!output_unmapped_) return;
    const std::string_view name = strip_suffix(r.name);
    size_t at;
    char* const p0 = sam_room(out_, name.size() + r.seq.size() + r.qual.size() + tail_.size() + 48, at);
    char* p = put_str(p0, name);
    *p++ = '\t';
    p = put_uint(p, flags);
    p = put_str(p, "\t*\t0\t0\t*\t*\t0\t0\t");
    p = put_str(p, r.seq.empty() ? std::string_view("*") : std::string_view(r.seq));
    *p++ = '\t';
    p = put_str(p, r.qual.empty() ? std::string_view("*") : std::string_view(r.qual));
    p = put_str(p, tail_);
    line_done(p0, p);
    sam_trim(out_, at, p0, p);
}

void Sam::add_unmapped_mate(const RecView& r, uint16_t flags, std::string_view mate_ref, uint32_t mate_pos) {
    const std::string_view name = strip_suffix(r.name);      // sam.cpp:94-116
    size_t at;
    char* const p0 =
        sam_room(out_, name.size() + mate_ref.size() + r.seq.size() + r.qual.size() + tail_.size() + 64, at);
    char* p = put_str(p0, name);
    *p++ = '\t';
    p = put_uint(p, flags);
    *p++ = '\t';
    p = put_str(p, mate_ref);
    *p++ = '\t';
    p = put_uint(p, (uint32_t)(mate_pos + 1));
    p = put_str(p, "\t0\t*\t=\t");
    p = put_uint(p, (uint32_t)(mate_pos + 1));
    p = put_str(p, "\t0\t");
    p = put_str(p, r.seq.empty() ? std::string_view("*") : std::string_view(r.seq));
    *p++ = '\t';
    p = put_str(p, r.qual.empty() ? std::string_view("*") : std::string_view(r.qual));
    p = put_str(p, tail_);
    line_done(p0, p);
    sam_trim(out_, at, p0, p);
}

void Sam::add_unmapped_pair(const RecView& r1, const RecView& r2) {
    add_unmapped(r1, 1 | 4 | 8 | 0x40);
    add_unmapped(r2, 1 | 4 | 8 | 0x80);
}

void Sam::add(const Alignment& a, const RecView& r, std::string_view rc, uint8_t mapq, bool primary,
              const Details& d) {                               // sam.cpp:124-139
    int flags = 0;
    if (!a.is_unaligned && a.is_rc) flags |= 0x10;
    if (!primary) { flags |= 0x100; mapq = 255; }
    add_record(r.name, (uint16_t)flags, refs_.names[a.ref_id], (uint32_t)a.ref_start, mapq, a.cigar, "*",
               (uint32_t)-1, 0, r.seq, rc, r.qual, a.edit_distance, a.score, d);
}

// CIGAR text straight into a sized buffer: `=`/`X` kept (eqx) or merged into M
// (Cigar::to_m, cigar.cpp:6-18)
static char* put_cigar(char* p, const Cigar& c, bool eqx) {
    if (eqx) {
        for (uint32_t x : c.ops) { p = put_uint(p, x >> 4); *p++ = "MIDNSHP=X"[x & 0xf]; }
        return p;
    }
    uint32_t cur = 0xff, len = 0;
    for (uint32_t x : c.ops) {
        uint32_t op = x & 0xf;
        if (op == C_EQ || op == C_X) op = C_M;
        if (op == cur) { len += x >> 4; continue; }
        if (cur != 0xff) { p = put_uint(p, len); *p++ = "MIDNSHP=X"[cur]; }
        cur = op;
        len = x >> 4;
    }
    if (cur != 0xff) { p = put_uint(p, len); *p++ = "MIDNSHP=X"[cur]; }
    return p;
}

void Sam::add_record(std::string_view qname, uint16_t flags, std::string_view rname, uint32_t pos, uint8_t mapq,
                     const Cigar& cigar, std::string_view mate_rname, uint32_t mate_pos, int32_t tlen,
                     std::string_view seq, std::string_view seq_rc, std::string_view qual, int ed, int score,
                     const Details& d) {                        // sam.cpp:141-213
    const std::string_view name = strip_suffix(qname);
    // upper bound of the record: fixed fields + numbers + CIGAR (<= 11 chars an op) + SEQ/QUAL + tags
    const size_t bound = name.size() + rname.size() + mate_rname.size() + std::max(seq.size(), seq_rc.size()) +
                         qual.size() + 11 * cigar.ops.size() + tail_.size() + 160 + (details_ ? kDetailsBound : 0);
    size_t at;
    char* const p0 = sam_room(out_, bound, at);
    char* p = p0;
    p = put_str(p, name);
    *p++ = '\t';
    p = put_uint(p, flags);
    *p++ = '\t';
    p = put_str(p, rname);
    *p++ = '\t';
    p = put_uint(p, (uint32_t)(pos + 1));
    *p++ = '\t';
    p = put_uint(p, mapq);
    *p++ = '\t';
    if (cigar.empty()) *p++ = '*';
    else p = put_cigar(p, cigar, eqx_);
    *p++ = '\t';
    p = put_str(p, mate_rname);
    *p++ = '\t';
    p = put_uint(p, (uint32_t)(mate_pos + 1));
    *p++ = '\t';
    p = put_int(p, tlen);
    *p++ = '\t';
    if (flags & 0x100) *p++ = '*';
    else if (flags & 0x10) p = put_str(p, seq_rc.empty() ? std::string_view("*") : seq_rc);
    else p = put_str(p, seq.empty() ? std::string_view("*") : seq);
    *p++ = '\t';
    if (!(flags & 4)) {
        if (flags & 0x100) *p++ = '*';
        else if (flags & 0x10) {
            if (qual.empty()) *p++ = '*';
            else { reverse_into(qual, p); p += qual.size(); }
        } else p = put_str(p, qual.empty() ? std::string_view("*") : std::string_view(qual));
        p = put_str(p, "\tNM:i:");
        p = put_int(p, ed);
        p = put_str(p, "\tAS:i:");
        p = put_int(p, score);
    } else {
        p = put_str(p, qual.empty() ? std::string_view("*") : std::string_view(qual));
    }
    if (details_) p = put_details(p, d, flags & 1);
    p = put_str(p, tail_);
    line_done(p0, p);
    sam_trim(out_, at, p0, p);
}

void Sam::add_pair(const Alignment& a1, const Alignment& a2, const RecView& r1, const RecView& r2, std::string_view rc1,
                   std::string_view rc2, uint8_t mapq1, uint8_t mapq2, bool proper, bool primary,
                   const Details d[2]) {                        // sam.cpp:215-313
    int f1 = 1 | 0x40, f2 = 1 | 0x80;
    if (!primary) { f1 |= 0x100; f2 |= 0x100; }
    int tlen1 = 0;
    bool both = !a1.is_unaligned && !a2.is_unaligned;
    if (both && a1.ref_id == a2.ref_id) {
        const int dist = a2.ref_start - a1.ref_start;
        if (dist > 0) tlen1 = dist + a2.length;
        else tlen1 = dist - a1.length;
    }
    if (proper) { f1 |= 2; f2 |= 2; }
    std::string_view rn1, rn2;
    int pos1 = a1.ref_start, pos2 = a2.ref_start;
    if (a1.is_unaligned) { f1 |= 4; f2 |= 8; pos1 = -1; rn1 = "*"; }
    else { if (a1.is_rc) { f1 |= 0x10; f2 |= 0x20; } rn1 = refs_.names[a1.ref_id]; }
    if (a2.is_unaligned) { f2 |= 4; f1 |= 8; pos2 = -1; rn2 = "*"; }
    else { if (a2.is_rc) { f1 |= 0x20; f2 |= 0x10; } rn2 = refs_.names[a2.ref_id]; }
    std::string_view mrn1 = rn1, mrn2 = rn2;
    if ((both && a1.ref_id == a2.ref_id) || (a1.is_unaligned != a2.is_unaligned)) { mrn1 = "="; mrn2 = "="; }
    if (a1.is_unaligned != a2.is_unaligned) {
        if (a1.is_unaligned) pos1 = pos2; else pos2 = pos1;
    }
    if (a1.is_unaligned) add_unmapped_mate(r1, (uint16_t)f1, rn2, (uint32_t)pos2);
    else add_record(r1.name, (uint16_t)f1, rn1, (uint32_t)a1.ref_start, mapq1, a1.cigar, mrn2, (uint32_t)pos2, tlen1,
                    r1.seq, rc1, r1.qual, a1.edit_distance, a1.score, d[0]);
    if (a2.is_unaligned) add_unmapped_mate(r2, (uint16_t)f2, rn1, (uint32_t)pos1);
    else add_record(r2.name, (uint16_t)f2, rn2, (uint32_t)a2.ref_start, mapq2, a2.cigar, mrn1, (uint32_t)pos1, -tlen1,
                    r2.seq, rc2, r2.qual, a2.edit_distance, a2.score, d[1]);
}

bool is_proper_pair(const Alignment& a1, const Alignment& a2, float mu, float sigma) {   // sam.cpp:315-325
    const int dist = a2.ref_start - a1.ref_start;
    const bool same_reference = a1.ref_id == a2.ref_id;
    const bool both_aligned = same_reference && !a1.is_unaligned && !a2.is_unaligned;
    const bool r1_r2 = !a1.is_rc && a2.is_rc && dist >= 0;
    const bool r2_r1 = !a2.is_rc && a1.is_rc && dist <= 0;
    const bool rel_orientation_good = r1_r2 || r2_r1;
    const bool insert_good = std::abs(dist) <= mu + 6 * sigma;
    return both_aligned && insert_good && rel_orientation_good;
}

std::string sam_header(const References& refs, const std::string& rg_id, const std::vector<std::string>& rg,
                       const std::string& cmd_line) {          // main.cpp:84-99
    std::string o = "@HD\tVN:1.6\tSO:unsorted\n";
    for (size_t i = 0; i < refs.size(); ++i) {
        o += "@SQ\tSN:" + refs.names[i] + "\tLN:";
        append_uint(o, (uint32_t)refs.seqs[i].size());
        o += "\n";
    }
    if (!rg_id.empty()) {
        o += "@RG\tID:" + rg_id;
        for (const auto& f : rg) o += "\t" + f;
        o += "\n";
    }
    o += "@PG\tID:rabbitsalign\tPN:rabbitsalign\tVN:0.1.0-mi355x\tCL:" + cmd_line + "\n";
    return o;
}

// ----------------------------------------------------------------- FASTA --
References References::from_fasta(const std::string& path) {   // refs.cpp:20-58
    std::ifstream in(path);
    if (!in) throw std::runtime_error("Cannot read from FASTA file " + path);
    if (in.peek() != '>') throw std::runtime_error("FASTA file must begin with '>' character");
    References r;
    std::string line, seq, name;
    bool eof = false;
    do {
        eof = !bool(std::getline(in, line));
        if (eof || (!line.empty() && line[0] == '>')) {
            if (!seq.empty()) {
                to_uppercase(seq);
                r.seqs.push_back(seq);
                r.names.push_back(name);
            }
            if (!eof) name = line.substr(1, line.find(' ') - 1);
            seq.clear();
        } else {
            seq += line;
        }
    } while (!eof);
    r.offsets.assign(1, 0);
    size_t total = 0;
    for (auto& s : r.seqs) { total += s.size(); r.offsets.push_back(total); }
    r.concat.reserve(total);
    for (auto& s : r.seqs) r.concat += s;
    r.make_hot();
    return r;
}

void References::make_hot() {
    const size_t total = concat.size();
    views.clear();
    hot.reset();
    if (total == 0) return;
    const size_t huge = 2u << 20;
    const size_t bytes = (total + huge - 1) / huge * huge;
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return;                    // plain strings keep serving seq(i)
    madvise(p, bytes, MADV_HUGEPAGE);               // before the first touch
    memcpy(p, concat.data(), total);
    hot = std::shared_ptr<char>((char*)p, [bytes](char* q) { munmap(q, bytes); });
    for (size_t i = 0; i < seqs.size(); ++i) views.emplace_back(hot.get() + offsets[i], offsets[i + 1] - offsets[i]);
}

// ------------------------------------------------------ IndexParameters --
struct Profile { int crl, r_threshold, k, s_offset, l, u; };
static const Profile kProfiles[] = {            // indexparameters.cpp:136-144
    {50, 90, 20, -4, -3, 2}, {100, 110, 20, -4, -2, 2}, {125, 135, 20, -4, -1, 4}, {150, 175, 20, -4, 1, 7},
    {250, 275, 20, -4, 4, 13}, {300, 375, 22, -4, 2, 12}, {400, INT32_MAX, 23, -6, 2, 12},
};

void IndexParameters::finalize() {
    t = (k - s) / 2 + 1;
    int wm = k / (k - s + 1) + l;
    w_min = (unsigned)std::max(0, wm);
    w_max = (unsigned)(k / (k - s + 1) + u);
    if (k <= 7 || k > 32) throw std::runtime_error("k not in [8,32]");
    if (s > k) throw std::runtime_error("s is larger than k");
    if ((k - s) % 2 != 0) throw std::runtime_error("(k - s) must be an even number");
    if (max_dist > 255) throw std::runtime_error("maximum seed length (-m) is larger than 255");
    if (w_min > w_max) throw std::runtime_error("w_min is greater than w_max");
}

IndexParameters IndexParameters::from_read_length(int read_length, int k, int s, int l, int u, int c,
                                                  int max_seed_len) {   // indexparameters.cpp:150-182
    const int DEF = INT32_MIN;
    int crl = 50;
    for (const auto& p : kProfiles) {
        if (read_length <= p.r_threshold) {
            if (k == DEF) k = p.k;
            if (s == DEF) s = k + p.s_offset;
            if (l == DEF) l = p.l;
            if (u == DEF) u = p.u;
            crl = p.crl;
            break;
        }
    }
    int max_dist;
    if (max_seed_len == DEF) {
        max_dist = std::max(crl - 70, k);
        max_dist = std::min(255, max_dist);
    } else {
        max_dist = max_seed_len - k;
    }
    int q = (int)std::pow(2, c == DEF ? 8 : c) - 1;
    IndexParameters ip;
    ip.canonical_read_length = crl; ip.k = k; ip.s = s; ip.l = l; ip.u = u; ip.q = q; ip.max_dist = max_dist;
    ip.finalize();
    return ip;
}

bool IndexParameters::operator==(const IndexParameters& o) const {
    return canonical_read_length == o.canonical_read_length && k == o.k && s == o.s && t == o.t && l == o.l &&
           u == o.u && q == o.q && max_dist == o.max_dist && w_min == o.w_min && w_max == o.w_max;
}

std::string IndexParameters::filename_extension() const {   // indexparameters.cpp:216-224
    std::string s;
    if (*this == from_read_length(canonical_read_length)) s = ".r" + std::to_string(canonical_read_length);
    return s + ".sti";
}

// ------------------------------------------------------------------ .sti --
template <class T> static void wr(std::ofstream& o, const T& v) { o.write((const char*)&v, sizeof(T)); }
template <class T> static T rd(std::ifstream& i) { T v{}; i.read((char*)&v, sizeof(T)); return v; }

void StiIndex::write(const std::string& path) const {   // index.cpp:73-89
    std::ofstream o(path, std::ios::binary);
    o.write("STI\1", 4);
    wr<int32_t>(o, 2);
    wr<uint64_t>(o, 8);
    const char reserved[8] = {0};
    o.write(reserved, 8);
    wr<int32_t>(o, filter_cutoff);
    wr<int32_t>(o, bits);
    const int32_t prm[7] = {params.canonical_read_length, params.k, params.s, params.l, params.u, params.q,
                            params.max_dist};
    o.write((const char*)prm, sizeof prm);
    wr<uint64_t>(o, randstrobes.size());
    o.write((const char*)randstrobes.data(), (std::streamsize)(randstrobes.size() * sizeof(rsa_ref_randstrobe)));
    wr<uint64_t>(o, bucket_starts.size());
    o.write((const char*)bucket_starts.data(), (std::streamsize)(bucket_starts.size() * 8));
    if (!o) throw std::runtime_error("cannot write " + path);
}

void StiIndex::read(const std::string& path) {          // index.cpp:91-132
    std::ifstream in(path, std::ios::binary);
    if (!in) throw std::runtime_error("cannot open index " + path);
    char magic[4];
    in.read(magic, 4);
    if (memcmp(magic, "STI\1", 4) != 0) throw std::runtime_error("Index file has incorrect format (magic number mismatch)");
    if (rd<int32_t>(in) != 2) throw std::runtime_error("Can only read index file format version 2");
    uint64_t reserved = rd<uint64_t>(in);
    in.seekg((std::streamoff)reserved, std::ios_base::cur);
    filter_cutoff = rd<int32_t>(in);
    bits = rd<int32_t>(in);
    int32_t prm[7];
    in.read((char*)prm, sizeof prm);
    params.canonical_read_length = prm[0]; params.k = prm[1]; params.s = prm[2]; params.l = prm[3];
    params.u = prm[4]; params.q = prm[5]; params.max_dist = prm[6];
    params.finalize();
    uint64_t n = rd<uint64_t>(in);
    randstrobes.resize(n);
    in.read((char*)randstrobes.data(), (std::streamsize)(n * sizeof(rsa_ref_randstrobe)));
    uint64_t ns = rd<uint64_t>(in);
    bucket_starts.resize(ns);
    in.read((char*)bucket_starts.data(), (std::streamsize)(ns * 8));
    if (!in) throw std::runtime_error("truncated index " + path);
    if (ns != (1ull << bits) + 1) throw std::runtime_error("randstrobe_start_indices vector is of the wrong size");
}

// --- index construction (index.cpp:141-309) --------------------------------
// Randstrobes of the forward reference (RandstrobeGenerator semantics equal the
// query iterator's: window [i+w_min, min(i+w_max, n-1)], first min popcount).
static uint64_t xxh64_u64(uint64_t input) {              // hash.hpp:105-118
    const uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL,
                   P4 = 0x85EBCA77C2B2AE63ULL, P5 = 0x27D4EB2F165667C5ULL;
    uint64_t acc = P5 + 8, k1 = input * P2;
    k1 = (k1 << 31) | (k1 >> 33);
    acc ^= k1 * P1;
    acc = ((acc << 27) | (acc >> 37)) * P1 + P4;
    acc ^= acc >> 33; acc *= P2; acc ^= acc >> 29; acc *= P3; acc ^= acc >> 32;
    return acc;
}

struct Syncmer { uint64_t hash; uint32_t pos; };

static void syncmers_of(std::string_view seq, const IndexParameters& p, std::vector<Syncmer>& out) {
    out.clear();
    const int k = p.k, s = p.s, t = p.t;
    const uint64_t kmask = (k == 32) ? ~0ULL : ((1ULL << (2 * k)) - 1), smask = (1ULL << (2 * s)) - 1;
    const int kshift = (k - 1) * 2, sshift = (s - 1) * 2, W = k - s + 1;
    uint64_t ring[64];
    int qn = 0, qh = 0, l = 0;
    uint64_t min_val = UINT64_MAX, xk0 = 0, xk1 = 0, xs0 = 0, xs1 = 0;
    long long min_pos = -1;
    for (size_t i = 0; i < seq.size(); ++i) {
        int c;
        switch (seq[i]) {
            case 'A': case 'a': c = 0; break;
            case 'C': case 'c': c = 1; break;
            case 'G': case 'g': c = 2; break;
            case 'T': case 't': case 'U': case 'u': c = 3; break;
            default: c = 4;
        }
        if (c < 4) {
            xk0 = ((xk0 << 2) | (uint64_t)c) & kmask;
            xk1 = (xk1 >> 2) | ((uint64_t)(3 - c) << kshift);
            xs0 = ((xs0 << 2) | (uint64_t)c) & smask;
            xs1 = (xs1 >> 2) | ((uint64_t)(3 - c) << sshift);
            if (++l < s) continue;
            uint64_t hs = xxh64_u64(std::min(xs0, xs1));
            ring[(qh + qn) & 63] = hs;
            qn++;
            if (qn < W) continue;
            long long ii = (long long)i;
            if (qn == W) {
                for (int j = 0; j < qn; ++j) {
                    uint64_t v = ring[(qh + j) & 63];
                    if (v < min_val) { min_val = v; min_pos = ii - k + j + 1; }
                }
            } else {
                qh = (qh + 1) & 63; qn--;
                if (min_pos == ii - k) {
                    min_val = UINT64_MAX; min_pos = ii - s + 1;
                    for (int j = qn - 1; j >= 0; --j) {
                        uint64_t v = ring[(qh + j) & 63];
                        if (v < min_val) { min_val = v; min_pos = ii - k + j + 1; }
                    }
                } else if (hs < min_val) { min_val = hs; min_pos = ii - s + 1; }
            }
            if (min_pos == ii - k + t) out.push_back(Syncmer{xxh64_u64(std::min(xk0, xk1)), (uint32_t)(ii - k + 1)});
        } else {
            min_val = UINT64_MAX; min_pos = -1; l = 0; xs0 = xs1 = xk0 = xk1 = 0; qn = 0; qh = 0;
        }
    }
}

void StiIndex::build(const References& refs, const IndexParameters& p, int bits_override, float f, int threads) {
    params = p;
    size_t total = 0;
    for (auto& s : refs.seqs) total += s.size();
    if (bits_override >= 0) bits = bits_override;
    else {   // pick_bits (index.cpp:135-139)
        size_t est = total / (size_t)(p.k - p.s + 1);
        bits = std::clamp((int)std::log2((double)est) - 1, 8, 31);
    }
    // per contig randstrobes (count, then assign), contigs distributed over threads
    std::vector<std::vector<rsa_ref_randstrobe>> per(refs.size());
    std::atomic<size_t> next{0};
    auto worker = [&]() {
        std::vector<Syncmer> sm;
        for (;;) {
            size_t j = next.fetch_add(1);
            if (j >= refs.size()) break;
            const std::string& seq = refs.seqs[j];
            if (seq.size() < p.w_max) continue;
            syncmers_of(seq, p, sm);
            auto& v = per[j];
            const size_t n = sm.size();
            for (size_t i = 0; i + p.w_min < n; ++i) {
                size_t w_end = std::min(i + p.w_max, n - 1);
                uint64_t maxp = (uint64_t)sm[i].pos + (unsigned)p.max_dist, min_val = UINT64_MAX;
                size_t best = i;
                for (size_t x = i + p.w_min; x <= w_end && sm[x].pos <= maxp; ++x) {
                    uint64_t res = (uint64_t)__builtin_popcountll((sm[i].hash ^ sm[x].hash) & (uint64_t)p.q);
                    if (res < min_val) { min_val = res; best = x; }
                }
                uint32_t packed = (uint32_t)(j << 8) + (sm[best].pos - sm[i].pos);
                v.push_back(rsa_ref_randstrobe{sm[i].hash + sm[best].hash, sm[i].pos, packed});
            }
        }
    };
    std::vector<std::thread> ws;
    for (int t = 0; t < std::max(1, threads); ++t) ws.emplace_back(worker);
    for (auto& w : ws) w.join();
    size_t n = 0;
    for (auto& v : per) n += v.size();
    randstrobes.clear();
    randstrobes.reserve(n);
    for (auto& v : per) { randstrobes.insert(randstrobes.end(), v.begin(), v.end()); std::vector<rsa_ref_randstrobe>().swap(v); }
    // RefRandstrobe::operator< orders by (hash, position) (randstrobes.hpp:32-35).
    // A fast parallel sort first; when two contigs hold an entry with equal hash
    // and position, their order is the one pdqsort_branchless's moves leave
    // (index.cpp:168), so the array goes back to generation order and the sort is
    // replayed (sti_order.hpp).
    auto lt = [](const rsa_ref_randstrobe& a, const rsa_ref_randstrobe& b) {
        if (a.hash != b.hash) return a.hash < b.hash;
        return a.position < b.position;
    };
    {   // parallel sort: sort slices, then pairwise merges
        const int T = std::max(1, threads);
        std::vector<size_t> cut(T + 1);
        for (int t = 0; t <= T; ++t) cut[t] = n * (size_t)t / (size_t)T;
        std::vector<std::thread> st;
        for (int t = 0; t < T; ++t)
            st.emplace_back([&, t]() { std::stable_sort(randstrobes.begin() + cut[t], randstrobes.begin() + cut[t + 1], lt); });
        for (auto& x : st) x.join();
        for (int width = 1; width < T; width *= 2) {
            std::vector<std::thread> mt;
            for (int t = 0; t + width < T; t += 2 * width) {
                size_t a = cut[t], m = cut[t + width], b = cut[std::min(T, t + 2 * width)];
                mt.emplace_back([&, a, m, b]() {
                    std::inplace_merge(randstrobes.begin() + a, randstrobes.begin() + m, randstrobes.begin() + b, lt);
                });
            }
            for (auto& x : mt) x.join();
        }
    }
    position_ties = sti_order::count_ties(randstrobes.data(), n, threads);
    if (position_ties) {
        sti_order::to_generation_order(randstrobes.data(), n, threads);
        sti_order::pdqsort_replay(randstrobes.data(), n, threads);
    }
    // bucket table + filter cutoff (index.cpp:174-238)
    bucket_starts.clear();
    bucket_starts.reserve((1ull << bits) + 1);
    uint64_t unique_mers = randstrobes.empty() ? 0 : 1;
    uint64_t prev = randstrobes.empty() ? 0 : randstrobes[0].hash;
    unsigned count = 0;
    std::vector<unsigned> counts;
    for (uint64_t pos = 0; pos < randstrobes.size(); ++pos) {
        const uint64_t h = randstrobes[pos].hash;
        if (h == prev) { ++count; continue; }
        ++unique_mers;
        if (count != 1) counts.push_back(count);
        count = 1;
        const uint64_t top = h >> (64 - bits);
        while (bucket_starts.size() <= top) bucket_starts.push_back(pos);
        prev = h;
    }
    if (count != 1 && !randstrobes.empty()) counts.push_back(count);
    else if (randstrobes.empty()) { /* nothing */ }
    while (bucket_starts.size() < (1ull << bits) + 1) bucket_starts.push_back(randstrobes.size());
    std::sort(counts.begin(), counts.end(), std::greater<int>());
    uint64_t index_cutoff = (uint64_t)(unique_mers * f);
    if (!counts.empty()) {
        unsigned fc = index_cutoff < counts.size() ? counts[index_cutoff] : counts.back();
        fc = std::max(30U, fc);
        fc = std::min(100U, fc);
        filter_cutoff = (int)fc;
    } else {
        filter_cutoff = 30;
    }
}

__attribute__((weak)) void build_default_index(StiIndex& idx, const References& refs, const IndexParameters& p,
                                               int bits_override, float f, int threads, int device, bool host_copy) {
    (void)device;
    (void)host_copy;
    idx.build(refs, p, bits_override, f, threads);
}

// ----------------------------------------------------------------- FASTQ --
struct FastxReader::Impl {
    // block reader: 4 MB gzread()s, lines found with memchr; a line is a view
    // into the buffer, valid until the next refill
    gzFile f = nullptr;
    const char* mem = nullptr;            // memory mode: bytes [mem_pos, mem_len) still to read
    size_t mem_len = 0, mem_pos = 0;
    std::vector<char> buf;
    size_t pos = 0, len = 0;
    bool eof = false;
    int last_char = -1;   // header char of the next record, if already consumed
    bool fill() {
        if (eof) return false;
        if (pos > 0) {
            memmove(buf.data(), buf.data() + pos, len - pos);
            len -= pos;
            pos = 0;
        }
        if (len == buf.size()) buf.resize(buf.size() * 2);
        size_t n = 0;
        if (f) {
            const int r = gzread(f, buf.data() + len, (unsigned)(buf.size() - len));
            n = r > 0 ? (size_t)r : 0;
        } else {
            n = std::min(buf.size() - len, mem_len - mem_pos);
            memcpy(buf.data() + len, mem + mem_pos, n);
            mem_pos += n;
        }
        if (n == 0) { eof = true; return false; }
        len += n;
        return true;
    }
    int getc() {
        if (pos >= len && !fill()) return -1;
        return (unsigned char)buf[pos++];
    }
    // the rest of the current line without its '\n'; false when nothing was left
    bool raw_line(std::string_view& out) {
        size_t from = pos;
        for (;;) {
            const char* e = (const char*)memchr(buf.data() + from, '\n', len - from);
            if (e) {
                const size_t n = (size_t)(e - (buf.data() + pos));
                out = std::string_view(buf.data() + pos, n);
                pos += n + 1;
                return true;
            }
            from = len - pos;                 // offset of the unscanned part after a refill
            if (!fill()) {
                if (pos < len) { out = std::string_view(buf.data() + pos, len - pos); pos = len; return true; }
                return false;
            }
            from += pos;
        }
    }
    // kseq getline: the line with one trailing '\r' removed
    bool getline(std::string_view& out) {
        if (!raw_line(out)) return false;
        if (!out.empty() && out.back() == '\r') out.remove_suffix(1);
        return true;
    }
};

FastxReader::FastxReader(const std::string& path) : impl_(new Impl) {
    impl_->f = gzopen(path == "-" ? "/dev/stdin" : path.c_str(), "r");
    if (!impl_->f) throw std::runtime_error("Could not open FASTQ file: " + path);
    impl_->buf.resize(4 << 20);
    (void)gzbuffer(impl_->f, 1 << 20);
}

FastxReader::FastxReader(const char* mem, size_t len) : impl_(new Impl) {
    impl_->mem = mem;
    impl_->mem_len = len;
    impl_->buf.resize(1 << 20);
}

FastxReader::~FastxReader() { if (impl_->f) gzclose(impl_->f); }

// kseq semantics: '@' or '>' header, name = up to the first whitespace, the
// rest of the header line (after that whitespace) is the comment; sequence
// lines are concatenated until '+' (FASTQ) or the next header (FASTA);
// quality is read until it is as long as the sequence.
bool FastxReader::next(Record& r) {
    Impl& I = *impl_;
    int c = I.last_char;
    if (c == -1) {
        for (;;) {                            // skip to the next '>' or '@' (any byte position)
            if (I.pos >= I.len && !I.fill()) return false;
            const char* s = I.buf.data() + I.pos;
            const size_t n = I.len - I.pos;
            size_t k = 0;
            while (k < n && s[k] != '>' && s[k] != '@') ++k;
            I.pos += k;
            if (k < n) { c = (unsigned char)I.buf[I.pos++]; break; }
        }
    }
    std::string_view line;
    I.getline(line);
    const size_t ws = line.find_first_of(" \t\v\f\r");
    if (ws == std::string_view::npos) { r.name.assign(line); r.comment.clear(); }
    else {
        r.name.assign(line.substr(0, ws));
        const size_t cs = line.find_first_not_of(" \t\v\f\r", ws);
        if (cs == std::string_view::npos) r.comment.clear();
        else r.comment.assign(line.substr(cs));
    }
    r.seq.clear();
    r.qual.clear();
    I.last_char = -1;
    for (;;) {                                // sequence lines
        c = I.getc();
        if (c == -1 || c == '>' || c == '@' || c == '+') break;
        if (c == '\n') continue;
        std::string_view rest;
        I.getline(rest);                      // '\r' stripped from the rest only (kseq reads c first)
        r.seq.push_back((char)c);
        r.seq.append(rest);
        while (!r.seq.empty() && (r.seq.back() == ' ' || r.seq.back() == '\t')) r.seq.pop_back();
    }
    if (c == '>' || c == '@') { I.last_char = c; return true; }
    if (c == -1) return true;
    I.getline(line);                          // rest of the '+' line
    while (r.qual.size() < r.seq.size()) {
        if (!I.getline(line)) break;
        r.qual.append(line);
    }
    if (r.qual.size() != r.seq.size()) throw std::runtime_error("FASTQ quality length differs from sequence length");
    return true;
}

namespace {

// Uncompressed FASTQ in the plain 4-line layout, parsed by several threads over
// byte ranges of the mapped file.  Every record must be header / one sequence
// line / '+' line / one quality line of the same length: then each range can
// find its first record (a line starting with '@' whose next-but-one line
// starts with '+': a quality line starting with '@' is followed two lines
// later by a sequence line) and the records are exactly what next() returns.
// Anything else (gzip, FASTA, wrapped lines, empty lines, length mismatch)
// returns false and the caller reads the file sequentially.
struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    ~Mapped() {
        if (p && n) munmap((void*)p, n);
        if (fd >= 0) close(fd);
    }
};

inline std::string_view strip_cr(std::string_view l) {
    if (!l.empty() && l.back() == '\r') l.remove_suffix(1);
    return l;
}

bool parse_range(const char* b, const char* e, std::vector<Record>& out) {
    auto next_line = [&](const char*& p, std::string_view& l) -> bool {
        if (p >= e) return false;
        const char* q = (const char*)memchr(p, '\n', (size_t)(e - p));
        const char* end = q ? q : e;
        l = std::string_view(p, (size_t)(end - p));
        p = q ? q + 1 : e;
        return true;
    };
    const char* p = b;
    std::string_view h, sq, pl, ql;
    while (p < e) {
        if (*p != '@') return false;
        if (!next_line(p, h) || !next_line(p, sq) || !next_line(p, pl) || !next_line(p, ql)) return false;
        if (pl.empty() || pl[0] != '+') return false;
        Record r;
        h = strip_cr(h.substr(1));
        const size_t ws = h.find_first_of(" \t\v\f\r");
        if (ws == std::string_view::npos) r.name.assign(h);
        else {
            r.name.assign(h.substr(0, ws));
            const size_t cs = h.find_first_not_of(" \t\v\f\r", ws);
            if (cs != std::string_view::npos) r.comment.assign(h.substr(cs));
        }
        // next(): '\r' is stripped from the sequence line after its first byte, then trailing blanks
        if (sq.empty()) return false;
        std::string_view body = sq.substr(1);
        body = strip_cr(body);
        r.seq.reserve(1 + body.size());
        r.seq.push_back(sq[0]);
        r.seq.append(body);
        if (r.seq[0] == '>' || r.seq[0] == '@' || r.seq[0] == '+' || r.seq[0] == '\r') return false;
        while (!r.seq.empty() && (r.seq.back() == ' ' || r.seq.back() == '\t')) r.seq.pop_back();
        r.qual.assign(strip_cr(ql));
        if (r.qual.size() != r.seq.size() || r.seq.empty()) return false;
        out.push_back(std::move(r));
    }
    return true;
}

bool parse_parallel(const std::string& path, int threads, std::vector<Record>& out) {
    if (path == "-" || threads < 2) return false;
    Mapped m;
    m.fd = open(path.c_str(), O_RDONLY);
    if (m.fd < 0) return false;
    struct stat st;
    if (fstat(m.fd, &st) != 0 || st.st_size < (1 << 20)) return false;       // small files: not worth it
    m.n = (size_t)st.st_size;
    // no MAP_POPULATE: the parsing threads fault their own ranges in, in parallel
    // (fault-around maps 64 KB a fault), instead of one thread mapping the whole file
    void* p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
    if (p == MAP_FAILED) { m.n = 0; return false; }
    m.p = (const char*)p;
    if ((unsigned char)m.p[0] == 0x1f && (unsigned char)m.p[1] == 0x8b) return false;   // gzip
    if (m.p[0] != '@') return false;
    const char* end = m.p + m.n;
    // range starts, each moved to the next record header
    std::vector<const char*> cut(threads + 1, end);
    cut[0] = m.p;
    auto line_after = [&](const char* q) -> const char* {
        const char* nl = (const char*)memchr(q, '\n', (size_t)(end - q));
        return nl ? nl + 1 : end;
    };
    for (int t = 1; t < threads; ++t) {
        const char* q = line_after(m.p + m.n * (size_t)t / (size_t)threads);
        while (q < end) {
            if (*q == '@') {
                const char* l2 = line_after(line_after(q));
                if (l2 < end && *l2 == '+') break;
            }
            q = line_after(q);
        }
        cut[t] = std::max(q, cut[t - 1]);
    }
    // records per range estimated from the first record's size (fewer vector regrowths)
    const char* r4 = m.p;
    for (int k = 0; k < 4 && r4 < end; ++k) r4 = line_after(r4);
    const size_t rec_bytes = std::max<size_t>(1, (size_t)(r4 - m.p));
    std::vector<std::vector<Record>> parts(threads);
    std::vector<char> ok(threads, 0);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t]() {
            parts[t].reserve((size_t)(cut[t + 1] - cut[t]) / rec_bytes + 16);
            ok[t] = parse_range(cut[t], cut[t + 1], parts[t]) ? 1 : 0;
        });
    for (auto& t : ts) t.join();
    for (char c : ok) if (!c) return false;
    size_t total = 0;
    for (auto& v : parts) total += v.size();
    out.clear();
    out.reserve(total);
    for (auto& v : parts) for (auto& r : v) out.push_back(std::move(r));
    return true;
}

// the CPUs this process may run on (its affinity mask: a rank's share of the node), at most 16
int reader_threads() {
    cpu_set_t cs;
    int n = 0;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(16, n));
}

}  // namespace

std::vector<Record> FastxReader::read_all(const std::string& path) {
    std::vector<Record> v;
    if (parse_parallel(path, reader_threads(), v)) return v;
    v.clear();
    FastxReader in(path);
    Record r;
    while (in.next(r)) { v.push_back(std::move(r)); r = Record(); }
    return v;
}

void FastxReader::read_pair(const std::string& p1, const std::string& p2, std::vector<Record>& r1,
                            std::vector<Record>& r2) {
    std::exception_ptr err;
    // each file on half of the reader threads (both parses run at once)
    const int half = std::max(1, reader_threads() / 2);
    auto read = [&](const std::string& p) {
        std::vector<Record> v;
        if (parse_parallel(p, half, v)) return v;
        v.clear();
        FastxReader in(p);
        Record r;
        while (in.next(r)) { v.push_back(std::move(r)); r = Record(); }
        return v;
    };
    std::thread t([&]() {
        try { r2 = read(p2); } catch (...) { err = std::current_exception(); }
    });
    try { r1 = read(p1); } catch (...) { t.join(); throw; }
    t.join();
    if (err) std::rethrow_exception(err);
}

}  // namespace rsa

namespace rsa {

}  // namespace rsa

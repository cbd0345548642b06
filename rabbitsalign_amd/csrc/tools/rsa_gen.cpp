// rsa_gen -- synthetic reference / read generator used by the benches and
// tests (spec: SURVEY.md Appendix D).  Deterministic for a given seed.
//
//   rsa_gen ref   <seed> <total_len> <n_contigs> <out.fa> [repeat_frac] [n_runs]
//   rsa_gen reads <seed> <ref.fa> <n_pairs> <L> <mu> <sigma> <out1.fq> <out2.fq> [n_rate]
//   rsa_gen se    <seed> <ref.fa> <n_reads> <L> <out.fq> [n_rate]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

static const char* B = "ACGT";

static std::vector<std::pair<std::string, std::string>> read_fa(const char* fn) {
    std::vector<std::pair<std::string, std::string>> out;
    FILE* f = fopen(fn, "r");
    if (!f) { perror(fn); exit(2); }
    char* line = nullptr;
    size_t cap = 0;
    ssize_t n;
    while ((n = getline(&line, &cap, f)) > 0) {
        while (n > 0 && (line[n - 1] == '\n' || line[n - 1] == '\r')) line[--n] = 0;
        if (line[0] == '>') out.push_back({std::string(line + 1), std::string()});
        else if (!out.empty()) out.back().second.append(line, (size_t)n);
    }
    free(line);
    fclose(f);
    return out;
}

static char comp(char c) {
    switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; default: return 'N'; }
}

static std::string revcomp(const std::string& s) {
    std::string r(s.size(), 'N');
    for (size_t i = 0; i < s.size(); ++i) r[i] = comp(s[s.size() - 1 - i]);
    return r;
}

struct Mutator {
    std::mt19937_64& rng;
    std::uniform_real_distribution<double> U{0.0, 1.0};
    double n_rate;
    std::string operator()(const std::string& s, size_t L) {
        std::string o;
        o.reserve(L + 8);
        for (char c : s) {
            double u = U(rng);
            if (u < 0.01) {
                char d;
                do { d = B[rng() & 3]; } while (d == c);
                o += d;
            } else if (u < 0.0115) {
                /* deletion */
            } else if (u < 0.013) {
                o += c;
                o += B[rng() & 3];
            } else {
                o += c;
            }
        }
        o.resize(L, 'A');
        if (n_rate > 0)
            for (auto& c : o) if (U(rng) < n_rate) c = 'N';
        return o;
    }
};

static int cmd_ref(int argc, char** argv) {
    if (argc < 6) return 2;
    std::mt19937_64 rng(strtoull(argv[2], nullptr, 10));
    uint64_t total = strtoull(argv[3], nullptr, 10);
    int nc = atoi(argv[4]);
    double repeat_frac = argc > 6 ? atof(argv[6]) : 0.0;
    int n_runs = argc > 7 ? atoi(argv[7]) : 0;
    std::string all(total, 'A');
    for (auto& c : all) c = B[rng() & 3];
    // optional repeats: copy random 300-3000 bp segments elsewhere (tests multi-mapping paths)
    uint64_t copied = 0;
    while (repeat_frac > 0 && copied < (uint64_t)(repeat_frac * (double)total)) {
        uint64_t len = 300 + rng() % 2700;
        if (len * 2 >= total) break;
        uint64_t a = rng() % (total - len), b = rng() % (total - len);
        all.replace(b, len, all, a, len);
        copied += len;
    }
    for (int r = 0; r < n_runs; ++r) {  // runs of N
        uint64_t len = 1 + rng() % 200, a = rng() % (total - len);
        for (uint64_t i = 0; i < len; ++i) all[a + i] = 'N';
    }
    FILE* f = fopen(argv[5], "w");
    uint64_t per = total / (uint64_t)nc;
    for (int c = 0; c < nc; ++c) {
        uint64_t a = per * (uint64_t)c, b = c == nc - 1 ? total : a + per;
        fprintf(f, ">chr%d\n", c + 1);
        for (uint64_t i = a; i < b; i += 80) {
            uint64_t e = i + 80 < b ? i + 80 : b;
            fwrite(all.data() + i, 1, e - i, f);
            fputc('\n', f);
        }
    }
    fclose(f);
    return 0;
}

static void write_fq(FILE* f, const std::string& name, const std::string& s) {
    fprintf(f, "@%s\n%s\n+\n", name.c_str(), s.c_str());
    std::string q(s.size(), 'I');
    fprintf(f, "%s\n", q.c_str());
}

static int cmd_reads(int argc, char** argv) {
    if (argc < 10) return 2;
    std::mt19937_64 rng(strtoull(argv[2], nullptr, 10));
    auto refs = read_fa(argv[3]);
    long n_pairs = atol(argv[4]);
    int L = atoi(argv[5]);
    double mu = atof(argv[6]), sigma = atof(argv[7]);
    double n_rate = argc > 10 ? atof(argv[10]) : 0.0;
    FILE* f1 = fopen(argv[8], "w");
    FILE* f2 = fopen(argv[9], "w");
    std::normal_distribution<double> N(mu, sigma);
    Mutator mut{rng, {}, n_rate};
    for (long p = 0; p < n_pairs; ++p) {
        int ins = (int)std::floor(N(rng));
        if (ins < L + 10) ins = L + 10;
        const auto& ref = refs[rng() % refs.size()].second;
        if ((long)ref.size() <= ins) continue;
        uint64_t start = rng() % (ref.size() - (size_t)ins);
        std::string frag = ref.substr(start, (size_t)ins);
        for (auto& c : frag) c = (char)toupper(c);
        std::string a = mut(frag.substr(0, (size_t)L + 5), (size_t)L);
        std::string b = mut(revcomp(frag).substr(0, (size_t)L + 5), (size_t)L);
        if (rng() & 1) std::swap(a, b);
        std::string nm = "r" + std::to_string(p);
        write_fq(f1, nm + "/1", a);
        write_fq(f2, nm + "/2", b);
    }
    fclose(f1);
    fclose(f2);
    return 0;
}

static int cmd_se(int argc, char** argv) {
    if (argc < 7) return 2;
    std::mt19937_64 rng(strtoull(argv[2], nullptr, 10));
    auto refs = read_fa(argv[3]);
    long n = atol(argv[4]);
    int L = atoi(argv[5]);
    double n_rate = argc > 7 ? atof(argv[7]) : 0.0;
    FILE* f = fopen(argv[6], "w");
    Mutator mut{rng, {}, n_rate};
    for (long p = 0; p < n; ++p) {
        const auto& ref = refs[rng() % refs.size()].second;
        if ((long)ref.size() <= L + 5) continue;
        uint64_t start = rng() % (ref.size() - (size_t)L - 5);
        std::string frag = ref.substr(start, (size_t)L + 5);
        if (rng() & 1) frag = revcomp(frag);
        write_fq(f, "r" + std::to_string(p), mut(frag, (size_t)L));
    }
    fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "rsa_gen ref|reads|se ...\n"); return 2; }
    int rc = 2;
    if (!strcmp(argv[1], "ref")) rc = cmd_ref(argc, argv);
    else if (!strcmp(argv[1], "reads")) rc = cmd_reads(argc, argv);
    else if (!strcmp(argv[1], "se")) rc = cmd_se(argc, argv);
    if (rc == 2) fprintf(stderr, "bad arguments\n");
    return rc;
}

// synth.hpp -- deterministic synthetic reference and reads:
// i.i.d. uniform ACGT reference cut into equal contigs chr1..chrN; pairs with
// insert ~ N(mu, sigma) (>= L+10), mate 1 = fragment prefix, mate 2 = prefix of
// the reverse-complemented fragment, swapped with p = 0.5; per base 1.0%
// substitution, 0.15% deletion, 0.15% insertion; truncated/padded to L; qual 'I'.
#pragma once
#include <cmath>
#include <cstdint>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace rsa {
namespace synth {

inline std::vector<std::string> reference(uint64_t seed, uint64_t total, int n_contigs, int threads = 8) {
    // generated in independent 1 Mb blocks (one mt19937_64 stream per block) so it parallelises
    const uint64_t BLK = 1 << 20;
    std::string all(total, 'A');
    const uint64_t nb = (total + BLK - 1) / BLK;
    auto work = [&](int t) {
        for (uint64_t b = (uint64_t)t; b < nb; b += (uint64_t)threads) {
            std::mt19937_64 rng(seed * 1000003ULL + b);
            const uint64_t e = std::min(total, (b + 1) * BLK);
            for (uint64_t i = b * BLK; i < e; i += 32) {
                uint64_t x = rng();
                for (uint64_t j = i; j < std::min(e, i + 32); ++j, x >>= 2) all[j] = "ACGT"[x & 3];
            }
        }
    };
    std::vector<std::thread> ws;
    for (int t = 0; t < threads; ++t) ws.emplace_back(work, t);
    for (auto& w : ws) w.join();
    std::vector<std::string> contigs;
    const uint64_t per = total / (uint64_t)n_contigs;
    for (int c = 0; c < n_contigs; ++c) {
        const uint64_t a = per * (uint64_t)c, b = c == n_contigs - 1 ? total : a + per;
        contigs.push_back(all.substr(a, b - a));
    }
    return contigs;
}

inline char comp(char c) {
    switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; default: return 'N'; }
}

inline std::string revcomp(const std::string& s) {
    std::string r(s.size(), 'N');
    for (size_t i = 0; i < s.size(); ++i) r[i] = comp(s[s.size() - 1 - i]);
    return r;
}

inline std::string mutate(std::mt19937_64& rng, const std::string& s, size_t L, double n_rate = 0.0) {
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::string o;
    o.reserve(L + 8);
    for (char c : s) {
        double u = U(rng);
        if (u < 0.01) {
            char d;
            do { d = "ACGT"[rng() & 3]; } while (d == c);
            o += d;
        } else if (u < 0.0115) {
        } else if (u < 0.013) {
            o += c;
            o += "ACGT"[rng() & 3];
        } else {
            o += c;
        }
    }
    o.resize(L, 'A');
    if (n_rate > 0)
        for (auto& c : o) if (U(rng) < n_rate) c = 'N';
    return o;
}

struct Pair { std::string a, b; };

// pair p is generated from its own stream (seed, p) so any subset can be regenerated
inline Pair pair(const std::vector<std::string>& contigs, uint64_t seed, uint64_t p, int L, double mu, double sigma,
                 double n_rate = 0.0) {
    std::mt19937_64 rng(seed * 0x9E3779B97F4A7C15ULL + p);
    std::normal_distribution<double> N(mu, sigma);
    for (;;) {
        int ins = (int)std::floor(N(rng));
        if (ins < L + 10) ins = L + 10;
        const std::string& ref = contigs[rng() % contigs.size()];
        if ((long)ref.size() <= ins) continue;
        uint64_t start = rng() % (ref.size() - (size_t)ins);
        std::string frag = ref.substr(start, (size_t)ins);
        Pair pr;
        pr.a = mutate(rng, frag.substr(0, (size_t)L + 5), (size_t)L, n_rate);
        pr.b = mutate(rng, revcomp(frag).substr(0, (size_t)L + 5), (size_t)L, n_rate);
        if (rng() & 1) std::swap(pr.a, pr.b);
        return pr;
    }
}

}  // namespace synth
}  // namespace rsa

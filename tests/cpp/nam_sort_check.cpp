// load_sorted_nams (csrc/host/aln.cpp) must give the permutation libstdc++'s
// std::sort(by_score) gives (src/aln.cpp sorts a read's NAMs that way; equal
// scores keep whatever order the introsort/insertion sort leaves them in).
#include <algorithm>
#include <cstdio>
#include <random>

#include "rsa_host.hpp"

using namespace rsa;

int main() {
    std::mt19937 g(1);
    long bad = 0;
    for (int it = 0; it < 200000; ++it) {
        const int n = (int)(g() % 41);
        std::vector<Nam> src(n);
        for (int i = 0; i < n; ++i) {
            src[i] = Nam{};
            src[i].nam_id = i;
            src[i].score = (float)(g() % 5);          // many ties
        }
        std::vector<Nam> a(src), b;
        std::sort(a.begin(), a.end(), [](const Nam& x, const Nam& y) { return x.score > y.score; });
        load_sorted_nams(b, src.data(), (size_t)n);
        for (int i = 0; i < n; ++i)
            if (a[i].nam_id != b[i].nam_id) { bad++; break; }
    }
    printf("mismatching lists: %ld\n", bad);
    return bad != 0;
}

// sti_order.hpp -- the .sti entry order exactly as the reference writes it.
//
// StrobemerIndex::populate sorts the RefRandstrobe array with
// pdqsort_branchless (src/index.cpp:168; ext/pdqsort, Orson Peters' pattern-
// defeating quicksort, commit b1ef26a per ext/README.md) under
// RefRandstrobe::operator< (src/randstrobes.hpp:32-35), which compares
// (hash, position) only.  Entries with equal hash and position in two contigs
// (duplicated sequence, e.g. the PAR regions of chrX/chrY) compare equal, and
// an unstable sort leaves them in whatever order its element moves produce.
// To write the reference's bytes we replay those moves: the routines below
// restate pdqsort_branchless step by step (insertion-sort threshold 24, Tukey
// ninther above 128 elements, median-of-3 below, block partitioning with 64-
// entry offset blocks, partition-left for runs equal to the previous pivot,
// the pattern-breaking swaps after an unbalanced split, heapsort after
// floor(log2 n) of them, the partial insertion sort after a split that found
// the range already partitioned).
//
// The recursion's two halves touch disjoint ranges and read only finished
// pivots outside them, so the left halves of large ranges run as tasks on a
// thread pool: the element moves -- and so the result -- are the same as one
// thread's.  Callers take this path only when ties exist (a fast sort + an
// adjacent-equal scan decides); the input must be the reference's generation
// order: contigs in order, each contig's randstrobes by strobe-1 position
// (index.cpp:244-303), which is (ref_id, position) order since one randstrobe
// starts at each syncmer.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "../../../include/rsa_gpu.h"

namespace rsa {
namespace sti_order {

using Entry = rsa_ref_randstrobe;

// RefRandstrobe::operator< (randstrobes.hpp:32-35)
inline bool key_lt(const Entry& a, const Entry& b) {
    return a.hash != b.hash ? a.hash < b.hash : a.position < b.position;
}

// equal (hash, position) neighbours in a sorted array: the entries whose order
// the sort leaves open
inline uint64_t count_ties(const Entry* a, size_t n, int threads) {
    if (n < 2) return 0;
    const int T = std::max(1, std::min<int>(threads, (int)(n >> 16) + 1));
    std::vector<uint64_t> part((size_t)T, 0);
    std::vector<std::thread> ws;
    for (int t = 0; t < T; ++t)
        ws.emplace_back([&, t] {
            const size_t b = 1 + (n - 1) * (size_t)t / (size_t)T, e = 1 + (n - 1) * (size_t)(t + 1) / (size_t)T;
            uint64_t c = 0;
            for (size_t i = b; i < e; ++i) c += a[i].hash == a[i - 1].hash && a[i].position == a[i - 1].position;
            part[(size_t)t] = c;
        });
    for (auto& w : ws) w.join();
    uint64_t s = 0;
    for (uint64_t c : part) s += c;
    return s;
}

class PdqReplay {
public:
    PdqReplay(Entry* base, int threads) : p_(base), threads_(std::max(1, threads)) {}

    void sort(size_t n) {
        if (n == 0) return;
        int budget = 0;                              // floor(log2 n) unbalanced splits
        for (size_t m = n; m >>= 1;) ++budget;
        if (threads_ == 1 || n < kTaskMin) {
            run(0, n, budget, true);
            return;
        }
        push(Task{0, n, budget, true});
        std::vector<std::thread> ws;
        for (int t = 0; t < threads_; ++t) ws.emplace_back([this] { drain(); });
        for (auto& w : ws) w.join();
    }

private:
    static constexpr ptrdiff_t kSmall = 24;          // insertion_sort_threshold
    static constexpr ptrdiff_t kNinther = 128;       // ninther_threshold
    static constexpr size_t kPartialLimit = 8;       // partial_insertion_sort_limit
    static constexpr int kBlock = 64;                // block_size
    static constexpr size_t kTaskMin = 1u << 15;     // left halves at least this long become tasks

    struct Task {
        size_t begin, end;
        int budget;
        bool leftmost;
    };

    Entry* p_;
    int threads_;
    std::mutex m_;
    std::condition_variable cv_;
    std::vector<Task> stack_;
    size_t open_ = 0;                                // tasks pushed and not finished

    void push(Task t) {
        {
            std::lock_guard<std::mutex> g(m_);
            stack_.push_back(t);
            ++open_;
        }
        cv_.notify_one();
    }
    void drain() {
        for (;;) {
            Task t;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return !stack_.empty() || open_ == 0; });
                if (stack_.empty()) return;
                t = stack_.back();
                stack_.pop_back();
            }
            run(t.begin, t.end, t.budget, t.leftmost);
            std::lock_guard<std::mutex> g(m_);
            if (--open_ == 0) cv_.notify_all();
        }
    }

    void swap_at(size_t i, size_t j) { std::swap(p_[i], p_[j]); }
    void order2(size_t i, size_t j) {
        if (key_lt(p_[j], p_[i])) swap_at(i, j);
    }
    void order3(size_t i, size_t j, size_t k) {
        order2(i, j);
        order2(j, k);
        order2(i, j);
    }

    // insertion sort of [b, e); `guarded` false: p_[b - 1] bounds the sift from below
    void insert_sort(size_t b, size_t e, bool guarded) {
        if (b == e) return;
        for (size_t cur = b + 1; cur != e; ++cur) {
            if (!key_lt(p_[cur], p_[cur - 1])) continue;
            const Entry v = p_[cur];
            size_t hole = cur;
            do {
                p_[hole] = p_[hole - 1];
                --hole;
            } while ((!guarded || hole != b) && key_lt(v, p_[hole - 1]));
            p_[hole] = v;
        }
    }
    // the insertion sort that gives up after more than kPartialLimit moved positions
    bool insert_sort_bounded(size_t b, size_t e) {
        if (b == e) return true;
        size_t moved = 0;
        for (size_t cur = b + 1; cur != e; ++cur) {
            if (key_lt(p_[cur], p_[cur - 1])) {
                const Entry v = p_[cur];
                size_t hole = cur;
                do {
                    p_[hole] = p_[hole - 1];
                    --hole;
                } while (hole != b && key_lt(v, p_[hole - 1]));
                p_[hole] = v;
                moved += cur - hole;
            }
            if (moved > kPartialLimit) return false;
        }
        return true;
    }

    // the misplaced pairs (left offsets from lbase, right offsets back from rbase)
    // exchanged: pairwise swaps when both blocks hold the same count, else one cycle
    void exchange(size_t lbase, size_t rbase, const unsigned char* lo, const unsigned char* ro, size_t cnt,
                  bool pairwise) {
        if (pairwise) {
            for (size_t i = 0; i < cnt; ++i) swap_at(lbase + lo[i], rbase - ro[i]);
            return;
        }
        if (cnt == 0) return;
        size_t l = lbase + lo[0], r = rbase - ro[0];
        const Entry first = p_[l];
        p_[l] = p_[r];
        for (size_t i = 1; i < cnt; ++i) {
            l = lbase + lo[i];
            p_[r] = p_[l];
            r = rbase - ro[i];
            p_[l] = p_[r];
        }
        p_[r] = first;
    }

    // p_[b] is the pivot; smaller keys end left of it, the others right.  Returns
    // the pivot's final index and whether no pair had to move.
    std::pair<size_t, bool> split_right(size_t b, size_t e) {
        const Entry piv = p_[b];
        size_t lo = b, hi = e;
        while (key_lt(p_[++lo], piv)) {}
        if (lo - 1 == b) {
            while (lo < hi && !key_lt(p_[--hi], piv)) {}
        } else {
            while (!key_lt(p_[--hi], piv)) {}
        }
        const bool clean = lo >= hi;
        if (!clean) {
            swap_at(lo, hi);
            ++lo;
            unsigned char left_off[kBlock], right_off[kBlock];
            size_t lbase = lo, rbase = hi;
            size_t nl = 0, nr = 0, sl = 0, sr = 0;
            while (lo < hi) {
                const size_t unknown = hi - lo;
                const size_t take_l = nl == 0 ? (nr == 0 ? unknown / 2 : unknown) : 0;
                const size_t take_r = nr == 0 ? unknown - take_l : 0;
                const size_t cl = take_l >= (size_t)kBlock ? (size_t)kBlock : take_l;
                for (size_t i = 0; i < cl; ++i) {
                    left_off[nl] = (unsigned char)i;
                    nl += !key_lt(p_[lo], piv);
                    ++lo;
                }
                const size_t cr = take_r >= (size_t)kBlock ? (size_t)kBlock : take_r;
                for (size_t i = 0; i < cr; ++i) {
                    right_off[nr] = (unsigned char)(i + 1);
                    nr += key_lt(p_[--hi], piv);
                }
                const size_t cnt = std::min(nl, nr);
                exchange(lbase, rbase, left_off + sl, right_off + sr, cnt, nl == nr);
                nl -= cnt;
                nr -= cnt;
                sl += cnt;
                sr += cnt;
                if (nl == 0) {
                    sl = 0;
                    lbase = lo;
                }
                if (nr == 0) {
                    sr = 0;
                    rbase = hi;
                }
            }
            if (nl) {
                const unsigned char* o = left_off + sl;
                while (nl--) swap_at(lbase + o[nl], --hi);
                lo = hi;
            }
            if (nr) {
                const unsigned char* o = right_off + sr;
                while (nr--) {
                    swap_at(rbase - o[nr], lo);
                    ++lo;
                }
                hi = lo;
            }
        }
        const size_t at = lo - 1;
        p_[b] = p_[at];
        p_[at] = piv;
        return {at, clean};
    }

    // keys equal to the pivot p_[b] end left of it (a run of keys equal to the
    // previous pivot); returns the pivot's final index
    size_t split_left(size_t b, size_t e) {
        const Entry piv = p_[b];
        size_t lo = b, hi = e;
        while (key_lt(piv, p_[--hi])) {}
        if (hi + 1 == e) {
            while (lo < hi && !key_lt(piv, p_[++lo])) {}
        } else {
            while (!key_lt(piv, p_[++lo])) {}
        }
        while (lo < hi) {
            swap_at(lo, hi);
            while (key_lt(piv, p_[--hi])) {}
            while (!key_lt(piv, p_[++lo])) {}
        }
        p_[b] = p_[hi];
        p_[hi] = piv;
        return hi;
    }

    void run(size_t b, size_t e, int budget, bool leftmost) {
        for (;;) {
            const ptrdiff_t size = (ptrdiff_t)(e - b);
            if (size < kSmall) {
                insert_sort(b, e, leftmost);
                return;
            }
            const size_t h = (size_t)(size / 2);
            if (size > kNinther) {
                order3(b, b + h, e - 1);
                order3(b + 1, b + (h - 1), e - 2);
                order3(b + 2, b + (h + 1), e - 3);
                order3(b + (h - 1), b + h, b + (h + 1));
                swap_at(b, b + h);
            } else {
                order3(b + h, b, e - 1);
            }
            if (!leftmost && !key_lt(p_[b - 1], p_[b])) {
                b = split_left(b, e) + 1;
                continue;
            }
            const std::pair<size_t, bool> sp = split_right(b, e);
            const size_t piv = sp.first;
            const ptrdiff_t ls = (ptrdiff_t)(piv - b), rs = (ptrdiff_t)(e - (piv + 1));
            if (ls < size / 8 || rs < size / 8) {
                if (--budget == 0) {
                    std::make_heap(p_ + b, p_ + e, key_lt);
                    std::sort_heap(p_ + b, p_ + e, key_lt);
                    return;
                }
                if (ls >= kSmall) {
                    const size_t q = (size_t)(ls / 4);
                    swap_at(b, b + q);
                    swap_at(piv - 1, piv - q);
                    if (ls > kNinther) {
                        swap_at(b + 1, b + (q + 1));
                        swap_at(b + 2, b + (q + 2));
                        swap_at(piv - 2, piv - (q + 1));
                        swap_at(piv - 3, piv - (q + 2));
                    }
                }
                if (rs >= kSmall) {
                    const size_t q = (size_t)(rs / 4);
                    swap_at(piv + 1, piv + (1 + q));
                    swap_at(e - 1, e - q);
                    if (rs > kNinther) {
                        swap_at(piv + 2, piv + (2 + q));
                        swap_at(piv + 3, piv + (3 + q));
                        swap_at(e - 2, e - (1 + q));
                        swap_at(e - 3, e - (2 + q));
                    }
                }
            } else if (sp.second && insert_sort_bounded(b, piv) && insert_sort_bounded(piv + 1, e)) {
                return;
            }
            // the left part (recursion in the reference), then the right part in this loop
            if (threads_ > 1 && piv - b >= kTaskMin) push(Task{b, piv, budget, leftmost});
            else run(b, piv, budget, leftmost);
            b = piv + 1;
            leftmost = false;
        }
    }
};

// The reference's order of a/n, given in generation order (see above).
inline void pdqsort_replay(Entry* a, size_t n, int threads) { PdqReplay(a, threads).sort(n); }

// Generation order back from any (hash, position)-sorted array: (ref_id, position)
// is unique per entry, so this is a permutation with one answer.
inline void to_generation_order(Entry* a, size_t n, int threads) {
    auto gen_lt = [](const Entry& x, const Entry& y) {
        const uint32_t cx = x.packed >> 8, cy = y.packed >> 8;
        return cx != cy ? cx < cy : x.position < y.position;
    };
    const int T = std::max(1, std::min<int>(threads, (int)(n >> 16) + 1));
    std::vector<size_t> cut((size_t)T + 1);
    for (int t = 0; t <= T; ++t) cut[(size_t)t] = n * (size_t)t / (size_t)T;
    std::vector<std::thread> ws;
    for (int t = 0; t < T; ++t) ws.emplace_back([&, t] { std::sort(a + cut[t], a + cut[t + 1], gen_lt); });
    for (auto& w : ws) w.join();
    for (int width = 1; width < T; width *= 2) {
        std::vector<std::thread> ms;
        for (int t = 0; t + width < T; t += 2 * width) {
            const size_t x = cut[t], y = cut[t + width], z = cut[std::min(T, t + 2 * width)];
            ms.emplace_back([=] { std::inplace_merge(a + x, a + y, a + z, gen_lt); });
        }
        for (auto& w : ms) w.join();
    }
}

}  // namespace sti_order
}  // namespace rsa

// Page-cache bandwidth of one SAM-sized file (740 MB in 3.7 MB chunks, the bench's
// step), written the ways a SAM sink can write it (profiling tool, no GPU):
//   write  : one thread, write() of each chunk in order (the OrderedSink writer)
//   mmapT  : ftruncate to the total, MAP_SHARED mapping, T threads each copying
//            every T-th chunk to its offset (each worker copying its own chunk)
//   mmapPT : the same with MADV_POPULATE_WRITE of each chunk's range before the copy
//   mmapFT : fallocate of the whole file first (blocks allocated up front), then as mmapPT
//   cold   : write() of 200 distinct chunks filled beforehand (source out of cache, as the
//            writer thread finds the chunks other workers formatted)
//   coldB  : the same while B background threads copy memory (a busy host)
//   --direct: T threads pwrite() 8 MiB blocks at disjoint offsets of one file, with O_DIRECT
//            (aligned source blocks, no page cache, no inode lock held across the copy) and
//            buffered (for comparison); the file is fsync'ed in neither mode's timing
// Build: g++ -O2 -pthread sam_sink_bw.cpp -o /tmp/sam_sink_bw ; run: sam_sink_bw DIR...
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static const size_t kChunk = 3700000, kN = 200, kTotal = kChunk * kN;

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double by_write(const std::string& path, const std::vector<char>& buf) {
    int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    const double t = now();
    for (size_t i = 0; i < kN; ++i) {
        size_t off = 0;
        while (off < kChunk) {
            ssize_t w = write(fd, buf.data() + off, kChunk - off);
            if (w <= 0) { perror("write"); return 0; }
            off += (size_t)w;
        }
    }
    const double dt = now() - t;
    close(fd);
    unlink(path.c_str());
    return kTotal / dt / 1e9;
}

static double by_mmap(const std::string& path, const std::vector<char>& buf, int threads, bool populate,
                      bool falloc = false) {
    int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
    const double t = now();
    if (falloc && fallocate(fd, 0, 0, (off_t)kTotal) != 0) { perror("fallocate"); return 0; }
    if (ftruncate(fd, (off_t)kTotal) != 0) { perror("ftruncate"); return 0; }
    char* m = (char*)mmap(nullptr, kTotal, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { perror("mmap"); return 0; }
    std::vector<std::thread> ws;
    for (int w = 0; w < threads; ++w)
        ws.emplace_back([&, w] {
            for (size_t i = (size_t)w; i < kN; i += (size_t)threads) {
                char* dst = m + i * kChunk;
                if (populate) {
                    const uintptr_t a = (uintptr_t)dst & ~(uintptr_t)4095;
                    madvise((void*)a, ((uintptr_t)dst + kChunk) - a, MADV_POPULATE_WRITE);
                }
                memcpy(dst, buf.data(), kChunk);
            }
        });
    for (auto& x : ws) x.join();
    munmap(m, kTotal);
    const double dt = now() - t;
    close(fd);
    unlink(path.c_str());
    return kTotal / dt / 1e9;
}

static double by_write_cold(const std::string& path, const std::vector<std::vector<char>>& bufs, int bg) {
    volatile bool stop = false;
    std::vector<std::thread> ts;
    for (int b = 0; b < bg; ++b)
        ts.emplace_back([&] {
            std::vector<char> x(64 << 20), y(64 << 20);
            while (!stop) memcpy(y.data(), x.data(), x.size());
        });
    if (bg) usleep(100000);
    int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    const double t = now();
    for (size_t i = 0; i < kN; ++i) {
        size_t off = 0;
        while (off < kChunk) {
            ssize_t w = write(fd, bufs[i].data() + off, kChunk - off);
            if (w <= 0) { perror("write"); return 0; }
            off += (size_t)w;
        }
    }
    const double dt = now() - t;
    stop = true;
    for (auto& x : ts) x.join();
    close(fd);
    unlink(path.c_str());
    return kTotal / dt / 1e9;
}

static double by_pwrite(const std::string& path, int threads, bool direct, size_t blk, size_t nblk, char* src) {
    int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | (direct ? O_DIRECT : 0), 0644);
    if (fd < 0) { perror("open"); return 0; }
    const double t = now();
    std::vector<std::thread> ws;
    std::vector<int> bad(threads, 0);
    for (int w = 0; w < threads; ++w)
        ws.emplace_back([&, w] {
            for (size_t i = (size_t)w; i < nblk; i += (size_t)threads) {
                size_t off = 0;
                while (off < blk) {
                    ssize_t r = pwrite(fd, src + (i % 16) * blk + off, blk - off, (off_t)(i * blk + off));
                    if (r <= 0) { bad[w] = 1; return; }
                    off += (size_t)r;
                }
            }
        });
    for (auto& x : ws) x.join();
    const double dt = now() - t;
    close(fd);
    unlink(path.c_str());
    for (int b : bad) if (b) { perror("pwrite"); return 0; }
    return (double)blk * nblk / dt / 1e9;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "--direct") {
        const size_t blk = 8u << 20, nblk = 96;   // 768 MiB, the size of a bench step's SAM
        char* src = nullptr;
        if (posix_memalign((void**)&src, 4096, 16 * blk) != 0) return 1;
        for (size_t i = 0; i < 16 * blk; ++i) src[i] = (char)('A' + (i * 7919) % 26);
        for (int a = 2; a < argc; ++a) {
            const std::string p = std::string(argv[a]) + "/ssbw_" + std::to_string(getpid());
            for (int rep = 0; rep < 2; ++rep) {
                printf("%s:", argv[a]);
                for (int t : {1, 2, 4, 8, 16}) printf(" direct%d %.2f", t, by_pwrite(p, t, true, blk, nblk, src));
                for (int t : {1, 4, 16}) printf(" buffered%d %.2f", t, by_pwrite(p, t, false, blk, nblk, src));
                printf(" GB/s\n");
                fflush(stdout);
            }
        }
        free(src);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "--cold") {
        std::vector<std::vector<char>> bufs(kN, std::vector<char>(kChunk));
        for (auto& b : bufs) for (size_t i = 0; i < kChunk; i += 64) b[i] = 'A';
        for (int a = 2; a < argc; ++a) {
            const std::string p = std::string(argv[a]) + "/ssbw_" + std::to_string(getpid());
            for (int rep = 0; rep < 2; ++rep) {
                printf("%s: cold %.2f", argv[a], by_write_cold(p, bufs, 0));
                for (int bg : {4, 8, 14}) printf(", cold+%d %.2f", bg, by_write_cold(p, bufs, bg));
                printf(" GB/s\n");
                fflush(stdout);
            }
        }
        return 0;
    }
    std::vector<char> buf(kChunk);
    for (size_t i = 0; i < kChunk; ++i) buf[i] = (char)('A' + (i * 7919) % 26);
    for (int a = 1; a < argc; ++a) {
        struct statfs sf;
        statfs(argv[a], &sf);
        const std::string p = std::string(argv[a]) + "/ssbw_" + std::to_string(getpid());
        for (int rep = 0; rep < 2; ++rep) {
            printf("%s (fs magic 0x%lx): write %.2f GB/s", argv[a], (unsigned long)sf.f_type, by_write(p, buf));
            for (int t : {1, 4, 8, 16}) printf(", mmap%d %.2f", t, by_mmap(p, buf, t, false));
            for (int t : {4, 8, 16}) printf(", mmapP%d %.2f", t, by_mmap(p, buf, t, true));
            for (int t : {4, 8, 16}) printf(", mmapF%d %.2f", t, by_mmap(p, buf, t, true, true));
            printf(" GB/s\n");
            fflush(stdout);
        }
    }
    return 0;
}

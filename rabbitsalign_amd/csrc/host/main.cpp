// main.cpp -- `rsalign`, the drop-in command line of the MI355X path.
// Options follow the reference's CLI (src/cmdline.cpp:9-158, src/arguments.hpp):
//   rsalign [options] <ref.fa> <reads1.fq[.gz]> [reads2.fq[.gz]]
// -t --chunk-size -o -v --eqx -U --rg-id --rg --details -N -i/--create-index
// --use-index -r -m -k -l -u -s -c -b -A -B -O -E -L -f -S -M -R, plus
// --device (GPU ordinal) and `rsalign index -r N -o out.sti ref.fa`.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <stdexcept>

#include "rsa_host.hpp"

namespace rsa {

namespace {

struct Opts {
    int threads = 3, chunk_size = 10000, device = 0, max_secondary = 0;
    int rank = 0, world = 1;           // --rank / --world: this process maps one part of the input
    std::string out_file, rg_id, ref, reads1, reads2, devices;
    std::vector<std::string> rg;
    bool verbose = false, eqx = false, no_unmapped = false, details = false, create_index = false,
         use_index = false, interleaved = false, cpu_index = false;
    int r = 150, m = INT32_MIN, k = INT32_MIN, l = INT32_MIN, u = INT32_MIN, s = INT32_MIN, c = INT32_MIN, bits = -1;
    bool r_set = false;
    int A = 2, B = 8, O = 12, E = 1, L = 10;
    float f = 0.0002f, S = 0.5f;
    int M = 20, R = 2;
    std::string index_out;
};

void usage(const char* prog) {
    fprintf(stderr,
            "usage: %s [options] <ref.fa> <reads1> [reads2]\n"
            "       %s index [-r INT] [-o out.sti] [-t INT] [-b INT] <ref.fa>\n"
            "  -t INT threads [3]   --chunk-size INT [10000]   -o PATH   --eqx   -U   --details\n"
            "  --rg-id ID  --rg TAG:VALUE   -N INT   -i/--create-index   --use-index   --device INT   --cpu-index\n"
            "  --devices LIST  map on several GPUs of this node (e.g. 0,1,2,3; index replicated per device)\n"
            "  --rank R --world W  map part R of W of the input (FASTQ, plain or gzip); the SAM parts of\n"
            "                      ranks 0..W-1 concatenated are the one-process SAM (rank 0's has the header;\n"
            "                      its @PG command line is the run's own, e.g. its -o)\n"
            "  seeding: -r -m -k -l -u -s -c -b      alignment: -A -B -O -E -L\n"
            "  search: -f FLOAT -S FLOAT -M INT -R INT\n",
            prog, prog);
}

Opts parse(int argc, char** argv, bool& ok) {
    Opts o;
    ok = true;
    std::vector<std::string> pos;
    auto need = [&](int& i) -> const char* {
        if (i + 1 >= argc) { fprintf(stderr, "option %s needs a value\n", argv[i]); ok = false; return "0"; }
        return argv[++i];
    };
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "-t" || a == "--threads") o.threads = atoi(need(i));
        else if (a == "--chunk-size") o.chunk_size = atoi(need(i));
        else if (a == "-o") o.out_file = need(i);
        else if (a == "-v") o.verbose = true;
        else if (a == "--no-progress") {}
        else if (a == "--eqx") o.eqx = true;
        else if (a == "-U") o.no_unmapped = true;
        else if (a == "--interleaved") o.interleaved = true;
        else if (a == "--rg-id") o.rg_id = need(i);
        else if (a == "--rg") o.rg.push_back(need(i));
        else if (a == "--details") o.details = true;
        else if (a == "-N") o.max_secondary = atoi(need(i));
        else if (a == "--index-statistics") (void)need(i);
        else if (a == "-i" || a == "--create-index") o.create_index = true;
        else if (a == "--use-index") o.use_index = true;
        else if (a == "--cpu-index") o.cpu_index = true;
        else if (a == "--device") o.device = atoi(need(i));
        else if (a == "--devices") o.devices = need(i);
        else if (a == "--rank") o.rank = atoi(need(i));
        else if (a == "--world") o.world = atoi(need(i));
        else if (a == "-r") { o.r = atoi(need(i)); o.r_set = true; }
        else if (a == "-m") o.m = atoi(need(i));
        else if (a == "-k") o.k = atoi(need(i));
        else if (a == "-l") o.l = atoi(need(i));
        else if (a == "-u") o.u = atoi(need(i));
        else if (a == "-s") o.s = atoi(need(i));
        else if (a == "-c") o.c = atoi(need(i));
        else if (a == "-b") o.bits = atoi(need(i));
        else if (a == "-A") o.A = atoi(need(i));
        else if (a == "-B") o.B = atoi(need(i));
        else if (a == "-O") o.O = atoi(need(i));
        else if (a == "-E") o.E = atoi(need(i));
        else if (a == "-L") o.L = atoi(need(i));
        else if (a == "-f") o.f = (float)atof(need(i));
        else if (a == "-S") o.S = (float)atof(need(i));
        else if (a == "-M") o.M = atoi(need(i));
        else if (a == "-R") o.R = atoi(need(i));
        else if (a == "-x") { fprintf(stderr, "-x (PAF output) is unreachable in the reference's async pipeline and not provided\n"); ok = false; }
        else if (a == "-h" || a == "--help") { ok = false; }
        else if (!a.empty() && a[0] == '-' && a.size() > 1) { fprintf(stderr, "unknown option %s\n", a.c_str()); ok = false; }
        else pos.push_back(a);
    }
    if (!pos.empty()) o.ref = pos[0];
    if (pos.size() > 1) o.reads1 = pos[1];
    if (pos.size() > 2) o.reads2 = pos[2];
    return o;
}


void write_sink(void* user, const char* chunk, size_t bytes) {
    fwrite(chunk, 1, bytes, (FILE*)user);
}

}  // namespace

int cli_main(int argc, char** argv, EngineFactory factory, const char* prog) {
    tune_malloc();
    try {
        bool index_cmd = argc > 1 && std::string(argv[1]) == "index";
        bool ok = true;
        Opts o = parse(argc - (index_cmd ? 1 : 0), argv + (index_cmd ? 1 : 0), ok);
        if (!ok || o.ref.empty()) { usage(prog); return 1; }
        if (o.c != INT32_MIN && (o.c >= 64 || o.c <= 0)) throw std::runtime_error("c must be greater than 0 and less than 64");
        if (o.interleaved && !o.reads2.empty())        // main.cpp:136-139
            throw std::runtime_error("Cannot specify both --interleaved and specify two read files");
        // the reads are streamed: a reader thread per file parses chunks while the
        // workers map (InputBuffer::read_records, pc.cpp:74-107).  The source opens
        // first: the read-length estimate (main.cpp:254-258, readlen.cpp:16-29: the
        // first read_records(500), i.e. 500 records of each file or 1000 of an
        // interleaved file) is taken from the records it has parsed, which stay queued
        // for mapping -- a pipe or stdin is read once, as the reference's
        // RewindableFile replays what the estimate read (fastq.cpp:1-65)
        if (o.world < 1 || o.rank < 0 || o.rank >= o.world) throw std::runtime_error("--rank must be in [0, --world)");
        const bool part = o.world > 1;
        if (part && o.interleaved) throw std::runtime_error("--rank/--world take two read files or one single-end file");
        std::unique_ptr<ReadSource> src;
        PartPlan plan;
        if (!o.reads1.empty() && !index_cmd) {
            if (part) {
                // no exchange between the ranks here: each counts every block of the files
                plan = plan_part(o.reads1, o.reads2, o.rank, o.world, (size_t)std::max(1, o.chunk_size), {}, {},
                                 std::max(1, o.threads));
                src = open_fastq_part_source(o.reads1, o.reads2, plan);
            } else {
                src = open_fastq_source(o.reads1, o.reads2, o.interleaved, (size_t)std::max(1, o.chunk_size));
            }
        }
        if (src && !o.r_set) o.r = src->estimate_read_length();
        IndexParameters ip = IndexParameters::from_read_length(o.r, o.k, o.s, o.l, o.u, o.c, o.m);
        auto t0 = std::chrono::steady_clock::now();
        References refs = References::from_fasta(o.ref);
        if (refs.size() == 0) throw std::runtime_error("No reference sequences found");
        for (auto& sq : refs.seqs)
            if (sq.size() >= (1ull << 31)) throw std::runtime_error("contigs must be shorter than 2^31 bp (int coordinates)");
        if (refs.size() >= (1u << 24)) throw std::runtime_error("at most 2^24 contigs");
        StiIndex idx;
        const std::string sti_path = o.ref + ip.filename_extension();
        // the index is built on the GPU (engine build) unless --cpu-index asks for the host build
        auto build_index = [&](bool host_copy) {
            if (o.cpu_index) idx.build(refs, ip, o.bits, o.f, std::max(1, o.threads));
            else build_default_index(idx, refs, ip, o.bits, o.f, std::max(1, o.threads), o.device, host_copy);
        };
        if (index_cmd || o.create_index) {
            build_index(true);
            std::string out = o.out_file.empty() ? sti_path : o.out_file;
            idx.write(out);
            if (o.verbose) {
                fprintf(stderr, "wrote %s (%zu randstrobes, bits %d, filter cutoff %d)\n", out.c_str(),
                        (size_t)idx.size(), idx.bits, idx.filter_cutoff);
                if (idx.built_on_device)
                    fprintf(stderr, "GPU build %.1f ms (upload %.1f, syncmers %.1f, randstrobes %.1f, sort %.1f, buckets "
                                    "%.1f); (hash, position) ties %lu, their order replayed on the host in %.1f ms\n",
                            idx.device_build_ms[5], idx.device_build_ms[0], idx.device_build_ms[1],
                            idx.device_build_ms[2], idx.device_build_ms[3], idx.device_build_ms[4],
                            (unsigned long)idx.position_ties, idx.ms_tie_replay);
                else
                    fprintf(stderr, "host build; (hash, position) ties %lu\n", (unsigned long)idx.position_ties);
            }
            return 0;
        }
        if (o.use_index) {
            idx.read(sti_path);
            if (!(idx.params == ip)) throw std::runtime_error("Index parameters in .sti file and those specified on command line differ");
        } else {
            build_index(false);   // a GPU build stays in HBM for the engine
        }
        const double t_index = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (o.reads1.empty()) throw std::runtime_error("At least one file with reads must be specified.");
        AlignmentParameters ap{o.A, o.B, o.O, o.E, o.L};
        MappingParameters mp;
        mp.r = o.r; mp.max_secondary = o.max_secondary; mp.dropoff_threshold = o.S; mp.rescue_level = o.R;
        mp.max_tries = o.M; mp.cigar_eqx = o.eqx; mp.output_unmapped = !o.no_unmapped; mp.details = o.details;
        if (mp.max_tries < 1) throw std::runtime_error("max_tries must be greater than zero");
        mp.rescue_cutoff = mp.rescue_level < 100 ? mp.rescue_level * idx.filter_cutoff : 1000;
        auto t1 = std::chrono::steady_clock::now();
        const std::vector<int> devs = o.devices.empty() ? std::vector<int>{o.device} : parse_devices(o.devices);
        std::unique_ptr<Engine> eng = open_engines(factory, refs, idx, devs);
        const double t_upload = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
        FILE* out = o.out_file.empty() ? stdout : fopen(o.out_file.c_str(), "wb");
        if (!out) throw std::runtime_error("cannot open " + o.out_file);
        // the @PG command line leaves --rank/--world out: rank 0's header is the one a
        // single process given the other arguments writes
        std::string cmd;
        for (int i = 0; i < argc; ++i) {
            const std::string a = argv[i];
            if ((a == "--rank" || a == "--world") && i + 1 < argc) { ++i; continue; }
            cmd += a;
            cmd += ' ';
        }
        std::string hdr = sam_header(refs, o.rg_id, o.rg, cmd);
        if (o.rank == 0) fwrite(hdr.data(), 1, hdr.size(), out);
        MapContext mc{refs, idx.params, ap, mp};
        PipelineOptions po;
        po.threads = o.threads; po.chunk_size = o.chunk_size; po.rg_id = o.rg_id;
        po.first_chunk = part ? (size_t)plan.first_chunk : 0;
        po.end_chunk = part ? (size_t)plan.end_chunk : SIZE_MAX;
        if (part && o.verbose)
            fprintf(stderr, "[%s] rank %d of %d: chunks [%lu, %lu) of %lu, pairs [%lu, %lu)\n", prog, o.rank, o.world,
                    (unsigned long)plan.first_chunk, (unsigned long)plan.end_chunk, (unsigned long)plan.n_chunks,
                    (unsigned long)plan.first_record, (unsigned long)(plan.first_record + plan.n_records));
        if (o.verbose) fprintf(stderr, "[%s] mapping %s%s%s%s\n", prog, o.reads1.c_str(), o.reads2.empty() ? "" : " + ",
                               o.reads2.c_str(), o.interleaved ? " (interleaved)" : "");
        PipelineResult res = src->paired() ? run_pipeline_pe(*src, *eng, mc, po, write_sink, out)
                                           : run_pipeline_se(*src, *eng, mc, po, write_sink, out);
        src.reset();
        if (o.interleaved && o.verbose)
            fprintf(stderr, "[%s] interleaved input: %lu unpaired records (not mapped, as in the reference's "
                            "paired-end task)\n", prog, (unsigned long)res.singletons);
        const bool bad = ferror(out) != 0;
        if ((out != stdout ? fclose(out) : fflush(out)) != 0 || bad)
            throw std::runtime_error("write failed: " + (o.out_file.empty() ? std::string("stdout") : o.out_file));
        fprintf(stderr,
                "[%s] engine %s | index %.2f s, upload %.2f s | mapped %lu reads in %.3f s = %.4f Mreads/s | "
                "SW calls %lu, tried %lu, inconsistent NAMs %lu, NAM rescue %lu, mate rescue %lu\n",
                prog, eng->name(), t_index, t_upload, (unsigned long)res.stats.n_reads, res.map_seconds,
                res.stats.n_reads / res.map_seconds / 1e6, (unsigned long)res.stats.tot_aligner_calls,
                (unsigned long)res.stats.tot_all_tried, (unsigned long)res.stats.inconsistent_nams,
                (unsigned long)res.stats.nam_rescue, (unsigned long)res.stats.tot_rescued);
        return 0;
    } catch (const std::exception& e) {
        fprintf(stderr, "%s: %s\n", prog, e.what());
        return 1;
    }
}

}  // namespace rsa

#ifndef RSA_NO_MAIN
int main(int argc, char** argv) { return rsa::cli_main(argc, argv, rsa::make_gpu_engine, "rsalign"); }
#endif

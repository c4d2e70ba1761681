// lzbench_amd/driver/lzbench_hip_main.cpp -- lzbench-compatible command line driver for the MI355X
// codec rows of liblzbench_hip.so.
//
// Mirrors the reference driver's semantics (/root/reference/_lzbench/lzbench.cpp):
//   * options -b -c -e -i -t -u -o -p -s -v -x -z -l -j and the "--compress-only" switch; -x
//     leaves the process priority alone, otherwise it is raised as SET_HIGH_PRIORITY does
//     (option parsing lzbench.cpp:824-934, usage :731-758)
//   * compressor_desc_t table with memcpy at index 0 (lzbench.h:113-219), name/level lookup
//     with '/' and ',' separated lists and aliases (lzbench.cpp:479-534)
//   * lzbench_test: init -> chunk list -> timed compress loop -> timed decompress loop with
//     length + memcmp verification -> print_stats (lzbench.cpp:332-476); MB = 1e6 B, speed =
//     size*1000/ns, ratio = 100*compr/orig (lzbench.cpp:104-106), fastest/average/median
//   * lzbench_compress / lzbench_decompress chunk loops with the raw-store rule
//     (lzbench.cpp:266-329), or ONE call per chunk list through a row's batched hook.
// Added: -g# = number of GPUs a HIP row shards the chunk list over (its additional_param).
#include <dirent.h>
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <strings.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/lzbench_hip.h"

#define PROGNAME "lzbench_hip"
#define PAD_SIZE (16 * 1024)
#define GET_COMPRESS_BOUND(n) ((n) + (n) / 6 + PAD_SIZE)
#define DEFAULT_LOOP_TIME (100 * 1000000ull)   // ns

typedef int64_t (*compress_func)(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char*);
typedef char* (*init_func)(size_t insize, size_t, size_t);
typedef void (*deinit_func)(char* workmem);
typedef int64_t (*compress_batch_func)(const char* in, const size_t* chunk_sizes, int nchunks, char* out, size_t outcap,
                                       size_t* compr_sizes, size_t, size_t, char*);
typedef int64_t (*decompress_batch_func)(const char* in, const size_t* compr_sizes, const size_t* chunk_sizes,
                                         int nchunks, char* out, size_t outcap, size_t, size_t, char*);

struct compressor_desc_t {
    const char* name;
    const char* version;
    int first_level, last_level, additional_param, max_block_size;
    compress_func compress, decompress;
    init_func init;
    deinit_func deinit;
    compress_batch_func compress_batch;
    decompress_batch_func decompress_batch;
};

// ---- CPU rows -------------------------------------------------------------------------
static int64_t lzb_return_0(char*, size_t, char*, size_t, size_t, size_t, char*) { return 0; }
static int64_t lzb_memcpy(char* in, size_t insize, char* out, size_t, size_t, size_t, char*) {
    memcpy(out, in, insize);
    return (int64_t)insize;
}
// system liblz4 (bit-identical to the bundled 1.9.3 on this image), if present
typedef int (*lz4c_t)(const char*, char*, int, int, int);
typedef int (*lz4d_t)(const char*, char*, int);
static lz4c_t sys_lz4_compress_fast = nullptr;
static lz4d_t sys_lz4_decompress_fast = nullptr;
static const char* sys_lz4_version = "n/a";
static void load_sys_lz4() {
    void* h = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    sys_lz4_compress_fast = (lz4c_t)dlsym(h, "LZ4_compress_fast");
    sys_lz4_decompress_fast = (lz4d_t)dlsym(h, "LZ4_decompress_fast");
    typedef const char* (*vs_t)(void);
    vs_t vs = (vs_t)dlsym(h, "LZ4_versionString");
    if (vs) sys_lz4_version = vs();
}
static int64_t cpu_lz4_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t, char*) {
    return sys_lz4_compress_fast(in, out, (int)insize, (int)outsize, level ? (int)level : 1);
}
static int64_t cpu_lz4_decompress(char* in, size_t, char* out, size_t outsize, size_t, size_t, char*) {
    sys_lz4_decompress_fast(in, out, (int)outsize);
    return (int64_t)outsize;
}

static compressor_desc_t comp_desc[] = {
    {"memcpy", "", 0, 0, 0, 0, lzb_return_0, lzb_memcpy, nullptr, nullptr, nullptr, nullptr},
    {"lz4", "sys", 0, 0, 0, 0, cpu_lz4_compress, cpu_lz4_decompress, nullptr, nullptr, nullptr, nullptr},
    {"lz4fast", "sys", 1, 99, 0, 0, cpu_lz4_compress, cpu_lz4_decompress, nullptr, nullptr, nullptr, nullptr},
    {"hipMemcpy", "", 0, 0, 1, 0, lzbench_hip_memcpy, lzbench_hip_memcpy, lzbench_hip_memcpy_init, lzbench_hip_deinit,
     lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
    {"hip_lz4", "1.9.3", 0, 0, 1, 0, lzbench_hip_lz4_compress, lzbench_hip_lz4_decompress, lzbench_hip_lz4_init,
     lzbench_hip_deinit, lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
    {"hip_lz4fast", "1.9.3", 1, 99, 1, 0, lzbench_hip_lz4fast_compress, lzbench_hip_lz4_decompress,
     lzbench_hip_lz4_init, lzbench_hip_deinit, lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
    {"hip_snappy", "2020-07-11", 0, 0, 1, 0, lzbench_hip_snappy_compress, lzbench_hip_snappy_decompress,
     lzbench_hip_snappy_init, lzbench_hip_deinit, lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
    // zstd / zstd_fast rows (lzbench.h:209-210) at the fast-strategy levels the GPU compressor covers
    {"hip_zstd", "1.5.2", 1, 2, 1, 0, lzbench_hip_zstd_compress, lzbench_hip_zstd_decompress, lzbench_hip_zstd_init,
     lzbench_hip_deinit, lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
    {"hip_zstd_fast", "1.5.2", -5, -1, 1, 0, lzbench_hip_zstd_compress, lzbench_hip_zstd_decompress,
     lzbench_hip_zstd_init, lzbench_hip_deinit, lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
    // framed formats: an LZ4 frame per chunk (level = LZH_LZ4F_PARAMS: 4..7 = block size 64 KiB..4 MiB), and
    // the nvcomp_lz4 row's container (lzbench.h:218, levels 0..5 = chunks of 32 KiB << level)
    {"hip_lz4frame", "1.9.3", 4, 7, 1, 0, lzbench_hip_lz4frame_compress, lzbench_hip_lz4frame_decompress,
     lzbench_hip_lz4frame_init, lzbench_hip_deinit, lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
    {"hip_nvcomp_lz4", "1.2.2", 0, 5, 1, 0, lzbench_hip_nvcomp_lz4_compress, lzbench_hip_nvcomp_lz4_decompress,
     lzbench_hip_nvcomp_lz4_init, lzbench_hip_deinit, lzbench_hip_compress_batch, lzbench_hip_decompress_batch},
};
static const int kRows = (int)(sizeof(comp_desc) / sizeof(comp_desc[0]));

struct alias_t { const char* name; const char* params; };
static const alias_t aliases[] = {
    {"hip", "hipMemcpy/hip_lz4/hip_lz4fast,3,17/hip_snappy/hip_zstd,1"},
    {"cuda", "hipMemcpy/hip_nvcomp_lz4,0,1,3,5"},   // the reference's GPU alias (lzbench.h:255) on its drop-in rows
    {"fast", "lz4/lz4fast,3,17/hip_lz4/hip_lz4fast,3,17/hip_snappy/hip_zstd_fast,-1/hip_zstd,1"},
    {"all", "lz4/lz4fast,3,17/hipMemcpy/hip_lz4/hip_lz4fast,3,17/hip_snappy/hip_zstd_fast/hip_zstd"},
};

// ---- parameters and results (lzbench.h:83-105) ------------------------------------------
enum textformat_e { MARKDOWN = 1, TEXT, TEXT_FULL, CSV, TURBOBENCH, MARKDOWN2 };
enum timetype_e { FASTEST = 1, AVERAGE, MEDIAN };
struct row_t {
    std::string alg;
    uint64_t ctime, dtime, csize, osize;
    std::string file;
};
struct params_t {
    int show_speed = 1, compress_only = 0, verbose = 2, ngpus = 1;
    int random_read = 0;        // -R: one random chunk-aligned block per file (lzbench.cpp:671-681)
    uint64_t mem_limit = 0;     // -m: read files in parts of this many bytes (lzbench.cpp:652-656, :699-713)
    timetype_e timetype = FASTEST;
    textformat_e textformat = TEXT;
    size_t chunk_size = (1ull << 31) - (1ull << 31) / 6;
    uint32_t c_iters = 1, d_iters = 1, cspeed = 0;
    uint64_t cmintime = 1000, dmintime = 2000;             // ms
    uint64_t cloop_time = DEFAULT_LOOP_TIME, dloop_time = DEFAULT_LOOP_TIME;
    std::vector<row_t> results;
    const char* in_filename = "";
};
#define LZB_PRINT(level, ...) do { if (P->verbose >= (level)) printf(__VA_ARGS__); } while (0)

static uint64_t now_ns() {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static bool g_gpu = false;
static void* alloc_touch(size_t size) {   // pinned when a GPU is present (faster H2D/D2H)
    void* p = nullptr;
    if (g_gpu && hipHostMalloc(&p, size, hipHostMallocDefault) == hipSuccess) {
        memset(p, 0, size);
        return p;
    }
    p = calloc(1, size);
    return p;
}
static void free_touch(void* p) {
    if (!p) return;
    if (g_gpu && hipHostFree(p) == hipSuccess) return;
    free(p);
}

static void print_header(params_t* P) {
    switch (P->textformat) {
    case CSV: printf("Compressor name,Compression speed,Decompression speed,Original size,Compressed size,Ratio,Filename\n"); break;
    case TURBOBENCH: printf("  Compressed  Ratio   Cspeed   Dspeed         Compressor name Filename\n"); break;
    case TEXT: printf("Compressor name         Compress. Decompress. Compr. size  Ratio Filename\n"); break;
    case TEXT_FULL: printf("Compressor name         Compress. Decompress.  Orig. size  Compr. size  Ratio Filename\n"); break;
    case MARKDOWN:
        printf("| Compressor name         | Compression| Decompress.| Compr. size | Ratio | Filename |\n");
        printf("| ---------------         | -----------| -----------| ----------- | ----- | -------- |\n");
        break;
    case MARKDOWN2:
        printf("| Compressor name         | Ratio | Compression| Decompress.|\n");
        printf("| ---------------         | ------| -----------| ---------- |\n");
        break;
    }
}

static void print_speed_field(double v) {
    if (v < 10) printf("%6.2f MB/s", v);
    else if (v < 100) printf("%6.1f MB/s", v);
    else printf("%6d MB/s", (int)v);
}

static void print_row(params_t* P, const row_t& r) {
    const double cs = r.ctime ? r.osize * 1000.0 / r.ctime : 0.0;
    const double ds = r.dtime ? r.osize * 1000.0 / r.dtime : 0.0;
    const double ratio = r.osize ? r.csize * 100.0 / r.osize : 0.0;
    if (!P->show_speed) {
        printf("%-23s %8.3f ms %8.3f ms %12llu %6.2f %s\n", r.alg.c_str(), r.ctime / 1e6, r.dtime / 1e6,
               (unsigned long long)r.csize, ratio, r.file.c_str());
        return;
    }
    switch (P->textformat) {
    case CSV:
        printf("%s,%.2f,%.2f,%llu,%llu,%.2f,%s\n", r.alg.c_str(), cs, ds, (unsigned long long)r.osize,
               (unsigned long long)r.csize, ratio, r.file.c_str());
        break;
    case TURBOBENCH:
        printf("%12llu %6.1f%9.2f%9.2f  %22s %s\n", (unsigned long long)r.csize, ratio, cs, ds, r.alg.c_str(), r.file.c_str());
        break;
    case MARKDOWN:
        printf("| %-23s |%8.0f MB/s |%8.0f MB/s |%12llu |%6.2f | %s |\n", r.alg.c_str(), cs, ds,
               (unsigned long long)r.csize, ratio, r.file.c_str());
        break;
    case MARKDOWN2:
        printf("| %-23s |%6.2f |%8.0f MB/s |%8.0f MB/s |\n", r.alg.c_str(), ratio, cs, ds);
        break;
    default:
        printf("%-23s", r.alg.c_str());
        print_speed_field(cs);
        if (!r.dtime) printf("      ERROR");
        else print_speed_field(ds);
        if (P->textformat == TEXT_FULL) printf("%12llu %12llu %6.2f %s\n", (unsigned long long)r.osize, (unsigned long long)r.csize, ratio, r.file.c_str());
        else printf("%12llu %6.2f %s\n", (unsigned long long)r.csize, ratio, r.file.c_str());
    }
}

static uint64_t pick_time(params_t* P, std::vector<uint64_t>& v) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    if (P->timetype == AVERAGE) return std::accumulate(v.begin(), v.end(), (uint64_t)0) / v.size();
    if (P->timetype == MEDIAN) return (v[(v.size() - 1) / 2] + v[v.size() / 2]) / 2;
    return v[0];
}

// ---- chunk loops (lzbench.cpp:266-329) ------------------------------------------------------
static int64_t run_compress(const compressor_desc_t* d, std::vector<size_t>& chunks, std::vector<size_t>& cs,
                            uint8_t* in, uint8_t* out, size_t outsize, size_t p1, size_t p2, char* wm) {
    cs.resize(chunks.size());
    if (d->compress_batch)
        return d->compress_batch((const char*)in, chunks.data(), (int)chunks.size(), (char*)out, outsize, cs.data(), p1, p2, wm);
    int64_t sum = 0;
    for (size_t i = 0; i < chunks.size(); i++) {
        const size_t part = chunks[i];
        size_t outpart = GET_COMPRESS_BOUND(part);
        if (outpart > outsize) outpart = outsize;
        int64_t clen = d->compress((char*)in, part, (char*)out, outpart, p1, p2, wm);
        if (clen <= 0 || (size_t)clen == part) {
            if (part > outsize) return 0;
            memcpy(out, in, part);
            clen = (int64_t)part;
        }
        in += part; out += clen; outsize -= (size_t)clen; cs[i] = (size_t)clen; sum += clen;
    }
    return sum;
}

static int64_t run_decompress(const compressor_desc_t* d, std::vector<size_t>& chunks, std::vector<size_t>& cs,
                              uint8_t* in, uint8_t* out, size_t outcap, size_t p1, size_t p2, char* wm) {
    if (d->decompress_batch)
        return d->decompress_batch((const char*)in, cs.data(), chunks.data(), (int)cs.size(), (char*)out, outcap, p1, p2, wm);
    int64_t sum = 0;
    for (size_t i = 0; i < cs.size(); i++) {
        const size_t part = cs[i];
        int64_t dlen;
        if (part == chunks[i]) { memcpy(out, in, part); dlen = (int64_t)part; }
        else dlen = d->decompress((char*)in, part, (char*)out, chunks[i], p1, p2, wm);
        if (dlen <= 0) return dlen;
        in += part; out += dlen; sum += dlen;
    }
    return sum;
}

// ---- lzbench_test (lzbench.cpp:332-476) -----------------------------------------------------
static void bench_one(params_t* P, std::vector<size_t>& file_sizes, const compressor_desc_t* d, int level, uint8_t* inbuf,
                      size_t insize, uint8_t* compbuf, size_t comprsize, uint8_t* decomp) {
    const size_t p1 = (size_t)level;
    const size_t p2 = d->additional_param ? (size_t)P->ngpus : 0;
    size_t chunk = P->chunk_size > insize ? insize : P->chunk_size;
    if (d->max_block_size && chunk > (size_t)d->max_block_size) chunk = (size_t)d->max_block_size;
    if (!d->compress || !d->decompress || !chunk) return;
    {   // GPU rows whose level the device codec does not cover for this chunk size (zstd level 2 is
        // double-fast above 256 KiB chunks): say so instead of an error row
        const int codec = d->init == lzbench_hip_zstd_init ? LZH_CODEC_ZSTD
                        : d->init == lzbench_hip_lz4frame_init ? LZH_CODEC_LZ4F
                        : d->init == lzbench_hip_nvcomp_lz4_init ? LZH_CODEC_NVLZ4 : -1;
        if (codec >= 0 && !lzh_level_supported(codec, level, chunk)) {
            LZB_PRINT(1, "%s %s -%d: level not supported by the GPU codec for %zu-byte chunks (skipped)\n", d->name,
                      d->version, level, chunk);
            return;
        }
    }
    char* wm = d->init ? d->init(chunk, p1, p2) : nullptr;
    if (d->init && !wm) { LZB_PRINT(1, "%s: init failed\n", d->name); return; }
    std::vector<size_t> chunks, cs;
    for (size_t f : file_sizes)
        for (size_t t = f; t > 0; t -= std::min(t, chunk)) chunks.push_back(std::min(t, chunk));
    std::vector<uint64_t> ctime, dtime;
    int64_t complen = 0, decomplen = 0;
    bool err = false;

    uint32_t iters = 0;
    const uint64_t t_start = now_ns();
    for (;;) {
        uint32_t i = 0;
        const uint64_t loop0 = now_ns();
        uint64_t t1;
        do {
            const uint64_t t0 = now_ns();
            complen = run_compress(d, chunks, cs, inbuf, compbuf, comprsize, p1, p2, wm);
            t1 = now_ns();
            if (t1 - t0 >= 10000) ctime.push_back(t1 - t0);
            i++;
        } while (t1 - loop0 < P->cloop_time);
        ctime.push_back((t1 - loop0) / i);
        iters += i;
        if (P->cspeed && (double)insize * i * 1000 / (t1 - loop0) < P->cspeed) goto done;
        if (iters >= P->c_iters && t1 - t_start > P->cmintime * 1000000ull) break;
    }
    if (complen <= 0) err = true;
    if (const char* dd = getenv("LZH_DUMP_DIR")) {   // test hook: the packed compbuf and compr_sizes of the row
        std::string nm = std::string(dd) + "/" + d->name + "_" + std::to_string(level);
        if (FILE* f = fopen((nm + ".bin").c_str(), "wb")) { fwrite(compbuf, 1, (size_t)std::max<int64_t>(complen, 0), f); fclose(f); }
        if (FILE* f = fopen((nm + ".sizes").c_str(), "wb")) { fwrite(cs.data(), sizeof(size_t), cs.size(), f); fclose(f); }
    }
    if (!P->compress_only) {
        iters = 0;
        const uint64_t t_dstart = now_ns();
        for (;;) {
            uint32_t i = 0;
            const uint64_t loop0 = now_ns();
            uint64_t t1;
            do {
                const uint64_t t0 = now_ns();
                decomplen = run_decompress(d, chunks, cs, compbuf, decomp, insize + PAD_SIZE, p1, p2, wm);
                t1 = now_ns();
                if (t1 - t0 >= 10000) dtime.push_back(t1 - t0);
                i++;
            } while (t1 - loop0 < P->dloop_time);
            dtime.push_back((t1 - loop0) / i);
            if ((size_t)decomplen != insize || memcmp(inbuf, decomp, insize) != 0) {
                err = true;
                LZB_PRINT(5, "ERROR in %s: decompressed data differs\n", d->name);
            }
            memset(decomp, 0, insize);
            if (err) break;
            iters += i;
            if (iters >= P->d_iters && t1 - t_dstart > P->dmintime * 1000000ull) break;
        }
    }
    {
        row_t r;
        char name[256];
        if (d->first_level == 0 && d->last_level == 0) snprintf(name, sizeof name, "%s %s", d->name, d->version);
        else snprintf(name, sizeof name, "%s %s -%d", d->name, d->version, level);
        r.alg = name;
        r.ctime = pick_time(P, ctime);
        r.dtime = err ? 0 : pick_time(P, dtime);
        r.csize = (uint64_t)std::max<int64_t>(complen, 0);
        r.osize = insize;
        r.file = P->in_filename;
        P->results.push_back(r);
        print_row(P, r);
    }
done:
    if (d->deinit) d->deinit(wm);
}

static const compressor_desc_t* find_row(const char* name) {
    for (int i = 1; i < kRows; i++)
        if (!strcmp(comp_desc[i].name, name)) return &comp_desc[i];
    return nullptr;
}

// '/'-separated list, each "name[,level[,level]]" (lzbench.cpp:479-534)
static void bench_list(params_t* P, std::vector<size_t>& fs, const char* list, uint8_t* in, size_t insize, uint8_t* comp,
                       size_t compsize, uint8_t* dec) {
    std::string s(list);
    size_t pos = 0;
    while (pos <= s.size()) {
        size_t e = s.find('/', pos);
        if (e == std::string::npos) e = s.size();
        std::string item = s.substr(pos, e - pos);
        pos = e + 1;
        if (item.empty()) continue;
        // an item naming an alias (case-insensitively) runs the alias' list (lzbench.cpp:493-501)
        const alias_t* al = nullptr;
        for (const alias_t& a : aliases)
            if (!strcasecmp(item.c_str(), a.name)) al = &a;
        if (al) {
            bench_list(P, fs, al->params, in, insize, comp, compsize, dec);
            continue;
        }
        std::vector<std::string> parts;
        size_t q = 0;
        while (q <= item.size()) {
            size_t c = item.find(',', q);
            if (c == std::string::npos) c = item.size();
            parts.push_back(item.substr(q, c - q));
            q = c + 1;
        }
        const compressor_desc_t* d = find_row(parts[0].c_str());
        if (!d || ((d == &comp_desc[1] || d == &comp_desc[2]) && !sys_lz4_compress_fast) ||
            (!g_gpu && d->init)) {
            // (lzbench.cpp:507-528: one line per requested level, "(null)" -- glibc's rendering of the
            // NULL level argument -- when none is given; memcpy, index 0, is never found by name)
            for (size_t k = 1; k == 1 || k < parts.size(); k++)
                printf("NOT FOUND: %s %s\n", parts[0].c_str(), k < parts.size() ? parts[k].c_str() : "(null)");
            continue;
        }
        if (parts.size() == 1) {
            for (int l = d->first_level; l <= d->last_level; l++) bench_one(P, fs, d, l, in, insize, comp, compsize, dec);
        } else {
            for (size_t k = 1; k < parts.size(); k++) {
                const int l = atoi(parts[k].c_str());
                if (l >= d->first_level && l <= d->last_level) bench_one(P, fs, d, l, in, insize, comp, compsize, dec);
            }
        }
    }
}

static void usage(params_t* P) {
    fprintf(stderr, "usage: " PROGNAME " [options] input [input2] [input3]\n\nwhere [options] are:\n");
    fprintf(stderr, " -b#   set block/chunk size to # KB (default = MIN(filesize,%d KB))\n", (int)(P->chunk_size >> 10));
    fprintf(stderr, " -c#   sort results by column # (1=algname, 2=ctime, 3=dtime, 4=comprsize)\n");
    fprintf(stderr, " -e#   #=compressors separated by '/' with parameters specified after ',' (deflt=hip)\n");
    fprintf(stderr, " -g#   number of GPUs a hip_* row shards the chunk list over (default = 1)\n");
    fprintf(stderr, " -iX,Y set min. number of compression and decompression iterations (default = %u, %u)\n", P->c_iters, P->d_iters);
    fprintf(stderr, " -j    join files in memory but compress them independently (for many small files)\n");
    fprintf(stderr, " -l    list of available compressors and aliases\n");
    fprintf(stderr, " -R    read block/chunk size from random blocks (to estimate for large files)\n");
    fprintf(stderr, " -m#   set memory limit to # MB (default = no limit)\n");
    fprintf(stderr, " -o#   output text format 1=Markdown, 2=text, 3=text+origSize, 4=CSV (default = %d)\n", P->textformat);
    fprintf(stderr, " -p#   print time for all iterations: 1=fastest 2=average 3=median (default = %d)\n", P->timetype);
    fprintf(stderr, " -r    operate recursively on directories\n");
    fprintf(stderr, " -s#   use only compressors with compression speed over # MB (default = %u MB)\n", P->cspeed);
    fprintf(stderr, " -tX,Y set min. time in seconds for compression and decompression (default = %.0f, %.0f)\n",
            P->cmintime / 1000.0, P->dmintime / 1000.0);
    fprintf(stderr, " -v    disable progress information\n -x    disable real-time process priority\n -z    show (de)compression times instead of speed\n");
    fprintf(stderr, "\ndebug (environment): LZH_DUMP_DIR=dir writes each GPU row's packed buffer and compressed sizes there\n");
}

static int read_file(const char* fn, std::vector<uint8_t>& out) {
    FILE* f = fopen(fn, "rb");
    if (!f) return -1;
    fseeko(f, 0, SEEK_END);
    const off_t n = ftello(f);
    fseeko(f, 0, SEEK_SET);
    out.resize((size_t)n);
    const size_t r = n ? fread(out.data(), 1, (size_t)n, f) : 0;
    fclose(f);
    return r == (size_t)n ? 0 : -1;
}

// inputs: files as given; directories expanded (sorted) when -r is set, else skipped
static void expand_inputs(const char* path, bool recursive, std::vector<std::string>& out) {
    struct stat st;
    if (stat(path, &st) != 0) { out.push_back(path); return; }      // (reported when opened)
    if (!S_ISDIR(st.st_mode)) { out.push_back(path); return; }
    if (!recursive) { fprintf(stderr, "%s is a directory (use -r)\n", path); return; }
    DIR* d = opendir(path);
    if (!d) return;
    std::vector<std::string> names;
    while (struct dirent* e = readdir(d))
        if (strcmp(e->d_name, ".") && strcmp(e->d_name, "..")) names.push_back(e->d_name);
    closedir(d);
    std::sort(names.begin(), names.end());
    for (const std::string& n : names) expand_inputs((std::string(path) + "/" + n).c_str(), true, out);
}

static void bench_buffer(params_t* P, std::vector<size_t>& fs, const std::vector<uint8_t>& data, const char* list) {
    const size_t insize = data.size();
    const size_t compsize = GET_COMPRESS_BOUND(insize);
    uint8_t* in = (uint8_t*)alloc_touch(insize + PAD_SIZE);
    uint8_t* comp = (uint8_t*)alloc_touch(compsize);
    uint8_t* dec = (uint8_t*)alloc_touch(insize + PAD_SIZE);
    if (!in || !comp || !dec) { fprintf(stderr, "Not enough memory!\n"); exit(1); }
    memcpy(in, data.data(), insize);
    if (P->results.empty()) {   // implicit memcpy row first (lzbench.cpp:685-697)
        params_t Q = *P;
        Q.cmintime = Q.dmintime = 0;
        Q.c_iters = Q.d_iters = 0;
        Q.cloop_time = Q.dloop_time = DEFAULT_LOOP_TIME;
        std::vector<size_t> one(1, insize);
        bench_one(&Q, one, &comp_desc[0], 0, in, insize, comp, compsize, dec);
        P->results.insert(P->results.end(), Q.results.begin(), Q.results.end());
    }
    bench_list(P, fs, list, in, insize, comp, compsize, dec);
    free_touch(in); free_touch(comp); free_touch(dec);
}

int main(int argc, char** argv) {
    params_t params;
    params_t* P = &params;
    const char* list = "hip";
    int sort_col = 0;
    bool join = false, recursive = false, real_time = true;
    int ngpu = 0;
    g_gpu = hipGetDeviceCount(&ngpu) == hipSuccess && ngpu > 0;
    load_sys_lz4();
    comp_desc[1].version = comp_desc[2].version = sys_lz4_version;

    while (argc > 1 && argv[1][0] == '-') {
        char* a = argv[1] + 1;
        if (!strcmp(a, "-compress-only")) { P->compress_only = 1; argv++; argc--; continue; }
        while (*a) {
            char* np = a + 1;
            unsigned num = 0;
            while (*np >= '0' && *np <= '9') num = num * 10 + (unsigned)(*np++ - '0');
            auto second = [&](unsigned& dst) {
                if (*np == ',') { np++; unsigned v = 0; while (*np >= '0' && *np <= '9') v = v * 10 + (unsigned)(*np++ - '0'); dst = v; return true; }
                return false;
            };
            switch (*a) {
            case 'b': P->chunk_size = (size_t)num << 10; break;
            case 'c': sort_col = (int)num; break;
            case 'e': list = strdup(a + 1); np += strlen(np); break;
            case 'g': P->ngpus = num ? (int)num : 1; break;
            case 'i': P->c_iters = num; { unsigned v = P->d_iters; if (second(v)) P->d_iters = v; } break;
            case 'j': join = true; break;
            case 'm': P->mem_limit = (uint64_t)num << 18; if (P->textformat == TEXT) P->textformat = TEXT_FULL; break;
            case 'r': recursive = true; break;
            case 'R': P->random_read = 1; srand((unsigned)time(NULL)); break;
            case 'o': P->textformat = (textformat_e)num; if (P->textformat == CSV) P->verbose = 0; break;
            case 'p': P->timetype = (timetype_e)num; break;
            case 's': P->cspeed = num; break;
            case 't': {
                P->cmintime = 1000ull * num;
                P->cloop_time = P->cmintime ? DEFAULT_LOOP_TIME : 0;
                unsigned v;
                if (second(v)) { P->dmintime = 1000ull * v; P->dloop_time = P->dmintime ? DEFAULT_LOOP_TIME : 0; }
                break;
            }
            case 'u': P->dmintime = 1000ull * num; P->dloop_time = P->dmintime ? DEFAULT_LOOP_TIME : 0; break;
            case 'v': P->verbose = (int)num; break;
            case 'x': real_time = false; break;
            case 'z': P->show_speed = 0; break;
            case 'l':
                printf("\nAvailable compressors for -e option:\n");
                for (const alias_t& al : aliases) printf("%s - alias for %s\n", al.name, al.params);
                for (int i = 1; i < kRows; i++) {
                    const compressor_desc_t& d = comp_desc[i];
                    if ((i == 1 || i == 2) && !sys_lz4_compress_fast) continue;
                    if (d.first_level < d.last_level) printf("%s %s [%d-%d]\n", d.name, d.version, d.first_level, d.last_level);
                    else printf("%s %s\n", d.name, d.version);
                }
                return 0;
            case 'h':
            case '-': usage(P); return 0;
            default: fprintf(stderr, "unknown option: %s\n", argv[1]); return 1;
            }
            a = np;
        }
        argv++;
        argc--;
    }
    if (argc < 2) { usage(P); return 1; }
    // SET_HIGH_PRIORITY unless -x (util.h:106, lzbench.cpp:948); needs privileges, so a refusal
    // (EACCES / EPERM) leaves the default priority, as in the reference
    if (real_time) (void)setpriority(PRIO_PROCESS, 0, -20);
    LZB_PRINT(2, PROGNAME " 1.8-hip (lzbench chunk loop, MI355X codec rows; %d GPU%s visible)\n\n", ngpu, ngpu == 1 ? "" : "s");
    print_header(P);

    std::vector<std::string> inputs;
    for (int i = 1; i < argc; i++) expand_inputs(argv[i], recursive, inputs);
    if (join) {
        std::vector<uint8_t> all;
        std::vector<size_t> fs;
        for (const std::string& fn : inputs) {
            std::vector<uint8_t> d;
            if (read_file(fn.c_str(), d)) { fprintf(stderr, "cannot read %s\n", fn.c_str()); continue; }
            fs.push_back(d.size());
            all.insert(all.end(), d.begin(), d.end());
        }
        P->in_filename = fs.size() == 1 ? inputs[0].c_str() : "(joined files)";
        bench_buffer(P, fs, all, list);
    } else {
        for (const std::string& fn : inputs) {
            FILE* f = fopen(fn.c_str(), "rb");
            if (!f) { perror(fn.c_str()); continue; }
            const char* base = strrchr(fn.c_str(), '/');
            const std::string name = base ? base + 1 : fn.c_str();
            fseeko(f, 0, SEEK_END);
            const uint64_t real = (uint64_t)ftello(f);
            rewind(f);
            uint64_t insize = (P->mem_limit && real > P->mem_limit) ? P->mem_limit : real;
            if (P->random_read) {                 // lzbench.cpp:671-681
                uint64_t pos = 0;
                if (P->chunk_size < real) {
                    pos = (uint64_t)(rand() % (int)(real / P->chunk_size)) * P->chunk_size;
                    insize = P->chunk_size;
                    fseeko(f, (off_t)pos, SEEK_SET);
                } else {
                    insize = real;
                }
                printf("Seeking to: %llu %llu %llu\n", (unsigned long long)pos, (unsigned long long)P->chunk_size,
                       (unsigned long long)insize);
            }
            std::vector<uint8_t> d((size_t)insize);
            d.resize(insize ? fread(d.data(), 1, (size_t)insize, f) : 0);
            if (P->mem_limit && real > P->mem_limit) {     // parts (lzbench.cpp:699-713)
                for (int part = 1; !d.empty(); part++) {
                    const std::string pn = name + " part " + std::to_string(part);
                    P->in_filename = pn.c_str();
                    std::vector<size_t> fs(1, d.size());
                    bench_buffer(P, fs, d, list);
                    d.resize((size_t)insize);
                    d.resize(fread(d.data(), 1, (size_t)insize, f));
                }
            } else {
                std::vector<size_t> fs(1, d.size());
                P->in_filename = name.c_str();
                bench_buffer(P, fs, d, list);
            }
            fclose(f);
        }
    }
    if (sort_col > 0 && sort_col <= 5) {
        std::vector<row_t> r = P->results;
        std::stable_sort(r.begin(), r.end(), [&](const row_t& x, const row_t& y) {
            switch (sort_col) {
            case 1: return x.alg < y.alg;
            case 2: return x.ctime > y.ctime;
            case 3: return x.dtime > y.dtime;
            case 4: return x.csize < y.csize;
            default: return x.osize < y.osize;
            }
        });
        printf("\nThe results sorted by column number %d:\n", sort_col);
        print_header(P);
        for (const row_t& x : r) print_row(P, x);
    }
    return 0;
}

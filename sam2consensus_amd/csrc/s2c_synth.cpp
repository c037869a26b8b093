// s2c_synth.cpp — deterministic synthetic SAM workloads (BASELINE.json configs C1..C5).
//
// uniform-ACGT references, 150 bp reads, FLAG 0, MAPQ 60, QUAL '*',
// 1 % substitutions, 0.1 % N calls, optional single I / D per read, no read crossing a
// reference end, no read ending in an I op, every SEQ char in {A,C,G,T,N}.
// Everything is derived from splitmix64 streams keyed by (seed, read index), so the
// bytes are identical on every machine; the same generator feeds the golden run of the
// reference (oracle/gen_golden_configs.py), the CLI tests and bench.py.
#include <thread>
#include "../../include/s2c.h"

#include <new>
#include <stdexcept>
#include <string>

int s2c_set_error(int code, const std::string &msg);
template <class F>
static int s2c_guarded(F &&f) {   // (as in s2c_host.cpp: no exception crosses the C-ABI)
    try {
        return f();
    } catch (const std::bad_alloc &) {
        return s2c_set_error(S2C_ERR_LIMIT, "out of host memory");
    } catch (const std::exception &e) {
        return s2c_set_error(S2C_ERR_IO, std::string("host exception: ") + e.what());
    }
}

#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

int s2c_set_error(int code, const std::string &msg);

namespace {
struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
};

inline uint64_t read_seed(uint64_t seed, uint64_t gi) { return seed * 0x2545F4914F6CDD1Dull ^ (gi + 1) * 0xD1B54A32D192ED03ull; }

struct ReadShape { int64_t start; int32_t a, k, b; char kind; int32_t span; };

ReadShape shape_of(const s2c_synth_spec &sp, const std::vector<int64_t> &amp_start, int64_t L, Rng &rng) {
    ReadShape s{};
    const int32_t RL = sp.read_len;
    double u = rng.uni();
    if (u < sp.ins_frac) {
        s.kind = 'I';
        s.k = 1 + (int32_t)rng.below(sp.ins_max);
        s.a = 1 + (int32_t)rng.below(RL - s.k - 1);
        s.b = RL - s.k - s.a;
        s.span = RL - s.k;
    } else if (u < sp.ins_frac + sp.del_frac) {
        s.kind = 'D';
        if (rng.uni() < sp.long_del_frac)
            s.k = RL + 1 + (int32_t)rng.below(RL);   // > read_len deleted bases (maxdel rule)
        else
            s.k = 1 + (int32_t)rng.below(sp.del_max);
        s.a = 1 + (int32_t)rng.below(RL - 1);
        s.b = RL - s.a;
        s.span = RL + s.k;
    } else {
        s.kind = 'M';
        s.a = RL;
        s.span = RL;
    }
    if (s.span > L) {  // never cross the reference end
        s.kind = 'M';
        s.a = (int32_t)std::min<int64_t>(RL, L);
        s.span = s.a;
    }
    if (!amp_start.empty()) {
        int64_t st = amp_start[rng.below(amp_start.size())];
        s.start = std::min<int64_t>(st, L - s.span);
    } else {
        s.start = (int64_t)rng.below((uint64_t)(L - s.span + 1));
    }
    return s;
}

inline char *put_u(char *o, uint64_t v) {
    char tmp[24];
    int n = 0;
    do { tmp[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (n) *o++ = tmp[--n];
    return o;
}

using Sink = std::function<int(const char *, size_t)>;

int generate(const s2c_synth_spec &sp, const Sink &sink, int64_t *n_out) {
    if (sp.n_refs <= 0 || sp.ref_len <= 0 || sp.read_len < 4)
        return s2c_set_error(S2C_ERR_ARG, "bad synth spec");
    const char *pre = sp.ref_prefix ? sp.ref_prefix : "gene";
    const int64_t L = sp.ref_len;
    const int64_t per_ref = (int64_t)((double)sp.depth * (double)L / (double)sp.read_len);
    std::string buf;
    buf.reserve(1 << 23);
    auto flush = [&]() -> int {
        int rc = sink(buf.data(), buf.size());
        buf.clear();
        return rc;
    };
    buf += sp.shuffle ? "@HD\tVN:1.6\tSO:unsorted\n" : "@HD\tVN:1.6\tSO:coordinate\n";
    for (int32_t r = 0; r < sp.n_refs; r++) {
        char line[256];
        snprintf(line, sizeof line, "@SQ\tSN:%s%d\tLN:%lld\n", pre, r, (long long)L);
        buf += line;
    }
    buf += "@PG\tID:s2c_synth\tPN:s2c_synth\n";
    std::vector<int64_t> amp;
    if (sp.amplicons > 1) {
        for (int32_t j = 0; j < sp.amplicons; j++) amp.push_back((L - sp.read_len) * j / (sp.amplicons - 1));
    }
    // record order: (ref, start, index) sorted, or a global shuffle
    const int64_t N = per_ref * sp.n_refs;
    std::vector<uint64_t> ord(N);
    {
        std::vector<std::pair<int64_t, int64_t>> key;
        key.reserve(sp.shuffle ? 0 : N);
        for (int64_t gi = 0; gi < N; gi++) {
            if (sp.shuffle) { ord[gi] = gi; continue; }
            Rng rng(read_seed(sp.seed, gi));
            ReadShape s = shape_of(sp, amp, L, rng);
            key.push_back({(gi / per_ref) * (L + 1) + s.start, gi});
        }
        if (sp.shuffle) {
            Rng rng(sp.seed ^ 0x5DEECE66Dull);
            for (int64_t i = N - 1; i > 0; i--) std::swap(ord[i], ord[rng.below(i + 1)]);
        } else {
            std::sort(key.begin(), key.end());
            for (int64_t i = 0; i < N; i++) ord[i] = key[i].second;
        }
    }
    // reference sequences
    std::vector<std::string> refseq(sp.n_refs);
    for (int32_t r = 0; r < sp.n_refs; r++) {
        Rng rng(sp.seed * 0x9E3779B97F4A7C15ull + 0x1234567ull * (uint64_t)(r + 1));
        refseq[r].resize(L);
        for (int64_t i = 0; i < L; i++) refseq[r][i] = "ACGT"[rng.next() >> 62];
    }
    static const char *OTHER[4] = {"CGT", "AGT", "ACT", "ACG"};
    std::vector<char> line(64 + 4 * (size_t)sp.read_len + 64);
    for (int64_t n = 0; n < N; n++) {
        const uint64_t gi = ord[n];
        const int32_t r = (int32_t)(gi / per_ref);
        Rng rng(read_seed(sp.seed, gi));
        ReadShape s = shape_of(sp, amp, L, rng);
        char *o = line.data();
        *o++ = 'r';
        o = put_u(o, gi);
        memcpy(o, "\t0\t", 3); o += 3;
        size_t pl = strlen(pre);
        memcpy(o, pre, pl); o += pl;
        o = put_u(o, (uint64_t)r);
        *o++ = '\t';
        o = put_u(o, (uint64_t)(s.start + 1));
        memcpy(o, "\t60\t", 4); o += 4;
        o = put_u(o, (uint64_t)s.a);
        *o++ = 'M';
        if (s.kind != 'M') {
            o = put_u(o, (uint64_t)s.k);
            *o++ = s.kind;
            o = put_u(o, (uint64_t)s.b);
            *o++ = 'M';
        }
        memcpy(o, "\t*\t0\t0\t", 7); o += 7;
        const std::string &ref = refseq[r];
        auto base = [&](int64_t p) -> char {
            double u = rng.uni();
            char c = ref[p];
            if (u < sp.sub_rate) return OTHER[c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3][rng.below(3)];
            if (u < sp.sub_rate + sp.n_rate) return 'N';
            return c;
        };
        int64_t p = s.start;
        for (int32_t j = 0; j < s.a; j++) *o++ = base(p++);
        if (s.kind == 'I') {
            for (int32_t j = 0; j < s.k; j++) *o++ = "ACGT"[rng.next() >> 62];
        } else if (s.kind == 'D') {
            p += s.k;
        }
        if (s.kind != 'M')
            for (int32_t j = 0; j < s.b; j++) *o++ = base(p++);
        memcpy(o, "\t*\n", 3); o += 3;
        buf.append(line.data(), o - line.data());
        if (buf.size() > (1u << 22)) {
            int rc = flush();
            if (rc) return rc;
        }
    }
    int rc = flush();
    if (rc) return rc;
    if (n_out) *n_out = N;
    return S2C_OK;
}
}  // namespace

static int s2c_synth_feed_impl(const s2c_synth_spec *spec, s2c_parser *p, int64_t *n_reads_out) {
    if (!spec || !p) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    return generate(*spec, [p](const char *b, size_t n) { return s2c_parser_feed(p, b, n); }, n_reads_out);
}
extern "C" int s2c_synth_feed(const s2c_synth_spec *spec, s2c_parser *p, int64_t *n_reads_out) {
    return s2c_guarded([&] { return s2c_synth_feed_impl(spec, p, n_reads_out); });
}

static int s2c_synth_write_impl(const s2c_synth_spec *spec, const char *path, int64_t *n_reads_out) {
    if (!spec || !path) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    size_t n = strlen(path);
    if (n >= 3 && strcmp(path + n - 3, ".gz") == 0) {
        // BGZF (the blocked gzip samtools / bgzip write: gzip members of <= 60000 text bytes,
        // each with a 'BC' extra field holding its size; 16 MB of text per host thread,
        // deflated at level 1): a valid .gz stream that zlib / gzip / Python read as one
        // file, and that s2c_parser_feed_file inflates block-parallel
        FILE *f = fopen(path, "wb");
        if (!f) return s2c_set_error(S2C_ERR_IO, std::string("cannot open ") + path);
        constexpr size_t BLK = (size_t)16 << 20, BGZF_IN = 60000;
        unsigned hw = std::thread::hardware_concurrency();
        const size_t nt = std::max<size_t>(1, std::min<unsigned>(hw ? hw : 1, 16));
        std::vector<std::string> in(1);
        auto deflate_all = [&]() -> int {
            std::vector<std::string> out(in.size());
            std::vector<int> ok(in.size(), 1);
            auto work = [&](size_t i) {
                z_stream z{};
                if (deflateInit2(&z, 1, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) { ok[i] = 0; return; }
                std::string &o = out[i];
                for (size_t a = 0; a < in[i].size(); a += BGZF_IN) {
                    const size_t n = std::min(BGZF_IN, in[i].size() - a), h = o.size();
                    const size_t cap = deflateBound(&z, n);
                    o.resize(h + 18 + cap + 8);
                    deflateReset(&z);
                    z.next_in = (Bytef *)in[i].data() + a;
                    z.avail_in = (uInt)n;
                    z.next_out = (Bytef *)&o[h + 18];
                    z.avail_out = (uInt)cap;
                    if (deflate(&z, Z_FINISH) != Z_STREAM_END) { ok[i] = 0; break; }
                    const size_t total = 18 + z.total_out + 8;
                    if (total > 65536) { ok[i] = 0; break; }
                    const unsigned char hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                                                   (unsigned char)((total - 1) & 0xff), (unsigned char)((total - 1) >> 8)};
                    memcpy(&o[h], hdr, 18);
                    const uint32_t crc = (uint32_t)crc32(0L, (const Bytef *)in[i].data() + a, (uInt)n), isz = (uint32_t)n;
                    for (int b = 0; b < 4; b++) {
                        o[h + 18 + z.total_out + b] = (char)(crc >> (8 * b));
                        o[h + 18 + z.total_out + 4 + b] = (char)(isz >> (8 * b));
                    }
                    o.resize(h + total);
                }
                deflateEnd(&z);
            };
            std::vector<std::thread> th;
            for (size_t i = 0; i < in.size(); i++)
                if (!in[i].empty()) th.emplace_back(work, i);
            for (auto &t : th) t.join();
            for (size_t i = 0; i < in.size(); i++) {
                if (in[i].empty()) continue;
                if (!ok[i]) return s2c_set_error(S2C_ERR_IO, "deflate failed");
                if (fwrite(out[i].data(), 1, out[i].size(), f) != out[i].size()) return s2c_set_error(S2C_ERR_IO, "write failed");
            }
            in.assign(1, std::string());
            return S2C_OK;
        };
        int rc = generate(*spec, [&](const char *b, size_t k) {
            in.back().append(b, k);
            if (in.back().size() >= BLK) {
                if (in.size() == nt) return deflate_all();
                in.emplace_back();
            }
            return S2C_OK;
        }, n_reads_out);
        if (!rc) rc = deflate_all();
        static const unsigned char eof_block[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0, 0x1b, 0,
                                                    3, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // BGZF end-of-file marker
        if (!rc && fwrite(eof_block, 1, sizeof(eof_block), f) != sizeof(eof_block)) rc = s2c_set_error(S2C_ERR_IO, "write failed");
        fclose(f);
        return rc;
    }
    FILE *f = fopen(path, "wb");
    if (!f) return s2c_set_error(S2C_ERR_IO, std::string("cannot open ") + path);
    int rc = generate(*spec, [f](const char *b, size_t k) {
        return fwrite(b, 1, k, f) == k ? S2C_OK : s2c_set_error(S2C_ERR_IO, "write failed");
    }, n_reads_out);
    fclose(f);
    return rc;
}
extern "C" int s2c_synth_write(const s2c_synth_spec *spec, const char *path, int64_t *n_reads_out) {
    return s2c_guarded([&] { return s2c_synth_write_impl(spec, path, n_reads_out); });
}

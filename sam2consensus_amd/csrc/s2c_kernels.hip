// s2c_kernels.hip — HIP kernels for gfx950 (MI355X) + their C-ABI launchers.
//
// The reference's hot path (sam2consensus.py) is a per-base Python dict increment
// (:210-218), an insertion motif aggregation (:256-311) and a per-position threshold
// vote (:232-253, :344-389).  Here it is four stream-ordered stages over the packed
// batch built by s2c_host.cpp:
//
//   k_zero_tiles / k_pileup   (2) CIGAR expansion + per-tile LDS histograms → counts[6][L]
//   k_ins_*                   (3) insertion hash table, column counts, insertion vote
//   k_consensus               (4) one pass per position for all thresholds: closed-form
//                                 Geneious vote, IUPAC LUT, min-depth / fill, stats
//   k_scan / k_assemble       device FASTA body assembly (block scan + byte scatter)
//
// Everything is integer counting; the single floating-point operation is the
// reference's `cov_nucs < t*coverage` (:362, :376), evaluated as
// (double)S < t * (double)cov — built with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/s2c.h"

int s2c_set_error(int code, const std::string &msg);

namespace {

constexpr int WG = 256;
constexpr uint32_t NSYM = S2C_NSYM;

// ----------------------------------------------------------------- IUPAC table (:317-329)
// mask bit i = symbol "-ACGNT"[i]; value = output char, 0xFF where the reference's amb
// dict has no key (mask 0 → KeyError '' ; {A,C,G,N,T} → KeyError 'ACGNT').
struct AmbTable {
    uint8_t v[64];
    constexpr AmbTable() : v{} {
        for (int m = 0; m < 64; m++) {
            const bool dash = m & 1, n = m & 16;
            const int b = ((m >> 1) & 1) | (((m >> 2) & 1) << 1) | (((m >> 3) & 1) << 2) | (((m >> 5) & 1) << 3);
            // b: bit0 A, bit1 C, bit2 G, bit3 T
            const char iupac[16] = {0, 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};
            uint8_t c = 0;
            if (m == 0) c = 0xFF;
            else if (b == 0) c = (dash && n) ? 'n' : (dash ? '-' : 'N');
            else if (b == 15) c = (n && !dash) ? 0xFF : 'N';
            else {
                c = (uint8_t)iupac[b];
                if (dash || n) c = (uint8_t)(c + ('a' - 'A'));
            }
            v[m] = c;
        }
    }
};
constexpr AmbTable AMB{};
__constant__ uint8_t c_amb[64] = {
#define E(i) AMB.v[i]
    E(0), E(1), E(2), E(3), E(4), E(5), E(6), E(7), E(8), E(9), E(10), E(11), E(12), E(13), E(14), E(15),
    E(16), E(17), E(18), E(19), E(20), E(21), E(22), E(23), E(24), E(25), E(26), E(27), E(28), E(29), E(30), E(31),
    E(32), E(33), E(34), E(35), E(36), E(37), E(38), E(39), E(40), E(41), E(42), E(43), E(44), E(45), E(46), E(47),
    E(48), E(49), E(50), E(51), E(52), E(53), E(54), E(55), E(56), E(57), E(58), E(59), E(60), E(61), E(62), E(63)
#undef E
};

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint32_t nibble(const uint32_t *__restrict__ w, uint64_t idx) {
    return (w[idx >> 3] >> ((idx & 7) * 4)) & 15u;
}

// Closed form of the group-sort vote (proven equal to :241-251 +
// :359-366 in tests/test_oracle.py): symbol i is taken iff c_i != 0 and the sum of the
// counts strictly greater than c_i is < t·cov (fp64 product, exact integer compare).
template <typename T>
__device__ __forceinline__ void greater_sums(const T (&c)[NSYM], int64_t (&s)[NSYM]) {
#pragma unroll
    for (int i = 0; i < (int)NSYM; i++) {
        int64_t a = 0;
#pragma unroll
        for (int j = 0; j < (int)NSYM; j++) a += (c[j] > c[i]) ? (int64_t)c[j] : 0;
        s[i] = a;
    }
}
template <typename T>
__device__ __forceinline__ uint32_t vote_mask(const T (&c)[NSYM], const int64_t (&s)[NSYM], double tc) {
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < (int)NSYM; i++) m |= ((c[i] != 0) && ((double)s[i] < tc)) ? (1u << i) : 0u;
    return m;
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
    return x;
}
// table entry: {key+1 (0 = empty), maxlen, colbase, unused}
__device__ __forceinline__ uint32_t ins_find(const uint32_t *__restrict__ tab, uint32_t cap, uint32_t key) {
    uint32_t h = hash32(key) & (cap - 1);
    for (uint32_t probe = 0; probe < cap; probe++) {
        uint32_t k = tab[4 * h];
        if (k == key + 1) return h;
        if (k == 0) return 0xFFFFFFFFu;
        h = (h + 1) & (cap - 1);
    }
    return 0xFFFFFFFFu;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ======================================================================= (2) pileup
// One workgroup per work item = (tile [a,b) of one reference, read range [lo,hi) +
// long-read extras).  Counts for the tile accumulate in LDS as [6][tile] u32 (symbol-
// major: consecutive lanes hit consecutive banks), each wave expanding one read's CIGAR
// at a time — lane j handles seqout char j (+64…).  Only the seqout window inside the
// tile is visited, so reads straddling tile edges cost no extra counting.  Tiles that
// hold the whole depth write their histogram with plain coalesced stores (no HBM
// atomics); tiles split into read chunks (ultra-deep, C4) add theirs atomically into a
// range zeroed by k_zero_tiles.
__global__ void k_zero_tiles(const s2c_dev d) {
    const uint32_t *it = d.items + (size_t)blockIdx.x * S2C_ITEM_WORDS;
    if ((it[6] & 3u) != 3u) return;  // atomic tile, first chunk
    const uint32_t a = it[0], n = it[1] - it[0];
    for (uint32_t c = 0; c < NSYM; c++)
        for (uint32_t i = threadIdx.x; i < n; i += WG) d.counts[(size_t)c * d.padded_len + a + i] = 0;
}

// Staged-chunk limits.  The host classifies a piece as "long" (per-tile extras, read
// straight from HBM) when its span > 1024 or it has > 64 op words, so every short read
// fits a chunk (≤ 129 base words, ≤ 64 ops).
constexpr int CH_READS = WG;      // reads per chunk (< 1023: a 10-bit field never overflows)
constexpr int CH_WORDS = 4096;    // 16 KiB of packed bases per chunk
constexpr int CH_OPS = 1024;      // op words per chunk
constexpr int MAX_WIN = 32;       // 64-position windows per tile (tile ≤ 2048 positions)

struct __attribute__((aligned(16))) ChunkLds {
    uint4 meta[CH_READS];         // x: start - a (signed), y: span | drop<<31,
                                  // z: op offset | nops<<16 | single-M<<31, w: base word offset
    uint32_t ops[CH_OPS];
    uint32_t bases[CH_WORDS];
    uint32_t win_lo[MAX_WIN], win_hi[MAX_WIN];
    uint32_t tot_words, tot_ops;
};

// code of seqout index j (lane-varying) of a read whose ops/bases sit at (ops, bases)
__device__ __forceinline__ uint32_t seqout_code(const uint32_t *ops, uint32_t nops, const uint32_t *bases, int j,
                                                bool mine) {
    uint32_t code = 15;
    int k = 0, q = 0;
    for (uint32_t o = 0; o < nops; o++) {
        const uint32_t w = uni(ops[o]);
        const int len = (int)(w >> 1);
        const bool m = (w & 1u) == 0;
        if (mine && (unsigned)(j - k) < (unsigned)len) {
            if (m) {
                const uint32_t qi = (uint32_t)(q + j - k);
                code = (bases[qi >> 3] >> ((qi & 7) * 4)) & 15u;
            } else {
                code = 0;
            }
        }
        k += len;
        q += m ? len : 0;
    }
    return code;
}

// One workgroup per work item = (tile [a,b) of one reference, read range [lo,hi) + long-read
// extras).  Position-major: lane ℓ of a wave owns tile position 64·w + ℓ of each of its
// windows and keeps its six counts in registers — a u64 of 10-bit fields per window
// (+1 << 10·code per covering read, no atomics), folded into u32 counts after every chunk.
// Reads are staged through LDS in chunks of ≤256 (coalesced global loads of their
// metadata, op words and packed bases), so a read costs no HBM round trip when its
// windows are visited.  Only windows inside the tile are visited: a read straddling a
// tile edge costs one extra window visit, never an extra count.  Tiles holding the whole
// depth store counts with plain coalesced stores; chunked (ultra-deep) tiles add them.
template <int WPW>
__global__ __launch_bounds__(WG) void k_pileup(const s2c_dev d) {
    __shared__ ChunkLds S;
    const uint32_t *it = d.items + (size_t)blockIdx.x * S2C_ITEM_WORDS;
    const uint32_t a = uni(it[0]), b = uni(it[1]), lo = uni(it[2]), hi = uni(it[3]);
    const uint32_t xlo = uni(it[4]), xhi = uni(it[5]), flags = uni(it[6]);
    const int n = (int)(b - a), nw = (n + 63) >> 6;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const int wbase = (int)uni(tid >> 6) * WPW;
    uint64_t acc[WPW];
    uint32_t cnt[WPW][NSYM];
#pragma unroll
    for (int wi = 0; wi < WPW; wi++) {
        acc[wi] = 0;
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) cnt[wi][c] = 0;
    }
    auto fold = [&]() {
#pragma unroll
        for (int wi = 0; wi < WPW; wi++) {
#pragma unroll
            for (uint32_t c = 0; c < NSYM; c++) cnt[wi][c] += (uint32_t)(acc[wi] >> (10 * c)) & 1023u;
            acc[wi] = 0;
        }
    };
    for (uint32_t r0 = lo; r0 < hi;) {
        // ---- stage one chunk: metadata, per-window read ranges, ops, bases ----
        if (tid < MAX_WIN) { S.win_lo[tid] = 0xFFFFFFFFu; S.win_hi[tid] = 0; }
        const uint32_t bw0 = uni(d.rd_base[r0]), op0 = uni(d.rd_op[r0]);
        const uint32_t rr = r0 + tid;
        const bool in = rr < hi;
        uint32_t bend = 0, oend = 0;
        if (in) { bend = d.rd_base[rr + 1]; oend = d.rd_op[rr + 1]; }
        const bool ok = in && bend - bw0 <= (uint32_t)CH_WORDS && oend - op0 <= (uint32_t)CH_OPS;
        const uint32_t nr = (uint32_t)__syncthreads_count(ok);
        if (tid < nr) {
            const uint32_t sp = d.rd_span[rr], o = d.rd_op[rr], bb = d.rd_base[rr];
            const int s_rel = (int)(d.rd_pos[rr] - a);
            const uint32_t nops = oend - o;
            const bool single = nops == 1 && (d.ops[o] & 1u) == 0;
            S.meta[tid] = make_uint4((uint32_t)s_rel, sp, (o - op0) | (nops << 16) | (single ? 0x80000000u : 0u),
                                     bb - bw0);
            const int e = s_rel + (int)(sp & 0x7FFFFFFFu);
            if (e > 0 && s_rel < n) {
                const int wf = (s_rel > 0 ? s_rel : 0) >> 6, wl = ((e < n ? e : n) - 1) >> 6;
                for (int i = wf; i <= wl; i++) { atomicMin(&S.win_lo[i], tid); atomicMax(&S.win_hi[i], tid + 1); }
            }
            if (tid == nr - 1) { S.tot_words = bend - bw0; S.tot_ops = oend - op0; }
        }
        __syncthreads();
        const uint32_t nwd = S.tot_words, nop = S.tot_ops;
        for (uint32_t i = tid; i < nop; i += WG) S.ops[i] = d.ops[op0 + i];
        {
            const uint32_t *src = d.bases + bw0;
            uint32_t i = tid;
            for (; i + 3 * WG < nwd; i += 4 * WG) {
                const uint32_t v0 = src[i], v1 = src[i + WG], v2 = src[i + 2 * WG], v3 = src[i + 3 * WG];
                S.bases[i] = v0; S.bases[i + WG] = v1; S.bases[i + 2 * WG] = v2; S.bases[i + 3 * WG] = v3;
            }
            for (; i < nwd; i += WG) S.bases[i] = src[i];
        }
        __syncthreads();
        // ---- count: every read overlapping one of this wave's windows ----
        if (wbase < nw) {
            uint32_t rlo = 0xFFFFFFFFu, rhi = 0;
#pragma unroll
            for (int wi = 0; wi < WPW; wi++)
                if (wbase + wi < nw) {
                    rlo = min(rlo, S.win_lo[wbase + wi]);
                    rhi = max(rhi, S.win_hi[wbase + wi]);
                }
            rlo = uni(rlo);
            rhi = uni(rhi);
            for (uint32_t t = rlo; t < rhi; t++) {
                const uint4 m = S.meta[t];
                const int s_rel = (int)uni(m.x);
                const uint32_t sp = uni(m.y), oo = uni(m.z), bo = uni(m.w);
                const int span = (int)(sp & 0x7FFFFFFFu);
                const bool drop = (sp >> 31) != 0;
#pragma unroll
                for (int wi = 0; wi < WPW; wi++) {
                    const int w0 = (wbase + wi) * 64;
                    if (wbase + wi >= nw || s_rel >= w0 + 64 || s_rel + span <= w0) continue;
                    const int j = w0 + (int)lane - s_rel;
                    const bool mine = (unsigned)j < (unsigned)span && w0 + (int)lane < n;
                    uint32_t code = 15;
                    if (oo >> 31) {   // single M op: seqout index = query index
                        if (mine) code = (S.bases[bo + ((uint32_t)j >> 3)] >> ((j & 7) * 4)) & 15u;
                    } else {
                        code = seqout_code(S.ops + (oo & 0xFFFFu), (oo >> 16) & 0x7FFFu, S.bases + bo, j, mine);
                    }
                    if (mine && !(drop && code == 0)) acc[wi] += 1ull << (10 * code);
                }
            }
        }
        fold();
        __syncthreads();
        r0 += nr;
    }
    // ---- long reads overlapping this tile (rare): metadata/ops/bases straight from HBM ----
    for (uint32_t x = xlo; x < xhi; x++) {
        const uint32_t r = uni(d.extras[x]);
        const int s_rel = (int)(uni(d.rd_pos[r]) - a);
        const uint32_t sp = uni(d.rd_span[r]);
        const int span = (int)(sp & 0x7FFFFFFFu);
        const bool drop = (sp >> 31) != 0;
        const uint32_t o = uni(d.rd_op[r]), nops = uni(d.rd_op[r + 1]) - o;
        const uint32_t *bw = d.bases + uni(d.rd_base[r]);
#pragma unroll
        for (int wi = 0; wi < WPW; wi++) {
            const int w0 = (wbase + wi) * 64;
            if (wbase + wi >= nw || s_rel >= w0 + 64 || s_rel + span <= w0) continue;
            const int j = w0 + (int)lane - s_rel;
            const bool mine = (unsigned)j < (unsigned)span && w0 + (int)lane < n;
            const uint32_t code = seqout_code(d.ops + o, nops, bw, j, mine);
            if (mine && !(drop && code == 0)) acc[wi] += 1ull << (10 * code);
        }
        if (((x - xlo) & 255u) == 255u) fold();
    }
    fold();
    // ---- tile counts → HBM (symbol-major, coalesced) ----
#pragma unroll
    for (int wi = 0; wi < WPW; wi++) {
        const int pl = (wbase + wi) * 64 + (int)lane;
        if (wbase + wi >= nw || pl >= n) continue;
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) {
            uint32_t *dst = d.counts + (size_t)c * d.padded_len + a + pl;
            if (flags & 1u) {
                if (cnt[wi][c]) atomicAdd(dst, cnt[wi][c]);
            } else {
                *dst = cnt[wi][c];
            }
        }
    }
}

// ======================================================================= (3) insertions
// (:264-271) motif multiplicities and (:284-287) per-column sums are additive, so the
// column counts are accumulated straight from the events: column c of key k gets +1 at
// motif[c] for every event at k with len > c.  The hash table maps key → slot with the
// longest motif (:278-281) and a column base from a wave-aggregated bump allocator.
__global__ void k_ins_insert(const s2c_dev d) {
    const uint32_t e = blockIdx.x * WG + threadIdx.x;
    if (e >= d.n_ins) return;
    const uint32_t key = d.ins_key[e];
    const uint32_t len = d.ins_off[e + 1] - d.ins_off[e];
    const uint32_t cap = (uint32_t)d.ins_cap;
    uint32_t h = hash32(key) & (cap - 1);
    for (uint32_t probe = 0; probe < cap; probe++) {
        const uint32_t prev = atomicCAS(&d.ins_table[4 * h], 0u, key + 1);
        if (prev == 0u || prev == key + 1) {
            atomicMax(&d.ins_table[4 * h + 1], len);
            break;
        }
        h = (h + 1) & (cap - 1);
    }
    atomicOr(&d.ins_bits[key >> 5], 1u << (key & 31));
}

__global__ void k_ins_alloc(const s2c_dev d) {
    const uint32_t s = blockIdx.x * WG + threadIdx.x;
    const uint32_t cap = (uint32_t)d.ins_cap;
    const uint32_t need = (s < cap && d.ins_table[4 * s] != 0u) ? d.ins_table[4 * s + 1] : 0u;
    // wave-inclusive scan of `need`, one atomic per wave
    uint32_t x = need;
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    const uint32_t total = __shfl(x, 63, 64);
    uint32_t base = 0;
    if (lane == 63 && total) base = atomicAdd(&d.scalars[0], total);
    base = __shfl(base, 63, 64);
    if (need) d.ins_table[4 * s + 2] = base + x - need;
}

__global__ void k_ins_scatter(const s2c_dev d) {
    const uint32_t e = blockIdx.x * WG + threadIdx.x;
    if (e >= d.n_ins) return;
    const uint32_t key = d.ins_key[e];
    const uint32_t o0 = d.ins_off[e], o1 = d.ins_off[e + 1];
    const uint32_t slot = ins_find(d.ins_table, (uint32_t)d.ins_cap, key);
    if (slot == 0xFFFFFFFFu) return;
    const uint32_t cb = d.ins_table[4 * slot + 2];
    for (uint32_t c = 0; o0 + c < o1; c++)
        atomicAdd(&d.ins_cols[(size_t)(cb + c) * NSYM + nibble(d.ins_bases, o0 + c)], 1u);
}

// (:290-309, :370-385) per key: '-' = cov[key] − Σ column (may be ≤ 0), vote each column
// for every threshold; emitted chars (vote != "-") are compacted per threshold.
__global__ void k_ins_vote(const s2c_dev d) {
    const uint32_t s = blockIdx.x * WG + threadIdx.x;
    const uint32_t cap = (uint32_t)d.ins_cap;
    if (s >= cap) return;
    const uint32_t k1 = d.ins_table[4 * s];
    const int T = d.n_thr;
    if (k1 == 0u) return;
    const uint32_t p = k1 - 1;
    uint64_t cov = 0;
    for (uint32_t c = 0; c < NSYM; c++) cov += d.counts[(size_t)c * d.padded_len + p];
    const bool called = cov > 0 && (int64_t)cov >= (int64_t)d.min_depth;
    const uint32_t ml = d.ins_table[4 * s + 1], cb = d.ins_table[4 * s + 2];
    // the key's reference: the consensus block containing p (blocks sorted by g_begin)
    int64_t lo = 0, hi = d.n_blocks - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (d.blocks[mid * S2C_BLOCK_WORDS] <= p) lo = mid; else hi = mid - 1;
    }
    const uint32_t ref = d.blocks[lo * S2C_BLOCK_WORDS + 2];
    for (int t = 0; t < T; t++) {
        uint32_t emitted = 0;
        if (called) {
            const double tc = d.thresholds[t] * (double)cov;
            for (uint32_t c = 0; c < ml; c++) {
                const uint32_t *col = d.ins_cols + (size_t)(cb + c) * NSYM;
                int64_t v[NSYM];
                int64_t tot = 0;
#pragma unroll
                for (uint32_t j = 0; j < NSYM; j++) { v[j] = col[j]; tot += v[j]; }
                v[0] = (int64_t)cov - tot;   // :294 (the column's own '-' count is in the sum)
                int64_t gs[NSYM];
                greater_sums(v, gs);
                const uint8_t ch = c_amb[vote_mask(v, gs, tc)];
                if (ch == 0xFF) {
                    atomicOr(&d.scalars[1], 1u);
                    atomicAdd((unsigned long long *)&d.stats[((size_t)ref * T + t) * 4 + 3], 1ull);
                    continue;
                }
                if (ch != '-') d.ins_chr[(size_t)t * d.n_ins_bases + cb + emitted++] = ch;
            }
        }
        d.ins_cnt[(size_t)t * cap + s] = emitted;
    }
}

__device__ __forceinline__ uint32_t ins_emitted(const s2c_dev &d, uint32_t p, int t, uint32_t *slot_out) {
    if (!(d.ins_bits[p >> 5] >> (p & 31) & 1u)) return 0;
    const uint32_t s = ins_find(d.ins_table, (uint32_t)d.ins_cap, p);
    if (s == 0xFFFFFFFFu) return 0;
    *slot_out = s;
    return d.ins_cnt[(size_t)t * d.ins_cap + s];
}

// ======================================================================= (4) consensus
// One workgroup per block (≤1024 positions of one ref); 4 positions per thread.
// Per position, the 6 counts are read once and voted for every threshold.
// Per (ref, t): sumcov (:357,:385), len and non-'-' chars of the record (:395-396).
template <typename T>
__device__ __forceinline__ T block_sum(T v, T *sh) {
    v = wave_sum(v);
    const uint32_t w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    T r = 0;
#pragma unroll
    for (int i = 0; i < WG / 64; i++) r += sh[i];
    return r;
}

__global__ __launch_bounds__(WG) void k_consensus(const s2c_dev d) {
    __shared__ uint64_t sh[WG / 64];
    const uint32_t *blk = d.blocks + (size_t)blockIdx.x * S2C_BLOCK_WORDS;
    const uint32_t g0 = uni(blk[0]), g1 = uni(blk[1]), ref = uni(blk[2]);
    const int T = d.n_thr;
    // positions handled by this thread
    uint32_t cnt[4][NSYM];
    uint64_t cov[4];
    int64_t gs[4][NSYM];
    bool valid[4], called[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t p = g0 + threadIdx.x + j * WG;
        valid[j] = p < g1;
        cov[j] = 0;
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) {
            cnt[j][c] = valid[j] ? d.counts[(size_t)c * d.padded_len + p] : 0u;
            cov[j] += cnt[j][c];
        }
        called[j] = cov[j] > 0 && (int64_t)cov[j] >= (int64_t)d.min_depth;
        greater_sums(cnt[j], gs[j]);
    }
    for (int t = 0; t < T; t++) {
        const double thr = d.thresholds[t];
        uint64_t len = 0, nondash = 0, sumcov = 0, nerr = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (!valid[j]) continue;
            const uint32_t p = g0 + threadIdx.x + j * WG;
            uint8_t code = S2C_CODE_FILL;
            if (called[j]) {
                const uint8_t ch = c_amb[vote_mask(cnt[j], gs[j], thr * (double)cov[j])];
                uint32_t slot;
                const uint32_t ne = ins_emitted(d, p, t, &slot);
                nerr += ch == 0xFF;
                code = ch;
                len += 1 + ne;
                nondash += (ch != '-') + ne;
                sumcov += cov[j] * (1 + ne);
            } else {
                len += (uint32_t)d.fill_len;
                nondash += (uint32_t)d.fill_nondash;
                sumcov += cov[j];
            }
            d.codes[(size_t)t * d.padded_len + p] = code;
        }
        len = block_sum(len, sh);
        nondash = block_sum(nondash, sh);
        sumcov = block_sum(sumcov, sh);
        nerr = block_sum(nerr, sh);
        if (threadIdx.x == 0) {
            uint64_t *st = d.stats + ((size_t)ref * T + t) * 4;
            atomicAdd((unsigned long long *)&st[0], (unsigned long long)sumcov);
            atomicAdd((unsigned long long *)&st[1], (unsigned long long)len);
            atomicAdd((unsigned long long *)&st[2], (unsigned long long)nondash);
            if (nerr) {
                atomicAdd((unsigned long long *)&st[3], (unsigned long long)nerr);
                atomicOr(&d.scalars[1], 1u);
            }
            d.blk_len[(size_t)t * d.n_blocks + blockIdx.x] = len;
        }
    }
}

// ======================================================================= assembly
// Exclusive scan of blk_len[T*n_blocks] (one workgroup, 1024 threads, chunked).
__global__ __launch_bounds__(1024) void k_scan(uint64_t *v, int64_t n) {
    __shared__ uint64_t sh[1024];
    const int64_t per = (n + 1023) / 1024;
    const int64_t b = threadIdx.x * per, e = (b + per < n) ? b + per : n;
    uint64_t s = 0;
    for (int64_t i = b; i < e; i++) s += v[i];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint64_t y = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0;
        __syncthreads();
        sh[threadIdx.x] += y;
        __syncthreads();
    }
    uint64_t run = sh[threadIdx.x] - s;
    for (int64_t i = b; i < e; i++) {
        const uint64_t x = v[i];
        v[i] = run;
        run += x;
    }
    if (threadIdx.x == 1023) v[n] = sh[1023];
}

// grid = n_blocks × T.  Record body of (ref, t) = concatenation over its positions of
// fill (uncalled) or the vote char followed by the emitted insertion chars (:367-389).
__global__ __launch_bounds__(WG) void k_assemble(const s2c_dev d) {
    __shared__ uint64_t sh[WG];
    const uint32_t bi = blockIdx.x;
    const int t = (int)blockIdx.y;
    const uint32_t *blk = d.blocks + (size_t)bi * S2C_BLOCK_WORDS;
    const uint32_t g0 = uni(blk[0]), g1 = uni(blk[1]);
    const uint64_t base = d.blk_len[(size_t)t * d.n_blocks + bi];
    const uint8_t *codes = d.codes + (size_t)t * d.padded_len;
    const uint32_t p0 = g0 + 4 * threadIdx.x;
    uint32_t lens[4], slots[4];
    uint64_t my = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t p = p0 + j;
        lens[j] = 0;
        slots[j] = 0xFFFFFFFFu;
        if (p < g1) {
            const uint8_t c = codes[p];
            lens[j] = c == S2C_CODE_FILL ? (uint32_t)d.fill_len : 1u + ins_emitted(d, p, t, &slots[j]);
        }
        my += lens[j];
    }
    // block exclusive scan of `my`
    uint64_t x = my;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint64_t wofs = 0;
    for (uint32_t i = 0; i < w; i++) wofs += sh[i];
    uint64_t off = base + wofs + x - my;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t p = p0 + j;
        if (p >= g1) break;
        const uint8_t c = codes[p];
        if (c == S2C_CODE_FILL) {
            for (int f = 0; f < d.fill_len; f++) d.out[off + f] = d.fill[f];
            off += (uint32_t)d.fill_len;
        } else {
            d.out[off++] = c;
            const uint32_t ne = lens[j] - 1;
            if (ne) {
                const uint32_t cb = d.ins_table[4 * slots[j] + 2];
                const uint8_t *src = d.ins_chr + (size_t)t * d.n_ins_bases + cb;
                for (uint32_t i = 0; i < ne; i++) d.out[off++] = src[i];
            }
        }
    }
}

inline int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return S2C_OK;
    return s2c_set_error(S2C_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + WG - 1) / WG); }

}  // namespace

// ======================================================================= C-ABI
extern "C" int s2c_workspace_sizes(const s2c_batch_info *info, int32_t n_thr, s2c_ws_sizes *o) {
    if (!info || !o || n_thr <= 0) return s2c_set_error(S2C_ERR_ARG, "bad workspace query");
    const int64_t L = info->padded_len, T = n_thr;
    int64_t cap = 64;
    while (cap < 2 * info->n_ins) cap <<= 1;
    const int64_t nib = info->n_ins_bases > 0 ? info->n_ins_bases : 1;
    o->counts = NSYM * L * 4;
    o->ins_cap = cap;
    o->ins_table = cap * 16;
    o->ins_cols = nib * NSYM * 4;
    o->ins_cnt = T * cap * 4;
    o->ins_chr = T * nib;
    o->ins_bits = (L / 32 + 2) * 4;
    o->scalars = 64;
    o->codes = T * L;
    o->blk_len = (T * info->n_blocks + 1) * 8;
    o->stats = info->n_refs * T * 32;
    return S2C_OK;
}

static int check_dev(const s2c_dev *d) {
    if (!d) return s2c_set_error(S2C_ERR_ARG, "s2c_dev is NULL");
    if (d->n_thr <= 0) return s2c_set_error(S2C_ERR_ARG, "no thresholds");
    if (d->tile_max <= 0 || d->tile_max > 64 * MAX_WIN) return s2c_set_error(S2C_ERR_ARG, "tile_max out of range");
    if (d->padded_len <= 0 || d->padded_len >= ((int64_t)1 << 32)) return s2c_set_error(S2C_ERR_ARG, "bad padded_len");
    if (d->ins_cap <= 0 || (d->ins_cap & (d->ins_cap - 1))) return s2c_set_error(S2C_ERR_ARG, "ins_cap not pow2");
    if (d->n_items > 0 && (!d->items || !d->counts)) return s2c_set_error(S2C_ERR_ARG, "missing pileup buffers");
    if (d->n_ins > 0 && (!d->ins_key || !d->ins_off || !d->ins_bases || !d->ins_table || !d->ins_cols))
        return s2c_set_error(S2C_ERR_ARG, "missing insertion buffers");
    return S2C_OK;
}

extern "C" int s2c_pileup(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    if (d->n_items == 0) return S2C_OK;
    hipStream_t s = (hipStream_t)stream;
    k_zero_tiles<<<(unsigned)d->n_items, WG, 0, s>>>(*d);
    const unsigned g = (unsigned)d->n_items;
    if (d->tile_max <= 256) k_pileup<1><<<g, WG, 0, s>>>(*d);
    else if (d->tile_max <= 512) k_pileup<2><<<g, WG, 0, s>>>(*d);
    else if (d->tile_max <= 1024) k_pileup<4><<<g, WG, 0, s>>>(*d);
    else k_pileup<8><<<g, WG, 0, s>>>(*d);
    return hip_check(hipGetLastError(), "k_pileup");
}

extern "C" int s2c_insertions(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    rc = hip_check(hipMemsetAsync(d->scalars, 0, 64, s), "memset scalars");
    if (rc) return rc;
    rc = hip_check(hipMemsetAsync(d->ins_bits, 0, (size_t)(d->padded_len / 32 + 2) * 4, s), "memset ins_bits");
    if (rc) return rc;
    // stats are accumulated by the insertion vote (errors) and then by the consensus
    rc = hip_check(hipMemsetAsync(d->stats, 0, (size_t)d->n_refs * d->n_thr * 32, s), "memset stats");
    if (rc || d->n_ins == 0) return rc;
    rc = hip_check(hipMemsetAsync(d->ins_table, 0, (size_t)d->ins_cap * 16, s), "memset ins_table");
    if (rc) return rc;
    rc = hip_check(hipMemsetAsync(d->ins_cols, 0, (size_t)d->n_ins_bases * NSYM * 4, s), "memset ins_cols");
    if (rc) return rc;
    k_ins_insert<<<grid_for(d->n_ins), WG, 0, s>>>(*d);
    k_ins_alloc<<<grid_for(d->ins_cap), WG, 0, s>>>(*d);
    k_ins_scatter<<<grid_for(d->n_ins), WG, 0, s>>>(*d);
    k_ins_vote<<<grid_for(d->ins_cap), WG, 0, s>>>(*d);
    return hip_check(hipGetLastError(), "k_ins_*");
}

extern "C" int s2c_consensus(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (d->n_blocks == 0) return S2C_OK;
    k_consensus<<<(unsigned)d->n_blocks, WG, 0, s>>>(*d);
    return hip_check(hipGetLastError(), "k_consensus");
}

extern "C" int s2c_assemble(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int64_t n = (int64_t)d->n_thr * d->n_blocks;
    k_scan<<<1, 1024, 0, s>>>(d->blk_len, n);
    if (d->n_blocks) k_assemble<<<dim3((unsigned)d->n_blocks, (unsigned)d->n_thr), WG, 0, s>>>(*d);
    return hip_check(hipGetLastError(), "k_assemble");
}

extern "C" int s2c_run(const s2c_dev *d, void *stream) {
    int rc;
    if ((rc = s2c_pileup(d, stream))) return rc;
    if ((rc = s2c_insertions(d, stream))) return rc;
    if ((rc = s2c_consensus(d, stream))) return rc;
    return s2c_assemble(d, stream);
}

extern "C" int s2c_device_error(const s2c_dev *d, void *stream, int *err_out) {
    if (!d || !err_out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    uint32_t v = 0;
    int rc = hip_check(hipMemcpyAsync(&v, d->scalars + 1, 4, hipMemcpyDeviceToHost, (hipStream_t)stream), "copy flags");
    if (rc) return rc;
    rc = hip_check(hipStreamSynchronize((hipStream_t)stream), "sync");
    if (rc) return rc;
    *err_out = v ? S2C_ERR_KEY : S2C_OK;
    return S2C_OK;
}

// s2c_tile.hip — per-tile pileup + insertion columns + vote (k_tile, k_consensus) and the
// C-ABI launchers of libs2c.so.
//
// The reference's hot path (sam2consensus.py) is a per-base Python dict increment
// (:210-218), an insertion motif aggregation (:256-311) and a per-position threshold vote
// (:232-253, :344-389).  Here the unit is the TILE (≤ 2048 positions of one reference):
//
//   k_reads (s2c_reads.hip)  parsecigar + maxdel per piece → run records; insertion events
//                            → per-tile hash tables
//   k_tile_dense (s2c_dense.hip)  shallow tiles without insertions: counts in registers,
//                            vote and body bytes straight from them
//   k_tile<NWP>              every other tile: bit-sliced counting of the runs covering each
//                            32-position word, then for a tile whose whole depth is in one
//                            work item the epilogue — its insertion layout built from its
//                            hash table (:262-294), the vote for all thresholds, IUPAC,
//                            min-depth / fill, insertion chars, tile statistics — counts
//                            never reach HBM; deep / general tiles add / store their counts
//   k_prep / k_consensus     deep / general tiles: zero their HBM counts, then the same
//                            insertion layout and vote with HBM columns
//
// Everything is integer counting; the single floating-point operation is the reference's
// `cov_nucs < t*coverage` (:362, :376), evaluated as (double)S < t * (double)cov — built
// with -ffp-contract=off.
#include <algorithm>

#include "s2c_common.h"

int s2c_launch_reads(const s2c_dev *d, hipStream_t s, bool all);
int s2c_launch_dense(const s2c_dev *d, hipStream_t s);

#ifdef S2C_PROF
// phase clocks of k_tile (diagnostic build `make prof`, scripts/prof_tile.py): Σ over sampled
// workgroups (one in 16, wave 0) of the s_memtime deltas of each phase; [15] = workgroups
__device__ unsigned long long g_tprof[16];
#define TPROF_MARK(i)                                                                                 \
    do {                                                                                              \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();                                   \
        if (threadIdx.x == 0 && (blockIdx.x & 15) == 0 && (i) > 0) atomicAdd(&g_tprof[(i)-1], _t - tprof_t); \
        tprof_t = _t;                                                                                 \
    } while (0)
extern "C" int s2c_prof_tile(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tprof), sizeof(g_tprof)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tprof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define TPROF_MARK(i) \
    do {              \
    } while (0)
#endif

namespace s2c {
namespace {

__constant__ uint8_t c_amb[64] = {
#define E(i) AMB.v[i]
    E(0), E(1), E(2), E(3), E(4), E(5), E(6), E(7), E(8), E(9), E(10), E(11), E(12), E(13), E(14), E(15),
    E(16), E(17), E(18), E(19), E(20), E(21), E(22), E(23), E(24), E(25), E(26), E(27), E(28), E(29), E(30), E(31),
    E(32), E(33), E(34), E(35), E(36), E(37), E(38), E(39), E(40), E(41), E(42), E(43), E(44), E(45), E(46), E(47),
    E(48), E(49), E(50), E(51), E(52), E(53), E(54), E(55), E(56), E(57), E(58), E(59), E(60), E(61), E(62), E(63)
#undef E
};

constexpr uint32_t PF = WG;                   // insertion keys per tile in k_tile's LDS (= S2C_EPI_KEYS)
constexpr uint32_t KMAX = S2C_TILE_MAX;       // keys per tile at most (one per position): k_consensus
constexpr int TILE_WORDS = S2C_TILE_MAX / 32;
constexpr int VT_ACC = 1 + 4 * VT_TMAX;       // LDS u64: position sumcov, {nondash, nerr, ins sumcov, ins len}[VT_TMAX]
static_assert(PF == S2C_EPI_KEYS, "k_tile key capacity");

// What the tile kernels read of s2c_dev, compact (kernel arguments stay in SGPRs).
// k_tile modes: the run (vote in the epilogue); counts stored (s2c_pileup_counts); counts
// added to running totals with the insertion tables cleared (a streamed batch) or kept for
// k_consensus (the last streamed batch)
constexpr uint32_t MODE_RUN = 0, MODE_STORE = 1, MODE_ADD = 2, MODE_ADD_KEEP = 3;

struct TileArgs {
    const uint32_t *rs, *runs, *bq, *bx, *tiles, *lp;
    uint32_t *ibkt, *ilong, *ilong_n;
    const double *thresholds;
    const uint8_t *fill;
    uint32_t *counts, *ins_cols;
    uint8_t *ins_chr;
    uint64_t *tile_stats, *blk_len;
    uint8_t *out;
    uint32_t padded_len, n_cols, n_tiles, kwin, chunk, n_qwords, runs_bytes, mode;   // MODE_* below
    int32_t n_thr, min_depth, fill_len, fill_nondash;
};

// Tile (t, tile)'s body region in `out`: a static slot — max(1, len(fill)) bytes per padded
// position plus the tile's insertion column slots; threshold t's region starts at t·stride.
template <class D>
__device__ __forceinline__ uint64_t body_stride(const D &d) {
    return (uint64_t)max(1, d.fill_len) * (uint64_t)d.padded_len + (uint64_t)d.n_cols;
}
template <class D>
__device__ __forceinline__ uint64_t body_slot(const D &d, uint32_t a, uint32_t cb0) {
    return (uint64_t)max(1, d.fill_len) * a + cb0;
}

// The tile record (16 words)
struct TileRec {
    uint32_t a, b, ref, flags, boff, bcap, loff, lcap, cb0, ccap, lp0, lp1, nev;
};
__device__ __forceinline__ TileRec tile_rec(const uint32_t *tiles, uint32_t t) {
    const uint4 *p = (const uint4 *)tiles + (size_t)t * (S2C_TILE_WORDS / 4);
    const uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];   // words 0-15 (13-19: the window)
    return {uni(v0.x), uni(v0.y), uni(v0.z), uni(v0.w), uni(v1.x), uni(v1.y), uni(v1.z), uni(v1.w),
            uni(v2.x), uni(v2.y), uni(v2.z), uni(v2.w), uni(v3.x)};
}

// symbol code ("-ACGNT" index) of query base q
__device__ __forceinline__ uint32_t base_code(const uint32_t *bq, const uint32_t *bx, uint64_t q) {
    const uint64_t w = q >> 5;
    const uint32_t sh = (uint32_t)(q & 31);
    const uint32_t p0 = (bq[2 * w] >> sh) & 1u, p1 = (bq[2 * w + 1] >> sh) & 1u, x = (bx[w] >> sh) & 1u;
    return x ? (p0 ? 0u : 4u) : ((p1 << 1 | p0) == 3u ? 5u : (p1 << 1 | p0) + 1u);
}

// ======================================================================= insertion layout
// A tile's insertion keys and columns from its hash table (k_reads): entry {key, count},
// key = position (11 bits) | length << 11 | 3-bit symbol codes << 16, and its long-motif
// events {position, length, query base}.  Keys sorted by position (a bitmap of the tile's
// words + ranks), per key the longest motif (:278-281) → column bases (a scan over keys),
// then every entry adds its count to column c's symbol (:284-287).  The table is left zero
// for the next run.  LDS arrays: bits/wrank [TILE_WORDS], klen/kpos [KCAP]; columns `cols`
// (LDS or the tile's HBM slots) and, if given, the column → key map `colkey`.
struct InsLayout {
    uint32_t nkeys, ncol;
};
template <uint32_t KCAP, bool HBMCOLS, class D>
__device__ InsLayout build_layout(const D &d, const TileRec &T, uint32_t t, uint32_t *bits, uint32_t *wrank,
                                  uint32_t *klen, uint4 *key, uint32_t *cols, uint16_t *colkey, uint32_t *scan) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t nwords = (T.b - T.a + 31) / 32;
    const uint32_t nlong = uni(d.ilong_n[t]);
    const uint4 *bk = (const uint4 *)d.ibkt + T.boff;
    const uint4 *lg = (const uint4 *)d.ilong + T.loff;
    // (1) key bitmap
    for (uint32_t e = tid; e < T.bcap; e += WG) {
        const uint4 v = bk[e];
        if (v.x | v.y) atomicOr(&bits[(v.x & 0x7FFu) >> 5], 1u << (v.x & 31u));
    }
    for (uint32_t e = tid; e < nlong; e += WG) {
        const uint32_t pos = lg[e].x;
        atomicOr(&bits[pos >> 5], 1u << (pos & 31u));
    }
    lds_sync();
    // (2) keys before each word
    if (wv == 0) {
        uint32_t carry = 0;
        for (uint32_t w0 = 0; w0 < nwords; w0 += 64) {
            const uint32_t w = w0 + lane;
            const uint32_t pc = w < nwords ? (uint32_t)__popc(bits[w]) : 0u;
            const uint32_t inc = __ockl_wfscan_add_u32(pc, true);
            if (w < nwords) wrank[w] = carry + inc - pc;
            carry += __shfl(inc, 63);
        }
        if (lane == 0) scan[8] = carry;
    }
    lds_sync();
    const uint32_t nkeys = scan[8];
    auto rank = [&](uint32_t pos) {
        return wrank[pos >> 5] + (uint32_t)__popc(bits[pos >> 5] & ((1u << (pos & 31u)) - 1u));
    };
    // (3) longest motif per key
    for (uint32_t e = tid; e < T.bcap; e += WG) {
        const uint4 v = bk[e];
        if (v.x | v.y) {
            const uint32_t pos = v.x & 0x7FFu, k = rank(pos);
            atomicMax(&klen[k], (v.x >> 11) & 31u);
            key[k].x = T.a + pos;
        }
    }
    for (uint32_t e = tid; e < nlong; e += WG) {
        const uint4 v = lg[e];
        const uint32_t k = rank(v.x);
        atomicMax(&klen[k], v.y);
        key[k].x = T.a + v.x;
    }
    lds_sync();
    // (4) column bases: exclusive scan of klen over keys (chunks of WG keys)
    uint32_t base = 0;
    for (uint32_t k0 = 0; k0 < nkeys; k0 += WG) {
        const uint32_t k = k0 + tid;
        const uint32_t l = k < nkeys ? klen[k] : 0u;
        const uint32_t inc = __ockl_wfscan_add_u32(l, true);
        if (lane == 63) scan[wv] = inc;
        lds_sync();
        const uint32_t wofs = (wv > 0 ? scan[0] : 0u) + (wv > 1 ? scan[1] : 0u) + (wv > 2 ? scan[2] : 0u);
        const uint32_t tot = scan[0] + scan[1] + scan[2] + scan[3];
        if (k < nkeys) {
            const uint32_t cb = base + wofs + inc - l;
            key[k].y = cb;
            key[k].z = l;
            key[k].w = 0;
            if (colkey)
                for (uint32_t c = 0; c < l; c++) colkey[cb + c] = (uint16_t)k;
        }
        base += tot;
        lds_sync();
    }
    const uint32_t ncol = base;
    // (5) column counts (:284-287); zero first when the columns are in HBM
    if constexpr (HBMCOLS) {
        for (uint32_t i = tid; i < ncol * NSYM; i += WG) cols[i] = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    for (uint32_t e = tid; e < T.bcap; e += WG) {
        const uint4 v = bk[e];
        if (v.x | v.y) {
            const uint32_t pos = v.x & 0x7FFu, len = (v.x >> 11) & 31u, k = rank(pos);
            const uint64_t m = ((uint64_t)v.x | ((uint64_t)v.y << 32)) >> 16;
            uint32_t *cc = cols + (size_t)key[k].y * NSYM;
            for (uint32_t c = 0; c < len; c++) atomicAdd(&cc[c * NSYM + ((m >> (3 * c)) & 7u)], v.z);
        }
    }
    for (uint32_t e = tid; e < nlong; e += WG) {
        const uint4 v = lg[e];
        const uint32_t k = rank(v.x);
        const uint64_t q = (uint64_t)v.z | ((uint64_t)v.w << 32);
        uint32_t *cc = cols + (size_t)key[k].y * NSYM;
        for (uint32_t c = 0; c < v.y; c++) atomicAdd(&cc[c * NSYM + base_code(d.bq, d.bx, q + c)], 1u);
    }
    // (6) leave the table zero for the next run
    for (uint32_t e = tid; e < T.bcap; e += WG) ((uint4 *)d.ibkt)[T.boff + e] = make_uint4(0, 0, 0, 0);
    if constexpr (HBMCOLS) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // atomics done before the readers
        __syncthreads();
    } else {
        lds_sync();
    }
    if (tid == 0) d.ilong_n[t] = 0;
    return {nkeys, ncol};
}

// ======================================================================= vote helpers
// Vote of one insertion column (:290-311) for up to 4 thresholds th[0..tn): counts v[6] of
// the column's motif symbols, the '-' count replaced by cov − Σ v (:294, signed: the
// column's own '-' count is in the sum); returns the 4 masks packed in bytes.
template <typename S, class V>
__device__ __forceinline__ uint32_t column_masks_t(const V &col, uint32_t cov, const double *th, int tn) {
    S v[NSYM], g[NSYM];
    S tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < NSYM; j++) { v[j] = (S)col[j]; tot += v[j]; }
    v[0] = (S)cov - tot;
    greater_sums(v, g);
    uint32_t m = 0;
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (u < tn) m |= vote_mask(v, g, th[u] * (double)cov) << (8 * u);
    return m;
}
template <class V>
__device__ __forceinline__ uint32_t column_masks(const V &col, uint32_t cov, const double *th, int tn) {
    uint32_t mx = cov;
#pragma unroll
    for (uint32_t j = 0; j < NSYM; j++) mx = max(mx, (uint32_t)col[j]);
    if (mx < (1u << 28)) return column_masks_t<int32_t>(col, cov, th, tn);   // |Σ| < 6·2^28 < 2^31
    return column_masks_t<int64_t>(col, cov, th, tn);
}

// LDS histogram of a tile: u16 counts in pairs, word s = 16·(word of 32) + i holds
// positions i (low half) and i + 16 (high half) of that word; one pad word per 16.
__device__ __forceinline__ uint32_t hslot(uint32_t s) { return s + (s >> 4); }
template <int NWP>
struct Hist {
    static constexpr int HP = 17 * NWP, CS = NSYM * HP + 8;
    static __device__ __forceinline__ uint32_t word(const uint32_t *h, uint32_t c, uint32_t s) { return h[c * HP + s]; }
    static __device__ __forceinline__ uint32_t get(const uint32_t *h, uint32_t c, uint32_t q) {
        return (word(h, c, hslot(((q >> 5) << 4) | (q & 15))) >> ((q & 16) ? 16 : 0)) & 0xFFFFu;
    }
    static __device__ __forceinline__ void add1(uint32_t *h, uint32_t c, uint32_t q, uint32_t v) {   // v ∈ {+1, −1}
        atomicAdd(h + c * HP + hslot(((q >> 5) << 4) | (q & 15)), (q & 16) ? (v << 16) : v);
    }
};

// ======================================================================= fast tile epilogue
// k_tile's epilogue (columns in LDS, ≤ PF keys, -f ≤ FILL_LDS bytes).  Per pass of ≤ 4
// thresholds and chunk of 512 positions:
//   A  the column votes (first chunk of a pass) and the position votes;
//   B  each position's body length per threshold (1 + its key's emitted insertion chars,
//      or len(fill)), a packed 16-bit row scan (DPP) per threshold, wave totals, the tile
//      statistics into LDS;
//   C  byte offsets → body bytes; the last chunk writes the tile statistics.
// A thread takes positions q and q + 16 of one 32-position word: their u16 counts share a
// histogram word.  The vote is the closed form (S9), evaluated in full only in waves
// holding a called position whose largest count is not a strict majority reaching t·cov of
// the pass's largest threshold; elsewhere the char is that symbol's for every threshold.
template <uint32_t ICOL>
struct FastLds {
    uint4 key[PF];                     // keys {position, column base, columns, 0}
    uint32_t klen[PF];                 // longest motif per key (layout build)
    unsigned long long acc[VT_ACC];
    alignas(16) uint32_t fsum[2][VT_TMAX][WG / 64];   // body-length scan: wave totals, by chunk parity
    uint32_t scan[12];
    uint32_t bits[TILE_WORDS];         // key bitmap of the tile's words
    uint32_t wrank[TILE_WORDS];        // keys of the tile before each word
    uint32_t kem2[2][PF];              // insertion chars emitted per key: u16 pairs (thresholds 0/2, 1/3)
    uint16_t colkey[ICOL];             // key of each tile column
    uint32_t vchr[ICOL];               // vote chars of each tile column, 4 thresholds per word
    uint8_t fill[FILL_LDS];
    uint8_t amb[64];
};

// Inclusive prefix sum inside each 16-lane row (DPP row_shr, zeros shifted in).
__device__ __forceinline__ uint32_t row_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    return x;
}

struct Pos {
    uint32_t c[NSYM];
    uint32_t cov, chars;
    uint32_t fl;   // bit 0 in the tile, bit 1 called, bit 2 slow
    __device__ __forceinline__ bool in() const { return fl & 1u; }
    __device__ __forceinline__ bool called() const { return fl & 2u; }
    __device__ __forceinline__ bool slow() const { return fl & 4u; }
};
__device__ __forceinline__ void pos_vote_fast(Pos &p, bool in, int32_t min_depth, uint32_t uq) {
    p.cov = 0;
#pragma unroll
    for (uint32_t s = 0; s < NSYM; s++) p.cov += p.c[s];
    const bool called = in && p.cov > 0 && (int64_t)p.cov >= (int64_t)min_depth;
    uint32_t k[NSYM];
#pragma unroll
    for (uint32_t s = 0; s < NSYM; s++) k[s] = (p.c[s] << 3) | s;
    const uint32_t mk = max(max(max(k[0], k[1]), k[2]), max(max(k[3], k[4]), k[5]));
    const bool fast = majority_fast(mk >> 3, p.cov, uq);
    p.chars = sym_char(mk & 7u) * 0x01010101u;
    p.fl = (in ? 1u : 0u) | (called ? 2u : 0u) | (called && !fast ? 4u : 0u);
}
template <class EL>
__device__ __forceinline__ void pos_vote_slow(Pos &p, const EL &L, const double (&th)[VT_TMAX], int tn) {
    uint32_t gs[NSYM];
    greater_sums(p.c, gs);
    uint32_t w = 0;
#pragma unroll
    for (int u = 0; u < VT_TMAX; u++)
        if (u < tn) w |= (uint32_t)L.amb[vote_mask_u32(p.c, gs, th[u] * (double)p.cov)] << (8 * u);
    if (p.slow()) p.chars = w;
}

// per byte of a vote-char word: 1 if the char is emitted (neither '-' nor a vote error),
// thresholds 0/2 in the 16-bit halves of the first result, 1/3 of the second
__device__ __forceinline__ void emitted4(uint32_t w, uint32_t &e02, uint32_t &e13) {
    const uint32_t x = w ^ 0x2D2D2D2Du, y = ~w;
    const uint32_t nzx = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;   // bit 7 of a byte: byte != 0
    const uint32_t nzy = ((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y;
    const uint32_t f = (nzx & nzy) >> 7;                          // bit 0 of each byte
    e02 += f & 0x00010001u;
    e13 += (f >> 8) & 0x00010001u;
}
__device__ __forceinline__ uint32_t em_of(uint32_t e02, uint32_t e13, int u) {
    return ((u & 1) ? (e13 >> (8 * (u & 2))) : (e02 >> (8 * (u & 2)))) & 0xFFFFu;
}

// Vote of one insertion column (:290-311) for the pass's thresholds; shortcut as for
// positions when every count is ≥ 0.
template <class EL>
__device__ __forceinline__ uint32_t column_word(const uint32_t *col, uint32_t cov, const EL &L, const double (&th)[VT_TMAX],
                                                int tn, uint32_t uq) {
    uint32_t v[NSYM], tot = 0;
#pragma unroll
    for (uint32_t c = 0; c < NSYM; c++) { v[c] = col[c]; tot += v[c]; }
    const int64_t dash = (int64_t)cov - (int64_t)tot;   // the column's own '-' count is in the sum
    if (uq && dash >= 0) {
        v[0] = (uint32_t)dash;
        uint32_t kk[NSYM];
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) kk[c] = (v[c] << 3) | c;
        const uint32_t mk = max(max(max(kk[0], kk[1]), kk[2]), max(max(kk[3], kk[4]), kk[5]));
        if (cov < (1u << 28) && majority_fast(mk >> 3, cov, uq)) return sym_char(mk & 7u) * 0x01010101u;
    }
    const uint32_t m = column_masks(col, cov, th, tn);
    uint32_t word = 0;
#pragma unroll
    for (int u = 0; u < VT_TMAX; u++) word |= (uint32_t)L.amb[(m >> (8 * u)) & 63u] << (8 * u);
    return word;
}

// hist: the tile's LDS histogram (Hist<NWP> layout); cols: LDS [ncol][6].
template <int NWP, class D, class EL>
__device__ __forceinline__ void tile_epilogue_fast(const D &d, uint32_t tile, const TileRec &T, const InsLayout &il,
                                                   const uint32_t *hist, const uint32_t *cols, EL &L) {
    using H = Hist<NWP>;
    constexpr uint32_t nwp = NWP;
    const uint32_t a = T.a, n = T.b - T.a;
    const int Tn = d.n_thr;
    const uint32_t F = (uint32_t)d.fill_len;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, row = lane >> 4;
    const uint32_t ncol = il.ncol;
    const bool has_ins = il.nkeys > 0;
    const uint32_t nchunk = (n + 2 * WG - 1) / (2 * WG);
    uint8_t *const obase = d.out + body_slot(d, a, T.cb0);
    const uint64_t ostride = body_stride(d);
    auto hget = [&](uint32_t q, uint32_t c) { return H::get(hist, c, q); };
    for (int t0 = 0; t0 < Tn; t0 += VT_TMAX) {
        const int tn = min(VT_TMAX, Tn - t0);
        double th[VT_TMAX];   // the pass's thresholds (uniform loads)
#pragma unroll
        for (int u = 0; u < VT_TMAX; u++) th[u] = u < tn ? d.thresholds[t0 + u] : 0.0;
        const uint32_t uq = pass_uq(th, tn);
        const bool more_pass = t0 + VT_TMAX < Tn;
        uint64_t base[VT_TMAX] = {};   // tile body bytes of the previous chunks, per threshold
        for (uint32_t ch = 0; ch < nchunk; ch++) {
            // ---- A: column votes (once per pass) and position votes
            uint32_t cs[VT_TMAX] = {};                      // Σ cov over emitted insertion chars (:385)
            uint32_t ec[VT_TMAX] = {}, nc[VT_TMAX] = {};    // emitted / error insertion chars (wave)
            if (ch == 0) {
                for (uint32_t i = tid; i < (uint32_t)VT_ACC; i += WG) L.acc[i] = 0;
                if (has_ins) {
                    for (uint32_t jb = 0; jb < ncol; jb += WG) {   // uniform trip count (ballots)
                        const uint32_t j = jb + tid;
                        uint32_t cov = 0, word = 0x2D2D2D2Du;   // '-': never emitted
                        uint32_t s = 0;
                        bool kc = false;
                        if (j < ncol) {
                            s = L.colkey[j];
                            const uint32_t kq = L.key[s].x - a;
#pragma unroll
                            for (uint32_t c = 0; c < NSYM; c++) cov += hget(kq, c);
                            kc = cov > 0 && (int64_t)cov >= (int64_t)d.min_depth;   // key called (:356-358)
                            if (kc) word = column_word(cols + (size_t)j * NSYM, cov, L, th, tn, uq);
                            L.vchr[j] = word;
                        }
                        uint32_t e02 = 0, e13 = 0;
                        if (kc) emitted4(word, e02, e13);
                        if (e02 | e13) {
                            atomicAdd(&L.kem2[0][s], e02);
                            atomicAdd(&L.kem2[1][s], e13);
                        }
#pragma unroll
                        for (int u = 0; u < VT_TMAX; u++) {
                            const uint32_t ic = (word >> (8 * u)) & 0xFFu;
                            const bool em = kc && ic != '-' && ic != 0xFFu;
                            ec[u] += (uint32_t)__popcll(__ballot(em));
                            nc[u] += (uint32_t)__popcll(__ballot(kc && ic == 0xFFu));
                            cs[u] += em ? cov : 0u;
                        }
                    }
                }
            }
            const uint32_t wd = 16 * ch + (tid >> 4), i16 = tid & 15;   // word, lane in its row
            const uint32_t q0 = 32 * wd + i16;                         // positions q0, q0 + 16
            Pos P[2];
            {
                const uint32_t s = hslot(16 * wd + i16);
#pragma unroll
                for (uint32_t c = 0; c < NSYM; c++) {
                    const uint32_t h = wd < nwp ? H::word(hist, c, s) : 0u;
                    P[0].c[c] = h & 0xFFFFu;
                    P[1].c[c] = h >> 16;
                }
            }
#pragma unroll
            for (int v = 0; v < 2; v++) pos_vote_fast(P[v], q0 + 16 * v < n, d.min_depth, uq);
            const bool any_slow = __ballot(P[0].slow() || P[1].slow()) != 0;
            if (any_slow) {
                pos_vote_slow(P[0], L, th, tn);
                pos_vote_slow(P[1], L, th, tn);
            }
            if (ch == 0) lds_sync();   // (1) column vote chars, per-key emitted counts, zeroed statistics
#pragma unroll
            for (int v = 0; v < 2; v++) asm volatile("" : "+v"(P[v].fl), "+v"(P[v].cov), "+v"(P[v].chars));
            // ---- B: body lengths, row scans, wave totals, statistics
            const uint32_t bw = (has_ins && wd < nwp) ? L.bits[wd] : 0u;
            uint32_t slot[2], em02[2], em13[2];
            bool hk[2];
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const uint32_t b = i16 + 16 * v;   // bit of the position in its word
                hk[v] = P[v].called() && ((bw >> b) & 1u);
                slot[v] = hk[v] ? L.wrank[wd] + (uint32_t)__popc(bw & ((1u << b) - 1u)) : 0u;
                em02[v] = hk[v] ? L.kem2[0][slot[v]] : 0u;
                em13[v] = hk[v] ? L.kem2[1][slot[v]] : 0u;
            }
            // lengths differ between thresholds only by emitted insertion chars
            const bool multi = __ballot((em02[0] | em13[0] | em02[1] | em13[1]) != 0) != 0;
            const uint32_t lin0 = P[0].in() ? (P[0].called() ? 1u : F) : 0u, lin1 = P[1].in() ? (P[1].called() ? 1u : F) : 0u;
            uint32_t off[VT_TMAX][2];
#pragma unroll
            for (int u = 0; u < VT_TMAX; u++) {
                if (u >= tn || (u > 0 && !multi)) continue;
                const uint32_t l0 = lin0 + em_of(em02[0], em13[0], u), l1 = lin1 + em_of(em02[1], em13[1], u);
                const uint32_t p = l0 | (l1 << 16);   // ≤ 16·64 + ICOL per row half: no carry
                const uint32_t incl = row_scan(p), excl = incl - p;
                const uint32_t r0 = __builtin_amdgcn_readlane(incl, 15), r1 = __builtin_amdgcn_readlane(incl, 31);
                const uint32_t r2 = __builtin_amdgcn_readlane(incl, 47), r3 = __builtin_amdgcn_readlane(incl, 63);
                const uint32_t w0 = (r0 & 0xFFFFu) + (r0 >> 16), w1 = (r1 & 0xFFFFu) + (r1 >> 16);
                const uint32_t w2 = (r2 & 0xFFFFu) + (r2 >> 16), w3 = (r3 & 0xFFFFu) + (r3 >> 16);
                const uint32_t rowoff = (row > 0 ? w0 : 0u) + (row > 1 ? w1 : 0u) + (row > 2 ? w2 : 0u);
                uint32_t rt = r3;
                rt = row == 2 ? r2 : rt;
                rt = row == 1 ? r1 : rt;
                rt = row == 0 ? r0 : rt;
                off[u][0] = rowoff + (excl & 0xFFFFu);
                off[u][1] = rowoff + (rt & 0xFFFFu) + (excl >> 16);
                if (lane == 0) {
                    const uint32_t wt = w0 + w1 + w2 + w3;
                    if (multi) {
                        L.fsum[ch & 1][u][wv] = wt;
                    } else {
#pragma unroll
                        for (int x = 0; x < VT_TMAX; x++) L.fsum[ch & 1][x][wv] = wt;
                    }
                }
            }
            if (!multi) {
#pragma unroll
                for (int u = 1; u < VT_TMAX; u++) { off[u][0] = off[0][0]; off[u][1] = off[0][1]; }
            }
            {   // statistics of this chunk's positions (and of the pass's columns, chunk 0)
                const uint32_t sc = wave_sum(P[0].cov + P[1].cov);   // ≤ 128 · 6 · 2^16 < 2^32
                const uint32_t nunc = (uint32_t)__popcll(__ballot((P[0].fl & 3u) == 1u)) +
                                      (uint32_t)__popcll(__ballot((P[1].fl & 3u) == 1u));
                uint32_t nd[VT_TMAX], ne[VT_TMAX];
#pragma unroll
                for (int u = 0; u < VT_TMAX; u++) {
                    nd[u] = ne[u] = 0;
                    if (u >= tn) continue;
                    if (u > 0 && !any_slow) {   // the same chars for every threshold
                        nd[u] = nd[0];
                        ne[u] = ne[0];
                        continue;
                    }
#pragma unroll
                    for (int v = 0; v < 2; v++) {
                        const uint32_t ch8 = (P[v].chars >> (8 * u)) & 0xFFu;
                        nd[u] += (uint32_t)__popcll(__ballot(P[v].called() && ch8 != '-'));
                        ne[u] += (uint32_t)__popcll(__ballot(P[v].called() && ch8 == 0xFFu));
                    }
                }
                uint64_t scs[VT_TMAX] = {};
                if (ch == 0 && has_ins) {
#pragma unroll
                    for (int u = 0; u < VT_TMAX; u++)
                        if (u < tn && ec[u]) scs[u] = wave_sum((uint64_t)cs[u]);
                }
                if (lane == 0) {
                    atomicAdd(&L.acc[0], (unsigned long long)sc);
#pragma unroll
                    for (int u = 0; u < VT_TMAX; u++) {
                        if (u >= tn) continue;
                        unsigned long long *at = L.acc + 1 + 4 * u;
                        atomicAdd(&at[0], (unsigned long long)(nd[u] + (uint64_t)d.fill_nondash * nunc));
                        if (ne[u] + nc[u]) atomicAdd(&at[1], (unsigned long long)(ne[u] + nc[u]));
                        if (ec[u]) {
                            atomicAdd(&at[2], (unsigned long long)scs[u]);
                            atomicAdd(&at[3], (unsigned long long)ec[u]);
                        }
                    }
                }
            }
            lds_sync();   // (2) wave totals, statistics
#pragma unroll
            for (int v = 0; v < 2; v++) asm volatile("" : "+v"(P[v].fl), "+v"(P[v].chars), "+v"(slot[v]), "+v"(em02[v]), "+v"(em13[v]));
            // ---- C: body bytes (:350-389): char, then the key's emitted insertion chars; fill
            const bool any_fill = F > 0 && __ballot((P[0].fl & 3u) == 1u || (P[1].fl & 3u) == 1u) != 0;
#pragma unroll
            for (int u = 0; u < VT_TMAX; u++) {
                if (u >= tn) continue;
                const uint4 fs = *(const uint4 *)&L.fsum[ch & 1][u][0];   // WG / 64 == 4 waves
                const uint32_t tot = fs.x + fs.y + fs.z + fs.w;
                const uint32_t wofs = (wv > 0 ? fs.x : 0u) + (wv > 1 ? fs.y : 0u) + (wv > 2 ? fs.z : 0u);
                uint8_t *const ob = obase + (size_t)(t0 + u) * ostride + base[u];
                const uint32_t o0 = wofs + off[u][0], o1 = wofs + off[u][1];
                if (P[0].called()) ob[o0] = (uint8_t)(P[0].chars >> (8 * u));
                if (P[1].called()) ob[o1] = (uint8_t)(P[1].chars >> (8 * u));
                if (any_fill) {   // fill (:356-359)
#pragma unroll
                    for (int v = 0; v < 2; v++) {
                        if ((P[v].fl & 3u) != 1u) continue;   // in the tile, not called: fill
                        const uint32_t o = v ? o1 : o0;
                        for (uint32_t f = 0; f < F; f++) ob[o + f] = f < (uint32_t)FILL_LDS ? L.fill[f] : d.fill[f];
                    }
                }
                if (multi) {   // insertion chars after the key's char (:370-385)
#pragma unroll
                    for (int v = 0; v < 2; v++) {
                        if (!em_of(em02[v], em13[v], u)) continue;
                        uint32_t o = (v ? o1 : o0) + 1;
                        const uint4 kr = L.key[slot[v]];
                        for (uint32_t c = 0; c < kr.z; c++) {
                            const uint32_t ic = (L.vchr[kr.y + c] >> (8 * u)) & 0xFFu;
                            if (ic != '-' && ic != 0xFFu) ob[o++] = (uint8_t)ic;
                        }
                    }
                }
                base[u] += tot;
            }
            if (ch + 1 == nchunk && more_pass) {   // next pass counts its emitted chars afresh
                L.kem2[0][tid] = 0;
                L.kem2[1][tid] = 0;
            }
            if (ch + 1 == nchunk && tid < (uint32_t)tn) {   // tile statistics (:352-397)
                uint64_t bl = 0;
#pragma unroll
                for (int u = 0; u < VT_TMAX; u++) bl = (uint32_t)u == tid ? base[u] : bl;
                const unsigned long long *at = L.acc + 1 + 4 * tid;
                const size_t j = (size_t)(t0 + tid) * d.n_tiles + tile;
                uint64_t *st = d.tile_stats + j * 4;
                st[0] = L.acc[0] + at[2];   // sumcov: positions + cov per insertion char
                st[1] = bl;                 // len
                st[2] = at[0] + at[3];      // non-'-' chars (insertion chars are never '-')
                st[3] = at[1];              // vote errors (KeyError, :367/:381)
                d.blk_len[j] = bl;
            }
            // (3) acc / vchr / kem2 reused by the next pass.  Between chunks no barrier: chunk k+1
            // writes the other fsum half, and chunk k+2's writes come after barrier (2) of k+1.
            if (ch + 1 == nchunk && more_pass) lds_sync();
        }
    }
}

// ======================================================================= k_tile
// One workgroup per work item = (tile [a, b) of ≤ 32·NWP positions, chunk k).  Lane L owns
// the 32-position word w = L / G of the tile (G = 256 / NWP lanes per word, a wave holds
// whole words) and takes candidate j ≡ L mod G of the word's candidates: the run slots of
// the short pieces starting in the kwin + 1 words up to w ([rs[W-kwin], rs[W+1])), then the
// tile's long-piece slots; the item takes candidates [k·chunk, (k+1)·chunk).  A candidate
// run covering the word gives one record: valid = the word positions it covers, planes =
// its query bases there (a funnel shift of two plane words).  Records are counted 8 at a
// time into bit-sliced counters X = C|T, Y = G|T, Z = T, V = covered A/C/G/T (and '-' as a
// rare ripple counter); non-ACGT bases of SEQ (N / '-') are taken off their A / C counts
// and added to N / '-' with LDS atomics.  The flush transposes the counters and adds, two
// u16 per LDS atomic, A = V − X − Y + Z, C = X − Z, G = Y − Z, T = Z, '-' into the tile's
// histogram.
constexpr int GS = 8;   // records per counting group
// A buffer offset past every buffer (their sizes stay below it, checked on the host) that
// still leaves room for the loads' immediate and group offsets: the hardware returns zeros.
constexpr uint32_t OOR = 0xF0000000u;

// PIPE: the count loop software-pipelined (next group's run records in flight during this
// group's base windows) at 2 waves/SIMD — it needs the registers; without, 3 waves/SIMD.
// Measured crossover (profiles/r02): deep batches (C3 1000x, C4) gain 3-11 %, C2 (500x with
// insertion epilogues) loses 7 %; launches pick PIPE for batches with >= 5 run slots per
// position (s2c_pileup).
#ifndef S2C_TILE_XCD
#define S2C_TILE_XCD 1
#endif
template <int NWP, bool PIPE>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(PIPE ? 2 : 3))) void k_tile(const TileArgs d, const uint32_t *items) {
    constexpr int G = WG / NWP, HP = 17 * NWP;
    using H = Hist<NWP>;
    constexpr uint32_t ICOL = S2C_LDS_COLS(NWP);
    __shared__ __attribute__((aligned(16))) uint32_t hist[H::CS];
    __shared__ uint32_t cols[ICOL * NSYM];
    __shared__ FastLds<ICOL> L;
    const uint32_t tid = threadIdx.x;
    const uint32_t w = tid / G, g = tid % G;
#ifdef S2C_PROF
    unsigned long long tprof_t = 0;
#endif
    TPROF_MARK(0);
    if (tid < 64) L.amb[tid] = c_amb[tid];
#if S2C_TILE_XCD
    // XCD-major: the blocks of one XCD (b ≡ x mod 8) take a contiguous range of items, so
    // neighbouring tiles' shared window reads meet in that XCD's L2
    const uint32_t bx8 = blockIdx.x & 7u, per = gridDim.x >> 3, rem = gridDim.x & 7u;
    const uint4 itv = ((const uint4 *)items)[bx8 * per + min(bx8, rem) + (blockIdx.x >> 3)];
#else
    const uint4 itv = ((const uint4 *)items)[blockIdx.x];
#endif
    const uint32_t tile = uni(itv.x), chunk = uni(itv.y);
    const TileRec T = tile_rec(d.tiles, tile);
    const uint32_t a = T.a, n = T.b - T.a;
    const uint32_t W = (a >> 5) + w;
    const bool active = 32u * w < n;
    const bool counts_only = d.mode != MODE_RUN;
    const bool accumulate = d.mode >= MODE_ADD;
    const bool finish = !(T.flags & (S2C_TILE_DEEP | S2C_TILE_GENERAL)) && !counts_only;
    const bool deep = (T.flags & S2C_TILE_DEEP) != 0;
    // ---- candidates of this lane: window slots [cw0, cw1) then long slots [lp0, lp1)
    const uint32_t K = d.kwin;
    const uint32_t cbase = uni(d.tiles[(size_t)tile * S2C_TILE_WORDS + 15]);   // the tile's first window slot (o0)
    uint32_t cw0 = 0, cw1 = 0;
    if (active) {
        cw0 = d.rs[W >= K ? W - K : 0u];
        cw1 = d.rs[W + 1];
    }
    const uint32_t nwin = cw1 - cw0, nlong = T.lp1 - T.lp0;
    const uint32_t j0 = chunk * d.chunk, j1 = min(j0 + d.chunk, active ? nwin + nlong : 0u);
    // window candidates of this lane: j = j0 + g + G·m < min(j1, nwin)
    const uint32_t jw1 = min(j1, nwin);
    const uint32_t nrec = j0 + g < jw1 ? (jw1 - j0 - g + G - 1) / G : 0u;
    const uint32_t ngrp = uni(__ockl_wfred_max_u32((nrec + GS - 1) / GS));
    const uint32_t voff = nrec ? (cw0 - cbase + j0 + g) * 16u : OOR;
    const __amdgpu_buffer_rsrc_t rrun = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(d.runs + 4 * (size_t)cbase), (short)0, (int)(d.runs_bytes - 16u * cbase), 0x00020000);
    const __amdgpu_buffer_rsrc_t rbq = __builtin_amdgcn_make_buffer_rsrc((void *)d.bq, (short)0, (int)(8u * d.n_qwords), 0x00020000);
    const __amdgpu_buffer_rsrc_t rbx = __builtin_amdgcn_make_buffer_rsrc((void *)d.bx, (short)0, (int)(4u * d.n_qwords), 0x00020000);

    // ---- zero the histogram (and, for a finished tile with insertions, the layout arrays)
    for (uint32_t i = tid; i < (uint32_t)H::CS / 4; i += WG) ((uint4 *)hist)[i] = make_uint4(0, 0, 0, 0);
    const bool has_ins = finish && T.nev > 0;
    if (has_ins) {
        L.klen[tid] = 0;
        L.kem2[0][tid] = 0;
        L.kem2[1][tid] = 0;
        if (tid < TILE_WORDS) L.bits[tid] = 0;
        for (uint32_t i = tid; i < T.ccap * NSYM && i < ICOL * NSYM; i += WG) cols[i] = 0;
    }
    if (finish && tid < (uint32_t)min(d.fill_len, FILL_LDS)) L.fill[tid] = d.fill[tid];
    lds_sync();
    InsLayout il = {0, 0};
    TPROF_MARK(1);
    if (has_ins) il = build_layout<PF, false>(d, T, tile, L.bits, L.wrank, L.klen, L.key, cols, L.colkey, L.scan);
    TPROF_MARK(2);
    if (counts_only && d.mode != MODE_ADD_KEEP && T.nev > 0 && chunk == 0) {   // no vote: leave the tile's tables zero for the next run
        for (uint32_t e = tid; e < T.bcap; e += WG) ((uint4 *)d.ibkt)[T.boff + e] = make_uint4(0, 0, 0, 0);
        if (tid == 0) d.ilong_n[tile] = 0;
    }

    uint32_t V[4][8], Dc[8];   // counters X, Y, Z, V; '-'
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int b = 0; b < 8; b++) V[c][b] = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) Dc[b] = 0;
    uint32_t nmax_rec = 0;
    // one record (run r at word W) → masks; rare parts ('-' runs, N / '-' of SEQ) applied here
    auto record = [&](const uint4 rv, const uint4 win, uint32_t xw0, uint32_t xw1, uint32_t &mx, uint32_t &my, uint32_t &mv) {
        mx = my = mv = 0;
        const Run r = run_of(rv);
        const uint32_t kd = r.kind & 3u;
        const RecGeom gm = rec_geom(r.gpos, r.len, W);
        if (kd == S2C_RUN_DASH) {
            ripple1(Dc, gm.valid);
        } else if (kd == S2C_RUN_BASES && gm.valid) {
            const uint64_t qs = r.q + gm.qs;
            const uint32_t sh = (uint32_t)(qs & 31);
            const uint32_t b0 = (funnel(win.z, win.x, sh) << gm.lo) & gm.valid;
            const uint32_t b1 = (funnel(win.w, win.y, sh) << gm.lo) & gm.valid;
            mv = gm.valid;
            mx = b0;
            my = b1;
            if (r.kind & S2C_RUN_XBIT) {
                const uint32_t xm = (funnel(xw1, xw0, sh) << gm.lo) & gm.valid;
                const uint32_t en = xm & ~b0 & ~b1, sd = xm & b0 & ~b1;   // 'N', '-' of SEQ
                mv &= ~xm;
                mx &= ~xm;
                my &= ~xm;
                if (sd && !(r.kind & S2C_RUN_DROP)) ripple1(Dc, sd);
                uint32_t e = en;
                while (e) {
                    const uint32_t bit = (uint32_t)__builtin_ctz(e);
                    e &= e - 1;
                    H::add1(hist, 4, 32 * w + bit, 1u);
                }
            }
        }
    };
    if constexpr (PIPE) {
    // ---- window records, GS at a time, software-pipelined: a group's run records become
    //      geometry (covered mask; first bit, funnel shift and kind packed) and base-window
    //      requests as they arrive, then the NEXT group's run records are requested, then this
    //      group's masks go into the counters (carry-save, one record at a time) — each group
    //      waits for one HBM round trip instead of two, in the registers of the old loop
    auto load_runs = [&](uint4 (&Rv)[GS], uint32_t gi) {
#pragma unroll
        for (int u = 0; u < GS; u++) {
            uint32_t vo = gi * GS + u < nrec ? voff : OOR;
            asm volatile("" : "+v"(vo));
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rrun, vo + (uint32_t)(u * 16 * G), gi * GS * 16 * G, 0);
            Rv[u] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    uint4 R[GS];
    if (ngrp) load_runs(R, 0);
    for (uint32_t gi = 0; gi < ngrp; gi++) {
        uint32_t gv[GS], gp[GS];   // covered bits; lo | sh << 8 | kind << 16 (kind 0: nothing)
        uint2 Wa[GS], Wb[GS];
        uint32_t X0[GS], X1[GS];
#pragma unroll
        for (int u = 0; u < GS; u++) {
            const Run r = run_of(R[u]);
            const uint32_t kind = (r.kind & S2C_RUN_LONG) ? 0u : r.kind;   // (long: reached through the long list)
            const RecGeom gm = rec_geom(r.gpos, r.len, W);
            const uint64_t qs = r.q + gm.qs;
            const bool bases = (kind & 3u) == S2C_RUN_BASES && gm.valid;
            const uint32_t wo = bases ? (uint32_t)(qs >> 5) * 8u : OOR;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rbq, wo, 0, 0);
            Wa[u] = make_uint2(v[0], v[1]);
            Wb[u] = make_uint2(v[2], v[3]);
            const uint32_t xo = (bases && (kind & S2C_RUN_XBIT)) ? (uint32_t)(qs >> 5) * 4u : OOR;
            const auto xv = __builtin_amdgcn_raw_buffer_load_b64(rbx, xo, 0, 0);
            X0[u] = xv[0];
            X1[u] = xv[1];
            gv[u] = ((kind & 3u) == S2C_RUN_BASES || (kind & 3u) == S2C_RUN_DASH) ? gm.valid : 0u;
            gp[u] = gm.lo | ((uint32_t)(qs & 31) << 8) | ((kind & 0xFFu) << 16);
        }
        uint4 Rn[GS];
        if (gi + 1 < ngrp) load_runs(Rn, gi + 1);
        uint32_t pend[4], t2a[4], t4a[4], t8[4];
#pragma unroll
        for (int u = 0; u < GS; u++) {
            const uint32_t valid = gv[u], lo = gp[u] & 0xFFu, sh = (gp[u] >> 8) & 31u, kind = gp[u] >> 16;
            uint32_t mx = 0, my = 0, mv = 0;
            if ((kind & 3u) == S2C_RUN_DASH) {
                ripple1(Dc, valid);
            } else if ((kind & 3u) == S2C_RUN_BASES && valid) {
                mx = (funnel(Wb[u].x, Wa[u].x, sh) << lo) & valid;
                my = (funnel(Wb[u].y, Wa[u].y, sh) << lo) & valid;
                mv = valid;
                if (kind & S2C_RUN_XBIT) {
                    const uint32_t xm = (funnel(X1[u], X0[u], sh) << lo) & valid;
                    const uint32_t en = xm & ~mx & ~my, sd = xm & mx & ~my;   // 'N', '-' of SEQ
                    mv &= ~xm;
                    mx &= ~xm;
                    my &= ~xm;
                    if (sd && !(kind & S2C_RUN_DROP)) ripple1(Dc, sd);
                    uint32_t e = en;
                    while (e) {
                        const uint32_t bit = (uint32_t)__builtin_ctz(e);
                        e &= e - 1;
                        H::add1(hist, 4, 32 * w + bit, 1u);
                    }
                }
            }
            const uint32_t mk[4] = {mx, my, mx & my, mv};
#pragma unroll
            for (int c = 0; c < 4; c++) {   // tree8 of the old loop, one record at a time
                if ((u & 1) == 0) {
                    pend[c] = mk[c];
                    continue;
                }
                uint32_t t2;
                csa(t2, V[c][0], V[c][0], pend[c], mk[c]);
                if ((u & 3) == 1) {
                    t2a[c] = t2;
                    continue;
                }
                uint32_t t4;
                csa(t4, V[c][1], V[c][1], t2a[c], t2);
                if ((u & 7) == 3) {
                    t4a[c] = t4;
                    continue;
                }
                csa(t8[c], V[c][2], V[c][2], t4a[c], t4);
            }
        }
#pragma unroll
        for (int c = 0; c < 4; c++) close8(V[c], t8[c]);
#pragma unroll
        for (int u = 0; u < GS; u++) R[u] = Rn[u];
    }
    } else {
    // ---- window records, GS at a time: run records, then their base windows
    for (uint32_t gi = 0; gi < ngrp; gi++) {
        uint4 R[GS];
#pragma unroll
        for (int u = 0; u < GS; u++) {
            uint32_t vo = gi * GS + u < nrec ? voff : OOR;
            asm volatile("" : "+v"(vo));
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rrun, vo + (uint32_t)(u * 16 * G), gi * GS * 16 * G, 0);
            R[u] = make_uint4(v[0], v[1], v[2], v[3]);
        }
        uint4 Wn[GS];
        uint32_t X0[GS], X1[GS];
#pragma unroll
        for (int u = 0; u < GS; u++) {
            const Run r = run_of(R[u]);
            const bool skip = (r.kind & 3u) != S2C_RUN_BASES || (r.kind & S2C_RUN_LONG);
            const RecGeom gm = rec_geom(r.gpos, r.len, W);
            const uint64_t qs = r.q + gm.qs;
            const uint32_t wo = (!skip && gm.valid) ? (uint32_t)(qs >> 5) * 8u : OOR;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rbq, wo, 0, 0);
            Wn[u] = make_uint4(v[0], v[1], v[2], v[3]);
            const uint32_t xo = (wo != OOR && (r.kind & S2C_RUN_XBIT)) ? (uint32_t)(qs >> 5) * 4u : OOR;
            const auto xv = __builtin_amdgcn_raw_buffer_load_b64(rbx, xo, 0, 0);
            X0[u] = xv[0];
            X1[u] = xv[1];
            if (r.kind & S2C_RUN_LONG) R[u].y = 0;   // reached through the long list instead
        }
        uint32_t mx[GS], my[GS], mz[GS], mv[GS];
#pragma unroll
        for (int u = 0; u < GS; u++) {
            record(R[u], Wn[u], X0[u], X1[u], mx[u], my[u], mv[u]);
            mz[u] = mx[u] & my[u];
        }
        const uint32_t t0 = tree8(V[0], mx), t1 = tree8(V[1], my), t2 = tree8(V[2], mz), t3 = tree8(V[3], mv);
        close8(V[0], t0);
        close8(V[1], t1);
        close8(V[2], t2);
        close8(V[3], t3);
    }
    }
    TPROF_MARK(3);
    nmax_rec = nrec;
    // ---- long-piece records (rare): one at a time
    {
        const uint32_t jl0 = max(j0, nwin);
        for (uint32_t j = jl0 + g; j < j1; j += G) {
            const uint32_t slot = d.lp[T.lp0 + (j - nwin)];
            const uint4 rv = ((const uint4 *)d.runs)[slot];
            const Run r = run_of(rv);
            const RecGeom gm = rec_geom(r.gpos, r.len, W);
            uint4 win = make_uint4(0, 0, 0, 0);
            uint32_t x0 = 0, x1 = 0;
            if ((r.kind & 3u) == S2C_RUN_BASES && gm.valid) {
                const uint64_t qw = (r.q + gm.qs) >> 5;
                win = make_uint4(d.bq[2 * qw], d.bq[2 * qw + 1], d.bq[2 * qw + 2], d.bq[2 * qw + 3]);
                if (r.kind & S2C_RUN_XBIT) { x0 = d.bx[qw]; x1 = d.bx[qw + 1]; }
            }
            uint32_t mx, my, mv;
            record(rv, win, x0, x1, mx, my, mv);
            ripple1(V[0], mx);
            ripple1(V[1], my);
            ripple1(V[2], mx & my);
            ripple1(V[3], mv);
            nmax_rec++;
        }
    }
    TPROF_MARK(4);
    // ---- flush: counters → symbol counts → LDS histogram
    {
        transpose8(V[0]);
        transpose8(V[1]);
        transpose8(V[2]);
        transpose8(V[3]);
        transpose8(Dc);
        // A = V − X − Y + Z, C = X − Z, G = Y − Z, T = Z (bytes: every difference is a count)
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const uint32_t x = V[0][r], y = V[1][r], z = V[2][r], v = V[3][r];
            V[3][r] = v - x - y + z;   // A
            V[0][r] = x - z;           // C
            V[1][r] = y - z;           // G
        }
        // the G lanes of a word sit side by side: pairs, then quads, pre-reduced with DPP row
        // shifts while a byte cannot carry (≤ 255), so that one lane in `red` adds into LDS
        uint32_t red = 1;
        auto shr1 = [](uint32_t &v) { v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true); };
        auto shr2 = [](uint32_t &v) { v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true); };
        const uint32_t nmax = uni(__ockl_wfred_max_u32(nmax_rec));
        if (nmax < 128) {
            red = 2;
#pragma unroll
            for (int r = 0; r < 8; r++) { shr1(V[0][r]); shr1(V[1][r]); shr1(V[2][r]); shr1(V[3][r]); shr1(Dc[r]); }
            if (nmax < 64) {
                red = 4;
#pragma unroll
                for (int r = 0; r < 8; r++) { shr2(V[0][r]); shr2(V[1][r]); shr2(V[2][r]); shr2(V[3][r]); shr2(Dc[r]); }
            }
        }
        if (active && (g % red) == red - 1) {
            uint32_t *h0 = hist + 17 * w;
            auto add = [&](uint32_t sym, const uint32_t (&R)[8]) {
                uint32_t *hw = h0 + sym * HP;
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const uint32_t lo = R[r] & 0x00FF00FFu, hi = (R[r] >> 8) & 0x00FF00FFu;
                    if (lo) atomicAdd(hw + r, lo);
                    if (hi) atomicAdd(hw + 8 + r, hi);
                }
            };
            add(1, V[3]);
            add(2, V[0]);
            add(3, V[1]);
            add(5, V[2]);
            add(0, Dc);
        }
    }
    lds_sync();
    TPROF_MARK(5);
    if (finish) {
        tile_epilogue_fast<NWP>(d, tile, T, il, hist, cols, L);
    } else {
        // deep tile: this chunk's counts → HBM (symbol-major, coalesced atomics); a general
        // tile's (and in counts-only mode every tile's) counts: plain stores; streamed
        // batches of unsorted input add every tile's counts to the running totals
        for (uint32_t q = tid; q < n; q += WG)
#pragma unroll
            for (uint32_t c = 0; c < NSYM; c++) {
                uint32_t *dst = d.counts + (size_t)c * d.padded_len + a + q;
                const uint32_t v = H::get(hist, c, q);
                if (deep || accumulate) {
                    if (v) atomicAdd(dst, v);
                } else {
                    *dst = v;
                }
            }
    }
    TPROF_MARK(6);
#ifdef S2C_PROF
    if (threadIdx.x == 0 && (blockIdx.x & 15) == 0) {
        atomicAdd(&g_tprof[15], 1ull);
        atomicAdd(&g_tprof[14], (unsigned long long)ngrp);
    }
#endif
}

// ======================================================================= k_prep / k_consensus
// Deep tiles add their work items' counts into HBM: their count ranges are zeroed first.
__global__ __launch_bounds__(WG) void k_prep(const TileArgs d, const uint32_t *deep) {
    const uint32_t t = deep[blockIdx.x];
    const TileRec T = tile_rec(d.tiles, t);
    if (!(T.flags & S2C_TILE_DEEP)) return;   // a general tile's item stores all its counts
    const uint32_t n = T.b - T.a;
    for (uint32_t c = 0; c < NSYM; c++)
        for (uint32_t i = threadIdx.x; i < n; i += WG) d.counts[(size_t)c * d.padded_len + T.a + i] = 0;
}

// The general epilogue of deep / general tiles: counts from HBM, keys (≤ one per position)
// in LDS, columns and column chars in the tile's HBM slots; thread per key for the column
// votes, 2 positions per thread for the body (a block scan of the lengths per chunk).
struct ConsLds {
    uint4 key[KMAX];
    uint32_t klen[KMAX];               // layout build; then per key its coverage if called, else 0
    uint16_t kem[VT_TMAX][KMAX];       // chars emitted per key (this pass)
    double thr[THR_MAX];
    unsigned long long acc[VT_ACC];
    uint64_t wsum[VT_TMAX][WG / 64];
    uint32_t scan[12];
    uint32_t bits[TILE_WORDS];
    uint32_t wrank[TILE_WORDS];
    uint8_t fill[FILL_LDS];
    uint8_t amb[64];
};

__global__ __launch_bounds__(WG) void k_consensus(const TileArgs d, const uint32_t *deep) {
    __shared__ ConsLds L;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t tile = deep[blockIdx.x];
    const TileRec T = tile_rec(d.tiles, tile);
    const uint32_t a = T.a, n = T.b - T.a;
    if (tid < 64) L.amb[tid] = c_amb[tid];
    for (uint32_t i = tid; i < KMAX; i += WG) L.klen[i] = 0;
    if (tid < TILE_WORDS) L.bits[tid] = 0;
    for (uint32_t i = tid; i < (uint32_t)d.n_thr; i += WG) L.thr[i] = d.thresholds[i];
    if (tid < (uint32_t)min(d.fill_len, FILL_LDS)) L.fill[tid] = d.fill[tid];
    __syncthreads();
    uint32_t *cols = d.ins_cols + (size_t)T.cb0 * NSYM;
    InsLayout il = {0, 0};
    if (T.nev > 0) il = build_layout<KMAX, true>(d, T, tile, L.bits, L.wrank, L.klen, L.key, cols, nullptr, L.scan);
    const uint32_t *cts = d.counts + a;
    const size_t Lp = d.padded_len;
    auto fetch = [&](uint32_t q, uint32_t c) { return cts[(size_t)c * Lp + q]; };
    const int Tn = d.n_thr;
    const uint32_t F = (uint32_t)d.fill_len;
    // key coverage (0 if the key position is not called, :356-358)
    for (uint32_t k = tid; k < il.nkeys; k += WG) {
        uint32_t cov = 0;
        for (uint32_t c = 0; c < NSYM; c++) cov += fetch(L.key[k].x - a, c);
        L.klen[k] = (cov > 0 && (int64_t)cov >= (int64_t)d.min_depth) ? cov : 0u;
    }
    __syncthreads();
    uint8_t *const obase = d.out + body_slot(d, a, T.cb0);
    const uint64_t ostride = body_stride(d);
    uint8_t *const chr = d.ins_chr;   // [T][n_cols]
    for (int t0 = 0; t0 < Tn; t0 += VT_TMAX) {
        const int tn = min(VT_TMAX, Tn - t0);
        for (uint32_t i = tid; i < (uint32_t)VT_ACC; i += WG) L.acc[i] = 0;
        __syncthreads();
        // ---- insertion columns of the called keys (:290-311, :370-385): thread per key
        for (uint32_t k = tid; k < il.nkeys; k += WG) {
            const uint4 kr = L.key[k];
            const uint32_t cov = L.klen[k];
            for (int u = 0; u < tn; u++) {
                const int t = t0 + u;
                uint32_t em = 0, ne = 0;
                for (uint32_t c = 0; cov && c < kr.z; c++) {
                    uint32_t v[NSYM];
#pragma unroll
                    for (uint32_t j = 0; j < NSYM; j++) v[j] = cols[(size_t)(kr.y + c) * NSYM + j];
                    const uint8_t ic = L.amb[column_masks(v, cov, &L.thr[t], 1) & 63u];
                    em += (ic != '-' && ic != 0xFF) ? 1u : 0u;
                    ne += ic == 0xFF ? 1u : 0u;
                    chr[(size_t)t * d.n_cols + T.cb0 + kr.y + c] = ic;
                }
                L.kem[u][k] = (uint16_t)min(em, 0xFFFFu);
                unsigned long long *at = L.acc + 1 + 4 * u;
                if (ne) atomicAdd(&at[1], (unsigned long long)ne);
                if (em) {
                    atomicAdd(&at[2], (unsigned long long)cov * em);
                    atomicAdd(&at[3], (unsigned long long)em);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // chars in HBM before other threads read them
        __syncthreads();
        // ---- positions: vote + body bytes, 2 consecutive positions per thread per chunk
        uint64_t base[VT_TMAX] = {};
        uint64_t sumcov = 0;
        for (uint32_t qb = 0; qb < n; qb += 2 * WG) {   // uniform trip count (scans, ballots)
            const uint32_t q0 = qb + 2 * tid;
            uint32_t cnt[2][NSYM], gs[2][NSYM], cov[2], slot[2];
            bool in[2], called[2], haskey[2];
            uint32_t n_unc = 0;
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t q = q0 + u;
                in[u] = q < n;
                cov[u] = 0;
#pragma unroll
                for (uint32_t c = 0; c < NSYM; c++) { cnt[u][c] = in[u] ? fetch(q, c) : 0u; cov[u] += cnt[u][c]; }
                called[u] = in[u] && cov[u] > 0 && (int64_t)cov[u] >= (int64_t)d.min_depth;   // :356-359
                sumcov += cov[u];
                n_unc += (uint32_t)__popcll(__ballot(in[u] && !called[u]));
                greater_sums(cnt[u], gs[u]);
                const uint32_t bw = (in[u] && il.nkeys) ? L.bits[q >> 5] : 0u;
                haskey[u] = called[u] && ((bw >> (q & 31)) & 1u);
                slot[u] = haskey[u] ? L.wrank[q >> 5] + (uint32_t)__popc(bw & ((1u << (q & 31)) - 1u)) : 0u;
            }
            uint8_t code[VT_TMAX][2];
            uint32_t my[VT_TMAX], incl[VT_TMAX];
#pragma unroll
            for (int u = 0; u < VT_TMAX; u++) {
                my[u] = 0;
                if (u >= tn) continue;
                const double th = L.thr[t0 + u];
                uint32_t nd = 0, ne = 0;
#pragma unroll
                for (int v = 0; v < 2; v++) {
                    code[u][v] = called[v] ? L.amb[vote_mask_u32(cnt[v], gs[v], th * (double)cov[v])] : (uint8_t)S2C_CODE_FILL;
                    my[u] += called[v] ? 1u + (haskey[v] ? L.kem[u][slot[v]] : 0u) : (in[v] ? F : 0u);
                    nd += (uint32_t)__popcll(__ballot(called[v] && code[u][v] != '-'));
                    ne += (uint32_t)__popcll(__ballot(called[v] && code[u][v] == 0xFF));
                }
                incl[u] = __ockl_wfscan_add_u32(my[u], true);
                if (lane == 63) L.wsum[u][wv] = incl[u];
                if (lane == 0) {   // non-'-' chars: called non-'-' codes + fill chars of uncalled positions
                    unsigned long long *at = L.acc + 1 + 4 * u;
                    atomicAdd(&at[0], (unsigned long long)(nd + (uint64_t)d.fill_nondash * n_unc));
                    if (ne) atomicAdd(&at[1], (unsigned long long)ne);
                }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < VT_TMAX; u++) {
                if (u >= tn) continue;
                uint64_t wofs = 0, tot = 0;
#pragma unroll
                for (uint32_t i = 0; i < WG / 64; i++) {
                    wofs += i < wv ? L.wsum[u][i] : 0ull;
                    tot += L.wsum[u][i];
                }
                uint8_t *dst = obase + (size_t)(t0 + u) * ostride + base[u] + wofs + incl[u] - my[u];
#pragma unroll
                for (int v = 0; v < 2; v++) {
                    if (!in[v]) continue;
                    if (!called[v]) {   // fill (:356-359)
                        for (uint32_t f = 0; f < F; f++) dst[f] = f < (uint32_t)FILL_LDS ? L.fill[f] : d.fill[f];
                        dst += F;
                    } else {            // vote char, then the key's insertion chars (:370-385)
                        *dst++ = code[u][v];
                        if (haskey[v]) {
                            const uint4 kr = L.key[slot[v]];
                            const uint8_t *src = chr + (size_t)(t0 + u) * d.n_cols + T.cb0 + kr.y;
                            for (uint32_t c = 0; c < kr.z; c++) {
                                const uint8_t ic = src[c];
                                if (ic != '-' && ic != 0xFF) *dst++ = ic;
                            }
                        }
                    }
                }
                base[u] += tot;
            }
            __syncthreads();   // wsum is rewritten by the next chunk
        }
        // tile totals per threshold (:352-397): len is the body length itself
        sumcov = wave_sum(sumcov);
        if (lane == 0) atomicAdd(&L.acc[0], (unsigned long long)sumcov);
        __syncthreads();
        if (tid < (uint32_t)tn) {
            uint64_t bl = 0;
#pragma unroll
            for (int u = 0; u < VT_TMAX; u++) bl = (uint32_t)u == tid ? base[u] : bl;
            const unsigned long long *at = L.acc + 1 + 4 * tid;
            const size_t j = (size_t)(t0 + tid) * d.n_tiles + tile;
            uint64_t *st = d.tile_stats + j * 4;
            st[0] = L.acc[0] + at[2];
            st[1] = bl;
            st[2] = at[0] + at[3];
            st[3] = at[1];
            d.blk_len[j] = bl;
        }
        __syncthreads();   // acc is rezeroed by the next pass
    }
}

inline int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return S2C_OK;
    return s2c_set_error(S2C_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

TileArgs tile_args(const s2c_dev &d) {
    TileArgs p;
    p.rs = d.rs; p.runs = d.runs; p.bq = d.bq; p.bx = d.bx; p.tiles = d.tiles; p.lp = d.lp;
    p.ibkt = d.ibkt; p.ilong = d.ilong; p.ilong_n = d.ilong_n;
    p.thresholds = d.thresholds; p.fill = d.fill; p.counts = d.counts; p.ins_cols = d.ins_cols; p.ins_chr = d.ins_chr;
    p.tile_stats = d.tile_stats; p.blk_len = d.blk_len; p.out = d.out;
    p.padded_len = (uint32_t)d.padded_len; p.n_cols = (uint32_t)d.n_cols; p.n_tiles = (uint32_t)d.n_tiles;
    p.kwin = (uint32_t)d.kwin; p.chunk = (uint32_t)d.chunk; p.n_qwords = (uint32_t)d.n_qwords;
    p.runs_bytes = (uint32_t)std::min<int64_t>(16 * std::max<int64_t>(d.n_ops, 1), 0xFFFFFFF0ll);
    p.mode = MODE_RUN;
    p.n_thr = d.n_thr; p.min_depth = d.min_depth; p.fill_len = d.fill_len; p.fill_nondash = d.fill_nondash;
    return p;
}

template <int NWP>
int launch_tile(const TileArgs &a, const uint32_t *items, int64_t n, hipStream_t s, bool pipe) {
    if (n <= 0) return S2C_OK;
    if (pipe) k_tile<NWP, true><<<(unsigned)n, WG, 0, s>>>(a, items);
    else k_tile<NWP, false><<<(unsigned)n, WG, 0, s>>>(a, items);
    return hip_check(hipGetLastError(), "k_tile");
}
// pipe: the software-pipelined count loop, for deep batches (>= 5 run slots per position)
int launch_tiles(const TileArgs &a, int32_t tile_max, const uint32_t *items, int64_t n, hipStream_t s, bool pipe) {
    if (tile_max <= 256) return launch_tile<8>(a, items, n, s, pipe);
    if (tile_max <= 512) return launch_tile<16>(a, items, n, s, pipe);
    if (tile_max <= 1024) return launch_tile<32>(a, items, n, s, pipe);
    return launch_tile<64>(a, items, n, s, pipe);
}
bool deep_batch(const s2c_dev *d) {
    const char *e = getenv("S2C_TILE_PIPE");   // (A/B diagnostic: 0 / 1 forces)
    if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
    return d->n_ops >= 5 * d->padded_len;
}

}  // namespace
}  // namespace s2c

using namespace s2c;

// ======================================================================= C-ABI
extern "C" int s2c_workspace_sizes(const s2c_batch_info *info, int32_t n_thr, s2c_ws_sizes *o) {
    if (!info || !o || n_thr <= 0) return s2c_set_error(S2C_ERR_ARG, "bad workspace query");
    const int64_t L = info->padded_len, T = n_thr, NB = T * info->n_tiles;
    const int64_t nc = std::max<int64_t>(info->n_cols, 1);
    o->runs = 16 * std::max<int64_t>(info->n_ops, 1);
    o->ibkt = 16 * std::max<int64_t>(info->n_bkt, 1);
    o->ilong = 16 * std::max<int64_t>(info->n_lng, 1);
    o->ilong_n = 4 * std::max<int64_t>(info->n_tiles, 1);
    o->counts = info->n_deep ? (int64_t)NSYM * L * 4 : 64;   // only deep / general tiles keep counts in HBM
    o->ins_cols = nc * (int64_t)NSYM * 4;
    o->ins_chr = T * nc;
    o->blk_len = std::max<int64_t>(NB, 1) * 8;
    o->tile_stats = std::max<int64_t>(NB, 1) * 32;
    // T body regions of max(1, len(fill))·L + n_cols bytes: the fill length is a run option
    o->out_per_fill = T * L;
    o->out_fixed = T * (info->n_cols + 16);
    return S2C_OK;
}

static int check_dev(const s2c_dev *d) {
    if (!d) return s2c_set_error(S2C_ERR_ARG, "s2c_dev is NULL");
    if (d->n_thr <= 0) return s2c_set_error(S2C_ERR_ARG, "no thresholds");
    if (d->n_thr > THR_MAX) return s2c_set_error(S2C_ERR_LIMIT, "more than 256 thresholds (-c values)");
    if (d->tile_max <= 0 || d->tile_max > S2C_TILE_MAX) return s2c_set_error(S2C_ERR_ARG, "tile_max out of range");
    if (d->padded_len <= 0 || d->padded_len >= ((int64_t)1 << 32)) return s2c_set_error(S2C_ERR_ARG, "bad padded_len");
    if (d->n_tiles >= ((int64_t)1 << 31) || (int64_t)d->n_thr * d->n_tiles >= ((int64_t)1 << 40))
        return s2c_set_error(S2C_ERR_LIMIT, "too many (threshold, tile) blocks");
    if (16 * d->n_ops >= 0xE0000000ll || 8 * d->n_qwords >= 0xE0000000ll)   // 32-bit buffer offsets below OOR
        return s2c_set_error(S2C_ERR_LIMIT, "run records or base planes beyond 3.5 GB (split the input)");
    if (d->n_pieces > 0 && (!d->pc || !d->ops || !d->bq || !d->bx || !d->runs))
        return s2c_set_error(S2C_ERR_ARG, "missing piece buffers");
    if (d->n_tiles > 0 && (!d->tiles || !d->rs || !d->wtile || !d->tile_stats || !d->blk_len || !d->out))
        return s2c_set_error(S2C_ERR_ARG, "missing tile / output buffers");
    if ((d->n_items > 0 && !d->items) || (d->n_dense > 0 && !d->dense)) return s2c_set_error(S2C_ERR_ARG, "missing items");
    if (!d->ibkt || !d->ilong || !d->ilong_n) return s2c_set_error(S2C_ERR_ARG, "missing insertion tables");
    {   // one flush per item: 8-bit counters hold ≤ FLUSH_RECS records per lane
        int64_t nwp = 8;
        while (nwp * 32 < d->tile_max) nwp *= 2;
        if (d->chunk <= 0 || d->chunk > (int64_t)FLUSH_RECS * (WG / nwp))
            return s2c_set_error(S2C_ERR_ARG, "chunk exceeds one flush per work item");
    }
    if (d->n_deep > 0 && (!d->deep || !d->counts || !d->ins_cols || !d->ins_chr))
        return s2c_set_error(S2C_ERR_ARG, "missing deep-tile buffers");
    if (d->fill_len < 0 || (d->fill_len > 0 && !d->fill)) return s2c_set_error(S2C_ERR_ARG, "bad fill");
    {   // every tile's body slot must fit: T regions of max(1, len(fill))·L + n_cols bytes
        const int64_t need = (int64_t)d->n_thr * ((int64_t)std::max(1, d->fill_len) * d->padded_len + d->n_cols);
        if (d->out_cap < need) return s2c_set_error(S2C_ERR_ARG, "out buffer smaller than the body slots");
    }
    return S2C_OK;
}

extern "C" int s2c_reads(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    // dense tiles walk their own pieces, unless len(-f) != 1 routes them to k_tile (which
    // reads run records): then every piece's runs are written
    return s2c_launch_reads(d, (hipStream_t)stream, d->n_dense > 0 && d->fill_len != 1);
}

extern "C" int s2c_pileup(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const TileArgs a = tile_args(*d);
    if (d->n_deep > 0) {
        k_prep<<<(unsigned)d->n_deep, WG, 0, s>>>(a, d->deep);
        if ((rc = hip_check(hipGetLastError(), "k_prep"))) return rc;
    }
    if (d->n_dense > 0) {
        // dense tiles emit exactly one char per position: len(fill) must be 1, else k_tile
        rc = d->fill_len == 1 ? s2c_launch_dense(d, s) : launch_tiles(a, d->tile_max, d->dense, d->n_dense, s, deep_batch(d));
        if (rc) return rc;
    }
    return launch_tiles(a, d->tile_max, d->items, d->n_items, s, deep_batch(d));
}

extern "C" int s2c_consensus(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    if (d->n_deep > 0) {
        k_consensus<<<(unsigned)d->n_deep, WG, 0, (hipStream_t)stream>>>(tile_args(*d), d->deep);
        return hip_check(hipGetLastError(), "k_consensus");
    }
    return S2C_OK;
}

extern "C" int s2c_run(const s2c_dev *d, void *stream) {
    int rc;
    if ((rc = s2c_reads(d, stream))) return rc;
    if ((rc = s2c_pileup(d, stream))) return rc;
    return s2c_consensus(d, stream);
}

extern "C" int s2c_pileup_counts(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    if (!d->counts) return s2c_set_error(S2C_ERR_ARG, "counts buffer required");
    hipStream_t s = (hipStream_t)stream;
    if ((rc = s2c_launch_reads(d, s, true))) return rc;   // run records of every piece
    TileArgs a = tile_args(*d);
    a.mode = MODE_STORE;
    if (d->n_deep > 0) {
        k_prep<<<(unsigned)d->n_deep, WG, 0, s>>>(a, d->deep);
        if ((rc = hip_check(hipGetLastError(), "k_prep"))) return rc;
    }
    if ((rc = launch_tiles(a, d->tile_max, d->dense, d->n_dense, s, deep_batch(d)))) return rc;
    return launch_tiles(a, d->tile_max, d->items, d->n_items, s, deep_batch(d));
}

extern "C" int s2c_accumulate(const s2c_dev *d, int keep_tables, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    if (!d->counts) return s2c_set_error(S2C_ERR_ARG, "counts buffer required");
    hipStream_t s = (hipStream_t)stream;
    if ((rc = s2c_launch_reads(d, s, true))) return rc;   // run records of every piece; events hashed
    TileArgs a = tile_args(*d);
    a.mode = keep_tables ? MODE_ADD_KEEP : MODE_ADD;
    if ((rc = launch_tiles(a, d->tile_max, d->dense, d->n_dense, s, deep_batch(d)))) return rc;
    return launch_tiles(a, d->tile_max, d->items, d->n_items, s, deep_batch(d));
}

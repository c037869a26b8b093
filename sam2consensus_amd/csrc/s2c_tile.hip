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
//   k_consensus              deep / general tiles: the same insertion layout and vote with HBM
//                            columns, then their HBM counts left zero for the next run (k_prep
//                            zeroes them before the counts-only modes)
//
// Everything is integer counting; the single floating-point operation is the reference's
// `cov_nucs < t*coverage` (:362, :376), evaluated as (double)S < t * (double)cov — built
// with -ffp-contract=off.
#include <algorithm>

#include "s2c_common.h"

int s2c_launch_reads(const s2c_dev *d, hipStream_t s, bool all, bool run);
int s2c_launch_dense(const s2c_dev *d, hipStream_t s);

#ifdef S2C_PROF
// phase clocks of k_tile (diagnostic build `make prof`, scripts/prof_tile.py): Σ over sampled
// workgroups (one in 16, wave 0) of the s_memtime deltas of each phase; [15] = workgroups
__device__ unsigned long long g_tprof[16];
__device__ uint32_t g_tabl;   // ablation bits (timing only; results wrong): 1 walk, 2 count, 4 flush atomics
#define TABL(b) ((tabl & (b)) != 0)   // (tabl: g_tabl read once per workgroup)
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
extern "C" int s2c_prof_tile_ablate(uint32_t bits) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tabl), &bits, sizeof(bits)) == hipSuccess ? 0 : -1;
}
#else
#define TABL(b) false
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
    const uint32_t *rs, *runs, *bq, *bx, *tiles, *lp, *pc, *ops, *ps;
    const uint32_t *lly, *lpc, *lops, *lbq, *lbx;
    const uint32_t *px, *lpx;   // S2C_PF_XFEW offsets of the pieces / of the layered pieces
    const void *bq_end, *bx_end, *ops_end, *pc_end;      // ends of the DMA sources (buffer ranges)
    const void *lbq_end, *lbx_end, *lops_end, *lpc_end;
    const void *px_end, *lpx_end;
    uint32_t maxdel_active, maxdel;
    uint32_t *ibkt, *ilong, *ilong_n;
    const double *thresholds;
    const uint8_t *fill;
    uint32_t *counts, *ins_cols;
    uint8_t *ins_chr;
    uint64_t *tile_stats, *blk_len;
    uint8_t *out;
    uint32_t padded_len, n_cols, n_tiles, kwin, chunk, n_qwords, runs_bytes, mode;   // MODE_* below
    uint32_t walk_queue;   // (host only: which k_tile instantiation)
    uint32_t tile_events;  // finish tiles record their short-motif insertion events (EvRec)
    uint32_t tables_empty; // MODE_RUN with tile_events and no piece for s2c_reads: no HBM table to read
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

// walk_piece's view of the batch in HBM (a dense tile's long pieces in counts-only modes)
struct TileMem {
    const uint32_t *ops, *bq, *bx;
    __device__ __forceinline__ uint32_t op(uint32_t j) const { return ops[j]; }
    __device__ __forceinline__ uint32_t p0(uint64_t w) const { return bq[2 * w]; }
    __device__ __forceinline__ uint32_t p1(uint64_t w) const { return bq[2 * w + 1]; }
    __device__ __forceinline__ uint32_t x(uint64_t w) const { return bx[w]; }
};

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
__device__ __forceinline__ InsLayout build_layout(   // (in line: an out-of-line call copies the kernel arguments to scratch)
    const D &d, const TileRec &T, uint32_t t, uint32_t *bits, uint32_t *wrank,
                                  uint32_t *klen, uint4 *key, uint32_t *cols, uint16_t *colkey, uint32_t *scan,
                                  const uint2 *evl = nullptr, uint32_t nevl = 0, bool tables = true) {
    // tables = false: k_reads hashed nothing this run (s2c_reads launched no piece): the tile's
    // HBM table and long-event list are empty, the LDS event list is everything
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t nwords = (T.b - T.a + 31) / 32;
    const uint32_t nlong = tables ? uni(d.ilong_n[t]) : 0u, bcap = tables ? T.bcap : 0u;
    const uint4 *bk = (const uint4 *)d.ibkt + T.boff;
    const uint4 *lg = (const uint4 *)d.ilong + T.loff;
    // (1) key bitmap
    for (uint32_t e = tid; e < bcap; e += WG) {
        const uint4 v = bk[e];
        if (v.x | v.y) atomicOr(&bits[(v.x & 0x7FFu) >> 5], 1u << (v.x & 31u));
    }
    for (uint32_t e = tid; e < nlong; e += WG) {
        const uint32_t pos = lg[e].x;
        atomicOr(&bits[pos >> 5], 1u << (pos & 31u));
    }
    for (uint32_t e = tid; e < nevl; e += WG) {   // (the events k_tile recorded: count 1 each)
        const uint32_t x = evl[e].x;
        atomicOr(&bits[(x & 0x7FFu) >> 5], 1u << (x & 31u));
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
    for (uint32_t e = tid; e < bcap; e += WG) {
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
    for (uint32_t e = tid; e < nevl; e += WG) {
        const uint32_t x = evl[e].x, pos = x & 0x7FFu, k = rank(pos);
        atomicMax(&klen[k], (x >> 11) & 31u);
        key[k].x = T.a + pos;
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
    for (uint32_t e = tid; e < bcap; e += WG) {
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
    for (uint32_t e = tid; e < nevl; e += WG) {
        const uint2 v = evl[e];
        const uint32_t pos = v.x & 0x7FFu, len = (v.x >> 11) & 31u, k = rank(pos);
        const uint64_t m = ((uint64_t)v.x | ((uint64_t)v.y << 32)) >> 16;
        uint32_t *cc = cols + (size_t)key[k].y * NSYM;
        for (uint32_t c = 0; c < len; c++) atomicAdd(&cc[c * NSYM + ((m >> (3 * c)) & 7u)], 1u);
    }
    // (6) leave the table zero for the next run
    for (uint32_t e = tid; e < bcap; e += WG) ((uint4 *)d.ibkt)[T.boff + e] = make_uint4(0, 0, 0, 0);
    if constexpr (HBMCOLS) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // atomics done before the readers
        __syncthreads();
    } else {
        lds_sync();
    }
    if (tid == 0 && tables) d.ilong_n[t] = 0;
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
// One workgroup per work item = (tile [a, b) of ≤ 32·NWP positions, its layers [l0, l1)).
// The tile's WINDOW — the short pieces starting in the kwin words before it and in it — is
// cut into nl LAYERS (host plan, s2c_host.cpp plan_layers): layer ℓ takes from every start
// word s of the window (a SEGMENT) its pieces [ps[s] + n_s·ℓ/nl, ps[s] + n_s·(ℓ+1)/nl), so
// every layer reaches every word of the tile alike.  Each WAVE of the workgroup takes every
// WV-th layer of the item into its own LDS chunk and runs it start to end with no
// workgroup barrier (the waves only meet in the shared histogram and difference arrays,
// by atomics), so one wave's DMA wait or walk overlaps the others' counting:
//   1 DMA    the layer's piece records, op words, base planes {p0, p1} and non-ACGT words,
//            each one contiguous range (16-byte LDS-DMA issued by the wave, the source
//            offset in SGPRs)
//   2 walk   lane per piece: the parsecigar token walk (:64-81) with the maxdel rule (:210)
//            → one run record per op word (rec_enc: packed ends, q − start; q: the run's first base in
//            the LDS planes); coverage and counted '-' runs (D/N/P) into position difference
//            arrays; the N / '-' chars of SEQ (:212, :217) into the histogram
//   3 count  lane (word w, g of G = 64 / NWP) takes the records of segments W-kwin .. W — one
//            contiguous LDS range — g, g + G, ..., 8 at a time: two plane words from LDS,
//            funnel shift, masks X = p0 (C|T), Y = p1 (G|T), Z = X & Y (T) into Harley–Seal
//            carry-save counters (8 bit-planes each)
// Counters are flushed (8×8 bit transposes, u16 pairs by LDS atomics) before they can
// overflow; coverage V comes from the difference array, so per position A = V − X − Y + Z −
// N, C = X − Z − '-'(SEQ), G = Y − Z, T = Z, N, '-' = D + counted '-'(SEQ).  Each base plane
// word is fetched from HBM once per tile (chunks are disjoint; neighbouring tiles share kwin
// start words).  Long pieces (span > the window) come from k_reads' run records through
// the tile's long list.  Then the epilogue (a single-item tile) or the counts to HBM.
// The walk (each measured against its alternative in round 5, profiles/r05/v8_*): the pieces'
// px words come with the layer's records (ahead DMA into LDS), so a walked piece with <= 2 'N'
// (S2C_PF_XFEW) adds them from px, no HBM scan (≤ 1024-position tiles); in the walk-queue
// instantiation the pieces walked op by op are queued and walked after the others by the
// wave's first lanes (one such walk per lane and layer); without '-' in SEQ the maxdel sum
// comes from the walk itself (one pass).

constexpr int GS = 8;                 // records per counting group
constexpr int CSEG = S2C_CHUNK_SEGS;  // segments of a window (≤ 64 words + kwin ≤ 32)
// zero records after a chunk's last: a counting group reads up to 7·G past it (G = 64 / NWP
// lanes per word), so 8·G (k_tile<16>: 32, 256 LDS bytes per wave left for its planes)
constexpr uint32_t rpad_of(int NWP) { return 8u * (64u / (uint32_t)NWP); }
constexpr uint32_t WV = WG / 64;      // waves per workgroup (each its own chunk)
// raw histogram slots while counting ("-ACGNT" slots after the reconstruction)
constexpr uint32_t SL_SDC = 0, SL_SD = 1, SL_X = 2, SL_Y = 3, SL_N = 4, SL_Z = 5;
// A buffer offset past every buffer (their sizes stay below it, checked on the host) that
// still leaves room for the loads' immediate offsets: the hardware returns zeros.
constexpr uint32_t OOR = 0xF0000000u;

// A wave's chunk in LDS: one layer of the tile's window, DMA'd as three contiguous ranges,
// each landing at its source's 16-byte phase — its piece records (pcb) and op words (ol) one
// layer AHEAD, during the previous layer's count (both are read by the walk only), and its
// base planes (pl;
// a 16-byte pad first, so plane word −1 is readable) at the top of its own, under its walk.
// The non-ACGT words stay in HBM (the few pieces that need them: S2C_PF_XFEW pieces take their
// 'N' from px).  runl: the run records; segR[σ]: the first run record of the layer's pieces
// starting in word S0 + σ (pieces are in start-word order).
// With EXT (px words in LDS / the walk queue, tiles of <= 1024 positions: the 2048-position
// instantiation keeps 2 workgroups per CU without them) also the pieces' px words (ahead,
// like pcb) and the queue of the pieces walked op by op.
template <bool EXT> struct ChunkExt {};
template <> struct ChunkExt<true> {
    alignas(16) uint32_t pxl[S2C_CHUNK_PIECES + 4];
    uint8_t wq[S2C_CHUNK_PIECES];
};
template <bool EXT, uint32_t QB, uint32_t RPAD>
struct ChunkLds : ChunkExt<EXT> {
    uint16_t segR[CSEG + 1];   // (u16: record offsets < S2C_CHUNK_RECS + RPAD; the LDS of 3 workgroups per CU)
    alignas(16) uint8_t pl[16 + QB + 16];   // (QB = S2C_CHUNK_QBYTES_OF(NWP, WQB))
    alignas(16) uint4 pcb[S2C_CHUNK_PIECES];
    alignas(16) uint8_t ol[S2C_CHUNK_OBYTES + 16];
    alignas(16) uint2 runl[S2C_CHUNK_RECS + RPAD];
};

typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_byte_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
// A DMA source array: its buffer descriptor (base = the array's 16-byte aligned start, range
// through its end rounded up to 16 bytes, < 4 GB: s2c_pileup checks), built once per kernel.
struct DmaSrc {
    v4i_t r;
    uintptr_t base;
};
__device__ __forceinline__ DmaSrc dma_src(const void *p, const void *end) {
    DmaSrc S;
    S.base = (uintptr_t)p & ~(uintptr_t)15;
    const uintptr_t eal = ((uintptr_t)end + 15) & ~(uintptr_t)15;
    S.r.x = (int)uni((uint32_t)S.base);
    S.r.y = (int)uni((uint32_t)(S.base >> 32) & 0xFFFFu);
    S.r.z = (int)uni((uint32_t)min((uint64_t)(eal - S.base), (uint64_t)0xFFFFFFF0u));
    S.r.w = 0x00020000;
    return S;
}
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0 (reserved) is set and clobbered by the DMA
// n dwords src[0..n) of source array S → the 16-byte aligned LDS region dst by 16-byte
// LDS-DMA issued by the calling wave, 1 KB per instruction (offsets in SGPRs); the copy
// starts at the 16-byte boundary below src, so the dwords land at dst + (src & 15).
// Arguments wave-uniform.  Completion: s_waitcnt vmcnt(0) (the compiler does not count these
// loads): the wave's own LDS reads then see the data.
// Returns the number of DMA instructions issued (each one vmcnt event).
// Cache policy of the layer DMA: nontemporal (C3 -3.5 % against the default policy,
// profiles/r05/v7_*)
#define S2C_TILE_DMA_POLICY " nt"
__device__ __forceinline__ uint32_t dma16_wave(uint8_t *dst, const DmaSrc &S, const uint32_t *src, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uintptr_t sal = (uintptr_t)src & ~(uintptr_t)15;
    const uint32_t nbytes = uni((uint32_t)((uintptr_t)src - sal) + 4 * n);
    const uint32_t soff = uni((uint32_t)(sal - S.base)), m0 = uni(lds_byte_addr(dst));
    uint32_t k = 0;
    for (uint32_t base = 0; base < nbytes; base += 1024, k++) {
        if (base + 16 * lane < nbytes)
            asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen" S2C_TILE_DMA_POLICY " lds"
                         :: "s"(m0 + base), "v"(16 * lane), "s"(S.r), "s"(soff + base) : "memory", "m0");
    }
    return k;
}
#pragma clang diagnostic pop
// s_waitcnt vmcnt(k) for a wave-uniform k (≤ 15 instructions younger than the ones waited
// for; more: all): the VMEM loads complete in order, so this waits for every load issued
// before the k youngest — the kernels' LDS-DMA loads, which the compiler does not count.
__device__ __forceinline__ void wait_vm(uint32_t k) {
    switch (uni(k)) {
#define S2C_WV(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
        S2C_WV(1) S2C_WV(2) S2C_WV(3) S2C_WV(4) S2C_WV(5) S2C_WV(6) S2C_WV(7) S2C_WV(8)
        S2C_WV(9) S2C_WV(10) S2C_WV(11) S2C_WV(12) S2C_WV(13) S2C_WV(14) S2C_WV(15)
#undef S2C_WV
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

template <uint32_t ICOL>
struct EpiLds {
    FastLds<ICOL> L;
    uint32_t cols[ICOL * NSYM];
};
template <uint32_t ICOL, bool EXT, uint32_t QB, uint32_t RPAD>
union TileLds {
    ChunkLds<EXT, QB, RPAD> c[WV];   // one chunk per wave
    EpiLds<ICOL> e;
};
// the non-ACGT words in HBM, as a global-address-space pointer (a uniform base + 32-bit lane
// offsets: global_load with an SGPR base, not flat loads with 64-bit lane addresses)
typedef const __attribute__((address_space(1))) uint32_t *gptr_u32;

// A wave's LDS hand-off between its own lanes (no other wave involved): the wave's LDS
// operations complete in order, and the compiler keeps its memory accesses on either side.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// The N / '-' chars of SEQ among LDS plane bases [q, q + l), whose first lies at
// tile-relative position r0: 'N' (counted as A by the planes) into SL_N; '-' (counted as C)
// into SL_SD and, unless the read's '-' are maxdel-dropped (:210), SL_SDC.  Runs of up to
// six plane words take an unrolled pass (their non-ACGT words read together, the rare set
// bits handled one by one); longer ones a loop.
template <int NWP>
__device__ __forceinline__ void x_bits(uint32_t xm, uint32_t p0, int32_t b0, uint32_t r0, bool drop, uint32_t *hist) {
    using H = Hist<NWP>;
    while (xm) {
        const uint32_t bit = (uint32_t)__builtin_ctz(xm);
        xm &= xm - 1;
        const uint32_t p = r0 + (uint32_t)(b0 + (int32_t)bit);
        if ((p0 >> bit) & 1u) {
            H::add1(hist, SL_SD, p, 1u);
            if (!drop) H::add1(hist, SL_SDC, p, 1u);
        } else {
            H::add1(hist, SL_N, p, 1u);
        }
    }
}
template <int NWP>
__device__ __forceinline__ void x_fix_body(const uint2 *bql, gptr_u32 xl, uint32_t xd, uint32_t q, uint32_t l, uint32_t r0, bool drop,
                      uint32_t *hist) {
    const uint32_t v0 = q >> 5, v1 = (q + l - 1) >> 5;
    for (uint32_t vb = v0; vb <= v1; vb += 4) {   // four HBM words per round trip, then one at a time
        uint32_t xs[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) xs[u] = vb + u <= v1 ? xl[vb + u + xd] : 0u;
#pragma unroll 1
        for (uint32_t v = vb; v < vb + 4; v++) {
            uint32_t xm = xs[0];
            xs[0] = xs[1];   // (shifted, not indexed: registers)
            xs[1] = xs[2];
            xs[2] = xs[3];
            if (!xm) continue;
            const int32_t b0 = (int32_t)(32 * v) - (int32_t)q;   // run offset of the word's bit 0
            if (b0 < 0) xm &= 0xFFFFFFFFu << (uint32_t)(-b0);
            if (b0 + 32 > (int32_t)l) xm &= 0xFFFFFFFFu >> (uint32_t)(b0 + 32 - (int32_t)l);
            x_bits<NWP>(xm, bql[v].x, b0, r0, drop, hist);
        }
    }
}
// x_fix in line, or (OOL) out of line: the walk-queue instantiation of k_tile spills 416
// bytes per lane with the rare non-ACGT scan in line (C2 0.075 -> 0.095 ms, profiles/r05/v9_*),
// the other one runs 2-4 % slower with it out of line
template <int NWP, bool OOL>
__device__ __forceinline__ void x_fix(const uint2 *bql, gptr_u32 xl, uint32_t xd, uint32_t q, uint32_t l, uint32_t r0, bool drop,
                                      uint32_t *hist);
template <int NWP>
__device__ __attribute__((noinline)) void x_fix_ool(const uint2 *bql, gptr_u32 xl, uint32_t xd, uint32_t q, uint32_t l, uint32_t r0,
                                                     bool drop, uint32_t *hist) {
    x_fix_body<NWP>(bql, xl, xd, q, l, r0, drop, hist);
}
template <int NWP, bool OOL>
__device__ __forceinline__ void x_fix(const uint2 *bql, gptr_u32 xl, uint32_t xd, uint32_t q, uint32_t l, uint32_t r0, bool drop,
                                      uint32_t *hist) {
    if constexpr (OOL) x_fix_ool<NWP>(bql, xl, xd, q, l, r0, drop, hist);
    else x_fix_body<NWP>(bql, xl, xd, q, l, r0, drop, hist);
}

// One piece of a chunk (record P, op words [P.z, oend) in LDS at opl[j + od], its SEQ[0] at
// LDS plane base 16·P.y + qadj): parsecigar (:64-81) + maxdel (:210) → run records
// runl[j + rd] (bases: rec_enc records; others zero); coverage / counted '-' of the
// tile part into dV / dD; N / '-' of SEQ via x_fix.  Everything from LDS.
// A finish tile's LDS event list (k_tile records the short-motif insertion events of its
// window's pieces keyed inside it; s2c_reads leaves exactly those to it, s2c_reads.hip
// add_event): key = tile position | length << 11 | 3-bit codes << 16 (k_reads' table key).
// The walking lane keeps up to two events of its piece in registers (EvOut: LDS plane base,
// position | length << 11 | non-ACGT << 16) and keys them once the layer's planes have landed
// (k_tile, after the planes wait), so the walk never waits for the planes; a third event of
// one piece flushes the first two with a wait of its own.
struct EvRec {
    uint2 *l;
    uint32_t *n;
    bool on;
};
struct EvOut {
    uint32_t n, q0, t0, q1, t1;
};

// One event's key: motif = LDS plane bases [q, q + take) (take <= 16), at tile position pos
__device__ __forceinline__ uint64_t ev_key(const uint2 *bql, gptr_u32 xl, uint32_t xd, uint32_t q, uint32_t take,
                                           uint32_t pos, bool x) {
    const uint32_t v = q >> 5, sh = q & 31u;
    const uint64_t p0 = (uint64_t)bql[v].x | ((uint64_t)bql[v + 1].x << 32);
    const uint64_t p1 = (uint64_t)bql[v].y | ((uint64_t)bql[v + 1].y << 32);
    const uint64_t px = x ? ((uint64_t)xl[v + xd] | ((uint64_t)xl[v + 1 + xd] << 32)) : 0ull;
    uint64_t key = (uint64_t)pos | ((uint64_t)take << 11);
    for (uint32_t c = 0; c < take; c++) {
        const uint32_t b0 = (uint32_t)(p0 >> (sh + c)) & 1u, b1 = (uint32_t)(p1 >> (sh + c)) & 1u;
        const uint32_t code = ((px >> (sh + c)) & 1u) ? (b0 ? 0u : 4u) : ((b1 << 1 | b0) == 3u ? 5u : (b1 << 1 | b0) + 1u);
        key |= (uint64_t)code << (16 + 3 * c);
    }
    return key;
}
__device__ __forceinline__ void ev_append(const uint2 *bql, gptr_u32 xl, uint32_t xd, uint32_t q, uint32_t t, const EvRec &ev) {
    const uint64_t k = ev_key(bql, xl, xd, q, (t >> 11) & 31u, t & 0x7FFu, (t >> 16) != 0);
    const uint32_t i = atomicAdd(ev.n, 1u);
    if (i < S2C_EPI_KEYS) ev.l[i] = make_uint2((uint32_t)k, (uint32_t)(k >> 32));
}
// the lane's held events keyed (the planes have landed)
__device__ __forceinline__ void ev_flush(const uint2 *bql, gptr_u32 xl, uint32_t xd, EvOut &eo, const EvRec &ev) {
    if (eo.n > 0) ev_append(bql, xl, xd, eo.q0, eo.t0, ev);
    if (eo.n > 1) ev_append(bql, xl, xd, eo.q1, eo.t1, ev);
    eo.n = 0;
}

template <int NWP, bool PXL, bool OOL, bool REC>
__device__ void walk_chunk_piece(const uint4 P, uint32_t oend, const uint32_t *opl, uint32_t od, uint2 *runl, uint32_t rd,
                                 const uint2 *bql, gptr_u32 xl, uint32_t xd, uint32_t qadj, bool maxdel_active,
                                 uint32_t maxdel, uint32_t a, uint32_t n, uint32_t *hist, int32_t *dV, int32_t *dD,
                                 uint32_t pxw, const EvRec &ev, EvOut &eo) {
    const uint32_t fl = P.w >> 24, slen = P.w & 0xFFFFFFu;
    uint32_t j = P.z;
    if (fl & S2C_PF_LONG) {   // (its runs come through the tile long lists)
        for (; j < oend; j++) runl[j + rd] = make_uint2(0u, 0u);
        return;
    }
    uint32_t ka = 0, kb = 0xFFFFFFFFu;
    if (fl & S2C_PF_RANGE) {
        ka = opl[j + od];
        kb = opl[j + 1 + od];
        runl[j + rd] = runl[j + 1 + rd] = make_uint2(0u, 0u);
        j += 2;
    }
    int64_t key0 = 0;   // (:74 start_ref = POS-1 + the seqout index; events before the ref start dropped)
    uint32_t roff = 0;
    const bool rec = REC && ev.on && (fl & S2C_PF_INS);
    if (fl & S2C_PF_INS) {   // (its events: the finish tiles' own, else k_reads)
        if (rec) {
            key0 = (int64_t)((uint64_t)opl[j + od] | ((uint64_t)opl[j + 1 + od] << 32));
            roff = opl[j + 2 + od];
        }
        runl[j + rd] = runl[j + 1 + rd] = runl[j + 2 + rd] = make_uint2(0u, 0u);
        j += 3;
    }
    const uint32_t ql = 16u * P.y + qadj;     // SEQ[0] in the LDS planes
    bool drop = false;
    // :210 — D/N/P lengths + '-' chars of the bases taken.  With '-' in SEQ a first pass over
    // the ops; otherwise the D/N/P lengths are summed by the one pass below,
    // which holds back the first two deletion runs' '-' counts until the sum is known
    const bool defer = maxdel_active && !(fl & S2C_PF_DASH);
    if (maxdel_active && (fl & S2C_PF_DASH)) {
        uint32_t dashes = 0, start = 0;
        for (uint32_t jj = j; jj < oend; jj++) {
            const uint32_t w = opl[jj + od], op = w & 15u, l = w >> 4;
            if (op_bases(op)) {
                uint32_t take = start < slen ? min(l, slen - start) : 0u;
                if (fl & S2C_PF_DASH) {   // '-' chars of SEQ: x = 1, p1 = 0, p0 = 1
                    uint32_t q = ql + start;
                    while (take) {
                        const uint32_t v = q >> 5, sh = q & 31u, nb = min(take, 32u - sh);
                        const uint32_t mask = (nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u)) << sh;
                        dashes += (uint32_t)__popc(xl[v + xd] & bql[v].x & ~bql[v].y & mask);
                        q += nb;
                        take -= nb;
                    }
                }
                start += l;
            } else if (op_dash(op)) {
                dashes += l;
            } else if (op == S2C_OP_I || op == S2C_OP_S) {
                start += l;
            }
        }
        drop = dashes > maxdel;
    }
    uint32_t dsum = 0, nd = 0, dr0 = 0, dr1 = 0;   // (deferred: '-' runs [c0, c1) - a packed c0 | c1 << 16)
    const uint32_t e_tile = a + n;
    uint32_t kk = 0, start = 0;
    // the next op word is read ahead of this op's LDS writes (records, atomics), which the
    // compiler must otherwise assume may alias it: one LDS round trip per piece, not per op
    uint32_t wn = j < oend ? opl[j + od] : 0u;
    for (uint32_t jj = j; jj < oend; jj++) {
        const uint32_t w = wn, op = w & 15u, l = w >> 4;
        wn = opl[min(jj + 1u, oend - 1u) + od];
        uint2 r = make_uint2(0u, 0u);
        const bool bases = op_bases(op);
        if (bases || op_dash(op)) {
            const uint32_t take = bases ? (start < slen ? min(l, slen - start) : 0u) : l;
            const uint32_t s = max(kk, ka), e = min(kk + take, kb);
            if (e > s) {
                const uint32_t gp = P.x + (s - ka), len = e - s;
                const uint32_t c0 = max(gp, a), c1 = min(gp + len, e_tile);   // the tile's part
                if (bases) {
                    const uint32_t q = ql + start + (s - kk);
                    r = rec_enc(gp - (a & ~31u), len, q);
                    if (c1 > c0) {
                        atomicAdd(&dV[c0 - a], 1);
                        atomicSub(&dV[c1 - a], 1);
                        if (PXL && (fl & (S2C_PF_X | S2C_PF_XFEW)) == (S2C_PF_X | S2C_PF_XFEW)) {
                            // ≤ 2 'N' at SEQ offsets px (s2c.h S2C_PF_XFEW): the run holds SEQ [so, so + len)
                            const uint32_t so = start + (s - kk);
#pragma unroll
                            for (int h = 0; h < 2; h++) {
                                const uint32_t off = (pxw >> (16 * h)) & 0xFFFFu, p = gp + (off - so);   // (0xFFFF: none)
                                if (off != 0xFFFFu && off - so < len && p >= c0 && p < c1) Hist<NWP>::add1(hist, SL_N, p - a, 1u);
                            }
                        } else if (fl & S2C_PF_X) {
                            x_fix<NWP, OOL>(bql, xl, xd, q + (c0 - gp), c1 - c0, c0 - a, drop, hist);
                        }
                    }
                } else if (defer && c1 > c0) {
                    const uint32_t pk = (c0 - a) | (c1 - a) << 16;
                    dr1 = nd == 1 ? pk : dr1;
                    dr0 = nd == 0 ? pk : dr0;
                    nd++;
                } else if (!drop && c1 > c0) {
                    atomicAdd(&dD[c0 - a], 1);
                    atomicSub(&dD[c1 - a], 1);
                }
            }
            kk += take;
        }
        if (op_dash(op)) dsum += l;
        if (REC && rec && op == S2C_OP_I) {   // an insertion event (:73-75) keyed in the tile, motif <= 16 bases
            const uint32_t take = start < slen ? min(l, slen - start) : 0u;
            const int64_t gk = key0 + (int64_t)kk;
            if (take && take <= S2C_SHORT_MOTIF && gk >= (int64_t)roff && gk >= (int64_t)a && gk < (int64_t)e_tile)
            {
                if (eo.n == 2) {   // (rare: a third event of the piece) the planes now
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    ev_flush(bql, xl, xd, eo, ev);
                }
                const uint32_t tq = (uint32_t)(gk - (int64_t)a) | take << 11 | ((fl & S2C_PF_X) ? 1u << 16 : 0u);
                if (eo.n == 0) { eo.q0 = ql + start; eo.t0 = tq; } else { eo.q1 = ql + start; eo.t1 = tq; }
                eo.n++;
            }
        }
        if (bases || op == S2C_OP_I || op == S2C_OP_S) start += l;
        runl[jj + rd] = r;
    }
    if (nd && dsum <= maxdel) {   // (defer: the read keeps its '-')
        atomicAdd(&dD[dr0 & 0xFFFFu], 1);
        atomicSub(&dD[dr0 >> 16], 1);
        if (nd > 1) {
            atomicAdd(&dD[dr1 & 0xFFFFu], 1);
            atomicSub(&dD[dr1 >> 16], 1);
        }
        if (nd > 2) {   // (rare) the third and later runs: the ops again
            uint32_t kk2 = 0, st2 = 0, m = 0;
            for (uint32_t jj = j; jj < oend; jj++) {
                const uint32_t w = opl[jj + od], op = w & 15u, l = w >> 4;
                const bool bs = op_bases(op);
                if (bs || op_dash(op)) {
                    const uint32_t take = bs ? (st2 < slen ? min(l, slen - st2) : 0u) : l;
                    const uint32_t s = max(kk2, ka), e = min(kk2 + take, kb);
                    if (!bs && e > s) {
                        const uint32_t gp = P.x + (s - ka), c0 = max(gp, a), c1 = min(gp + (e - s), e_tile);
                        if (c1 > c0 && m++ >= 2) {
                            atomicAdd(&dD[c0 - a], 1);
                            atomicSub(&dD[c1 - a], 1);
                        }
                    }
                    kk2 += take;
                }
                if (bs || op == S2C_OP_I || op == S2C_OP_S) st2 += l;
            }
        }
    }
}

// Exclusive prefix sum and total over the 4 lanes of a lane group (lane & 3 = sub) by DPP
// quad permutes (no LDS round trip); every lane of the wave takes part.
template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t xscan4(uint32_t x, uint32_t sub) {
    // (each permute taken by every lane, then selected: a permute inside the select could be
    // predicated to the selecting lanes, leaving its source lanes off)
    const uint32_t t1 = quad_perm<0x90>(x);   // [0,0,1,2]: lane i − 1's
    uint32_t v = x + (sub >= 1u ? t1 : 0u);
    const uint32_t t2 = quad_perm<0x44>(v);   // [0,1,0,1]: lane i − 2's
    v += sub >= 2u ? t2 : 0u;
    return v - x;
}
__device__ __forceinline__ uint32_t sum4(uint32_t x) {
    x += quad_perm<0xB1>(x);      // [1,0,3,2]
    return x + quad_perm<0x4E>(x);   // [2,3,0,1]
}

// walk_chunk_piece for a piece of at most 4 op words (after its insertion-key prefix), walked
// by the 4 lanes of a group, one op word each (the walk-queue instantiation: C2's indel reads
// are 3-op pieces).  The serial walk's running values come from two group scans — the query
// offset `start` over the query-consuming ops, then the seqout offset `kk` over the taken
// lengths, which depend on `start` (a base op takes min(l, len(SEQ) − start), :64-69) — and
// the read's D/N/P total (:210) from a group sum, so each op's run, coverage, '-' run and
// insertion event are the serial walk's.  No shard range (ka = 0, kb = ∞) and no '-' in SEQ
// (drop = false; the maxdel rule then keeps the '-' runs iff their total ≤ maxdel, as the
// serial walk's deferred runs do).  `mine`: this lane holds op word jj of such a piece.
template <int NWP, bool PXL, bool OOL, bool REC>
__device__ __forceinline__ void walk_op_coop(const uint4 P, bool mine, uint32_t jj, uint32_t sub, const uint32_t *opl,
                                             uint32_t od, uint2 *runl, uint32_t rd, const uint2 *bql, gptr_u32 xl,
                                             uint32_t xd, uint32_t qadj, bool maxdel_active, uint32_t maxdel, uint32_t a,
                                             uint32_t n, uint32_t *hist, int32_t *dV, int32_t *dD, uint32_t pxw,
                                             int64_t key0, uint32_t roff, bool rec, const EvRec &ev, EvOut &eo) {
    const uint32_t fl = P.w >> 24, slen = P.w & 0xFFFFFFu;
    const uint32_t w = mine ? opl[jj + od] : 0u, op = w & 15u, l = w >> 4;
    const bool bases = mine && op_bases(op), dash = mine && op_dash(op);
    const bool qop = bases || (mine && (op == S2C_OP_I || op == S2C_OP_S));
    const uint32_t start = xscan4(qop ? l : 0u, sub);
    const uint32_t take = bases ? (start < slen ? min(l, slen - start) : 0u) : (dash ? l : 0u);
    const uint32_t kk = xscan4(take, sub);
    const uint32_t dsum = sum4(dash ? l : 0u);
    if (!mine) return;
    const uint32_t ql = 16u * P.y + qadj;   // SEQ[0] in the LDS planes
    const uint32_t e_tile = a + n;
    uint2 r = make_uint2(0u, 0u);
    if (take) {
        const uint32_t gp = P.x + kk;
        const uint32_t c0 = max(gp, a), c1 = min(gp + take, e_tile);   // the tile's part
        if (bases) {
            const uint32_t q = ql + start;
            r = rec_enc(gp - (a & ~31u), take, q);
            if (c1 > c0) {
                atomicAdd(&dV[c0 - a], 1);
                atomicSub(&dV[c1 - a], 1);
                if (PXL && (fl & (S2C_PF_X | S2C_PF_XFEW)) == (S2C_PF_X | S2C_PF_XFEW)) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint32_t off = (pxw >> (16 * h)) & 0xFFFFu, p = gp + (off - start);   // (0xFFFF: none)
                        if (off != 0xFFFFu && off - start < take && p >= c0 && p < c1) Hist<NWP>::add1(hist, SL_N, p - a, 1u);
                    }
                } else if (fl & S2C_PF_X) {
                    x_fix<NWP, OOL>(bql, xl, xd, q + (c0 - gp), c1 - c0, c0 - a, false, hist);
                }
            }
        } else if (c1 > c0 && !(maxdel_active && dsum > maxdel)) {
            atomicAdd(&dD[c0 - a], 1);
            atomicSub(&dD[c1 - a], 1);
        }
    }
    if (REC && rec && op == S2C_OP_I) {   // an insertion event (:73-75) keyed in the tile, motif <= 16 bases
        const uint32_t ti = start < slen ? min(l, slen - start) : 0u;
        const int64_t gk = key0 + (int64_t)kk;
        if (ti && ti <= S2C_SHORT_MOTIF && gk >= (int64_t)roff && gk >= (int64_t)a && gk < (int64_t)e_tile) {
            if (eo.n == 2) {   // (a lane's third held event: the planes now)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                ev_flush(bql, xl, xd, eo, ev);
            }
            const uint32_t tq = (uint32_t)(gk - (int64_t)a) | ti << 11 | ((fl & S2C_PF_X) ? 1u << 16 : 0u);
            if (eo.n == 0) { eo.q0 = ql + start; eo.t0 = tq; } else { eo.q1 = ql + start; eo.t1 = tq; }
            eo.n++;
        }
    }
    runl[jj + rd] = r;
}

template <int NWP, bool WQB>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(NWP <= 16 ? 3 : 2))) void k_tile(const TileArgs d, const uint32_t *items) {
    constexpr int HP = 17 * NWP;
    constexpr uint32_t NPOS = 32 * NWP;
    using H = Hist<NWP>;
    constexpr uint32_t ICOL = S2C_LDS_COLS(NWP);
    static_assert(NWP + 32 < CSEG, "segments of a window");
    __shared__ __attribute__((aligned(16))) uint32_t hist[H::CS];
    __shared__ int32_t dV[NPOS + 1], dD[NPOS + 1];
    __shared__ uint32_t wtot[2][WG / 64];
    // WQB: the launch's batch has pieces walked op by op (s2c_dev n_walked); without them the
    // queue's code costs C3 / C4 4 % (profiles/r05/v9_*), so it is a separate instantiation
    constexpr bool PXL = NWP <= 32, WQ = WQB && NWP <= 32;   // (ChunkLds' EXT)
    __shared__ __attribute__((aligned(16))) TileLds<ICOL, PXL || WQ, S2C_CHUNK_QBYTES_OF(NWP, WQB), rpad_of(NWP)> U;
    // a finish tile's own short-motif insertion events (EvRec; the 2048-position instantiation
    // leaves them to k_reads: its LDS)
    constexpr bool REC = WQB && NWP <= 32;   // (the walk-queue instantiation's LDS has room for the list)
    __shared__ uint2 evl[REC ? S2C_EPI_KEYS : 1];
    __shared__ uint32_t evn;
    S2C_POISON(hist, sizeof(hist));
    S2C_POISON(dV, sizeof(dV));
    S2C_POISON(dD, sizeof(dD));
    S2C_POISON(wtot, sizeof(wtot));
    S2C_POISON(&U, sizeof(U));
    S2C_POISON(evl, sizeof(evl));
    S2C_POISON(&evn, sizeof(evn));
    S2C_POISON_DONE();
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#ifdef S2C_PROF
    const uint32_t tabl = uni(*(volatile uint32_t *)&g_tabl);
#endif
#ifdef S2C_PROF
    unsigned long long tprof_t = 0;
#endif
    TPROF_MARK(0);
    // XCD-major: the blocks of one XCD (b ≡ x mod 8) take a contiguous range of items, so
    // neighbouring tiles' shared window reads meet in that XCD's L2
    const uint32_t bx8 = blockIdx.x & 7u, per = gridDim.x >> 3, rem = gridDim.x & 7u;
    const uint4 itv = ((const uint4 *)items)[bx8 * per + min(bx8, rem) + (blockIdx.x >> 3)];
    const uint32_t tile = uni(itv.x), chunk = uni(itv.y), l0 = uni(itv.z), l1 = uni(itv.w);
    const TileRec T = tile_rec(d.tiles, tile);
    const uint32_t nl = uni(d.tiles[(size_t)tile * S2C_TILE_WORDS + 19]);
    const uint32_t a = T.a, n = T.b - T.a;
    const uint32_t W0 = a >> 5, nwords = (n + 31) / 32;
    const uint32_t K = d.kwin;
    const uint32_t S0 = W0 >= K ? W0 - K : 0u, NS = W0 + nwords - S0;
    const bool counts_only = d.mode != MODE_RUN;
    const bool accumulate = d.mode >= MODE_ADD;
    const bool finish = !(T.flags & (S2C_TILE_DEEP | S2C_TILE_GENERAL)) && !counts_only;
    const bool deep = (T.flags & S2C_TILE_DEEP) != 0;

    // ---- zero the histogram and the difference arrays; the window's piece CSR
    for (uint32_t i = tid; i < (uint32_t)H::CS / 4; i += WG) ((uint4 *)hist)[i] = make_uint4(0, 0, 0, 0);
    for (uint32_t i = tid; i <= NPOS; i += WG) {
        dV[i] = 0;
        dD[i] = 0;
    }
    const bool rec_ev = REC && d.tile_events && finish && T.nev > 0;   // (s2c_reads.hip add_event leaves these to the walk)
    EvRec evr;
    evr.l = evl;
    evr.n = &evn;
    evr.on = rec_ev;
    if (tid == 0) evn = 0;

    if (counts_only && d.mode != MODE_ADD_KEEP && T.nev > 0 && chunk == 0) {   // no vote: leave the tile's tables zero for the next run
        for (uint32_t e = tid; e < T.bcap; e += WG) ((uint4 *)d.ibkt)[T.boff + e] = make_uint4(0, 0, 0, 0);
        if (tid == 0) d.ilong_n[tile] = 0;
    }
    lds_sync();
    TPROF_MARK(1);

    uint32_t X[8], Y[8], Z[8];
#pragma unroll
    for (int b = 0; b < 8; b++) X[b] = Y[b] = Z[b] = 0;
    uint32_t acc = 0;   // records counted per lane since the last flush (wave-uniform bound)
    // flush: counters → bytes (R[r] byte j = count of position 8j + r) → u16 pairs of the
    // histogram for the lane's word wd (lane gg of gn of the word, consecutive lanes); the
    // gn lanes pre-reduced by DPP row shifts while a byte cannot carry
    auto flush = [&](uint32_t wd, uint32_t gg, uint32_t gn, bool act) {
        transpose8(X);
        transpose8(Y);
        transpose8(Z);
        uint32_t red = 1;
        auto shr1 = [](uint32_t &v) { v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true); };
        auto shr2 = [](uint32_t &v) { v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true); };
        if (acc < 128 && gn >= 2) {
            red = 2;
#pragma unroll
            for (int r = 0; r < 8; r++) { shr1(X[r]); shr1(Y[r]); shr1(Z[r]); }
            if (acc < 64 && gn >= 4) {
                red = 4;
#pragma unroll
                for (int r = 0; r < 8; r++) { shr2(X[r]); shr2(Y[r]); shr2(Z[r]); }
            }
        }
        if (act && (gg % red) == red - 1 && !TABL(4)) {
            uint32_t *h0 = hist + 17 * wd;
            auto add = [&](uint32_t sym, const uint32_t (&R)[8]) {
                uint32_t *hw = h0 + sym * HP;
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const uint32_t lo = R[r] & 0x00FF00FFu, hi = (R[r] >> 8) & 0x00FF00FFu;
                    if (lo) atomicAdd(hw + r, lo);
                    if (hi) atomicAdd(hw + 8 + r, hi);
                }
            };
            add(SL_X, X);
            add(SL_Y, Y);
            add(SL_Z, Z);
        }
#pragma unroll
        for (int b = 0; b < 8; b++) X[b] = Y[b] = Z[b] = 0;
        acc = 0;
    };

    // ---- the wave's layers: lane (word ww, ga of GW) of the wave's own chunk
    constexpr uint32_t GW = 64 / NWP;
    const uint32_t ww = lane / GW, ga = lane % GW, Ww = W0 + ww;
    const bool wact = ww < nwords;
    auto &C = U.c[wv];
    // this lane's word reads the records of segments [sa, sb] (start words Ww - K .. Ww)
    const uint32_t sa = wact ? (Ww >= S0 + K ? Ww - K : S0) - S0 : 1u, sb = wact ? Ww - S0 : 0u;
    const uint2 *bql = (const uint2 *)(C.pl + 16);
    const int16_t wbias = (int16_t)(32 * ww + REC_BIAS);     // the word's first position, biased (rec_enc)
    const v2s wpk = (v2s){wbias, wbias};
    const uint2 *bqw = bql + ((32 * ww + REC_BIAS) >> 5);    // plane word of query y + wbias, less y >> 5
    // one group's records → carry-save trees of X, Y, Z; NR = 8: weight-8 carries in t8o,
    // NR = 4 (a tail group): weight-4 carries
    auto count_group = [&](const uint2 (&rv)[GS], uint32_t (&t8o)[3], auto nr) {
        constexpr int NR = decltype(nr)::value;
        uint32_t pend[3], t2a[3], t4a[3];
#pragma unroll
        for (int h = 0; h < NR; h += 2) {
            uint32_t bm[GS], fx[GS], sh[GS];
            uint2 pa[GS], pb[GS];
#pragma unroll
            for (int u = h; u < h + 2; u++) {
                rec_mask(rv[u].x, wpk, bm[u], fx[u]);   // the word's covered bits (rec_enc)
                sh[u] = rv[u].y;                       // (the funnel shift takes the low 5 bits)
                const uint2 *pw = bqw + ((int32_t)rv[u].y >> 5);
                pa[u] = pw[0];
                pb[u] = pw[1];
            }
#pragma unroll
            for (int u = h; u < h + 2; u++) {
                uint32_t x, y;   // plane & (bm | fx)
                asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe0" : "=v"(x) : "v"(funnel(pb[u].x, pa[u].x, sh[u])), "v"(bm[u]), "v"(fx[u]));
                asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe0" : "=v"(y) : "v"(funnel(pb[u].y, pa[u].y, sh[u])), "v"(bm[u]), "v"(fx[u]));
                auto chain = [&](uint32_t (&Cc)[8], int c, uint32_t mk) {
                    if ((u & 1) == 0) {
                        pend[c] = mk;
                        return;
                    }
                    uint32_t t2;
                    csa(t2, Cc[0], Cc[0], pend[c], mk);
                    if ((u & 3) == 1) {
                        t2a[c] = t2;
                        return;
                    }
                    uint32_t t4;
                    csa(t4, Cc[1], Cc[1], t2a[c], t2);
                    if ((u & 7) == 3) {
                        t4a[c] = t4;
                        if constexpr (NR == 4) t8o[c] = t4;
                        return;
                    }
                    csa(t8o[c], Cc[2], Cc[2], t4a[c], t4);
                };
                chain(X, 0, x);
                chain(Y, 1, y);
                chain(Z, 2, x & y);
            }
        }
    };
    using Full = std::integral_constant<int, 8>;
    using Half = std::integral_constant<int, 4>;

    // the layers: in place (one layer: the window of the sorted arrays) or the tile's copies
    // in the layered arrays
    const uint32_t ly0 = sload1(d.tiles + (size_t)tile * S2C_TILE_WORDS + 20);
    const bool inplace = ly0 == S2C_LY_MAIN;
    const uint32_t *const spc = inplace ? d.pc : d.lpc, *const sops = inplace ? d.ops : d.lops;
    const uint32_t *const sbq = inplace ? d.bq : d.lbq, *const sbx = inplace ? d.bx : d.lbx;
    const uint32_t *const spx = inplace ? d.px : d.lpx;
    const DmaSrc Dpc = dma_src(spc, inplace ? d.pc_end : d.lpc_end), Dops = dma_src(sops, inplace ? d.ops_end : d.lops_end);
    const DmaSrc Dbq = dma_src(sbq, inplace ? d.bq_end : d.lbq_end);
    const DmaSrc Dpx = dma_src(spx, inplace ? d.px_end : d.lpx_end);
    const uint4 *const pcr = C.pcb;
    // a layer's bounds: pieces [P0, P1), op words [O0, O1), plane words [qa, qb) (scalar loads)
    struct Lay {
        uint32_t P0, P1, O0, O1, qa, qb;
    };
    auto layer_of = [&](uint32_t ly) {
        Lay L;
        if (inplace) {
            const uint32_t *tw = d.tiles + (size_t)tile * S2C_TILE_WORDS;
            const uint4 A = sload4(tw + 12), B = sload4(tw + 16);   // words 13-18
            L.P0 = A.y; L.P1 = A.z; L.O0 = A.w; L.O1 = B.x; L.qa = B.y; L.qb = B.z;
        } else {
            const uint4 A = sload4(d.lly + 4 * (size_t)(ly0 + ly)), B = sload4(d.lly + 4 * (size_t)(ly0 + ly + 1));
            L.P0 = A.x; L.P1 = B.x; L.O0 = A.y; L.O1 = B.y;
            L.qa = A.z >> 1;
            L.qb = ((B.z + 1u) >> 1) + 1u;   // through the word after the last base (funnel)
        }
        return L;
    };
    // the ahead part of layer ly: its piece records and op words; returns the vmcnt events
    // issued
    auto issue_ahead = [&](const Lay &L) -> uint32_t {
        uint32_t k = dma16_wave((uint8_t *)C.pcb, Dpc, spc + 4 * (size_t)L.P0, 4 * (L.P1 - L.P0));
        if constexpr (PXL) k += dma16_wave((uint8_t *)C.pxl, Dpx, spx + L.P0, L.P1 - L.P0);
        return k + dma16_wave(C.ol, Dops, sops + L.O0, L.O1 - L.O0);
    };
    uint32_t ly = l0 + wv;
    Lay cur = {0, 0, 0, 0, 0, 0};
    if (ly < l1) {
        cur = layer_of(ly);
        issue_ahead(cur);
    }
    for (; ly < l1; ly += WV) {
        // ---- 1. the lane's pieces' 'N' offsets (S2C_PF_XFEW; read after the walk), the layer's
        //      planes (their buffer is free: the previous count is done), then the wait for
        //      what was issued ahead (older: everything but the planes)
        const uint32_t P0 = cur.P0, O0 = cur.O0, O1 = cur.O1, qa = cur.qa;
        const uint32_t NPc = cur.P1 - cur.P0, NR = O1 - O0;
        uint32_t pxr[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
        const uint32_t *pxl = nullptr;   // (PXL: px of layer piece i at pxl[i], ahead with the records)
        if constexpr (PXL) {
            pxl = C.pxl + (P0 & 3u);
        } else {
#pragma unroll
            for (int u = 0; u < 2; u++) pxr[u] = spx[lane + 64 * u < NPc ? P0 + lane + 64 * u : (NPc ? P0 : 0u)];   // (in bounds)
            asm volatile("" ::: "memory");   // (the loads stay ahead of the planes' DMA)
        }
        const uint32_t nq = dma16_wave(C.pl + 16, Dbq, sbq + 2 * (size_t)qa, 2 * (cur.qb - qa));
        wait_vm(nq);
        TPROF_MARK(2);
        const uint32_t *const opl = (const uint32_t *)C.ol;
        // ---- 2. walk: lane per piece (records to registers first); the per-word record
        //      ranges from the pieces' start words
        const uint32_t od = (O0 & 3u) - O0;                     // op word j at opl[j + od]
        const uint32_t qadj = 32u * (qa & 1u) - 32u * qa;       // SEQ[0] at LDS plane base 16·qh + qadj
        const gptr_u32 xg = (gptr_u32)(sbx + (qa - (qa & 1u)));   // non-ACGT word of LDS plane word v: xg[v] (HBM)
        uint4 Pw[2];
        uint32_t oe[2];
        bool planes = false;   // a piece of the lane reads the planes in its walk
        EvOut eo;              // (REC: the lane's insertion events, keyed after the planes wait)
        eo.n = 0;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t i = lane + 64 * u;
            Pw[u] = make_uint4(0u, 0u, 0u, 0u);
            oe[u] = 0;
            if (i < NPc) {
                Pw[u] = pcr[i];
                if constexpr (PXL) pxr[u] = pxl[i];
                oe[u] = i + 1 < NPc ? pcr[i + 1].z : O1;
                const int32_t sw = (int32_t)(Pw[u].x >> 5) - (int32_t)S0;
                const int32_t pw = i > 0 ? (int32_t)(pcr[i - 1].x >> 5) - (int32_t)S0 : -1;
                for (int32_t sg = pw + 1; sg <= sw; sg++) C.segR[sg] = (uint16_t)(Pw[u].z - O0);
                if (i + 1 == NPc)
                    for (uint32_t sg = (uint32_t)(sw + 1); sg <= NS; sg++) C.segR[sg] = (uint16_t)NR;
                const uint32_t f = Pw[u].w >> 24;
                if constexpr (PXL)   // (x_fix and the maxdel '-' count read the planes; S2C_PF_XFEW pieces take px;
                                     //  recorded events are keyed after the walk)
                    planes |= (f & S2C_PF_X) && !(f & (S2C_PF_XFEW | S2C_PF_LONG));
                else
                    planes |= (f & S2C_PF_SIMPLE) ? ((f & S2C_PF_X) && !(f & S2C_PF_XFEW)) : !(f & S2C_PF_LONG);
            }
        }
        if (NPc == 0)
            for (uint32_t sg = lane; sg <= NS; sg += 64) C.segR[sg] = 0;
        if (__ballot(planes)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the planes, for those walks)
        for (uint32_t i = lane; i < rpad_of(NWP); i += 64) C.runl[NR + i] = make_uint2(0u, 0u);
        TPROF_MARK(10);    // (the records, segments and any planes wait of the walk)
        if (TABL(1))   // (ablated walk: zero records)
            for (uint32_t i = lane; i < NR; i += 64) C.runl[i] = make_uint2(0u, 0u);
        // (WQ) the pieces walked op by op go to a queue, walked after the others by the wave's
        // first lanes: one such walk per lane and layer, not one for each of a lane's two pieces
        uint32_t nwq = 0;
        if constexpr (WQ) {
            bool cx[2];
#pragma unroll
            for (int u = 0; u < 2; u++)
                cx[u] = lane + 64 * u < NPc && !TABL(1) && !((Pw[u].w >> 24) & (S2C_PF_SIMPLE | S2C_PF_LONG));
            const uint64_t m0 = __ballot(cx[0]), m1 = __ballot(cx[1]);
            const uint32_t n0 = (uint32_t)__popcll(m0);
            auto below = [&](uint64_t m) {
                return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            };
            if (cx[0]) C.wq[below(m0)] = (uint8_t)lane;
            if (cx[1]) C.wq[n0 + below(m1)] = (uint8_t)(lane + 64);
            nwq = uni(n0 + (uint32_t)__popcll(m1));
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            if (lane + 64 * u >= NPc || TABL(1)) continue;
            const uint4 P = Pw[u];
            const uint32_t fl = P.w >> 24, len = P.w & 0xFFFFFFu, rPre = P.z - O0;
            const uint32_t ql = 16u * P.y + qadj;
            if (fl & S2C_PF_SIMPLE) {   // one run of SEQ[0:take] (:64-69)
                const uint32_t c0 = max(P.x, a), c1 = min(P.x + len, a + n);
                C.runl[rPre] = len ? rec_enc(P.x - 32u * W0, len, ql) : make_uint2(0u, 0u);
                if (c1 > c0) {
                    atomicAdd(&dV[c0 - a], 1);
                    atomicSub(&dV[c1 - a], 1);
                    if (PXL && (fl & (S2C_PF_X | S2C_PF_XFEW)) == (S2C_PF_X | S2C_PF_XFEW)) {   // ≤ 2 'N' at SEQ offsets px
#pragma unroll
                        for (int h = 0; h < 2; h++) {
                            const uint32_t off = (pxr[u] >> (16 * h)) & 0xFFFFu, p = P.x + off;   // (0xFFFF: none)
                            if (off != 0xFFFFu && p >= c0 && p < c1) H::add1(hist, SL_N, p - a, 1u);
                        }
                    } else if ((fl & S2C_PF_X) && !(fl & S2C_PF_XFEW)) {   // (without PXL: S2C_PF_XFEW after the walk)
                        x_fix<NWP, WQ>(bql, xg, 0u, ql + (c0 - P.x), c1 - c0, c0 - a, false, hist);
                    }
                }
            } else if (fl & S2C_PF_LONG) {   // (its runs come through the tile long lists)
                for (uint32_t j = P.z; j < oe[u]; j++) C.runl[j - O0] = make_uint2(0u, 0u);
            } else if constexpr (!WQ) {
                walk_chunk_piece<NWP, PXL, WQ, REC>(P, oe[u], opl, od, C.runl, 0u - O0, bql, xg, 0u, qadj, d.maxdel_active != 0,
                                               (uint32_t)d.maxdel, a, n, hist, dV, dD, pxr[u], evr, eo);
            }
        }
        TPROF_MARK(11);    // (the one-token pieces; MARK(9) below: the op walks)
        if constexpr (WQ) {
            if (nwq) wave_lds_sync();   // (the queue)
            // 16 queued pieces per pass, 4 lanes each: a piece of ≤ 4 op words (no shard range,
            // no '-' in SEQ) one op word per lane (walk_op_coop); any other by its group's first lane
            constexpr bool COOP = NWP >= 16;   // (k_tile<8, true>: the serial walks only; the cooperative one spills there)
            const uint32_t sub = lane & 3u;
            bool serial = !COOP;   // (uniform) some queued piece takes the serial walk
            for (uint32_t kb = 0; kb < (COOP ? nwq : 0u); kb += 16) {
                const uint32_t k = kb + (lane >> 2);
                const bool have = k < nwq;
                const uint32_t i = have ? (uint32_t)C.wq[k] : 0u;
                const uint4 P = have ? pcr[i] : make_uint4(0u, 0u, 0u, 0u);
                const uint32_t oend = have ? (i + 1 < NPc ? pcr[i + 1].z : O1) : 0u;
                const uint32_t fl = P.w >> 24;
                const bool ins = (fl & S2C_PF_INS) != 0u;
                const uint32_t j0 = P.z + (ins ? 3u : 0u);
                const bool coop = have && !(fl & (S2C_PF_RANGE | S2C_PF_DASH)) && oend - j0 <= 4u;
                const uint32_t pxw = have && PXL ? pxl[i] : 0xFFFFFFFFu;
                serial = serial || __ballot(have && !coop) != 0ull;
                if (__ballot(coop)) {
                    const bool rec = REC && evr.on && coop && ins;
                    int64_t key0 = 0;
                    uint32_t roff = 0;
                    if (rec) {
                        key0 = (int64_t)((uint64_t)opl[P.z + od] | ((uint64_t)opl[P.z + 1 + od] << 32));
                        roff = opl[P.z + 2 + od];
                    }
                    if (coop && ins && sub < 3u) C.runl[P.z + sub - O0] = make_uint2(0u, 0u);   // (the key words' slots)
                    walk_op_coop<NWP, PXL, WQ, REC>(P, coop && sub < oend - j0, j0 + sub, sub, opl, od, C.runl, 0u - O0, bql, xg,
                                                    0u, qadj, d.maxdel_active != 0, (uint32_t)d.maxdel, a, n, hist, dV, dD,
                                                    pxw, key0, roff, rec, evr, eo);
                }
            }
            // the other queued pieces (rare): one lane each, the serial walk
            for (uint32_t k = lane; k < (serial ? nwq : 0u); k += 64) {
                const uint32_t i = C.wq[k];
                const uint4 P = pcr[i];
                const uint32_t oend = i + 1 < NPc ? pcr[i + 1].z : O1, fl = P.w >> 24;
                const bool coop = COOP && !(fl & (S2C_PF_RANGE | S2C_PF_DASH)) && oend - (P.z + ((fl & S2C_PF_INS) ? 3u : 0u)) <= 4u;
                if (!coop)
                    walk_chunk_piece<NWP, PXL, WQ, REC>(P, oend, opl, od, C.runl, 0u - O0, bql, xg, 0u, qadj, d.maxdel_active != 0,
                                               (uint32_t)d.maxdel, a, n, hist, dV, dD, PXL ? pxl[i] : 0xFFFFFFFFu, evr, eo);
            }
        }
        wave_lds_sync();   // every run record written; the piece records and op words read
        TPROF_MARK(9);     // (the walk's own work; MARK(3) below: the wait for the planes)
        // this layer's planes (and 'N' offsets) have landed from here on
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (REC) {   // the lane's held events keyed from the landed planes (EvOut)
            if (eo.n) ev_flush(bql, xg, 0u, eo, evr);
        }
#pragma unroll
        for (int u = 0; u < 2 && !PXL; u++) {   // ≤ 2 'N' of an S2C_PF_XFEW piece at its SEQ offsets px: no plane scan
            const uint4 P = Pw[u];
            const uint32_t fl = P.w >> 24;
            if (lane + 64 * u >= NPc || TABL(1) || (fl & (S2C_PF_SIMPLE | S2C_PF_XFEW)) != (S2C_PF_SIMPLE | S2C_PF_XFEW))
                continue;
            const uint32_t c0 = max(P.x, a), c1 = min(P.x + (P.w & 0xFFFFFFu), a + n);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t off = (pxr[u] >> (16 * h)) & 0xFFFFu, p = P.x + off;   // (0xFFFF: none)
                if (off != 0xFFFFu && p >= c0 && p < c1) H::add1(hist, SL_N, p - a, 1u);
            }
        }
        TPROF_MARK(3);
        // ---- 3. the next layer's piece records and op words, under this layer's count
        if (ly + WV < l1) {
            cur = layer_of(ly + WV);
            issue_ahead(cur);
        }
        // ---- 4. count this lane's records cw0 + ga + GW·m < cw1 (reads past them: records of
        //      pieces starting after Ww, or the zero pad — they cover nothing of Ww)
        const uint32_t cw0 = C.segR[sa], cw1 = C.segR[sb + 1];
        const uint32_t nrec = cw0 + ga < cw1 ? (cw1 - cw0 - ga + GW - 1) / GW : 0u;
        const uint32_t nmx = TABL(2) ? 0u : uni(__ockl_wfred_max_u32(nrec));
        const uint32_t ngrp = nmx / GS + ((nmx % GS) > 4u ? 1u : 0u);
        const bool half = (nmx % GS) != 0u && (nmx % GS) <= 4u;
        const uint32_t add_recs = GS * ngrp + (half ? 4u : 0u);
        if (acc + add_recs > 255u) flush(ww, ga, GW, wact);
        acc += add_recs;
        const uint32_t rend = NR;
        auto load_runs = [&](uint2 (&rv)[GS], uint32_t gi) {   // (64-bit loads: two records per ds_read2_b64)
            const unsigned long long *rb = (const unsigned long long *)(C.runl + min(cw0 + ga + GW * GS * gi, rend));
#pragma unroll
            for (int u = 0; u < GS; u++) {
                unsigned long long r = rb[GW * u];
                asm("" : "+v"(r));   // (kept one 64-bit load: its halves are used as different types)
                rv[u] = make_uint2((uint32_t)r, (uint32_t)(r >> 32));
            }
        };
        uint2 ra[GS], rb2[GS];
        if (ngrp) load_runs(ra, 0);
        for (uint32_t gi = 0; gi < ngrp; gi += 2) {
            uint32_t t8a[3], t8b[3];
            if (gi + 1 < ngrp) load_runs(rb2, gi + 1);
            count_group(ra, t8a, Full{});
            if (gi + 1 >= ngrp) {
                close8(X, t8a[0]);
                close8(Y, t8a[1]);
                close8(Z, t8a[2]);
                break;
            }
            if (gi + 2 < ngrp) load_runs(ra, gi + 2);
            count_group(rb2, t8b, Full{});
            close16(X, t8a[0], t8b[0]);
            close16(Y, t8a[1], t8b[1]);
            close16(Z, t8a[2], t8b[2]);
        }
        if (half) {   // records 8·ngrp .. 8·ngrp + 3 of each lane
            uint32_t t4[3];
            load_runs(ra, ngrp);
            count_group(ra, t4, Half{});
            close4(X, t4[0]);
            close4(Y, t4[1]);
            close4(Z, t4[2]);
        }
        wave_lds_sync();   // the planes and run records are rewritten by the wave's next layer
        TPROF_MARK(4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (nothing of this wave's in flight past here)
    if (acc) flush(ww, ga, GW, wact);
    lds_sync();   // every wave's layers counted (hist, dV, dD complete but for the long pieces)

    // the workgroup's lanes for the long pieces: word w, lane g of G = 256 / NWP
    constexpr uint32_t G = WG / NWP;
    const uint32_t w = tid / G, g = tid % G, W = W0 + w;
    const bool active = w < nwords;
    // ---- long pieces (rare), counted once per tile (by its first item), one list entry per
    //      lane and round: k_reads' run records through the tile's long list of run slots, or
    //      for a dense tile (run here in counts-only modes) its long pieces themselves, walked
    //      from HBM (walk_piece) — each run's part in the lane's word W
    {
        auto one_run = [&](uint32_t gpos, uint32_t len, uint32_t kind, uint64_t q) {
            const RecGeom gm = rec_geom(gpos, len, W);
            if (!gm.valid) return;
            const uint32_t p0 = 32 * w + gm.lo, p1 = p0 + (uint32_t)__popc(gm.valid);
            if ((kind & 3u) == S2C_RUN_DASH) {
                atomicAdd(&dD[p0], 1);
                atomicSub(&dD[p1], 1);
            } else if ((kind & 3u) == S2C_RUN_BASES) {
                const uint64_t qs = q + gm.qs, qw = qs >> 5;
                const uint32_t sh = (uint32_t)(qs & 31);
                const uint32_t mx = (funnel(d.bq[2 * qw + 2], d.bq[2 * qw], sh) << gm.lo) & gm.valid;
                const uint32_t my = (funnel(d.bq[2 * qw + 3], d.bq[2 * qw + 1], sh) << gm.lo) & gm.valid;
                ripple1(X, mx);
                ripple1(Y, my);
                ripple1(Z, mx & my);
                atomicAdd(&dV[p0], 1);
                atomicSub(&dV[p1], 1);
                if (kind & S2C_RUN_XBIT) {
                    uint32_t xm = (funnel(d.bx[qw + 1], d.bx[qw], sh) << gm.lo) & gm.valid;
                    while (xm) {
                        const uint32_t bit = (uint32_t)__builtin_ctz(xm);
                        xm &= xm - 1;
                        if ((mx >> bit) & 1u) {   // '-' of SEQ (p0 = 1)
                            H::add1(hist, SL_SD, 32 * w + bit, 1u);
                            if (!(kind & S2C_RUN_DROP)) H::add1(hist, SL_SDC, 32 * w + bit, 1u);
                        } else {
                            H::add1(hist, SL_N, 32 * w + bit, 1u);
                        }
                    }
                }
            }
        };
        const bool lpieces = (T.flags & S2C_TILE_DENSE) != 0;
        const uint32_t nlong = l0 == 0 ? T.lp1 - T.lp0 : 0u;
        const uint32_t ntr = uni(__ockl_wfred_max_u32(active && g < nlong ? (nlong - g + G - 1) / G : 0u));
        for (uint32_t m = 0; m < ntr; m++) {
            // (a walked piece adds at most one to a position: its runs cover disjoint positions)
            if (acc >= 255u) flush(w, g, G, active);
            acc++;
            const uint32_t j = g + G * m;
            if (!(active && j < nlong)) continue;
            const uint32_t e = d.lp[T.lp0 + j];
            if (lpieces) {
                const uint4 P = ((const uint4 *)d.pc)[e];
                walk_piece(TileMem{d.ops, d.bq, d.bx}, P, d.pc[4 * (size_t)e + 6], d.maxdel_active != 0, d.maxdel,
                           [&](uint32_t, uint32_t gp, uint32_t l, uint32_t kind, uint64_t q) {
                               if (kind != S2C_RUN_EMPTY) one_run(gp, l, kind, q);
                           },
                           [](uint64_t, uint64_t, uint32_t) {});   // (a dense tile holds no insertion keys)
            } else {
                const Run r = run_of(((const uint4 *)d.runs)[e]);
                one_run(r.gpos, r.len, r.kind, r.q);
            }
        }
    }
    if (acc) flush(w, g, G, active);
    lds_sync();
    TPROF_MARK(5);
    // ---- difference arrays → coverage and '-' per position (inclusive scans, thread blocks
    //      of NPOS / WG positions)
    {
        constexpr uint32_t PER = NPOS / WG;   // NWP / 8
        const uint32_t p0 = tid * PER;
        int32_t sv = 0, sd = 0;
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            sv += dV[p0 + i];
            sd += dD[p0 + i];
        }
        uint32_t tv, td;
        const uint32_t iv = __ockl_wfscan_add_u32((uint32_t)sv, true), idd = __ockl_wfscan_add_u32((uint32_t)sd, true);
        if (lane == 63) {
            wtot[0][wv] = iv;
            wtot[1][wv] = idd;
        }
        lds_sync();
        uint32_t ov = 0, od = 0;
#pragma unroll
        for (uint32_t k = 0; k < WG / 64; k++) {
            ov += k < wv ? wtot[0][k] : 0u;
            od += k < wv ? wtot[1][k] : 0u;
        }
        tv = ov + iv - (uint32_t)sv;
        td = od + idd - (uint32_t)sd;
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            tv += (uint32_t)dV[p0 + i];
            td += (uint32_t)dD[p0 + i];
            dV[p0 + i] = (int32_t)tv;
            dD[p0 + i] = (int32_t)td;
        }
    }
    lds_sync();
    // ---- raw slots → "-ACGNT" counts in place (u16 pairs: positions 32·v + i, + 16)
    for (uint32_t s = tid; s < 16u * NWP; s += WG) {
        const uint32_t hs = hslot(s);
        uint32_t raw[NSYM];
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) raw[c] = hist[c * HP + hs];
        const uint32_t q0 = 32 * (s >> 4) + (s & 15);
        uint32_t outw[NSYM] = {};
#pragma unroll
        for (int hh = 0; hh < 2; hh++) {
            const uint32_t sh = 16 * hh, q = q0 + 16 * hh;
            auto f = [&](uint32_t c) { return (raw[c] >> sh) & 0xFFFFu; };
            const uint32_t x = f(SL_X), y = f(SL_Y), z = f(SL_Z), nn = f(SL_N), sd = f(SL_SD), sdc = f(SL_SDC);
            const uint32_t v = (uint32_t)dV[q], dd = (uint32_t)dD[q];
            const uint32_t cnt[NSYM] = {dd + sdc, v - x - y + z - nn, x - z - sd, y - z, nn, z};
#pragma unroll
            for (uint32_t c = 0; c < NSYM; c++) outw[c] |= (cnt[c] & 0xFFFFu) << sh;
        }
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) hist[c * HP + hs] = outw[c];
    }
    lds_sync();
    TPROF_MARK(6);
    if (finish) {
        // the epilogue's LDS (aliases the chunk): layout arrays zeroed, tables, fill
        FastLds<ICOL> &L = U.e.L;
        uint32_t *cols = U.e.cols;
        if (tid < 64) L.amb[tid] = c_amb[tid];
        const bool has_ins = T.nev > 0;
        if (has_ins) {
            L.klen[tid] = 0;
            L.kem2[0][tid] = 0;
            L.kem2[1][tid] = 0;
            if (tid < TILE_WORDS) L.bits[tid] = 0;
            for (uint32_t i = tid; i < T.ccap * NSYM && i < ICOL * NSYM; i += WG) cols[i] = 0;
        }
        if (tid < (uint32_t)min(d.fill_len, FILL_LDS)) L.fill[tid] = d.fill[tid];
        lds_sync();
        InsLayout il = {0, 0};
        if (has_ins)
            il = build_layout<PF, false>(d, T, tile, L.bits, L.wrank, L.klen, L.key, cols, L.colkey, L.scan, evl,
                                         rec_ev ? min(evn, (uint32_t)S2C_EPI_KEYS) : 0u, !(rec_ev && d.tables_empty));
        TPROF_MARK(12);   // (the epilogue's LDS set up and the insertion layout; MARK(7): the votes and stores)
        tile_epilogue_fast<NWP>(d, tile, T, il, hist, cols, L);
    } else {
        // deep tile: this item's counts → HBM (symbol-major, coalesced atomics); a general
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
    TPROF_MARK(7);
#ifdef S2C_PROF
    if (threadIdx.x == 0 && (blockIdx.x & 15) == 0) {
        atomicAdd(&g_tprof[15], 1ull);
        atomicAdd(&g_tprof[14], (unsigned long long)(l1 - l0));
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
    S2C_POISON(&L, sizeof(L));
    S2C_POISON_DONE();
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t tile = deep[blockIdx.x];
    const TileRec T = tile_rec(d.tiles, tile);
    const uint32_t a = T.a, n = T.b - T.a;
    if (tid < 64) L.amb[tid] = c_amb[tid];
    for (uint32_t i = tid; i < KMAX; i += WG) L.klen[i] = 0;
    if (tid < TILE_WORDS) L.bits[tid] = 0;
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
                    const uint8_t ic = L.amb[column_masks(v, cov, d.thresholds + t, 1) & 63u];
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
                const double th = d.thresholds[t0 + u];
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
    // the tile's HBM counts read for the last time: left zero for the next run, whose deep items
    // add into them (s2c_dev.counts; round 6 — a k_prep launch zeroed them before every run)
    for (uint32_t c = 0; c < NSYM; c++)
        for (uint32_t i = tid; i < n; i += WG) d.counts[(size_t)c * d.padded_len + a + i] = 0u;
}

inline int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return S2C_OK;
    return s2c_set_error(S2C_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

TileArgs tile_args(const s2c_dev &d) {
    TileArgs p;
    p.rs = d.rs; p.runs = d.runs; p.bq = d.bq; p.bx = d.bx; p.tiles = d.tiles; p.lp = d.lp;
    p.pc = d.pc; p.ops = d.ops; p.ps = d.ps; p.bq_end = d.bq + 2 * d.n_qwords; p.bx_end = d.bx + d.n_qwords;
    p.ops_end = d.ops + std::max<int64_t>(d.n_ops, 1); p.pc_end = d.pc + 4 * (d.n_pieces + 1);
    p.lly = d.lly; p.lpc = d.lpc; p.lops = d.lops; p.lbq = d.lbq; p.lbx = d.lbx;
    p.px = d.px; p.lpx = d.lpx;
    p.px_end = d.px + std::max<int64_t>(d.n_pieces, 1); p.lpx_end = d.lpx ? d.lpx + std::max<int64_t>(d.n_lpieces, 1) : nullptr;
    p.lbq_end = d.lbq + 2 * d.n_lqwords; p.lbx_end = d.lbx + d.n_lqwords;
    p.lops_end = d.lops + std::max<int64_t>(d.n_lops, 4); p.lpc_end = d.lpc + 4 * (d.n_lpieces + 1);
    p.maxdel_active = d.maxdel_active ? 1u : 0u;
    p.maxdel = d.maxdel < 0 ? 0u : (uint32_t)d.maxdel;
    p.ibkt = d.ibkt; p.ilong = d.ilong; p.ilong_n = d.ilong_n;
    p.thresholds = d.thresholds; p.fill = d.fill; p.counts = d.counts; p.ins_cols = d.ins_cols; p.ins_chr = d.ins_chr;
    p.tile_stats = d.tile_stats; p.blk_len = d.blk_len; p.out = d.out;
    p.padded_len = (uint32_t)d.padded_len; p.n_cols = (uint32_t)d.n_cols; p.n_tiles = (uint32_t)d.n_tiles;
    p.kwin = (uint32_t)d.kwin; p.chunk = (uint32_t)d.chunk; p.n_qwords = (uint32_t)d.n_qwords;
    p.runs_bytes = (uint32_t)std::min<int64_t>(16 * std::max<int64_t>(d.n_ops, 1), 0xFFFFFFF0ll);
    p.mode = MODE_RUN;
    p.walk_queue = d.walk_queue ? 1u : 0u;
    p.tile_events = d.walk_queue && d.tile_events ? 1u : 0u;
    p.tables_empty = p.tile_events && d.n_rlist_run == 0 ? 1u : 0u;
    p.n_thr = d.n_thr; p.min_depth = d.min_depth; p.fill_len = d.fill_len; p.fill_nondash = d.fill_nondash;
    return p;
}

template <int NWP>
int launch_tile(const TileArgs &a, const uint32_t *items, int64_t n, hipStream_t s) {
    if (n <= 0) return S2C_OK;
    if (a.walk_queue) k_tile<NWP, true><<<(unsigned)n, WG, 0, s>>>(a, items);
    else k_tile<NWP, false><<<(unsigned)n, WG, 0, s>>>(a, items);
    return hip_check(hipGetLastError(), "k_tile");
}
int launch_tiles(const TileArgs &a, int32_t tile_max, const uint32_t *items, int64_t n, hipStream_t s) {
    if (tile_max <= 256) return launch_tile<8>(a, items, n, s);
    if (tile_max <= 512) return launch_tile<16>(a, items, n, s);
    if (tile_max <= 1024) return launch_tile<32>(a, items, n, s);
    return launch_tile<64>(a, items, n, s);
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
    if (d->tile_max <= 0 || d->tile_max > S2C_TILE_MAX) return s2c_set_error(S2C_ERR_ARG, "tile_max out of range");
    if (d->padded_len <= 0 || d->padded_len >= ((int64_t)1 << 32)) return s2c_set_error(S2C_ERR_ARG, "bad padded_len");
    if (d->n_tiles >= ((int64_t)1 << 31) || (int64_t)d->n_thr * d->n_tiles >= ((int64_t)1 << 40))
        return s2c_set_error(S2C_ERR_LIMIT, "too many (threshold, tile) blocks");
    if (16 * d->n_ops >= 0xE0000000ll || 8 * d->n_qwords >= 0xE0000000ll || 16 * d->n_pieces >= 0xE0000000ll ||
        8 * d->n_lqwords >= 0xE0000000ll || 16 * d->n_lpieces >= 0xE0000000ll || 4 * d->n_lops >= 0xE0000000ll)
        return s2c_set_error(S2C_ERR_LIMIT, "run records, pieces or base planes beyond 3.5 GB (split the input)");   // 32-bit buffer offsets
    if (d->n_layers > 0 && (!d->lly || !d->lpc || !d->lops || !d->lbq || !d->lbx || !d->lpx))
        return s2c_set_error(S2C_ERR_ARG, "missing layered windows");
    // k_tile reads every work item's tile through its layered windows (tile word 20): a batch
    // whose layers were never built (e.g. a fresh s2c_batch_shard) holds no valid ones
    if (d->n_items > 0 && !d->layers_built)
        return s2c_set_error(S2C_ERR_ARG, "the batch's layered windows are not built (s2c_batch_layers before upload)");
    if (d->n_pieces > 0 && (!d->pc || !d->ops || !d->bq || !d->bx || !d->runs || !d->px))
        return s2c_set_error(S2C_ERR_ARG, "missing piece buffers");
    if (d->n_tiles > 0 && (!d->tiles || !d->rs || !d->wtile || !d->tile_stats || !d->blk_len || !d->out))
        return s2c_set_error(S2C_ERR_ARG, "missing tile / output buffers");
    if ((d->n_items > 0 && !d->items) || (d->n_dense > 0 && (!d->dense || !d->dwin)))
        return s2c_set_error(S2C_ERR_ARG, "missing items");
    if (!d->ibkt || !d->ilong || !d->ilong_n) return s2c_set_error(S2C_ERR_ARG, "missing insertion tables");
    if (d->n_tiles > 0 && !d->ps) return s2c_set_error(S2C_ERR_ARG, "missing piece CSR (ps)");
    // (ABI 13) the per-word entries the device copies hold: a batch with tiles has some
    if (d->word_lo < 0 || d->word_hi < d->word_lo || 32 * d->word_hi > d->padded_len || d->word_hi >= ((int64_t)1 << 32) ||
        (d->n_tiles > 0 && d->word_hi == d->word_lo))
        return s2c_set_error(S2C_ERR_ARG, "bad per-word span word_lo / word_hi (s2c_batch_info, ABI 13)");
    {   // k_tile's segments: a window of ≤ 64 words and kwin start words before it
        int64_t nwp = 8;
        while (nwp * 32 < d->tile_max) nwp *= 2;
        if (d->kwin < 0 || d->kwin + nwp > S2C_CHUNK_SEGS) return s2c_set_error(S2C_ERR_ARG, "kwin beyond k_tile's segments");
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
    // the tile kernels walk their windows' pieces themselves: k_reads takes the insertion
    // emitters and the long pieces (rlist)
    return s2c_launch_reads(d, (hipStream_t)stream, false, true);
}

extern "C" int s2c_pileup(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    // dense tiles emit exactly one char per position: len(fill) must be 1, else k_tile (which
    // reads their layered windows) — refused before anything is launched
    if (d->n_dense > 0 && d->fill_len != 1 && !d->layers_dense)
        return s2c_set_error(S2C_ERR_ARG, "a fill of length != 1 runs the dense tiles through k_tile: their layered "
                                          "windows are needed (s2c_batch_layers_mode(b, 1))");
    hipStream_t s = (hipStream_t)stream;
    const TileArgs a = tile_args(*d);
    // (the deep tiles' HBM counts are zero: before the first run by the caller, after every
    // run by s2c_consensus — s2c_dev.counts)
    if (d->n_dense > 0) {
        rc = d->fill_len == 1 ? s2c_launch_dense(d, s) : launch_tiles(a, d->tile_max, d->dense, d->n_dense, s);
        if (rc) return rc;
    }
    return launch_tiles(a, d->tile_max, d->items, d->n_items, s);
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
    if (d->n_dense > 0 && !d->layers_dense)   // (k_tile takes the dense tiles here: their layers)
        return s2c_set_error(S2C_ERR_ARG, "counts-only modes need the dense tiles' layered windows (s2c_batch_layers_mode(b, 1))");
    hipStream_t s = (hipStream_t)stream;
    if ((rc = s2c_launch_reads(d, s, true, false))) return rc;   // run records of every piece (compared by the tests)
    TileArgs a = tile_args(*d);
    a.mode = MODE_STORE;
    if (d->n_deep > 0) {
        k_prep<<<(unsigned)d->n_deep, WG, 0, s>>>(a, d->deep);
        if ((rc = hip_check(hipGetLastError(), "k_prep"))) return rc;
    }
    if ((rc = launch_tiles(a, d->tile_max, d->dense, d->n_dense, s))) return rc;
    return launch_tiles(a, d->tile_max, d->items, d->n_items, s);
}

extern "C" int s2c_accumulate(const s2c_dev *d, int keep_tables, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    if (!d->counts) return s2c_set_error(S2C_ERR_ARG, "counts buffer required");
    if (d->n_dense > 0 && !d->layers_dense)   // (k_tile takes the dense tiles here: their layers)
        return s2c_set_error(S2C_ERR_ARG, "counts-only modes need the dense tiles' layered windows (s2c_batch_layers_mode(b, 1))");
    hipStream_t s = (hipStream_t)stream;
    if ((rc = s2c_launch_reads(d, s, false, false))) return rc;   // every event hashed, long pieces' runs
    TileArgs a = tile_args(*d);
    a.mode = keep_tables ? MODE_ADD_KEEP : MODE_ADD;
    if ((rc = launch_tiles(a, d->tile_max, d->dense, d->n_dense, s))) return rc;
    return launch_tiles(a, d->tile_max, d->items, d->n_items, s);
}

// s2c_dense.hip — k_tile_dense: shallow tiles without insertion keys (-f of one char).
//
// Such a tile's body is one char per position (:355-389 with no insertion columns and a
// one-char fill), so the byte offset of position q is q: no length scan.  One wave per tile
// walks the tile's window itself (the short pieces starting up to kwin words before it):
// the window's op words, base planes {p0, p1} and non-ACGT plane (one contiguous range
// each) arrive in LDS by one LDS-DMA sweep, one lane per piece runs parsecigar + maxdel
// (walk_piece, :46-82, :210) into run records in LDS, and the G = 64 / (tile words) lanes
// of a word count the records covering it — A C G T into bit-sliced counters (as in
// k_tile), a group of 8 records at a time; the rare '-' and 'N' into per-position byte
// counters in LDS.  The word's lanes all-reduce their byte counters with DPP (every
// position's total is ≤ 255, host plan), and each lane votes its 32/G consecutive
// positions for every threshold (closed form of :241-251 / :359-366 with the
// strict-majority shortcut) and stores their chars with wide stores.  Counts never touch
// HBM.  The host sizes the tiles so the window takes ≤ S2C_DENSE_LDS bytes
// (S2C_DENSE_BYTES; ≈ 1024 positions at 30x coverage).
#include "s2c_common.h"

#ifdef S2C_PROF
// phase clocks (diagnostic build `make prof`, scripts/prof_dense.py): Σ over sampled waves
// (one tile in 64) of the s_memtime deltas of each phase
__device__ unsigned long long g_prof[16];
__device__ uint32_t g_abl;   // ablation bits (timing only; results wrong): 1 events, 2 count, 4 walk, 8 vote
#define ABL(b) ((g_abl & (b)) != 0)
#define PROF_MARK(i)                                                                               \
    do {                                                                                           \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();                                \
        if (threadIdx.x == 0 && (blockIdx.x & 63) == 0 && (i) > 0) atomicAdd(&g_prof[(i)-1], _t - prof_t); \
        prof_t = _t;                                                                               \
    } while (0)
#else
#define ABL(b) false
#define PROF_MARK(i) \
    do {             \
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

struct DenseArgs {
    const uint32_t *rs, *pc, *ops, *bq, *bx, *tiles, *items;
    const double *thresholds;
    uint64_t *tile_stats, *blk_len;
    uint8_t *out;
    uint32_t padded_len, n_cols, n_tiles, kwin, fill_nondash, maxdel_active, maxdel;
    int32_t n_thr, min_depth;
    const uint8_t *fill;   // the one -f char
};

// The token walk of walk_piece (s2c_common.h: parsecigar :64-81 + maxdel :210) in 32-bit
// window-relative coordinates (klen, len(SEQ) < 2^24; the window's query bases < 2^17),
// without insertion events (a dense tile holds no keys).  q0: window-relative query base of
// SEQ[0]; op words j are window-relative; run(j, gpos, len, kind, q) as in walk_piece with
// q window-relative.
template <class RunFn>
__device__ __forceinline__ void walk_window(const uint32_t *opl, const uint2 *bql, const uint32_t *bxl, const uint4 P,
                                            uint32_t j0, uint32_t j1, uint32_t q0, bool maxdel_active, uint32_t maxdel,
                                            RunFn &&run) {
    const uint32_t slen = P.w & 0xFFFFFFu, fl = P.w >> 24;
    uint32_t j = j0;
    uint32_t ka = 0, kb = 0xFFFFFFFFu;
    if (fl & S2C_PF_RANGE) {
        ka = opl[j];
        kb = opl[j + 1];
        run(j, 0u, 0u, S2C_RUN_EMPTY, 0u);
        run(j + 1, 0u, 0u, S2C_RUN_EMPTY, 0u);
        j += 2;
    }
    if (fl & S2C_PF_INS) {   // key words: its events are keyed in other tiles
        for (uint32_t i = 0; i < 3; i++) run(j + i, 0u, 0u, S2C_RUN_EMPTY, 0u);
        j += 3;
    }
    bool drop = false;
    if (maxdel_active) {   // :210
        uint32_t dashes = 0, start = 0;
        for (uint32_t i = j; i < j1; i++) {
            const uint32_t w = opl[i], op = w & 15u, l = w >> 4;
            if (op_bases(op)) {
                uint32_t take = start < slen ? min(l, slen - start) : 0u;
                if (fl & S2C_PF_X) {   // '-' chars of SEQ: x = 1, p1 = 0, p0 = 1
                    uint32_t q = q0 + start;
                    while (take) {
                        const uint32_t qw = q >> 5, sh = q & 31u, nb = min(take, 32u - sh);
                        const uint32_t mask = (nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u)) << sh;
                        dashes += (uint32_t)__popc(bxl[qw] & bql[qw].x & ~bql[qw].y & mask);
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
    const uint32_t bkind = S2C_RUN_BASES | ((fl & S2C_PF_X) ? S2C_RUN_XBIT : 0u) | (drop ? S2C_RUN_DROP : 0u);
    uint32_t k = 0, start = 0;
    for (; j < j1; j++) {
        const uint32_t w = opl[j], op = w & 15u, l = w >> 4;
        uint32_t rg = 0, rl = 0, rk = S2C_RUN_EMPTY, rq = 0;
        const bool bases = op_bases(op);
        if (bases || op_dash(op)) {
            const uint32_t take = bases ? (start < slen ? min(l, slen - start) : 0u) : l;
            const uint32_t s = max(k, ka), e = min(k + take, kb);
            if (e > s && (bases || !drop)) {
                rg = P.x + (s - ka);
                rl = e - s;
                rk = bases ? bkind : S2C_RUN_DASH;
                rq = bases ? q0 + start + (s - k) : 0u;
            }
            k += take;
        }
        if (bases || op == S2C_OP_I || op == S2C_OP_S) start += l;
        run(j, rg, rl, rk, rq);
    }
}

// n dwords src[0..n) → LDS dst[0..n) by LDS-DMA (no VGPR round trip; the wave's 64 lanes copy
// 64 consecutive dwords per instruction; lanes past n re-copy src[n-1] into the 64-dword slack
// after dst).  Completion: s_waitcnt vmcnt(0).
__device__ __forceinline__ void dma_dwords(uint32_t *dst, const uint32_t *src, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = 0; base < n; base += 64) {
        const uint32_t i = min(base + lane, n - 1);
        __builtin_amdgcn_global_load_lds(src + i, dst + base, 4, 0, 0);
    }
}

constexpr int WGD = 64;   // one wave per tile
constexpr int GSD = 8;    // records per counting group (one Harley–Seal tree)

// all-reduce of one register over the G adjacent lanes of a word
template <int G>
__device__ __forceinline__ uint32_t word_allreduce(uint32_t v) {
    if constexpr (G >= 2) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    if constexpr (G >= 4) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);   // row_half_mirror
    static_assert(G <= 8, "at most 8 lanes per word");
    return v;
}

// +1 at the tile-relative positions [r0, r1) (clipped to [0, lim)), one byte counter per
// position: byte adds at the ends, 4 positions per add in between
__device__ __forceinline__ void lds_range(uint32_t *cnt, int32_t r0, int32_t r1, int32_t lim) {
    uint32_t q = (uint32_t)max(r0, 0);
    const uint32_t e = (uint32_t)max(min(r1, lim), 0);
    for (; q < e && (q & 3); q++) atomicAdd(&cnt[q >> 2], 1u << (8 * (q & 3)));
    for (; q + 4 <= e; q += 4) atomicAdd(&cnt[q >> 2], 0x01010101u);
    for (; q < e; q++) atomicAdd(&cnt[q >> 2], 1u << (8 * (q & 3)));
}

// The non-ACGT chars of SEQ in a run of bases (window-relative query bases [q, q + l), tile-
// relative position r0 of q): 'N' (p0 0) into ncnt, '-' (p0 1) into ccnt and, unless maxdel
// drops the read's '-', into dcnt.  The run's x-plane words are read 4 at a time (one LDS
// round trip), the base planes only of words holding such chars.
__device__ __forceinline__ void x_events(const uint32_t *bxl, const uint2 *bql, uint32_t q, uint32_t l, int32_t r0,
                                         int32_t lim, bool drop, uint32_t *dcnt, uint32_t *ncnt, uint32_t *ccnt) {
    const uint32_t wa = q >> 5, wb = (q + l - 1) >> 5;
    for (uint32_t w0 = wa; w0 <= wb; w0 += 4) {
        uint32_t xs[4];
#pragma unroll
        for (int u = 0; u < 4; u++) xs[u] = bxl[min(w0 + u, wb)];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t qw = w0 + u;
            const int32_t b0 = (int32_t)(32 * qw) - (int32_t)q;   // run offset of the word's bit 0
            uint32_t xm = qw <= wb ? xs[u] : 0u;
            if (b0 < 0) xm &= 0xFFFFFFFFu << (uint32_t)(-b0);
            if (b0 + 32 > (int32_t)l) xm &= 0xFFFFFFFFu >> (uint32_t)(b0 + 32 - (int32_t)l);
            if (!xm) continue;
            const uint2 pp = bql[qw];
            while (xm) {
                const uint32_t bit = (uint32_t)__builtin_ctz(xm);
                xm &= xm - 1;
                const int32_t r = r0 + b0 + (int32_t)bit;
                if (r < 0 || r >= lim || ((pp.y >> bit) & 1u)) continue;
                const uint32_t one = 1u << (8 * (r & 3));
                if ((pp.x >> bit) & 1u) {
                    atomicAdd(&ccnt[r >> 2], one);
                    if (!drop) atomicAdd(&dcnt[r >> 2], one);
                } else {
                    atomicAdd(&ncnt[r >> 2], one);
                }
            }
        }
    }
}

// One wave per tile of NWP words; G = 64 / NWP lanes per word.
template <int NWP>
__global__ __launch_bounds__(WGD) void k_tile_dense(const DenseArgs d) {
    constexpr int G = WGD / NWP, PPL = 32 / G;
    static_assert(PPL >= 4 && PPL % 4 == 0, "a lane votes whole dwords of positions");
    extern __shared__ uint4 arena[];          // the window (S2C_DENSE_BYTES layout)
    // one byte per position: '-' (D/N/P runs, '-' of SEQ unless maxdel drops the read's), 'N'
    // of SEQ, '-' of SEQ (all: the planes count them as C, and 'N' as A)
    __shared__ uint32_t dcnt[8 * NWP], ncnt[8 * NWP], ccnt[8 * NWP];
    __shared__ uint8_t amb[64];
#ifdef S2C_PROF
    unsigned long long prof_t = 0;
#endif
    PROF_MARK(0);
    const uint32_t lane = threadIdx.x;
    const uint32_t w = lane / G, g = lane % G;
    const uint32_t tile = uni(d.items[4 * (size_t)blockIdx.x]);
    const uint32_t *twp = d.tiles + (size_t)tile * S2C_TILE_WORDS;
    const uint4 tw = *(const uint4 *)twp;
    const uint4 tw3 = *(const uint4 *)(twp + 12), tw4 = *(const uint4 *)(twp + 16);
    const uint32_t cb0 = uni(twp[8]);
    const uint32_t a = uni(tw.x), n = uni(tw.y) - a;
    const uint32_t pf0 = uni(tw3.y), pf1 = uni(tw3.z), o0 = uni(tw3.w), o1 = uni(tw4.x), qw0 = uni(tw4.y), qw1 = uni(tw4.z);
    const uint32_t W0 = a >> 5, nwords = (n + 31) / 32, W = W0 + w;
    const bool active = w < nwords;
    const uint32_t K = d.kwin;
    const uint32_t nslot = o1 - o0, npc = pf1 - pf0, nqw = qw1 - qw0;
    // ---- one round trip: the window's op words and planes by LDS-DMA, this lane's first
    //      piece record and its word's run-slot range
    uint32_t *opl = (uint32_t *)arena;
    uint2 *bql = (uint2 *)(opl + ((nslot + 65) & ~1u));
    uint32_t *bxl = (uint32_t *)(bql + nqw + 32);
    uint2 *runl = (uint2 *)(bxl + ((nqw + 65) & ~1u));
    if (nslot) dma_dwords(opl, d.ops + o0, nslot);
    if (nqw) {
        dma_dwords((uint32_t *)bql, d.bq + 2 * (size_t)qw0, 2 * nqw);
        dma_dwords(bxl, d.bx + qw0, nqw);
    }
    constexpr int PFN = 4;   // piece records per lane in flight with the DMA
    uint4 Pp[PFN];
    uint32_t oe[PFN];
#pragma unroll
    for (int i = 0; i < PFN; i++) {
        const uint32_t k = lane + WGD * i;
        Pp[i] = make_uint4(0u, 0u, 0u, 0u);
        oe[i] = 0;
        if (k < npc) {
            Pp[i] = ((const uint4 *)d.pc)[pf0 + k];
            oe[i] = d.pc[4 * (size_t)(pf0 + k + 1) + 2];
        }
    }
    uint32_t cw0 = 0, cw1 = 0;
    if (active) {
        cw0 = d.rs[W >= K ? W - K : 0u] - o0;
        cw1 = d.rs[W + 1] - o0;
    }
    for (uint32_t i = lane; i < 8 * NWP; i += WGD) {
        dcnt[i] = 0;
        ncnt[i] = 0;
        ccnt[i] = 0;
    }
    amb[lane] = c_amb[lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();
    PROF_MARK(1);
    // ---- parsecigar + maxdel of the window's pieces (one lane per piece) → run records of the
    //      bases {gpos, (query base − 32·qw0) << 15 | len << 4 | kind}; '-' runs and the
    //      non-ACGT chars of SEQ straight into the byte counters
    const int32_t T0 = (int32_t)(32 * W0), TL = (int32_t)(32 * nwords);   // the tile's words
    auto walk = [&](const uint4 &P, uint32_t oend) {
        const bool lng = ((P.w >> 24) & S2C_PF_LONG) != 0;   // (a long piece starting here does not overlap the tile)
        walk_window(opl, bql, bxl, P, P.z - o0, oend - o0, (uint32_t)((uint64_t)P.y * 16 - 32ull * qw0),
                    d.maxdel_active != 0, d.maxdel, [&](uint32_t j, uint32_t gp, uint32_t l, uint32_t kind, uint32_t q) {
                        const uint32_t kd = (lng || kind == S2C_RUN_EMPTY) ? 0u : (kind & 3u);
                        runl[j] = kd == S2C_RUN_BASES ? make_uint2(gp, (q << 15) | (l << 4) | kind) : make_uint2(0u, 0u);
                        const int32_t r0 = (int32_t)gp - T0;
                        if (kd == S2C_RUN_DASH) lds_range(dcnt, r0, r0 + (int32_t)l, TL);
                        if (kd == S2C_RUN_BASES && (kind & S2C_RUN_XBIT))
                            x_events(bxl, bql, q, l, r0, TL, (kind & S2C_RUN_DROP) != 0, dcnt, ncnt, ccnt);
                    });
    };
    const uint32_t nit = ABL(4) ? 0u : (npc + WGD - 1) / WGD;
    for (uint32_t i = 0; i < nit; i++) {   // (one copy of the walk: the prefetched records by a select chain)
        const uint32_t k = lane + WGD * i;
        uint4 P = Pp[0];
        uint32_t oend = oe[0];
#pragma unroll
        for (int u = 1; u < PFN; u++) {
            P.x = i == (uint32_t)u ? Pp[u].x : P.x;
            P.y = i == (uint32_t)u ? Pp[u].y : P.y;
            P.z = i == (uint32_t)u ? Pp[u].z : P.z;
            P.w = i == (uint32_t)u ? Pp[u].w : P.w;
            oend = i == (uint32_t)u ? oe[u] : oend;
            asm volatile("" : "+v"(P.x), "+v"(P.y), "+v"(P.z), "+v"(P.w), "+v"(oend));
        }
        if (i >= (uint32_t)PFN && k < npc) {   // (windows of more than 256 pieces)
            P = ((const uint4 *)d.pc)[pf0 + k];
            oend = d.pc[4 * (size_t)(pf0 + k + 1) + 2];
        }
        if (k < npc) walk(P, oend);
    }
    lds_sync();
    PROF_MARK(2);

    // ---- count the base records of this lane's word (candidates cw0 + g + G·m < cw1),
    //      bit-sliced by the planes (non-ACGT chars of SEQ as A / C: taken back in the vote), a
    //      group's records read together from LDS
    uint32_t C[4][8];   // X = p0 (C|T), Y = p1 (G|T), Z = T, V = covered
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int b = 0; b < 8; b++) C[c][b] = 0;
    const uint32_t nrec = cw0 + g < cw1 ? (cw1 - cw0 - g + G - 1) / G : 0u;
    const uint32_t ngrp = ABL(2) ? 0u : uni(__ockl_wfred_max_u32((nrec + GSD - 1) / GSD));
    for (uint32_t gi = 0; gi < ngrp; gi++) {
        uint32_t vd[GSD], gk[GSD];   // covered bits; first bit | shift << 5
        uint2 pa[GSD], pb[GSD];
#pragma unroll
        for (int u = 0; u < GSD; u++) {
            const uint32_t m = gi * GSD + u;
            uint2 rv = runl[m < nrec ? cw0 + g + G * m : 0u];   // (unconditional: the group's reads in flight together)
            if (m >= nrec) rv = make_uint2(0u, 0u);
            const RecGeom gm = rec_geom(rv.x, (rv.y >> 4) & 0x7FFu, W);   // (zero records: valid 0)
            const uint32_t qs = (rv.y >> 15) + gm.qs;
            const uint32_t kw = gm.valid ? qs >> 5 : 0u;   // window-relative plane word (uncovered: one broadcast address)
            vd[u] = gm.valid;
            gk[u] = gm.lo | (qs & 31u) << 5;
            pa[u] = bql[kw];
            pb[u] = bql[kw + 1];
        }
        // one Harley–Seal tree per plane (tree8 + close8), fed a pair of records at a time
        uint32_t pend[4], t2a[4], t4a[4];
#pragma unroll
        for (int u = 0; u < GSD; u++) {
            const uint32_t v0 = vd[u], lo = gk[u] & 31u, sh = gk[u] >> 5;
            const uint32_t x = (funnel(pb[u].x, pa[u].x, sh) << lo) & v0;
            const uint32_t y = (funnel(pb[u].y, pa[u].y, sh) << lo) & v0;
            const uint32_t mk[4] = {x, y, x & y, v0};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                if ((u & 1) == 0) {
                    pend[c] = mk[c];
                    continue;
                }
                uint32_t t2;
                csa(t2, C[c][0], C[c][0], pend[c], mk[c]);
                if ((u & 3) == 1) {
                    t2a[c] = t2;
                    continue;
                }
                uint32_t t4;
                csa(t4, C[c][1], C[c][1], t2a[c], t2);
                if ((u & 7) == 3) {
                    t4a[c] = t4;
                    continue;
                }
                uint32_t t8;
                csa(t8, C[c][2], C[c][2], t4a[c], t4);
                close8(C[c], t8);
            }
        }
    }
    PROF_MARK(3);
    // ---- counters → byte counts: R[r] byte j = count of position 8j + r
#pragma unroll
    for (int c = 0; c < 4; c++) transpose8(C[c]);
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const uint32_t x = C[0][r], y = C[1][r], z = C[2][r], v = C[3][r];
        C[3][r] = v - x - y + z;   // A
        C[0][r] = x - z;           // C
        C[1][r] = y - z;           // G
    }
    if constexpr (G > 1) {
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int r = 0; r < 8; r++) C[c][r] = word_allreduce<G>(C[c][r]);
    }
    PROF_MARK(4);

    // ---- vote of this lane's PPL consecutive positions p0 .. p0+PPL-1 of its word
    const uint32_t p0 = g * PPL;                 // word-relative
    const uint32_t jb = p0 >> 3, rs0 = p0 & 7;   // PPL ≥ 8: bytes jb.. of every R[r]; PPL = 4: R[rs0 + i] byte jb
    const uint32_t q0 = 32 * w + p0;             // tile-relative
    const uint32_t npos = active ? (q0 < n ? min((uint32_t)PPL, n - q0) : 0u) : 0u;
    uint32_t dv[PPL / 4], nv[PPL / 4], cv[PPL / 4];   // '-', 'N', '-' of SEQ counts, 4 positions a dword
#pragma unroll
    for (int v = 0; v < PPL / 4; v++) {
        dv[v] = dcnt[(q0 >> 2) + v];
        nv[v] = ncnt[(q0 >> 2) + v];
        cv[v] = ccnt[(q0 >> 2) + v];
    }
    uint32_t jbt = jb;   // (re-made opaque per threshold: the counts stay packed, not hoisted)
    // count of symbol sym (A C G T = C[3] C[0] C[1] C[2]) at p0 + i: byte jb + i/8 of
    // R[i % 8] (PPL ≥ 8), byte jb of R[rs0 + i] (PPL = 4)
    auto cnt = [&](int sym, int i) -> uint32_t {
        if constexpr (PPL >= 8) {
            return (C[sym][i & 7] >> (8 * (jbt + (uint32_t)(i >> 3)))) & 0xFFu;
        } else {
            const uint32_t v = rs0 ? C[sym][4 + i] : C[sym][i];
            return (v >> (8 * jbt)) & 0xFFu;
        }
    };
    // the same for a run-time i (rare paths: a select chain, no indexed registers)
    auto sel = [&](const auto &R, uint32_t r) -> uint32_t {
        constexpr int nr = (int)(sizeof(R) / sizeof(R[0]));
        uint32_t v = R[0];
#pragma unroll
        for (int k = 1; k < nr; k++) {
            v = r == (uint32_t)k ? R[k] : v;
            asm volatile("" : "+v"(v));   // keeps the chain of selects (no indexed copy)
        }
        return v;
    };
    auto cnt_rt = [&](int sym, uint32_t i) -> uint32_t {
        const uint32_t r = PPL >= 8 ? (i & 7u) : rs0 + i, by = PPL >= 8 ? jb + (i >> 3) : jb;
        return (sel(C[sym], r) >> (8 * by)) & 0xFFu;
    };
    const uint64_t ostride = (uint64_t)d.padded_len + d.n_cols;   // max(1, len(fill)) = 1
    const uint32_t fill0 = d.fill[0];
    uint8_t *const obase = d.out + (uint64_t)a + cb0 + q0;
    const uint32_t inmask = npos >= 32 ? 0xFFFFFFFFu : (1u << npos) - 1u;
    uint32_t sc = 0;
    for (int t = 0; t < (ABL(8) ? 0 : d.n_thr); t++) {
        const double th = d.thresholds[t];
        const uint32_t uq = pass_uq(&th, 1);
        const bool uqok = uq != 0;
        jbt = jb;
        asm volatile("" : "+v"(jbt));
        uint32_t ow[PPL / 4];
        uint32_t nd = 0, ne = 0, slow = 0;
        // fast path: fill, or the strict-majority symbol
#pragma unroll
        for (int i = 0; i < PPL; i++) {
            uint32_t c6[NSYM];   // "-ACGNT"
            c6[0] = (dv[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            c6[4] = (nv[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            c6[1] = cnt(3, i) - c6[4];
            c6[2] = cnt(0, i) - ((cv[i >> 2] >> (8 * (i & 3))) & 0xFFu);
            c6[3] = cnt(1, i);
            c6[5] = cnt(2, i);
            const bool in = (uint32_t)i < npos;
            const uint32_t cov = c6[0] + c6[1] + c6[2] + c6[3] + c6[4] + c6[5];
            if (t == 0) sc += in ? cov : 0u;   // Σ cov, uncalled positions included (:357)
            const bool called = (cov > 0) & ((int32_t)cov >= d.min_depth);   // :356-359
            uint32_t k6[NSYM];
#pragma unroll
            for (uint32_t s = 0; s < NSYM; s++) k6[s] = (c6[s] << 3) | s;
            const uint32_t mk = max(max(max(k6[0], k6[1]), k6[2]), max(max(k6[3], k6[4]), k6[5]));
            // majority_fast in 32 bits (counts ≤ 255: m1·2^15 and uq·cov < 2^24)
            const uint32_t m1 = mk >> 3;
            const bool fast = uqok & (2u * m1 > cov) & ((m1 << 15) >= uq * cov);
            slow |= (called && !fast) ? (1u << i) : 0u;
            // "-ACGNT"[mk & 7] by a byte permute
            const uint32_t sc6 = __builtin_amdgcn_perm(0x0000544Eu, 0x4743412Du, (mk & 7u) | 0x0C0C0C00u);
            const uint32_t ch = called ? sc6 : fill0;
            nd += (in && (!called || fast)) ? (called ? (ch != '-') : d.fill_nondash) : 0u;
            if ((i & 3) == 0) ow[i >> 2] = 0;
            ow[i >> 2] |= ch << (8 * (i & 3));
        }
        // the other called positions: closed form of the group-sort vote
        slow &= inmask;
        while (slow) {
            const uint32_t i = (uint32_t)__builtin_ctz(slow);
            slow &= slow - 1;
            uint32_t c6[NSYM];
            c6[0] = (sel(dv, i >> 2) >> (8 * (i & 3))) & 0xFFu;
            c6[4] = (sel(nv, i >> 2) >> (8 * (i & 3))) & 0xFFu;
            c6[1] = cnt_rt(3, i) - c6[4];
            c6[2] = cnt_rt(0, i) - ((sel(cv, i >> 2) >> (8 * (i & 3))) & 0xFFu);
            c6[3] = cnt_rt(1, i);
            c6[5] = cnt_rt(2, i);
            const uint32_t cov = c6[0] + c6[1] + c6[2] + c6[3] + c6[4] + c6[5];
            uint32_t gs[NSYM];
            greater_sums(c6, gs);
            const uint32_t ch = amb[vote_mask_u32(c6, gs, th * (double)cov)];
            nd += ch != '-';
            ne += ch == 0xFFu;
            const uint32_t sh = 8 * (i & 3), keep = ~(0xFFu << sh);
#pragma unroll
            for (int v = 0; v < PPL / 4; v++) {
                ow[v] = (i >> 2) == (uint32_t)v ? (ow[v] & keep) | (ch << sh) : ow[v];
                asm volatile("" : "+v"(ow[v]));
            }
        }
        uint8_t *dst = obase + (uint64_t)t * ostride;
        if (npos == (uint32_t)PPL) {
            if constexpr (PPL >= 16) {
#pragma unroll
                for (int v = 0; v < PPL / 4; v += 4) *(uint4 *)(dst + 4 * v) = make_uint4(ow[v], ow[v + 1], ow[v + 2], ow[v + 3]);
            } else if constexpr (PPL == 8) {
                *(uint2 *)dst = make_uint2(ow[0], ow[1]);
            } else {
                *(uint32_t *)dst = ow[0];
            }
        } else {
#pragma unroll
            for (int i = 0; i < PPL; i++)
                if ((uint32_t)i < npos) dst[i] = (uint8_t)(ow[i >> 2] >> (8 * (i & 3)));
        }
        if (t == 0) sc = wave_sum(sc);
        nd = wave_sum(nd);
        ne = wave_sum(ne);
        if (lane == 0) {   // tile statistics (:352-397)
            const size_t j = (size_t)t * d.n_tiles + tile;
            uint64_t *st = d.tile_stats + j * 4;
            st[0] = sc;
            st[1] = n;
            st[2] = nd;
            st[3] = ne;
            d.blk_len[j] = n;
        }
    }
    PROF_MARK(5);
#ifdef S2C_PROF
    if (threadIdx.x == 0 && (blockIdx.x & 63) == 0) {
        atomicAdd(&g_prof[8], 1ull);
        atomicAdd(&g_prof[9], (unsigned long long)ngrp);
        atomicAdd(&g_prof[10], (unsigned long long)npc);
        atomicAdd(&g_prof[11], (unsigned long long)(nslot + 3 * nqw));
    }
#endif
}

template <int NWP>
int launch(const DenseArgs &a, int64_t n, int64_t lds, hipStream_t s) {
    k_tile_dense<NWP><<<(unsigned)n, WGD, (unsigned)lds, s>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? S2C_OK : s2c_set_error(S2C_ERR_HIP, std::string("k_tile_dense: ") + hipGetErrorString(e));
}

}  // namespace
}  // namespace s2c

#ifdef S2C_PROF
extern "C" int s2c_prof_ablate(uint32_t bits) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_abl), &bits, sizeof(bits)) == hipSuccess ? 0 : -1;
}
extern "C" int s2c_prof_dense(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

int s2c_launch_dense(const s2c_dev *dv, hipStream_t st) {
    using namespace s2c;
    if (dv->n_dense <= 0) return S2C_OK;
    if (dv->fill_len != 1) return s2c_set_error(S2C_ERR_ARG, "dense tiles need a one-char fill");
    DenseArgs a;
    a.rs = dv->rs; a.pc = dv->pc; a.ops = dv->ops; a.bq = dv->bq; a.bx = dv->bx; a.tiles = dv->tiles; a.items = dv->dense;
    a.thresholds = dv->thresholds; a.tile_stats = dv->tile_stats; a.blk_len = dv->blk_len; a.out = dv->out;
    a.padded_len = (uint32_t)dv->padded_len; a.n_cols = (uint32_t)dv->n_cols; a.n_tiles = (uint32_t)dv->n_tiles;
    a.kwin = (uint32_t)dv->kwin; a.fill_nondash = (uint32_t)dv->fill_nondash;
    a.maxdel_active = dv->maxdel_active ? 1u : 0u;
    a.maxdel = dv->maxdel < 0 ? 0u : (uint32_t)dv->maxdel;
    a.n_thr = dv->n_thr; a.min_depth = dv->min_depth;
    a.fill = dv->fill;
    const int64_t n = dv->n_dense;
    // LDS: the largest window of the batch (S2C_DENSE_BYTES, host plan)
    const int64_t lds = dv->dense_lds;
    if (lds <= 0 || lds > S2C_DENSE_LDS) return s2c_set_error(S2C_ERR_ARG, "dense_lds outside (0, S2C_DENSE_LDS]");
    if (dv->tile_max <= 256) return launch<8>(a, n, lds, st);
    if (dv->tile_max <= 512) return launch<16>(a, n, lds, st);
    if (dv->tile_max <= 1024) return launch<32>(a, n, lds, st);
    return launch<64>(a, n, lds, st);   // tile_max ≤ 2048 (host plan)
}

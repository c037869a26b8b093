// s2c_dense.hip — k_tile_dense: shallow tiles without insertion keys (-f of one char).
//
// Such a tile's body is one char per position (:355-389 with no insertion columns and a
// one-char fill), so the byte offset of position q is q: no length scan.  The tile walks
// its window's pieces itself (the short pieces starting up to kwin words before it): the
// base planes of the window — one contiguous range — are staged in LDS with one coalesced
// sweep, one thread per piece runs parsecigar + maxdel (walk_piece, :46-82, :210) into run
// records in LDS, each lane counts the records covering its word (bit-sliced counters as in
// k_tile), and — every position's total being ≤ 255 (host plan) — the word's G lanes
// all-reduce their byte counters with DPP, so each lane holds the counts of the whole word.  Lane g
// of a word then votes its 32/G consecutive positions for every threshold (closed form of
// :241-251 / :359-366 with the strict-majority shortcut) and stores their chars with one
// wide store.  Counts never touch LDS or HBM.
#include "s2c_common.h"

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

// walk_piece's view of the window staged in LDS
struct LdsMem {
    const uint32_t *ops;    // op words from o0
    const uint2 *bql;       // base planes {p0, p1} from qw0
    const uint32_t *bxl;    // non-ACGT plane from qw0
    uint32_t o0, qw0;
    __device__ __forceinline__ uint32_t op(uint32_t j) const { return ops[j - o0]; }
    __device__ __forceinline__ uint32_t p0(uint64_t w) const { return bql[(uint32_t)w - qw0].x; }
    __device__ __forceinline__ uint32_t p1(uint64_t w) const { return bql[(uint32_t)w - qw0].y; }
    __device__ __forceinline__ uint32_t x(uint64_t w) const { return bxl[(uint32_t)w - qw0]; }
};

// n dwords src[0..n) → LDS dst[0..n) by LDS-DMA (no VGPR round trip; the wave's 64 lanes copy
// 64 consecutive dwords per instruction; lanes past n re-copy src[n-1] into the 64-dword slack
// after dst).  Completion: s_waitcnt vmcnt(0) + a barrier.
__device__ __forceinline__ void dma_dwords(uint32_t *dst, const uint32_t *src, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t base = 64 * wv; base < n; base += WG) {
        const uint32_t i = min(base + lane, n - 1);
        __builtin_amdgcn_global_load_lds(src + i, dst + base, 4, 0, 0);
    }
}

constexpr int GSD = 4;   // records per counting group

// all-reduce of one register over the G adjacent lanes of a word
template <int G>
__device__ __forceinline__ uint32_t word_allreduce(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);   // row_half_mirror
    if constexpr (G >= 16) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    if constexpr (G >= 32) v += (uint32_t)__shfl_xor((int)v, 16);
    return v;
}

template <int NWP>
__global__ __launch_bounds__(WG) void k_tile_dense(const DenseArgs d) {
    constexpr int G = WG / NWP, PPL = 32 / G;
    __shared__ uint4 arena[S2C_DENSE_LDS / 16 + 4];   // the tile's window (layout below)
    __shared__ uint32_t nb[8 * NWP];                   // 'N' counts of SEQ, one byte per position
    __shared__ uint32_t acc[2 * THR_MAX + 1];          // sumcov; per threshold {non-'-', vote errors}
    __shared__ uint8_t amb[64];
    const uint32_t tid = threadIdx.x;
    const uint32_t w = tid / G, g = tid % G;
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
    const uint32_t nqw = qw1 - qw0, nslot = o1 - o0, npc = pf1 - pf0;
    // ---- one round of LDS-DMA: piece records, base planes, non-ACGT plane, op words (each
    //      region 16-B aligned with 64 dwords of slack); the run records are written later
    auto up4 = [](uint32_t x) { return (x + 3u) & ~3u; };
    uint32_t *L0 = (uint32_t *)arena;
    uint32_t *pcl = L0;
    uint32_t *bq_l = pcl + up4(4 * npc + 64);
    uint32_t *bx_l = bq_l + up4(2 * nqw + 64);
    uint32_t *op_l = bx_l + up4(nqw + 64);
    uint2 *runl = (uint2 *)(op_l + up4(nslot + 64));
    if (npc) dma_dwords(pcl, d.pc + 4 * (size_t)pf0, 4 * npc);
    if (nqw) {
        dma_dwords(bq_l, d.bq + 2 * (size_t)qw0, 2 * nqw);
        dma_dwords(bx_l, d.bx + (size_t)qw0, nqw);
    }
    if (nslot) dma_dwords(op_l, d.ops + (size_t)o0, nslot);
    uint32_t cw0 = 0, cw1 = 0;
    if (active) {
        cw0 = d.rs[W >= K ? W - K : 0u] - o0;
        cw1 = d.rs[W + 1] - o0;
    }
    for (uint32_t i = tid; i < 8 * NWP; i += WG) nb[i] = 0;
    for (uint32_t i = tid; i < 2 * (uint32_t)d.n_thr + 1; i += WG) acc[i] = 0;
    if (tid < 64) amb[tid] = c_amb[tid];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();
    // ---- parsecigar + maxdel of the window's pieces (one thread per piece) → run records:
    //      {gpos, (query bit − 32·qw0) << 15 | len << 4 | kind}
    const uint2 *bql = (const uint2 *)bq_l;
    const LdsMem mem{op_l, bql, bx_l, o0, qw0};
    for (uint32_t k = tid; k < npc; k += WG) {
        const uint4 P = ((const uint4 *)pcl)[k];
        const uint32_t oend = k + 1 < npc ? pcl[4 * (k + 1) + 2] : o1;
        walk_piece(mem, P, oend, d.maxdel_active != 0, d.maxdel,
                   [&](uint32_t j, uint32_t gp, uint32_t l, uint32_t kind, uint64_t q) {
                       uint2 r = make_uint2(0u, 0u);
                       if (kind != S2C_RUN_EMPTY && !(kind & S2C_RUN_LONG))   // a long piece here does not overlap the tile
                           r = make_uint2(gp, ((uint32_t)(q - 32ull * qw0) << 15) | (l << 4) | (kind & 15u));
                       runl[j - o0] = r;
                   },
                   [&](uint64_t, uint64_t, uint32_t) {});   // dense tiles hold no insertion keys
    }
    lds_sync();
    const uint32_t *bxl = bx_l;

    // ---- count the records of this lane's word: candidates cw0 + g + G·m < cw1
    uint32_t C[5][8];   // X, Y, Z, V, '-'
#pragma unroll
    for (int c = 0; c < 5; c++)
#pragma unroll
        for (int b = 0; b < 8; b++) C[c][b] = 0;
    const uint32_t nrec = cw0 + g < cw1 ? (cw1 - cw0 - g + G - 1) / G : 0u;
    const uint32_t ngrp = uni(__ockl_wfred_max_u32((nrec + GSD - 1) / GSD));
    for (uint32_t gi = 0; gi < ngrp; gi++) {
        uint32_t mx[8], my[8], mz[8], mv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) mx[u] = my[u] = mz[u] = mv[u] = 0;
#pragma unroll
        for (int u = 0; u < GSD; u++) {
            const uint32_t m = gi * GSD + u;
            const uint2 rv = m < nrec ? runl[cw0 + g + G * m] : make_uint2(0u, 0u);
            const uint32_t kind = rv.y & 15u, kd = kind & 3u, len = (rv.y >> 4) & 0x7FFu;
            const RecGeom gm = rec_geom(rv.x, len, W);
            if (kd == S2C_RUN_DASH) {
                ripple1(C[4], gm.valid);
            } else if (kd == S2C_RUN_BASES && gm.valid) {
                const uint32_t qs = (rv.y >> 15) + (uint32_t)gm.qs, k = qs >> 5, sh = qs & 31u;
                const uint2 lo = bql[k], hi = bql[k + 1];
                const uint32_t vd = gm.valid;
                const uint32_t b0 = (funnel(hi.x, lo.x, sh) << gm.lo) & vd;
                const uint32_t b1 = (funnel(hi.y, lo.y, sh) << gm.lo) & vd;
                uint32_t v = vd, x = b0, y = b1;
                if (kind & S2C_RUN_XBIT) {
                    const uint32_t xm = (funnel(bxl[k + 1], bxl[k], sh) << gm.lo) & vd;
                    const uint32_t en = xm & ~b0 & ~b1, sd = xm & b0 & ~b1;   // 'N', '-' of SEQ
                    v &= ~xm;
                    x &= ~xm;
                    y &= ~xm;
                    if (sd && !(kind & S2C_RUN_DROP)) ripple1(C[4], sd);
                    uint32_t e = en;
                    while (e) {
                        const uint32_t bit = (uint32_t)__builtin_ctz(e);
                        e &= e - 1;
                        const uint32_t q = 32 * w + bit;
                        atomicAdd(&nb[q >> 2], 1u << (8 * (q & 3)));
                    }
                }
                mx[u] = x;
                my[u] = y;
                mz[u] = x & y;
                mv[u] = v;
            }
        }
        close8(C[0], tree8(C[0], mx));
        close8(C[1], tree8(C[1], my));
        close8(C[2], tree8(C[2], mz));
        close8(C[3], tree8(C[3], mv));
    }
    // ---- counters → byte counts of the whole word in every lane of it
#pragma unroll
    for (int c = 0; c < 5; c++) transpose8(C[c]);
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const uint32_t x = C[0][r], y = C[1][r], z = C[2][r], v = C[3][r];
        C[3][r] = v - x - y + z;   // A
        C[0][r] = x - z;           // C
        C[1][r] = y - z;           // G
    }
#pragma unroll
    for (int c = 0; c < 5; c++)
#pragma unroll
        for (int r = 0; r < 8; r++) C[c][r] = word_allreduce<G>(C[c][r]);
    lds_sync();   // 'N' counts complete

    // ---- vote of this lane's PPL consecutive positions p0 .. p0+PPL-1 of its word
    const uint32_t p0 = g * PPL;                 // word-relative
    const uint32_t jb = p0 >> 3, rs0 = p0 & 7;   // byte j of R[r], r = rs0 + i
    const uint32_t q0 = 32 * w + p0;             // tile-relative
    const uint32_t npos = active ? (q0 < n ? min((uint32_t)PPL, n - q0) : 0u) : 0u;
    auto cnt = [&](int sym, int i) -> uint32_t {   // count of symbol (A C G T '-' = C[3] C[0] C[1] C[2] C[4]) at p0 + i
        uint32_t v = 0;
#pragma unroll
        for (int s = 0; s < 8 / PPL; s++) v = (rs0 == (uint32_t)(s * PPL)) ? C[sym][s * PPL + i] : v;
        return (v >> (8 * jb)) & 0xFFu;
    };
    uint32_t c6[PPL][NSYM], cov[PPL];
#pragma unroll
    for (int i = 0; i < PPL; i++) {
        const uint32_t q = q0 + i;
        c6[i][0] = cnt(4, i);
        c6[i][1] = cnt(3, i);
        c6[i][2] = cnt(0, i);
        c6[i][3] = cnt(1, i);
        c6[i][4] = (nb[q >> 2] >> (8 * (q & 3))) & 0xFFu;
        c6[i][5] = cnt(2, i);
        cov[i] = 0;
#pragma unroll
        for (int s = 0; s < (int)NSYM; s++) cov[i] += c6[i][s];
        if ((uint32_t)i >= npos) cov[i] = 0;
    }
    uint32_t sc = 0;
#pragma unroll
    for (int i = 0; i < PPL; i++) sc += cov[i];   // Σ cov, uncalled positions included (:357)
    sc = wave_sum(sc);
    if ((tid & 63) == 0) atomicAdd(&acc[0], sc);
    const uint64_t ostride = (uint64_t)d.padded_len + d.n_cols;   // max(1, len(fill)) = 1
    const uint32_t fill0 = d.fill[0];
    uint8_t *const obase = d.out + (uint64_t)a + cb0 + q0;
    for (int t = 0; t < d.n_thr; t++) {
        const double th = d.thresholds[t];
        const uint32_t uq = pass_uq(&th, 1);
        uint64_t word = 0;
        uint32_t nd = 0, ne = 0;
#pragma unroll
        for (int i = 0; i < PPL; i++) {
            const bool called = cov[i] > 0 && (int64_t)cov[i] >= (int64_t)d.min_depth;   // :356-359
            uint32_t k[NSYM];
#pragma unroll
            for (uint32_t s = 0; s < NSYM; s++) k[s] = (c6[i][s] << 3) | s;
            const uint32_t mk = max(max(max(k[0], k[1]), k[2]), max(max(k[3], k[4]), k[5]));
            uint32_t ch = sym_char(mk & 7u);
            if (called && !majority_fast(mk >> 3, cov[i], uq)) {
                uint32_t gs[NSYM];
                greater_sums(c6[i], gs);
                ch = amb[vote_mask_u32(c6[i], gs, th * (double)cov[i])];
            }
            if (!called) ch = fill0;
            const bool in = (uint32_t)i < npos;
            nd += in ? (called ? (ch != '-') : d.fill_nondash) : 0u;
            ne += (in && called && ch == 0xFFu) ? 1u : 0u;
            word |= (uint64_t)ch << (8 * i);
        }
        uint8_t *dst = obase + (uint64_t)t * ostride;
        if (npos == (uint32_t)PPL) {
            if constexpr (PPL == 8) *(uint2 *)dst = make_uint2((uint32_t)word, (uint32_t)(word >> 32));
            else if constexpr (PPL == 4) *(uint32_t *)dst = (uint32_t)word;
            else if constexpr (PPL == 2) *(uint16_t *)dst = (uint16_t)word;
            else *dst = (uint8_t)word;
        } else {
            for (uint32_t i = 0; i < npos; i++) dst[i] = (uint8_t)(word >> (8 * i));
        }
        nd = wave_sum(nd);
        ne = wave_sum(ne);
        if ((tid & 63) == 0) {
            atomicAdd(&acc[1 + 2 * t], nd);
            if (ne) atomicAdd(&acc[2 + 2 * t], ne);
        }
    }
    lds_sync();
    for (uint32_t t = tid; t < (uint32_t)d.n_thr; t += WG) {   // tile statistics (:352-397)
        const size_t j = (size_t)t * d.n_tiles + tile;
        uint64_t *st = d.tile_stats + j * 4;
        st[0] = acc[0];
        st[1] = n;
        st[2] = acc[1 + 2 * t];
        st[3] = acc[2 + 2 * t];
        d.blk_len[j] = n;
    }
}

template <int NWP>
int launch(const DenseArgs &a, int64_t n, hipStream_t s) {
    k_tile_dense<NWP><<<(unsigned)n, WG, 0, s>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? S2C_OK : s2c_set_error(S2C_ERR_HIP, std::string("k_tile_dense: ") + hipGetErrorString(e));
}

}  // namespace
}  // namespace s2c

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
    if (dv->tile_max <= 256) return launch<8>(a, n, st);
    if (dv->tile_max <= 512) return launch<16>(a, n, st);
    if (dv->tile_max <= 1024) return launch<32>(a, n, st);
    return launch<64>(a, n, st);
}

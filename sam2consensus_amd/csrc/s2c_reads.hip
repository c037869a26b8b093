// s2c_reads.hip — k_reads: the reference's parsecigar (:46-82), maxdel rule (:210) and
// insertion collection (:73-75, :221, :262-271) on the device, one thread per piece.
//
// Input: the packed batch of s2c_host.cpp — per piece its global start, its read's CIGAR
// tokens (:58 regex matches) and SEQ as query-order base planes.  The thread walks the
// tokens exactly as parsecigar does (start = query index, k = seqout index):
//   M / = / X   take = min(l, len(SEQ) - start) bases (SEQ truncation, :67), k += take
//   D / N / P   l '-' (:70-72), k += l
//   I           event (start_ref, SEQ[start:start+l]) if the slice is non-empty (:73-75)
//   S           start += l (:76-77);  H nothing (:78-79)
// and writes one run record per token (parallel to ops[]): the seqout interval of the
// token inside the piece, mapped to query bases or to counted '-' — the maxdel rule drops
// the '-' of a read whose seqout holds more than maxdel of them (:210, '-' chars of SEQ
// included).  Insertion events go to the piece's tile: motifs of ≤ 16 bases into the
// tile's open-addressing table keyed by (position, length, 3-bit codes) with a count per
// entry (the reference's ins_tmp1[pos][motif] += 1, :264-271); longer motifs into the
// tile's long-event list (multiplicity 1; the column sums of :284-287 are additive).
#include "s2c_common.h"

namespace s2c {
namespace {

struct ReadsArgs {
    const uint32_t *pc, *ops, *bq, *bx, *tiles, *wtile, *rlist;
    uint32_t *runs, *ibkt, *ilong, *ilong_n;
    uint32_t n, maxdel_active, maxdel, all;   // all: every piece (else the pieces of rlist)
    uint32_t word_lo, word_hi;                // wtile holds words [word_lo, word_hi) (s2c_dev, ABI 13)
    uint32_t skip_fin, kwin;                  // s2c_reads: events k_tile records are left to it (below)
};

struct GlobalMem {   // walk_piece's view of the batch in HBM
    const uint32_t *ops, *bq, *bx;
    __device__ __forceinline__ uint32_t op(uint32_t j) const { return ops[j]; }
    __device__ __forceinline__ uint32_t p0(uint64_t w) const { return bq[2 * w]; }
    __device__ __forceinline__ uint32_t p1(uint64_t w) const { return bq[2 * w + 1]; }
    __device__ __forceinline__ uint32_t x(uint64_t w) const { return bx[w]; }
};

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// One insertion event (global key gkey, motif = query bases [q, q + len)) of the piece starting
// in word ws into its tile.  With skip_fin (s2c_reads, k_tile recording events: the launch's
// walk_queue) a short motif keyed in a finish tile whose window holds the piece is left
// to that tile's k_tile walk (s2c_tile.hip, the LDS event list): exactly the events it records.
__device__ void add_event(const ReadsArgs &d, uint64_t gkey, uint64_t q, uint32_t len, uint32_t ws, bool lng) {
    // a short motif's codes from its (at most two) plane words, loaded with the tile lookup
    uint64_t c01[3] = {0, 0, 0};   // p0, p1, x of bases q .. q + 63
    if (len <= S2C_SHORT_MOTIF) {
        const uint64_t wq = q >> 5;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            c01[0] |= (uint64_t)d.bq[2 * (wq + h)] << (32 * h);
            c01[1] |= (uint64_t)d.bq[2 * (wq + h) + 1] << (32 * h);
            c01[2] |= (uint64_t)d.bx[wq + h] << (32 * h);
        }
    }
    const uint64_t W = gkey >> 5;
    if (W < d.word_lo || W >= d.word_hi) return;   // keyed outside a multi-GPU shard's words
    const uint32_t t = d.wtile[W - d.word_lo];
    if (t == 0xFFFFFFFFu) return;   // keyed outside this batch's tiles (padding, another shard's tile)
    const uint4 tw0 = ((const uint4 *)d.tiles)[(size_t)t * (S2C_TILE_WORDS / 4)];
    const uint4 tw1 = ((const uint4 *)d.tiles)[(size_t)t * (S2C_TILE_WORDS / 4) + 1];
    if (d.skip_fin && len <= S2C_SHORT_MOTIF && !lng && !(tw0.w & (S2C_TILE_DEEP | S2C_TILE_GENERAL | S2C_TILE_DENSE))) {
        const uint32_t W0 = tw0.x >> 5, W1 = (tw0.y + 31) >> 5;
        if (ws + d.kwin >= W0 && ws < W1) return;   // (the window [max(W0 - kwin, 0), W1) holds the piece)
    }
    const uint32_t pos = (uint32_t)(gkey - tw0.x);   // tile-relative (< 2048)
    if (len <= S2C_SHORT_MOTIF) {
        uint64_t key = (uint64_t)pos | ((uint64_t)len << 11);
        const uint32_t sh = (uint32_t)(q & 31);
        for (uint32_t c = 0; c < len; c++) {
            const uint32_t p0 = (uint32_t)(c01[0] >> (sh + c)) & 1u, p1 = (uint32_t)(c01[1] >> (sh + c)) & 1u,
                           x = (uint32_t)(c01[2] >> (sh + c)) & 1u;
            const uint32_t code = x ? (p0 ? 0u : 4u) : ((p1 << 1 | p0) == 3u ? 5u : (p1 << 1 | p0) + 1u);
            key |= (uint64_t)code << (16 + 3 * c);
        }
        const uint32_t boff = tw1.x, bcap = tw1.y;
        uint32_t s = (uint32_t)mix64(key) & (bcap - 1u);
        for (uint32_t probe = 0; probe < bcap; probe++) {   // bcap ≥ 2 × the tile's short events
            unsigned long long *slot = (unsigned long long *)(d.ibkt + 4 * ((size_t)boff + s));
            const unsigned long long prev = atomicCAS(slot, 0ull, (unsigned long long)key);
            if (prev == 0ull || prev == key) {
                atomicAdd(d.ibkt + 4 * ((size_t)boff + s) + 2, 1u);
                return;
            }
            s = (s + 1u) & (bcap - 1u);
        }
    } else {
        const uint32_t loff = tw1.z, lcap = tw1.w;
        const uint32_t i = atomicAdd(d.ilong_n + t, 1u);
        if (i < lcap)
            ((uint4 *)d.ilong)[(size_t)loff + i] = make_uint4(pos, len, (uint32_t)q, (uint32_t)(q >> 32));
    }
}

// The insertion events of a piece walked for them only (no run records; the maxdel rule does
// not touch events): its op words read together (one round trip), the walk in registers;
// per event the motif's plane words and the tile lookup together, then the table.  Pieces of
// more than EV_OPS op words take walk_piece.
constexpr uint32_t EV_OPS = 12;
__device__ __forceinline__ bool piece_events(const ReadsArgs &d, const uint4 P, uint32_t oend) {
    const uint32_t fl = P.w >> 24, slen = P.w & 0xFFFFFFu, nw = oend - P.z;
    if (nw > EV_OPS || !(fl & S2C_PF_INS)) return false;
    uint32_t w[EV_OPS];
#pragma unroll
    for (uint32_t i = 0; i < EV_OPS; i++) w[i] = i < nw ? d.ops[P.z + i] : 0u;
    const bool rg = (fl & S2C_PF_RANGE) != 0;
    const uint32_t first = rg ? 5u : 3u;   // (prefix words: {ka, kb}, then {key0 lo, key0 hi, ref_off})
    const int64_t key0 = (int64_t)((uint64_t)(rg ? w[2] : w[0]) | ((uint64_t)(rg ? w[3] : w[1]) << 32));
    const uint32_t roff = rg ? w[4] : w[2];
    const uint64_t q0 = (uint64_t)P.y * 16;
    int64_t k = 0;
    uint32_t start = 0;
#pragma unroll
    for (uint32_t i = 0; i < EV_OPS; i++) {
        if (i < first || i >= nw) continue;
        const uint32_t op = w[i] & 15u, l = w[i] >> 4;
        const uint32_t take = start < slen ? min(l, slen - start) : 0u;
        if (op_bases(op)) {
            k += take;
            start += l;
        } else if (op_dash(op)) {
            k += l;
        } else if (op == S2C_OP_I) {
            if (take && key0 + k >= (int64_t)roff) add_event(d, (uint64_t)(key0 + k), q0 + start, take, P.x >> 5, false);
            start += l;
        } else if (op == S2C_OP_S) {
            start += l;
        }
    }
    return true;
}

__global__ __launch_bounds__(WG) void k_reads(const ReadsArgs d) {
    const uint32_t n = blockIdx.x * WG + threadIdx.x;
    if (n >= d.n) return;
    const uint32_t i = d.all ? n : d.rlist[n];
    const uint4 P = ((const uint4 *)d.pc)[i];
    const uint32_t oend = d.pc[4 * (size_t)i + 6];   // next piece's opoff (sentinel at the end)
    const bool runs = d.all || ((P.w >> 24) & S2C_PF_RUNS);
    if (!runs && piece_events(d, P, oend)) return;
    uint4 *out = (uint4 *)d.runs;
    walk_piece(GlobalMem{d.ops, d.bq, d.bx}, P, oend, d.maxdel_active != 0, d.maxdel,
               [&](uint32_t j, uint32_t g, uint32_t l, uint32_t k, uint64_t q) {
                   if (runs) out[j] = make_uint4(g, l | (k << S2C_RUN_KSHIFT), (uint32_t)q, (uint32_t)(q >> 32));
               },
               [&](uint64_t gkey, uint64_t q, uint32_t len) {
                   add_event(d, gkey, q, len, P.x >> 5, ((P.w >> 24) & S2C_PF_LONG) != 0);
               });
}

}  // namespace
}  // namespace s2c

// Launcher (called by s2c_reads in s2c_tile.hip): the pieces of rlist, or all of them
// all: every piece (s2c_pileup_counts); run: s2c_reads (rlist's run prefix, the events k_tile
// records skipped); neither: all of rlist (s2c_accumulate)
int s2c_launch_reads(const s2c_dev *dv, hipStream_t st, bool all, bool run) {
    using namespace s2c;
    const bool rec = run && dv->walk_queue && dv->tile_events;   // (k_tile records its finish tiles' short-motif events)
    const int64_t n = all ? dv->n_pieces : rec ? dv->n_rlist_run : dv->n_rlist;
    if (n == 0) return S2C_OK;
    ReadsArgs a;
    a.pc = dv->pc; a.ops = dv->ops; a.bq = dv->bq; a.bx = dv->bx; a.tiles = dv->tiles; a.wtile = dv->wtile;
    a.rlist = dv->rlist;
    a.runs = dv->runs; a.ibkt = dv->ibkt; a.ilong = dv->ilong; a.ilong_n = dv->ilong_n;
    a.n = (uint32_t)n;
    a.maxdel_active = dv->maxdel_active ? 1u : 0u;
    a.maxdel = dv->maxdel < 0 ? 0u : (uint32_t)dv->maxdel;
    a.all = all ? 1u : 0u;
    a.word_lo = (uint32_t)dv->word_lo;
    a.word_hi = (uint32_t)dv->word_hi;
    a.skip_fin = rec ? 1u : 0u;
    a.kwin = (uint32_t)dv->kwin;
    k_reads<<<(unsigned)((n + WG - 1) / WG), WG, 0, st>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? S2C_OK : s2c_set_error(S2C_ERR_HIP, std::string("k_reads: ") + hipGetErrorString(e));
}

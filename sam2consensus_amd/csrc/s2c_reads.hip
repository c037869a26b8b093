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
    const uint32_t *pc, *ops, *bq, *bx, *tiles, *wtile;
    uint32_t *runs, *ibkt, *ilong, *ilong_n;
    uint32_t n_pieces, maxdel_active, maxdel;
};

__device__ __forceinline__ bool op_bases(uint32_t op) { return op == S2C_OP_M || op == S2C_OP_EQ || op == S2C_OP_X; }
__device__ __forceinline__ bool op_dash(uint32_t op) { return op == S2C_OP_D || op == S2C_OP_N || op == S2C_OP_P; }

// '-' chars of SEQ in query bases [q, q + n): x = 1, p1 = 0, p0 = 1
__device__ uint32_t seq_dashes(const ReadsArgs &d, uint64_t q, uint64_t n) {
    uint32_t c = 0;
    while (n) {
        const uint64_t w = q >> 5;
        const uint32_t sh = (uint32_t)(q & 31), m = (uint32_t)(n < 32 - sh ? n : 32 - sh);
        const uint32_t mask = (m >= 32 ? 0xFFFFFFFFu : ((1u << m) - 1u)) << sh;
        c += (uint32_t)__popc(d.bx[w] & d.bq[2 * w] & ~d.bq[2 * w + 1] & mask);
        q += m;
        n -= m;
    }
    return c;
}

// symbol code ("-ACGNT" index) of query base q
__device__ __forceinline__ uint32_t base_code(const ReadsArgs &d, uint64_t q) {
    const uint64_t w = q >> 5;
    const uint32_t sh = (uint32_t)(q & 31);
    const uint32_t p0 = (d.bq[2 * w] >> sh) & 1u, p1 = (d.bq[2 * w + 1] >> sh) & 1u, x = (d.bx[w] >> sh) & 1u;
    // x = 0: A C G T → 1 2 3 5;  x = 1: p0 = 0 'N' → 4, p0 = 1 '-' → 0
    return x ? (p0 ? 0u : 4u) : ((p1 << 1 | p0) == 3u ? 5u : (p1 << 1 | p0) + 1u);
}

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// One insertion event (global key gkey, motif = query bases [q, q + len)) into its tile.
__device__ void add_event(const ReadsArgs &d, uint64_t gkey, uint64_t q, uint32_t len) {
    const uint32_t t = d.wtile[gkey >> 5];
    if (t == 0xFFFFFFFFu) return;   // keyed outside this batch's tiles (a multi-GPU shard)
    const uint4 tw0 = ((const uint4 *)d.tiles)[(size_t)t * (S2C_TILE_WORDS / 4)];
    const uint4 tw1 = ((const uint4 *)d.tiles)[(size_t)t * (S2C_TILE_WORDS / 4) + 1];
    const uint32_t pos = (uint32_t)(gkey - tw0.x);   // tile-relative (< 2048)
    if (len <= S2C_SHORT_MOTIF) {
        uint64_t key = (uint64_t)pos | ((uint64_t)len << 11);
        for (uint32_t c = 0; c < len; c++) key |= (uint64_t)base_code(d, q + c) << (16 + 3 * c);
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

__global__ __launch_bounds__(WG) void k_reads(const ReadsArgs d) {
    const uint32_t i = blockIdx.x * WG + threadIdx.x;
    if (i >= d.n_pieces) return;
    const uint4 P = ((const uint4 *)d.pc)[i];
    const uint32_t oend = d.pc[4 * (size_t)i + 6];   // next piece's opoff (sentinel at the end)
    const uint32_t slen = P.w & 0xFFFFFFu, fl = P.w >> 24;
    const uint64_t q0 = (uint64_t)P.y * 16;
    uint4 *runs = (uint4 *)d.runs;
    const uint4 EMPTY = make_uint4(0u, 0u, 0u, 0u);
    uint32_t o = P.z;
    int64_t ka = 0, kb = INT64_MAX;
    if (fl & S2C_PF_RANGE) {
        ka = d.ops[o];
        kb = d.ops[o + 1];
        runs[o] = EMPTY;
        runs[o + 1] = EMPTY;
        o += 2;
    }
    int64_t key0 = 0;
    uint32_t roff = 0;
    const bool ins = (fl & S2C_PF_INS) != 0;
    if (ins) {
        key0 = (int64_t)((uint64_t)d.ops[o] | ((uint64_t)d.ops[o + 1] << 32));
        roff = d.ops[o + 2];
        runs[o] = EMPTY;
        runs[o + 1] = EMPTY;
        runs[o + 2] = EMPTY;
        o += 3;
    }
    // ---- the maxdel rule (:210): '-' in seqout = D/N/P lengths + '-' chars of the bases taken
    bool drop = false;
    if (d.maxdel_active) {
        uint64_t dashes = 0, start = 0;
        for (uint32_t j = o; j < oend; j++) {
            const uint32_t w = d.ops[j], op = w & 15u;
            const uint64_t l = w >> 4;
            if (op_bases(op)) {
                const uint64_t take = start < slen ? (l < slen - start ? l : slen - start) : 0;
                if ((fl & S2C_PF_X) && take) dashes += seq_dashes(d, q0 + start, take);
                start += l;
            } else if (op_dash(op)) {
                dashes += l;
            } else if (op == S2C_OP_I || op == S2C_OP_S) {
                start += l;
            }
        }
        drop = dashes > (uint64_t)d.maxdel;
    }
    // ---- runs of the piece's seqout range [ka, kb), insertion events
    const uint32_t lng = (fl & S2C_PF_LONG) ? S2C_RUN_LONG : 0u;
    const uint32_t bkind = S2C_RUN_BASES | ((fl & S2C_PF_X) ? S2C_RUN_XBIT : 0u) | (drop ? S2C_RUN_DROP : 0u) | lng;
    int64_t k = 0;
    uint64_t start = 0;
    for (uint32_t j = o; j < oend; j++) {
        const uint32_t w = d.ops[j], op = w & 15u;
        const uint64_t l = w >> 4;
        uint4 r = EMPTY;
        if (op_bases(op) || op_dash(op)) {
            const bool bases = op_bases(op);
            const uint64_t take = bases ? (start < slen ? (l < slen - start ? l : slen - start) : 0) : l;
            const int64_t s = k > ka ? k : ka, e = (k + (int64_t)take) < kb ? k + (int64_t)take : kb;
            if (e > s && (bases || !drop)) {
                const uint32_t gpos = P.x + (uint32_t)(s - ka);
                if (bases) {
                    const uint64_t q = q0 + start + (uint64_t)(s - k);
                    r = make_uint4(gpos, (uint32_t)(e - s) | (bkind << 24), (uint32_t)q, (uint32_t)(q >> 32));
                } else {
                    r = make_uint4(gpos, (uint32_t)(e - s) | ((S2C_RUN_DASH | lng) << 24), 0u, 0u);
                }
            }
            k += (int64_t)take;
            if (bases) start += l;
        } else if (op == S2C_OP_I) {
            const uint64_t take = start < slen ? (l < slen - start ? l : slen - start) : 0;
            if (ins && take) {
                const int64_t gkey = key0 + k;   // start_ref (:74) = POS-1 + seqout index here
                if (gkey >= (int64_t)roff) add_event(d, (uint64_t)gkey, q0 + start, (uint32_t)take);
            }
            start += l;
        } else if (op == S2C_OP_S) {
            start += l;
        }
        runs[j] = r;
    }
}

}  // namespace
}  // namespace s2c

// Launcher (called by s2c_reads in s2c_tile.hip)
int s2c_launch_reads(const s2c_dev *dv, hipStream_t st) {
    using namespace s2c;
    if (dv->n_pieces == 0) return S2C_OK;
    ReadsArgs a;
    a.pc = dv->pc; a.ops = dv->ops; a.bq = dv->bq; a.bx = dv->bx; a.tiles = dv->tiles; a.wtile = dv->wtile;
    a.runs = dv->runs; a.ibkt = dv->ibkt; a.ilong = dv->ilong; a.ilong_n = dv->ilong_n;
    a.n_pieces = (uint32_t)dv->n_pieces;
    a.maxdel_active = dv->maxdel_active ? 1u : 0u;
    a.maxdel = dv->maxdel < 0 ? 0u : (uint32_t)dv->maxdel;
    const unsigned grid = (unsigned)((dv->n_pieces + WG - 1) / WG);
    k_reads<<<grid, WG, 0, st>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? S2C_OK : s2c_set_error(S2C_ERR_HIP, std::string("k_reads: ") + hipGetErrorString(e));
}

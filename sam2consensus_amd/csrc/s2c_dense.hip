// s2c_dense.hip — k_tile_dense: shallow tiles without insertion keys (-f of one char).
//
// Such a tile's body is one char per position (:355-389 with no insertion columns and a
// one-char fill), so the byte offset of position q is q: no length scan.  One wave per tile:
//
//   1. DMA     the tile's window — the op words, base planes {p0, p1} and non-ACGT plane of
//              the short pieces starting up to kwin words before the tile (one contiguous
//              range each) — into LDS by buffer LDS-DMA with SGPR offsets (no per-lane address
//              arithmetic); the lane's piece records into registers.
//   2. walk    one lane per piece.  The common piece — one M / = / X token, no range, prefix
//              or long flag — is one run of min(l, len(SEQ)) bases (parsecigar :64-69) and
//              takes a few instructions; every other piece (D / I / S / H tokens, wrap ranges,
//              maxdel with '-' chars in SEQ) is queued, and the queue is walked afterwards by
//              the general parsecigar + maxdel walk (:46-82, :210) with all lanes busy.  Runs
//              of reads holding N / '-' chars are queued too: their SEQ chars go into the
//              per-position byte counters in one dense pass.
//   3. count   the G = 64 / (tile words) lanes of a word count the runs covering it — A C G T
//              into bit-sliced Harley–Seal counters, 8 records at a time.
//   4. vote    each lane holds 8 / G counter rows (a row = positions 8j + r, j = 0..3, one
//              byte each — the transposed counters' own layout, and the byte counters' layout
//              in LDS) and votes them four positions per register: coverage by byte adds, the
//              largest count by packed 16-bit max over (count << 3 | symbol) keys, the strict
//              majority (2·m1 > cov) by a packed subtract — for thresholds in (0, 0.5] that
//              alone decides the char (fl(t·cov) ≤ cov/2 < m1), for (0.5, 1] one more integer
//              test per position; the rest take the closed form of :241-251 / :359-366.
//              Chars come from a byte permute, rows are byte-transposed into consecutive
//              positions and stored.  Counts never touch HBM.
//
// Tiles are mapped XCD-major (blocks b, b + 8, ... — one XCD — take consecutive tiles), so
// the window overlap of neighbouring tiles is served by that XCD's L2.  The host sizes the
// tiles so the window takes ≤ S2C_DENSE_LDS bytes (S2C_DENSE_BYTES).
#include <algorithm>
#include <type_traits>

#include "s2c_common.h"

#ifdef S2C_PROF
// phase clocks (diagnostic build `make prof`, scripts/prof_dense.py): Σ over sampled waves
// (one tile in 64) of the s_memtime deltas of each phase
__device__ unsigned long long g_prof[16];
__device__ uint32_t g_abl;   // ablation bits (timing only; results wrong): 1 events, 2 count, 4 walk, 8 vote, 64 slow votes,
                             // 16 queued walk, 32 N / '-' events
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

__constant__ __attribute__((aligned(16))) uint8_t c_amb[64] = {
#define E(i) AMB.v[i]
    E(0), E(1), E(2), E(3), E(4), E(5), E(6), E(7), E(8), E(9), E(10), E(11), E(12), E(13), E(14), E(15),
    E(16), E(17), E(18), E(19), E(20), E(21), E(22), E(23), E(24), E(25), E(26), E(27), E(28), E(29), E(30), E(31),
    E(32), E(33), E(34), E(35), E(36), E(37), E(38), E(39), E(40), E(41), E(42), E(43), E(44), E(45), E(46), E(47),
    E(48), E(49), E(50), E(51), E(52), E(53), E(54), E(55), E(56), E(57), E(58), E(59), E(60), E(61), E(62), E(63)
#undef E
};

struct DenseArgs {
    const uint32_t *rs, *pc, *ops, *bq, *bx, *tiles, *items, *lp, *dwin, *dpc;
    const double *thresholds;
    uint64_t *tile_stats, *blk_len;
    uint8_t *out;
    uint32_t padded_len, n_cols, n_tiles, kwin, fill_nondash, maxdel_active, maxdel, n_items;
    uint32_t word_lo;               // rs holds entries word_lo .. (s2c_dev, ABI 13)
    const void *ops_end, *bq_end;   // ends of the DMA sources
    uint32_t buf_bytes;                                        // the window's LDS (16-byte multiple)
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
                if (fl & S2C_PF_DASH) {   // '-' chars of SEQ: x = 1, p1 = 0, p0 = 1
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
    // the next op word read ahead of run()'s LDS writes (which the compiler must assume alias it)
    uint32_t wn = j < j1 ? opl[j] : 0u;
    for (; j < j1; j++) {
        const uint32_t w = wn, op = w & 15u, l = w >> 4;
        wn = opl[min(j + 1u, j1 - 1u)];
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

// walk_piece's view of the batch in HBM (the tile's long pieces)
struct DenseMem {
    const uint32_t *ops, *bq, *bx;
    __device__ __forceinline__ uint32_t op(uint32_t j) const { return ops[j]; }
    __device__ __forceinline__ uint32_t p0(uint64_t w) const { return bq[2 * w]; }
    __device__ __forceinline__ uint32_t p1(uint64_t w) const { return bq[2 * w + 1]; }
    __device__ __forceinline__ uint32_t x(uint64_t w) const { return bx[w]; }
};

// A compact piece record of the item's window (s2c.h S2C_DPC_WORDS; ABI 12) decoded: rs = its
// start relative to the tile's first word + REC_BIAS, q = query base of SEQ[0] in the window's
// planes, its op slots [j, j + nops) in the window, len(SEQ), flags (x: word 0, y: word 1)
struct DPiece {
    uint32_t rs, q, nops, j, slen, fl;
};
__device__ __forceinline__ DPiece dpc_dec(uint32_t c0, uint32_t c1) {
    return DPiece{c0 & 0xFFFu, 16u * ((c0 >> 12) & 0x1FFFu), c0 >> 25, c1 & 0x1FFFu, (c1 >> 13) & 0x7FFu, c1 >> 24};
}
// FASTA body stores (written once, fetched by the host): nontemporal (−1.2 % on C5,
// profiles/r05/v6_nt_loads_stores_ab.txt; the same policy on the compact records' loads cost +2 %)
template <class T>
__device__ __forceinline__ void body_st(T *p, T v) {
    if constexpr (std::is_same_v<T, uint2>) {
        __builtin_nontemporal_store(v.x, (uint32_t *)p);
        __builtin_nontemporal_store(v.y, (uint32_t *)p + 1);
    } else {
        __builtin_nontemporal_store(v, p);
    }
}
// (a 3-vector takes 16 bytes: the record is addressed by dwords, 3 per record, 4-byte aligned)
__device__ __forceinline__ uint3 dpc_load(const DenseArgs &d, uint32_t i) {
    return ((const uint3 *)d.dpc)[i];
}
// rec_enc from a biased start (rs = tile-relative start + REC_BIAS)
__device__ __forceinline__ uint2 rec_enc_b(uint32_t rs, uint32_t len, uint32_t q) {
    return make_uint2(rs | ((rs + len) << 16), q - rs);
}

constexpr int WGD = 64;   // one wave per tile
constexpr int GSD = 8;    // records per counting group (one Harley–Seal tree)
constexpr int CNT_PART = 2;   // records whose geometry and plane words are in registers at once

// LDS byte address of a shared-memory pointer
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
// Scalar loads of uniform read-only words (tile records, items): s_load through the scalar
// cache, waited here — the compiler would otherwise emit vector loads (the kernel stores to
// global memory) and wait on vmcnt, i.e. on the window DMA in flight.
__device__ __forceinline__ double sload_f64(const double *p) {
    uint64_t r;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(uni_ptr((const uint32_t *)p)) : "memory");
    return __builtin_bit_cast(double, r);
}

// cache policy bits of the window DMA: nt (streamed; measured −2.5 % on C5 against the
// default policy and sc0 / sc1, profiles/r05/v5_dma_policy_ab.txt)
#define S2C_DMA_POLICY " nt"
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0 (reserved) is set and clobbered by the DMA
// n dwords src[0..n) of an array ending at `end` → LDS by 16-byte LDS-DMA (1 KB per wave
// instruction, the source offset in an SGPR: no per-lane address arithmetic).  The copy
// starts at the 16-byte boundary below src into the 16-byte aligned LDS region `dst`, so the
// dwords land at dst + (src & 15); lanes past the copy's end are masked off (the region
// needs dma16_bytes(n)).  The buffer range ends at `end` rounded up to 16 bytes (device
// arrays are allocated in 512-byte granules).  Issued as inline asm: the compiler neither
// sees the LDS writes nor counts these loads, so it never waits on them; completion is an
// explicit s_waitcnt vmcnt(0) before the window is read.
template <int WPT>
__device__ __forceinline__ void dma16(uint8_t *dst, const uint32_t *src, uint32_t n, const void *end) {
    const uint32_t lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);   // the waves share the 1 KB blocks
    const uintptr_t s0 = (uintptr_t)src, sal = s0 & ~(uintptr_t)15, delta = s0 - sal;
    const uintptr_t eal = ((uintptr_t)end + 15) & ~(uintptr_t)15;
    const uint32_t nbytes = (uint32_t)delta + 4 * n;
    v4i r;
    r.x = (int)uni((uint32_t)sal);
    r.y = (int)uni((uint32_t)(sal >> 32) & 0xFFFFu);
    r.z = (int)uni((uint32_t)min((uint64_t)(eal - sal), (uint64_t)0x7FFFFFF0u));
    r.w = 0x00020000;
    const uint32_t m0 = uni(lds_addr(dst));
    for (uint32_t base = 1024 * wv; base < nbytes; base += 1024 * WPT) {
        if (base + 16 * lane < nbytes)
            asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen" S2C_DMA_POLICY " lds"
                         :: "s"(uni(m0 + base)), "v"(16 * lane), "s"(r), "s"(uni(base)) : "memory", "m0");
    }
}
#pragma clang diagnostic pop
// LDS bytes of a dma16 region for n dwords (16-byte phase of the source + rounding)
__host__ __device__ constexpr uint32_t dma16_bytes(uint32_t n) { return (4 * n + 15 + 15) & ~15u; }

// Sum of N bit-sliced counters (mod 256: a word's counts are ≤ 255) whose planes NP .. 7 are
// zero, into 8 planes.  N = 4: two carry-save layers (a + b + c → s + 2k; s + d + 2k → s2 +
// 2k2), then one ripple s2 + 2k2; one v_bitop3 per full-adder output (xor3 0x96, majority
// 0xE8), the known-zero inputs folded at compile time.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// a + b + c with zero-ness known at compile time (za / zb / zc): sum and carry bits
template <bool ZA, bool ZB, bool ZC>
__device__ __forceinline__ void fadd(uint32_t a, uint32_t b, uint32_t c, uint32_t &s, uint32_t &k) {
    constexpr int nz = (ZA ? 0 : 1) + (ZB ? 0 : 1) + (ZC ? 0 : 1);
    if constexpr (nz == 3) {
        s = xor3(a, b, c);
        k = maj3(a, b, c);
    } else if constexpr (nz == 0) {
        s = 0u;
        k = 0u;
    } else if constexpr (nz == 1) {
        s = ZA ? (ZB ? c : b) : a;
        k = 0u;
    } else {   // two live inputs
        const uint32_t x = ZA ? b : a, y = ZC ? b : c;
        s = x ^ y;
        k = x & y;
    }
}
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}
template <int N, int NP>
__device__ __forceinline__ void bsum(const uint32_t (&in)[N][8], uint32_t (&o)[8]) {
    static_assert(N == 1 || N == 2 || N == 4, "counters summed");
    if constexpr (N == 1) {
#pragma unroll
        for (int i = 0; i < 8; i++) o[i] = in[0][i];
    } else if constexpr (N == 2) {   // ripple a + b: the carry into plane i is live for 1 ≤ i ≤ NP
        uint32_t cy = 0;
        static_for<0, 8>([&](auto ic) {
            constexpr int I = decltype(ic)::value;
            uint32_t k;
            fadd<(I >= NP), (I >= NP), (I == 0 || I > NP)>(in[0][I], in[1][I], cy, o[I], k);
            cy = k;
        });
    } else {
        // s / k live for planes < NP; s2 for planes ≤ NP, k2 for planes < NP; the ripple's carry
        // into plane i is live for 2 ≤ i ≤ NP + 1
        uint32_t s[8], k[8], s2[8], k2[8], cy = 0;
        static_for<0, 8>([&](auto ic) {
            constexpr int I = decltype(ic)::value;
            fadd<(I >= NP), (I >= NP), (I >= NP)>(in[0][I], in[1][I], in[2][I], s[I], k[I]);
        });
        static_for<0, 8>([&](auto ic) {
            constexpr int I = decltype(ic)::value;
            fadd<(I >= NP), (I >= NP), (I == 0 || I > NP)>(s[I], in[3][I], I ? k[(I + 7) % 8] : 0u, s2[I], k2[I]);
        });
        static_for<0, 8>([&](auto ic) {
            constexpr int I = decltype(ic)::value;
            uint32_t c2;
            fadd<(I > NP), (I == 0 || I > NP), (I < 2 || I > NP + 1)>(s2[I], I ? k2[(I + 7) % 8] : 0u, cy, o[I], c2);
            cy = c2;
        });
    }
}

// LDS hand-off between the lanes of one wave (its LDS operations execute in order: no wait)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The counters' exchange in the window's LDS once the count is done (k_tile_dense, after the
// barrier that ends the count): per wave, plane pairs [4][4 counters][XCH_STRIDE lanes] of
// uint2 (a padded lane stride: the lanes of a word read different counters on distinct
// banks), then aliased by the summed rows [word][4 counters][8 rows] at XCH_VROW dwords a word
constexpr uint32_t XCH_STRIDE = 65;
constexpr uint32_t XCH_NCH_MAX = 4;
constexpr uint32_t XCH_WAVE_BYTES = XCH_NCH_MAX * 4 * XCH_STRIDE * 8;   // 8,320
constexpr uint32_t XCH_VROW = 40;                              // 32 row dwords + 8 (conflict-free b64 reads)

// Per-position byte counters in the ROW layout of the transposed counters: tile-relative
// position p = 32w + 8j + r is byte j of dword 8w + r.
__device__ __forceinline__ void cnt_add1(uint32_t *cnt, uint32_t p) {
    atomicAdd(&cnt[((p >> 5) << 3) | (p & 7u)], 1u << (8 * ((p >> 3) & 3u)));
}
// +1 at the tile-relative positions [r0, r1) clipped to [0, lim), a word at a time: the
// word's covered positions m add (m >> r) & 0x01010101 to its row dword r (byte j of row r
// is position 8j + r), at most 8 atomics per word instead of one per position at its ends
__device__ __forceinline__ void cnt_range(uint32_t *cnt, int32_t r0, int32_t r1, int32_t lim) {
    const int32_t p0 = max(r0, 0), e = max(min(r1, lim), 0);
    for (int32_t wd = p0 >> 5; p0 < e && wd <= (e - 1) >> 5; wd++) {
        const int32_t lo = max(p0 - 32 * wd, 0), hi = min(e - 32 * wd, 32);
        const uint32_t m = (hi - lo >= 32 ? 0xFFFFFFFFu : ((1u << (hi - lo)) - 1u)) << lo;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const uint32_t inc = (m >> r) & 0x01010101u;
            if (inc) atomicAdd(&cnt[((uint32_t)wd << 3) + r], inc);
        }
    }
}

// The non-ACGT chars of SEQ in a run of bases (window-relative query bases [q, q + l), tile-
// relative position r0 of q): 'N' (p0 0) into ncnt, '-' (p0 1) into ccnt and, unless maxdel
// drops the read's '-', into dcnt.  Eight x-plane and base-plane words per round trip.
__device__ __forceinline__ void x_events(const uint32_t *bxl, const uint2 *bql, uint32_t q, uint32_t l, int32_t r0,
                                         int32_t lim, bool drop, uint32_t *dcnt, uint32_t *ncnt, uint32_t *ccnt) {
    const uint32_t wa = q >> 5, wb = (q + l - 1) >> 5;
    for (uint32_t w0 = wa; w0 <= wb; w0 += 8) {
        uint32_t xs[8];
        uint2 ps[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t qw = min(w0 + u, wb);
            xs[u] = bxl[qw];
            ps[u] = bql[qw];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t qw = w0 + u;
            const int32_t b0 = (int32_t)(32 * qw) - (int32_t)q;   // run offset of the word's bit 0
            uint32_t xm = qw <= wb ? xs[u] : 0u;
            if (b0 < 0) xm &= 0xFFFFFFFFu << (uint32_t)(-b0);
            if (b0 + 32 > (int32_t)l) xm &= 0xFFFFFFFFu >> (uint32_t)(b0 + 32 - (int32_t)l);
            xm &= ~ps[u].y;   // (p1 = 0 for every non-ACGT char)
            while (xm) {
                const uint32_t bit = (uint32_t)__builtin_ctz(xm);
                xm &= xm - 1;
                const int32_t r = r0 + b0 + (int32_t)bit;
                if (r < 0 || r >= lim) continue;
                if ((ps[u].x >> bit) & 1u) {
                    cnt_add1(ccnt, (uint32_t)r);
                    if (!drop) cnt_add1(dcnt, (uint32_t)r);
                } else {
                    cnt_add1(ncnt, (uint32_t)r);
                }
            }
        }
    }
}

// lane index among the active lanes of a ballot below this one
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// 16-bit halves (positions j = 0, 2 / j = 1, 3) of a register of 4 byte counts
__device__ __forceinline__ uint32_t lo16(uint32_t v) { return v & 0x00FF00FFu; }
__device__ __forceinline__ uint32_t hi16(uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0C030C01u); }
// the low bytes of the halves of e (j = 0, 2) and o (j = 1, 3) back into j order
__device__ __forceinline__ uint32_t merge16(uint32_t o, uint32_t e) { return __builtin_amdgcn_perm(o, e, 0x06020400u); }
// ... and their high bytes
__device__ __forceinline__ uint32_t merge16h(uint32_t o, uint32_t e) { return __builtin_amdgcn_perm(o, e, 0x07030501u); }
// vote keys count << 8 | symbol in the 16-bit halves of byte counts c (one byte permute each;
// sb = symbol · 0x01010101): e = positions j = 0, 2, o = j = 1, 3
__device__ __forceinline__ uint32_t key_e(uint32_t c, uint32_t sb) { return __builtin_amdgcn_perm(sb, c, 0x02040004u); }
__device__ __forceinline__ uint32_t key_o(uint32_t c, uint32_t sb) { return __builtin_amdgcn_perm(sb, c, 0x03040104u); }
typedef unsigned short v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(v2u, a), __builtin_bit_cast(v2u, b)));
}
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u, a) - __builtin_bit_cast(v2u, b));
}
template <int S>
__device__ __forceinline__ uint32_t pk_shr(uint32_t a) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u, a) >> (v2u){S, S});
}
// 0xFFFF in each half whose bit 15 is set
__device__ __forceinline__ uint32_t pk_sign(uint32_t a) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s, a) >> (v2s){15, 15});
}
// bit j (j = 0..3) = top bit of byte j
__device__ __forceinline__ uint32_t byte_bits(uint32_t m) { return ((m & 0x80808080u) * 0x00204081u) >> 28; }

// A tile's window (uniform values from its tile record; S2C_TILE_WORDS layout)
struct Win {
    uint32_t tile, a, n, cb0, pf0, npc, o0, nslot, qw0, nqw, W0, nwords, lp0, nlong, dpc0;
};
__device__ __forceinline__ Win win_of(const DenseArgs &d, uint32_t item) {
    Win v;
    // the item's window (S2C_DWIN_WORDS, built by the host from the tile record) in one
    // scalar round trip
    v16i r;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(r) : "s"(uni_ptr(d.dwin + (size_t)item * S2C_DWIN_WORDS)) : "memory");
    v.tile = (uint32_t)r[0];
    v.a = (uint32_t)r[1];
    v.n = (uint32_t)r[2] - v.a;
    v.cb0 = (uint32_t)r[3];
    v.lp0 = (uint32_t)r[4];
    v.nlong = (uint32_t)r[5] - v.lp0;
    v.pf0 = (uint32_t)r[6];
    v.npc = (uint32_t)r[7] - v.pf0;
    v.o0 = (uint32_t)r[8];
    v.nslot = (uint32_t)r[9] - v.o0;
    v.qw0 = (uint32_t)r[10];
    v.nqw = (uint32_t)r[11] - v.qw0;
    v.dpc0 = (uint32_t)r[12];
    v.W0 = v.a >> 5;
    v.nwords = (v.n + 31) / 32;
    return v;
}
// The window's arrays in LDS (S2C_DENSE_BYTES layout): op words, planes (each at its
// source's 16-byte phase, dma16), run records + RUN_PAD zero records, the walk's queues.
constexpr uint32_t RUN_PAD = 64;   // zero records after the last: a count group's reads past it
struct WinLds {
    const uint32_t *opl;
    const uint2 *bql;
    uint2 *runl;
    uint32_t *q;   // [nslot]: queued pieces (window index) from the front, X-run slots from the back
};
__device__ __forceinline__ const uint32_t *phase16(const uint8_t *region, const void *src) {
    return (const uint32_t *)(region + ((uintptr_t)src & 15));
}
__device__ __forceinline__ WinLds win_lds(const DenseArgs &d, const Win &v, uint8_t *buf) {
    WinLds L;
    const uint32_t *sop = d.ops + v.o0, *sbq = d.bq + 2 * (size_t)v.qw0;
    L.opl = phase16(buf, sop);
    buf += dma16_bytes(v.nslot);
    L.bql = (const uint2 *)phase16(buf, sbq);
    buf += dma16_bytes(2 * v.nqw);
    L.runl = (uint2 *)buf;
    L.q = (uint32_t *)(L.runl + v.nslot + RUN_PAD);
    return L;
}
// issue the LDS-DMA of window v into buf, shared by the tile's waves (completion: every wave's
// s_waitcnt vmcnt(0), then a barrier)
template <int WPT>
__device__ __forceinline__ void win_issue(const DenseArgs &d, const Win &v, uint8_t *buf) {
    dma16<WPT>(buf, d.ops + v.o0, v.nslot, d.ops_end);
    buf += dma16_bytes(v.nslot);
    dma16<WPT>(buf, d.bq + 2 * (size_t)v.qw0, 2 * v.nqw, d.bq_end);
}

// One tile of NWP words from its window in LDS, WPT waves (WT threads): a wave holds NWP / WPT
// words, G lanes per word, RPL = 8 / G counter rows (4 positions each) voted per lane.
// dcnt / ncnt / ccnt: zeroed byte counters; stl: the waves' partial tile statistics.
constexpr int WPT = 2;   // waves per tile (they share the window)
constexpr int WT = WGD * WPT;     // threads per tile
constexpr int PFN = 2;   // piece records per thread loaded with the DMA (windows of ≤ PFN·WT pieces)
template <int NWP>
__device__ __forceinline__ void dense_tile(const DenseArgs &d, const Win &v, const WinLds &L, uint32_t *dcnt,
                                           uint32_t *ncnt, uint32_t *ccnt, const uint8_t *amb, uint32_t fill0,
                                           const uint3 (&Pc)[PFN],
                                           uint32_t cw0, uint32_t cw1, unsigned long long t_entry,
                                           uint32_t (*stl)[WPT][4], uint32_t tid, uint8_t *scratch) {
    constexpr int NWPW = NWP / WPT, G = WGD / NWPW, RPL = 8 / G;
#ifdef S2C_PROF
    unsigned long long prof_t = t_entry;
#else
    (void)t_entry;
#endif
    PROF_MARK(1);   // phase 0: entry → window landed (scalar tile loads, DMA, piece records)
    const uint32_t lane = tid & 63, wv = tid >> 6;
    const uint32_t w = wv * NWPW + lane / G, g = lane % G;   // tile-relative word of this lane
    const uint32_t tile = v.tile, a = v.a, n = v.n, cb0 = v.cb0, npc = v.npc, o0 = v.o0, qw0 = v.qw0;
    const uint32_t W0 = v.W0, nwords = v.nwords, W = W0 + w;
    const bool active = w < nwords;
    const uint32_t K = d.kwin;
    const uint32_t pf0 = v.pf0;
    // the non-ACGT plane stays in HBM (read only for the ~14 % of runs with N / '-' in SEQ, in
    // one round trip per queue pass); window-relative word index as for the planes
    const uint32_t *opl = L.opl, *bxl = d.bx + qw0;
    const uint2 *bql = L.bql;
    uint2 *runl = L.runl;
    // this wave's queue: 64 entries per walk iteration (its pieces' share of the window)
    const uint32_t nitw = (npc + WT - 1) / WT, qcap = WGD * nitw;
    uint32_t *queue = L.q + wv * qcap;

    // ---- walk: one lane per piece → run records {gpos, (query base − 32·qw0) << 15 | len << 4
    //      | kind} of the bases; the common piece here, the others queued
    const int32_t T0 = (int32_t)(32 * W0), TL = (int32_t)(32 * nwords);   // the tile's words
    const bool mda = d.maxdel_active != 0;
    uint32_t nslow = 0, nx = 0;   // queue lengths (uniform)
    const uint32_t nit = ABL(4) ? 0u : nitw;
    uint32_t opw[PFN];   // the pieces' first op words, read together
#pragma unroll
    for (int u = 0; u < PFN; u++) opw[u] = (tid + WT * u < npc) ? opl[Pc[u].y & 0x1FFFu] : 0u;
    for (uint32_t it = 0; it < nit; it++) {
        const uint32_t k = tid + WT * it;
        uint3 P = Pc[0];
        uint32_t w0 = opw[0];
#pragma unroll
        for (int u = 1; u < PFN; u++) {   // (the loaded records by a select chain)
            P.x = it == (uint32_t)u ? Pc[u].x : P.x;
            P.y = it == (uint32_t)u ? Pc[u].y : P.y;
            P.z = it == (uint32_t)u ? Pc[u].z : P.z;
            w0 = it == (uint32_t)u ? opw[u] : w0;
        }
        const bool in = k < npc;
        if (it >= (uint32_t)PFN && in) {   // (windows of more than WT·PFN pieces)
            P = dpc_load(d, v.dpc0 + k);
            w0 = opl[P.y & 0x1FFFu];
        }
        const DPiece D = dpc_dec(P.x, P.y);
        const uint32_t pxv = P.z, fl = D.fl, slen = D.slen, j = D.j, nops = D.nops;
        const uint32_t op = w0 & 15u, l = w0 >> 4;
        const bool xf = (fl & S2C_PF_X) != 0;
        // (no maxdel count to take: the rule is off, or SEQ holds no '-'; S2C_PF_SIMPLE marks the
        // one-token pieces, whose length field already holds take)
        const bool plain = in && (fl & ~(uint32_t)(S2C_PF_X | S2C_PF_DASH | S2C_PF_SIMPLE | S2C_PF_XFEW)) == 0u && op_bases(op) &&
                           !((fl & S2C_PF_DASH) && mda);
        // one M / = / X token and nothing else: seqout = SEQ[0 : min(l, len(SEQ))] (:64-69)
        const bool fast = plain && nops == 1u;
        const uint32_t take = min(l, slen), q = D.q;
        if (fast) runl[j] = rec_enc_b(D.rs, take, q);
        // bases, D / N / P, bases (the deletion reads): two base runs here (:64-72: k = take,
        // then l1 '-', then SEQ[l : l + min(l2, len(SEQ) − l)]), the '-' run queued for the byte
        // counters unless maxdel drops it (:210: l1 dashes); with N / '-' in SEQ (no maxdel
        // count to take: `plain`) both base runs go to the X-run queue
        bool fdel = false, fdash = false;
        uint32_t da = 0, db = 0, t2 = 0, l1 = 0;   // the '-' run's tile-relative range, clipped to the tile
        if (plain && nops == 3u) {
            const uint32_t w1 = opl[j + 1], w2 = opl[j + 2];
            if (op_dash(w1 & 15u) && op_bases(w2 & 15u)) {
                l1 = w1 >> 4;
                t2 = l < slen ? min(w2 >> 4, slen - l) : 0u;
                const int32_t r0 = (int32_t)(D.rs + take) - REC_BIAS;
                da = (uint32_t)min(max(r0, 0), TL);
                db = (uint32_t)min(max(r0 + (int32_t)l1, 0), TL);
                fdel = true;
                fdash = db > da && !(mda && l1 > d.maxdel);
                runl[j] = rec_enc_b(D.rs, take, q);
                runl[j + 1] = make_uint2(0u, 0u);
                runl[j + 2] = rec_enc_b(D.rs + take + l1, t2, q + l);
            }
        }
        // queue: pieces for the general walk (their index) and the '-' runs of the deletion
        // reads (1 << 31 | begin << 12 | end, tile-relative: TL ≤ 2048) from the front; the X
        // runs' slots from the back.  A lane adds ≤ 3 entries (an X deletion read), so while
        // that could overrun the wave's queue (64 entries kept per walk iteration left) such
        // reads take the general walk instead (≤ 1 entry per lane)
        // the 'N' chars of a read whose SEQ holds at most two (S2C_PF_XFEW: their SEQ offsets in
        // px) straight into the 'N' counters through its runs: SEQ[0 : take) from P.x, the
        // deletion read's SEQ[l : l + t2) from P.x + take + l1; other reads with non-ACGT chars
        // queue their runs for the plane scan
        const bool xfew = (fl & S2C_PF_XFEW) != 0u && (fast || fdel);
        if (xfew) {
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t off = (pxv >> (16 * u)) & 0xFFFFu;
                int32_t r = -1;
                if (off < take) r = (int32_t)(D.rs + off) - REC_BIAS;
                else if (fdel && off >= l && off - l < t2) r = (int32_t)(D.rs + take + l1 + (off - l)) - REC_BIAS;
                if (off != 0xFFFFu && r >= 0 && r < TL) cnt_add1(ncnt, (uint32_t)r);
            }
        }
        bool x1 = (fast || fdel) && xf && !xfew, x2 = fdel && xf && !xfew && t2 > 0u;
        bool qd = (in && !fast && !fdel) || fdash;
        uint64_t bs = __ballot(qd), bxm = __ballot(x1), bx2 = __ballot(x2);
        if (nslow + nx + (uint32_t)(__popcll(bs) + __popcll(bxm) + __popcll(bx2)) > qcap - WGD * (nitw - 1u - it)) {
            if (fdel && xf && !xfew) {
                fdel = false;
                fdash = false;
            }
            x1 = fast && xf && !xfew;
            x2 = false;
            qd = (in && !fast && !fdel) || fdash;
            bs = __ballot(qd);
            bxm = __ballot(x1);
            bx2 = 0;
        }
        if (qd) queue[nslow + mbcnt(bs)] = fdel ? 0x80000000u | (da << 12) | db : k;
        if (x1) queue[qcap - 1u - nx - mbcnt(bxm)] = j;
        nx += (uint32_t)__popcll(bxm);
        if (x2) queue[qcap - 1u - nx - mbcnt(bx2)] = j + 2u;
        nx += (uint32_t)__popcll(bx2);
        nslow += (uint32_t)__popcll(bs);
    }
    // (the queued work below is this wave's own — its queue, its pieces' run records, atomic
    // byte-counter adds — so its LDS writes completing is enough: the other wave's records are
    // needed only by the count, after the barrier that ends the queued walks)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PROF_MARK(2);
    // queued pieces: the general walk; '-' runs and SEQ N / '-' straight into the byte counters.
    // A queued piece's record comes from the lane that loaded it (ds_bpermute, all lanes on).
    for (uint32_t base = 0; base < (ABL(16) ? 0u : nslow); base += WGD) {
        const uint32_t i = base + lane;
        const uint32_t qe = i < nslow ? queue[i] : 0u;
        if (i < nslow && (qe >> 31)) cnt_range(dcnt, (int32_t)((qe >> 12) & 0xFFFu), (int32_t)(qe & 0xFFFu), TL);
        const bool gen = i < nslow && !(qe >> 31);
        if (!__ballot(gen)) continue;   // (only '-' runs in this round)
        const uint32_t k = gen ? qe : 0u, it = k / WT;
        const int src = (int)(4 * (k % WGD));   // (k ≡ this wave's lane mod 64: WT is a multiple of 64)
        uint32_t c0 = 0, c1 = 0;
#pragma unroll
        for (int u = 0; u < PFN; u++) {
            const uint32_t px = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)Pc[u].x);
            const uint32_t py = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)Pc[u].y);
            const bool me = it == (uint32_t)u;
            c0 = me ? px : c0;
            c1 = me ? py : c1;
        }
        if (gen) {
            if (it >= (uint32_t)PFN) {   // (windows of more than WT·PFN pieces)
                const uint3 R = dpc_load(d, v.dpc0 + k);
                c0 = R.x;
                c1 = R.y;
            }
            const DPiece D = dpc_dec(c0, c1);
            // (walk_window's view: the global start position and len(SEQ) | flags << 24)
            const uint4 P = make_uint4((uint32_t)T0 + D.rs - (uint32_t)REC_BIAS, 0u, 0u, D.slen | D.fl << 24);
            const bool lng = (D.fl & S2C_PF_LONG) != 0;   // (a long piece starting here does not overlap the tile)
            walk_window(opl, bql, bxl, P, D.j, D.j + D.nops, D.q, mda, d.maxdel,
                        [&](uint32_t j, uint32_t gp, uint32_t l, uint32_t kind, uint32_t q) {
                            const uint32_t kd = (lng || kind == S2C_RUN_EMPTY) ? 0u : (kind & 3u);
                            runl[j] = kd == S2C_RUN_BASES ? rec_enc(gp - (uint32_t)T0, l, q) : make_uint2(0u, 0u);
                            const int32_t r0 = (int32_t)gp - T0;
                            if (kd == S2C_RUN_DASH) cnt_range(dcnt, r0, r0 + (int32_t)l, TL);
                            if (kd == S2C_RUN_BASES && (kind & S2C_RUN_XBIT))
                                x_events(bxl, bql, q, l, r0, TL, (kind & S2C_RUN_DROP) != 0, dcnt, ncnt, ccnt);
                        });
        }
    }
    lds_sync();   // every run record written
    PROF_MARK(3);

    // ---- count the base records of this lane's word (candidates cw0 + g + G·m < cw1),
    //      bit-sliced by the planes (non-ACGT chars of SEQ as A / C: taken back in the vote), a
    //      group's records read together from LDS
    uint32_t C[4][8];   // X = p0 (C|T), Y = p1 (G|T), Z = T, V = covered
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int b = 0; b < 8; b++) C[c][b] = 0;
    const uint32_t nrec = cw0 + g < cw1 ? (cw1 - cw0 - g + G - 1) / G : 0u;
    // full groups of 8, then (when the wave's longest lane has 1-4 records left) a group of 4
    const uint32_t nmx = ABL(2) ? 0u : uni(__ockl_wfred_max_u32(nrec));
    const uint32_t ngrp = nmx / GSD + ((nmx % GSD) > 4u ? 1u : 0u);
    const bool half = (nmx % GSD) != 0u && (nmx % GSD) <= 4u;
    // Group gi reads records cw0 + g + G·(8 gi + u), u < 8, by immediate offsets from one base
    // clamped to the end of the records: every slot past this lane's candidates is a record of
    // a piece starting in a later word (or a zero pad record), so it covers nothing here.
    // The planes are aligned to the word's bit 0 (query base b of position 32·W; a record
    // outside the word reads any LDS word, masked off).
    const uint32_t rend = v.nslot;
    const int16_t wbias = (int16_t)(32 * w + REC_BIAS);     // the word's first position, biased (rec_enc)
    const v2s wpk = (v2s){wbias, wbias};
    const uint2 *bqw = bql + ((32 * w + REC_BIAS) >> 5);    // plane word of query y + wbias, less y >> 5
    auto load_runs = [&](uint2 (&rv)[GSD], uint32_t gi) {
        // (64-bit loads: two records per ds_read2_b64)
        const unsigned long long *rb = (const unsigned long long *)(runl + min(cw0 + g + G * GSD * gi, rend));
#pragma unroll
        for (int u = 0; u < GSD; u++) {
            unsigned long long r = rb[G * u];
            asm("" : "+v"(r));   // (kept one 64-bit load: its halves are used as different types)
            rv[u] = make_uint2((uint32_t)r, (uint32_t)(r >> 32));
        }
    };
    // one group's 8 records → Harley–Seal tree of each plane; returns the weight-8 carries
    // NR = 8: returns the weight-8 carries in t8o; NR = 4 (a tail group): the weight-4 carries
    auto count_group = [&](const uint2 (&rv)[GSD], uint32_t (&t8o)[4], auto nr) {
        constexpr int NR = decltype(nr)::value;
        uint32_t pend[4], t2a[4], t4a[4];
#pragma unroll
        for (int h = 0; h < NR; h += CNT_PART) {   // (parts of CNT_PART records: fewer live registers)
        uint32_t bm[GSD], fx[GSD], sh[GSD];
        uint2 pa[GSD], pb[GSD];
#pragma unroll
        for (int u = h; u < h + CNT_PART; u++) {
            rec_mask(rv[u].x, wpk, bm[u], fx[u]);   // the word's covered bits (rec_enc)
            // query base of the word's bit 0 = y + (biased word start): word offset y >> 5 from
            // the lane's base, bit offset y mod 32 (the funnel shift takes the low 5 bits)
            sh[u] = rv[u].y;
            const uint2 *pw = bqw + ((int32_t)rv[u].y >> 5);
            pa[u] = pw[0];
            pb[u] = pw[1];
        }
#pragma unroll
        for (int u = h; u < h + CNT_PART; u++) {
            uint32_t x, y;   // x & (bm | fx)
            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe0" : "=v"(x) : "v"(funnel(pb[u].x, pa[u].x, sh[u])), "v"(bm[u]), "v"(fx[u]));
            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe0" : "=v"(y) : "v"(funnel(pb[u].y, pa[u].y, sh[u])), "v"(bm[u]), "v"(fx[u]));
            const uint32_t mk[4] = {x, y, x & y, bm[u] | fx[u]};
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
                    if constexpr (NR == 4) t8o[c] = t4;
                    continue;
                }
                csa(t8o[c], C[c][2], C[c][2], t4a[c], t4);
            }
        }
        }
    };
    using Full = std::integral_constant<int, 8>;
    using Half = std::integral_constant<int, 4>;
    // two groups per trip (ping-pong record buffers; the next group's records are read while
    // this group's plane words are in flight), their weight-8 carries closed together
    uint2 ra[GSD], rb2[GSD];
    auto trip = [&](uint32_t gi) -> bool {   // groups gi, gi + 1; false: the last group counted
        uint32_t t8a[4], t8b[4];
        if (gi + 1 < ngrp) load_runs(rb2, gi + 1);
        count_group(ra, t8a, Full{});
        if (gi + 1 >= ngrp) {
#pragma unroll
            for (int c = 0; c < 4; c++) close8(C[c], t8a[c]);
            return false;
        }
        if (gi + 2 < ngrp) load_runs(ra, gi + 2);
        count_group(rb2, t8b, Full{});
#pragma unroll
        for (int c = 0; c < 4; c++) close16(C[c], t8a[c], t8b[c]);
        return true;
    };
    if (ngrp) {   // the first trip peeled: its counters start at zero (folded, no initialising moves)
        load_runs(ra, 0);
        if (trip(0))
            for (uint32_t gi = 2; gi < ngrp; gi += 2)
                if (!trip(gi)) break;
    }
    if (half) {   // records 8·ngrp .. 8·ngrp + 3 of each lane
        uint32_t t4[4];
        load_runs(ra, ngrp);
        count_group(ra, t4, Half{});
#pragma unroll
        for (int c = 0; c < 4; c++) close4(C[c], t4[c]);
    }
    // long pieces over the tile (rare: spans past the window, C5's long deletions): the tile's
    // long list holds their piece indices; the lanes of each word take them one per lane and
    // round and walk each from HBM (parsecigar :64-81 + maxdel :210, walk_piece), keeping the
    // runs' parts in the lane's word — bases into the counters (planes from HBM), '-' runs and
    // the N / '-' chars of SEQ into the byte counters (the host keeps a dense tile's candidate
    // runs + long runs ≤ 255 per word)
    uint32_t ntr = 0;   // long-piece rounds (each adds ≤ 1 per position to a lane's counters)
    if (v.nlong) {
        const int32_t wr = (int32_t)(32 * w);   // tile-relative first position of the lane's word
        ntr = uni(__ockl_wfred_max_u32(active && g < v.nlong ? (v.nlong - g + G - 1) / G : 0u));
        for (uint32_t m = 0; m < ntr; m++) {
            const uint32_t j = g + G * m;
            if (!(active && j < v.nlong)) continue;
            const uint32_t k = d.lp[v.lp0 + j];
            const uint4 P = ((const uint4 *)d.pc)[k];
            const uint32_t oend = d.pc[4 * (size_t)k + 6];   // next piece's op offset
            walk_piece(DenseMem{d.ops, d.bq, d.bx}, P, oend, mda, d.maxdel,
                       [&](uint32_t, uint32_t gp, uint32_t l, uint32_t kind, uint64_t q) {
                           const uint32_t kd = kind & 3u;
                           if (kd != S2C_RUN_BASES && kd != S2C_RUN_DASH) return;
                           const RecGeom gm = rec_geom(gp, l, W);
                           if (!gm.valid) return;
                           const int32_t p0 = wr + (int32_t)gm.lo, p1 = p0 + __popc(gm.valid);
                           if (kd == S2C_RUN_DASH) {
                               cnt_range(dcnt, p0, p1, TL);
                               return;
                           }
                           const uint64_t qs = q + gm.qs, qw = qs >> 5;
                           const uint32_t sh = (uint32_t)(qs & 31);
                           const uint32_t mx = (funnel(d.bq[2 * qw + 2], d.bq[2 * qw], sh) << gm.lo) & gm.valid;
                           const uint32_t my = (funnel(d.bq[2 * qw + 3], d.bq[2 * qw + 1], sh) << gm.lo) & gm.valid;
                           ripple1(C[0], mx);
                           ripple1(C[1], my);
                           ripple1(C[2], mx & my);
                           ripple1(C[3], gm.valid);
                           if (kind & S2C_RUN_XBIT) {
                               uint32_t xm = (funnel(d.bx[qw + 1], d.bx[qw], sh) << gm.lo) & gm.valid;
                               while (xm) {
                                   const uint32_t bit = (uint32_t)__builtin_ctz(xm);
                                   xm &= xm - 1;
                                   if ((mx >> bit) & 1u) {   // '-' of SEQ (p0 = 1)
                                       cnt_add1(ccnt, (uint32_t)(wr + (int32_t)bit));
                                       if (!(kind & S2C_RUN_DROP)) cnt_add1(dcnt, (uint32_t)(wr + (int32_t)bit));
                                   } else {
                                       cnt_add1(ncnt, (uint32_t)(wr + (int32_t)bit));
                                   }
                               }
                           }
                       },
                       [](uint64_t, uint64_t, uint32_t) {});   // (a dense tile holds no insertion keys)
        }
    }
    PROF_MARK(5);
    // queued single-token runs of reads with N / '-' in SEQ (never dropped: maxdel is off; 0.08
    // per C5 wave: read here, where their registers are not live through the count)
    for (uint32_t i = lane; i < (ABL(32) ? 0u : nx); i += WGD) {
        const Rec rc = rec_dec(runl[queue[qcap - 1u - i]]);
        x_events(bxl, bql, rc.q, rc.l, rc.r0, TL, false, dcnt, ncnt, ccnt);
    }
    lds_sync();   // the byte counters are final, and every wave's count is done: the window's LDS is scratch
    PROF_MARK(4);
    // the byte counters of this lane's rows: read now, used by the vote
    const uint32_t rbase = 8 * w + g * RPL;   // the rows' dword index in the byte counters
    uint32_t rD[RPL], rN[RPL], rX[RPL];       // '-', 'N', '-' of SEQ
#pragma unroll
    for (int rr = 0; rr < RPL; rr++) {
        rD[rr] = active ? dcnt[rbase + rr] : 0u;
        rN[rr] = active ? ncnt[rbase + rr] : 0u;
        rX[rr] = active ? ccnt[rbase + rr] : 0u;
    }
    // ---- counters → byte counts of this lane's rows g·RPL .. g·RPL + RPL − 1 (row r byte j =
    //      position 8j + r), summed over the word's G lanes.  The sum is taken while the counters
    //      are still bit-sliced: every lane puts its four counters' planes into the scratch,
    //      then each lane adds ONE counter of its word over the SRC lanes that hold it (a
    //      carry-save sum of bit planes, ~45 instructions) and transposes that one counter —
    //      where each lane used to transpose all four (192 instructions) and reduce-scatter the
    //      bytes by DPP (72).  The word's rows go back through the scratch to the lanes voting them.
    uint32_t rA[RPL], rC[RPL], rG[RPL], rT[RPL];
    {
        constexpr int SRC = G < 4 ? G : 4;   // lanes summed per counter
        constexpr int CPL = 4 / SRC;         // counters each lane sums (G = 2: two)
        constexpr int PARTS = G / SRC;       // G = 8: two half-groups of 4, added by DPP
        const uint32_t wl = lane / G;        // the lane's word within the wave
        // G = 8: lanes g and 7 − g (row_half_mirror partners) take the same counter, g < 4 over
        // lanes 0-3 of the word and 7 − g over lanes 4-7
        const uint32_t part = PARTS == 2 ? (g >= 4 ? 1u : 0u) : 0u;
        const uint32_t cb = PARTS == 2 ? min(g, 7u - g) : (g % (uint32_t)SRC) * (uint32_t)CPL;
        const uint32_t src0 = wl * G + part * SRC;
        uint2 *xp = (uint2 *)(scratch + wv * XCH_WAVE_BYTES);   // this wave's scratch
        uint32_t *vp = (uint32_t *)xp;   // the rows (aliases the planes: read before, in wave order)
        // a lane's count ≤ its record slots + long rounds: planes 0 .. 2·NCH − 1 carry it
        const uint32_t mxc = 8 * ngrp + (half ? 4u : 0u) + ntr;
        const uint32_t npl = 32u - (uint32_t)__builtin_clz(mxc | 1u);
        auto xchg = [&](auto nch_c) {
            constexpr int NCH = decltype(nch_c)::value;   // plane pairs exchanged
#pragma unroll
            for (int ch = 0; ch < NCH; ch++)
#pragma unroll
                for (int c = 0; c < 4; c++) xp[(ch * 4 + c) * XCH_STRIDE + lane] = make_uint2(C[c][2 * ch], C[c][2 * ch + 1]);
            wave_lds_sync();
            uint32_t S[CPL][8];
#pragma unroll
            for (int k = 0; k < CPL; k++) {
                uint32_t in[SRC][8];
#pragma unroll
                for (int j = 0; j < SRC; j++) {
#pragma unroll
                    for (int ch = 0; ch < 4; ch++) {
                        uint2 pv = make_uint2(0u, 0u);
                        if (ch < NCH) pv = xp[(ch * 4 + cb + k) * XCH_STRIDE + src0 + j];
                        in[j][2 * ch] = pv.x;
                        in[j][2 * ch + 1] = pv.y;
                    }
                }
                constexpr int NP = 2 * NCH < 8 ? 2 * NCH : 8;   // planes exchanged
                bsum<SRC, NP>(in, S[k]);
                // (the sum's planes: ≤ NP + 2 for four counters, NP + 1 for two)
                transpose8z<(SRC == 4 ? (NP + 2 < 8 ? NP + 2 : 8) : SRC == 2 ? (NP + 1 < 8 ? NP + 1 : 8) : NP)>(S[k]);
                if constexpr (PARTS == 2) {
#pragma unroll
                    for (int r = 0; r < 8; r++) S[k][r] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)S[k][r], 0x141, 0xF, 0xF, true);
                }
            }
            wave_lds_sync();
            if (part == 0) {
#pragma unroll
                for (int k = 0; k < CPL; k++) {
                    uint4 *dst = (uint4 *)(vp + wl * XCH_VROW + (cb + k) * 8);
                    dst[0] = make_uint4(S[k][0], S[k][1], S[k][2], S[k][3]);
                    dst[1] = make_uint4(S[k][4], S[k][5], S[k][6], S[k][7]);
                }
            }
            wave_lds_sync();
        };
        if (npl <= 2) xchg(std::integral_constant<int, 1>{});
        else if (npl <= 4) xchg(std::integral_constant<int, 2>{});
        else if (npl <= 6) xchg(std::integral_constant<int, 3>{});
        else xchg(std::integral_constant<int, 4>{});
        const uint32_t *vr = vp + wl * XCH_VROW + g * RPL;
#pragma unroll
        for (int rr = 0; rr < RPL; rr++) {   // counts from the planes' sums: X = C|T, Y = G|T, Z = T, V = covered
            const uint32_t x = vr[rr], y = vr[8 + rr], z = vr[16 + rr], v = vr[24 + rr];
            rA[rr] = v - x - y + z;
            rC[rr] = x - z;
            rG[rr] = y - z;
            rT[rr] = z;
        }
    }
    PROF_MARK(6);

    // ---- vote of this lane's rows: row rr = word positions 8j + g·RPL + rr (j = 0..3)
    const uint32_t md = (uint32_t)min(max(d.min_depth, 1), 0x7FFF);   // called: cov ≥ max(-m, 1) (:356-359)
    const uint32_t md16 = md | (md << 16);
    // per row: chars of the largest count, masks (one byte per position) of strict majority
    // and of "not called", the largest count m1 and coverage (bytes), in-tile bytes
    uint32_t chr[RPL], fmk[RPL], ncm[RPL], m1b[RPL], cvb[RPL], inb[RPL];
    uint32_t sc = 0;
    const bool wave_full = uni(n >= 32u * (wv * NWPW + NWPW) ? 1u : 0u) != 0u;   // (uniform)
#pragma unroll
    for (int rr = 0; rr < RPL; rr++) {
        const uint32_t cA = rA[rr] - rN[rr], cC = rC[rr] - rX[rr];   // 'N' counted as A, SEQ '-' as C
        const uint32_t cv = cA + cC + rG[rr] + rT[rr] + rD[rr] + rN[rr];   // ≤ 255 per byte
        // in-tile positions: p = 32w + 8j + r < n
        // (bytes j < ⌈(n − pr) / 8⌉, at most 4)
        // (a wave whose words are all inside the tile — every wave of a full tile: all bytes)
        uint32_t im = 0xFFFFFFFFu;
        if (!wave_full) {
            const int32_t nj = min(max(((int32_t)n - (int32_t)(32 * w + g * RPL + rr) + 7) >> 3, 0), 4);
            im = (active && nj) ? 0xFFFFFFFFu >> (32 - 8 * nj) : 0u;
        }
        inb[rr] = im;
        cvb[rr] = cv;
        sc = __builtin_amdgcn_udot4(cv & im, 0x01010101u, sc, false);   // Σ cov over the tile (:357)
        // keys count << 8 | symbol ("-ACGNT" index), halves e (j = 0, 2) and o (j = 1, 3); the
        // largest key's symbol is the char wherever the count is a strict majority (elsewhere
        // the tie order does not matter: fill, or the closed form below)
        const uint32_t cnt[NSYM] = {rD[rr], cA, cC, rG[rr], rN[rr], rT[rr]};
        uint32_t ke = key_e(cnt[0], 0u), ko = key_o(cnt[0], 0u);
#pragma unroll
        for (uint32_t s = 1; s < NSYM; s++) {
            ke = pk_max(ke, key_e(cnt[s], s * 0x01010101u));
            ko = pk_max(ko, key_o(cnt[s], s * 0x01010101u));
        }
        const uint32_t ce = lo16(cv), co = hi16(cv);
        // strict majority 2·m1 > cov: the half's bit 15 of cov − 2·m1 (key >> 7 = 2·m1)
        const uint32_t mje = pk_sign(pk_sub(ce, pk_shr<7>(ke))), mjo = pk_sign(pk_sub(co, pk_shr<7>(ko)));
        // not called: cov < md
        const uint32_t nce = pk_sign(pk_sub(ce, md16)), nco = pk_sign(pk_sub(co, md16));
        const uint32_t sym = merge16(ko, ke);
        chr[rr] = __builtin_amdgcn_perm(0x0000544Eu, 0x4743412Du, sym);   // "-ACGNT"[sym]
        fmk[rr] = merge16(mjo, mje);
        ncm[rr] = merge16(nco, nce) | ~im;
        m1b[rr] = merge16h(ko, ke);
    }
    const uint32_t fill4 = fill0 * 0x01010101u;
    const uint64_t ostride = (uint64_t)d.padded_len + d.n_cols;   // max(1, len(fill)) = 1
    uint8_t *const obase = d.out + (uint64_t)a + cb0 + 32 * w + g * RPL;
    const bool full = active && 32 * w + 32 <= n;
    // the count of symbol s at row rr, byte j (slow path: run-time indices, select chains)
    auto sel = [&](const uint32_t (&R)[RPL], uint32_t r) -> uint32_t {
        uint32_t v = R[0];
#pragma unroll
        for (int k = 1; k < RPL; k++) {
            v = r == (uint32_t)k ? R[k] : v;
            asm volatile("" : "+v"(v));   // keeps the chain of selects (no indexed copy)
        }
        return v;
    };
    for (int t = 0; t < (ABL(8) ? 0 : d.n_thr); t++) {
        const double th = sload_f64(d.thresholds + t);
        // threshold class: (0, 0.5] the majority decides; (0.5, 1] plus m1·2^15 ≥ uq·cov; else none
        const bool clsA = th > 0.0 && th <= 0.5, clsB = th > 0.5 && th <= 1.0;
        const uint32_t uq = clsB ? (uint32_t)ceil(th * 32768.0) + 1u : 0u;
        uint32_t ow[RPL], slow = 0, nd = 0, ne = 0;
#pragma unroll
        for (int rr = 0; rr < RPL; rr++) {
            uint32_t fm = (clsA || clsB) ? fmk[rr] & ~ncm[rr] : 0u;
            if (clsB) {   // m1·2^15 ≥ uq·cov per position (m1, cov ≤ 255: 32-bit products)
                uint32_t ok = 0, mb = m1b[rr], cb = cvb[rr];
                asm volatile("" : "+v"(mb), "+v"(cb));   // (kept here: not hoisted for every class)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t m1 = (mb >> (8 * j)) & 0xFFu, cv = (cb >> (8 * j)) & 0xFFu;
                    ok |= (m1 << 15) >= uq * cv ? (0xFFu << (8 * j)) : 0u;
                }
                fm &= ok;
            }
            ow[rr] = (chr[rr] & fm) | (fill4 & ncm[rr]);   // fast chars; fill; slow bytes 0 for now
            slow |= byte_bits(~(fm | ncm[rr])) << (4 * rr);
            // non-'-' chars: fast chars ≠ '-' and in-tile fill chars
            const uint32_t nz = (chr[rr] ^ 0x2D2D2D2Du) & fm;   // nonzero byte ⟺ fast char ≠ '-'
            const uint32_t nzb = (((nz & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | nz) & 0x80808080u;
            nd += (uint32_t)__popc(nzb) + d.fill_nondash * (uint32_t)__popc(ncm[rr] & inb[rr] & 0x01010101u);
        }
        // the other called positions: closed form of the group-sort vote (:241-251, :359-366)
        if (ABL(64)) slow = 0;
        while (slow) {
            const uint32_t i = (uint32_t)__builtin_ctz(slow);
            slow &= slow - 1;
            const uint32_t rr = i >> 2, sh = 8 * (i & 3);
            uint32_t c6[NSYM];   // "-ACGNT"
            c6[0] = (sel(rD, rr) >> sh) & 0xFFu;
            c6[4] = (sel(rN, rr) >> sh) & 0xFFu;
            c6[1] = ((sel(rA, rr) >> sh) & 0xFFu) - c6[4];
            c6[2] = ((sel(rC, rr) >> sh) & 0xFFu) - ((sel(rX, rr) >> sh) & 0xFFu);
            c6[3] = (sel(rG, rr) >> sh) & 0xFFu;
            c6[5] = (sel(rT, rr) >> sh) & 0xFFu;
            const uint32_t cov = c6[0] + c6[1] + c6[2] + c6[3] + c6[4] + c6[5];
            uint32_t gs[NSYM];
            greater_sums(c6, gs);
            const uint32_t ch = amb[vote_mask_u32(c6, gs, th * (double)cov)];
            nd += ch != '-';
            ne += ch == 0xFFu;
#pragma unroll
            for (int v = 0; v < RPL; v++) {
                ow[v] = rr == (uint32_t)v ? ow[v] | (ch << sh) : ow[v];
                asm volatile("" : "+v"(ow[v]));
            }
        }
        // rows → consecutive positions: byte j of row rr is position 8j + g·RPL + rr
        uint8_t *dst = obase + (uint64_t)t * ostride;
        uint32_t cj[4];   // RPL ≤ 4 bytes of each j (RPL = 8: two halves, below)
        auto tr4 = [](uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t (&o)[4]) {   // 4×4 byte transpose
            const uint32_t t0 = __builtin_amdgcn_perm(r1, r0, 0x05010400u);
            const uint32_t t1 = __builtin_amdgcn_perm(r1, r0, 0x07030602u);
            const uint32_t t2 = __builtin_amdgcn_perm(r3, r2, 0x05010400u);
            const uint32_t t3 = __builtin_amdgcn_perm(r3, r2, 0x07030602u);
            o[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);
            o[1] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);
            o[2] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
            o[3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
        };
        if constexpr (RPL == 8) {
            uint32_t c2[4];
            tr4(ow[0], ow[1], ow[2], ow[3], cj);
            tr4(ow[4 % RPL], ow[5 % RPL], ow[6 % RPL], ow[7 % RPL], c2);
            if (full) {
#pragma unroll
                for (int j = 0; j < 4; j++) body_st((uint2 *)(dst + 8 * j), make_uint2(cj[j], c2[j]));
            } else if (active) {   // (the tile's last word; bounds kept here, not hoisted)
                uint32_t nn = n - 32 * w;
                asm volatile("" : "+v"(nn));
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int b = 0; b < 8; b++)
                        if (8 * j + b < nn) dst[8 * j + b] = (uint8_t)((b < 4 ? cj[j] : c2[j]) >> (8 * (b & 3)));
            }
        } else {
            tr4(ow[0], RPL > 1 ? ow[1 % RPL] : 0u, RPL > 2 ? ow[2 % RPL] : 0u, RPL > 3 ? ow[3 % RPL] : 0u, cj);
            if (full) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if constexpr (RPL == 4) body_st((uint32_t *)(dst + 8 * j), cj[j]);
                    else if constexpr (RPL == 2) body_st((uint16_t *)(dst + 8 * j), (uint16_t)cj[j]);
                    else body_st(dst + 8 * j, (uint8_t)cj[j]);
                }
            } else if (active) {   // (the tile's last word; bounds kept here, not hoisted)
                uint32_t nn = n - 32 * w - g * RPL;
                asm volatile("" : "+v"(nn));
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int b = 0; b < RPL; b++)
                        if ((int32_t)(8 * j + b) < (int32_t)nn) dst[8 * j + b] = (uint8_t)(cj[j] >> (8 * b));
            }
        }
        // one reduction: at t = 0 Σcov (≤ 4·RPL·255 per lane: 17 bits per wave for RPL ≤ 2, 18
        // for 4) with the non-'-' count (≤ 256·RPL) above it; later thresholds the non-'-'
        // count alone; the vote-error count (almost always 0 in the whole wave) only when some
        // lane has one (round 5: two reductions per threshold)
        uint32_t nde;
        constexpr uint32_t SCB = RPL <= 2 ? 17u : 18u;
        static_assert(RPL <= 4, "Σcov and the non-'-' count share 32 bits");
        if (t == 0) {
            const uint32_t s2 = wave_sum(sc | (nd << SCB));
            sc = s2 & ((1u << SCB) - 1u);
            nde = s2 >> SCB;
        } else {
            nde = wave_sum(nd);
        }
        if (__ballot(ne != 0u)) nde |= wave_sum(ne) << 16;
        if (lane == 0) {   // this wave's share (by threshold parity: one barrier per threshold)
            stl[t & 1][wv][0] = sc;
            stl[t & 1][wv][1] = nde & 0xFFFFu;
            stl[t & 1][wv][2] = nde >> 16;
        }
        lds_sync();
        if (tid == 0) {   // tile statistics (:352-397); ≤ 2048 positions: u32 partial sums
            uint64_t s0 = 0, s2 = 0, s3 = 0;
#pragma unroll
            for (int k = 0; k < WPT; k++) {
                s0 += stl[t & 1][k][0];
                s2 += stl[t & 1][k][1];
                s3 += stl[t & 1][k][2];
            }
            const size_t jt = (size_t)t * d.n_tiles + tile;
            uint64_t *st = d.tile_stats + jt * 4;
            st[0] = s0;
            st[1] = n;
            st[2] = s2;
            st[3] = s3;
            d.blk_len[jt] = n;
        }
    }
    PROF_MARK(7);
#ifdef S2C_PROF
    if (threadIdx.x == 0 && (blockIdx.x & 63) == 0) {
        atomicAdd(&g_prof[8], 1ull);
        atomicAdd(&g_prof[9], (unsigned long long)ngrp);
        atomicAdd(&g_prof[10], (unsigned long long)npc);
        atomicAdd(&g_prof[11], (unsigned long long)(v.nslot + 3 * v.nqw));
        atomicAdd(&g_prof[12], (unsigned long long)nslow);
        atomicAdd(&g_prof[13], (unsigned long long)nx);
    }
#endif
}

// One wave per tile (block b → item, XCD-major: the blocks of one XCD, b ≡ x mod 8, take a
// contiguous range of items, so neighbouring windows meet in that XCD's L2).  Everything the
// tile needs arrives by one LDS-DMA round trip after the scalar loads of its tile record.
template <int NWP>
__global__ __launch_bounds__(WT) void k_tile_dense(const DenseArgs d) {
    extern __shared__ uint4 arena[];   // the window (S2C_DENSE_BYTES layout)
    // one byte per position (row layout): '-' (D/N/P runs, '-' of SEQ unless maxdel drops
    // the read's), 'N' of SEQ, '-' of SEQ (all: the planes count them as C, and 'N' as A)
    __shared__ __attribute__((aligned(16))) uint32_t dcnt[8 * NWP], ncnt[8 * NWP], ccnt[8 * NWP];
    __shared__ __attribute__((aligned(16))) uint8_t amb[64];
    __shared__ uint32_t stl[2][WPT][4];
    S2C_POISON(arena, d.buf_bytes);   // (before the window's DMA lands there)
    S2C_POISON(dcnt, sizeof(dcnt));
    S2C_POISON(ncnt, sizeof(ncnt));
    S2C_POISON(ccnt, sizeof(ccnt));
    S2C_POISON(amb, sizeof(amb));
    S2C_POISON(stl, sizeof(stl));
    S2C_POISON_DONE();
#ifdef S2C_PROF
    const unsigned long long t_entry = __builtin_amdgcn_s_memtime();
#else
    const unsigned long long t_entry = 0;
#endif
    const uint32_t tid = threadIdx.x, b = blockIdx.x;
    const uint32_t x = b & 7u, per = d.n_items >> 3, rem = d.n_items & 7u;
    const uint32_t item = x * per + min(x, rem) + (b >> 3);
    const Win v = win_of(d, item);
    uint8_t *const buf = (uint8_t *)arena;
    win_issue<WPT>(d, v, buf);
    const WinLds wl = win_lds(d, v, buf);
    if (tid < RUN_PAD) wl.runl[v.nslot + tid] = make_uint2(0u, 0u);   // (the DMA does not write there)
    // with the DMA: the thread's piece records and its word's run-slot range
    constexpr int G = WGD / (NWP / WPT);
    uint3 Pc[PFN];   // (compact records: s2c.h S2C_DPC_WORDS)
#pragma unroll
    for (int i = 0; i < PFN; i++) {
        const uint32_t k = tid + WT * i;
        Pc[i] = make_uint3(0u, 0u, 0u);
        if (k < v.npc) Pc[i] = dpc_load(d, v.dpc0 + k);
    }
    const uint32_t w = (tid >> 6) * (NWP / WPT) + (tid & 63) / G, W = v.W0 + w, K = d.kwin;
    uint32_t cw0 = 0, cw1 = 0;
    if (w < v.nwords) {   // (window-relative after the wait below: no early wait on the DMA)
        cw0 = d.rs[(W >= K ? W - K : 0u) - d.word_lo];   // (rs holds entries word_lo ..: s2c_dev)
        cw1 = d.rs[W + 1 - d.word_lo];
    }
    // the ambiguity table and the fill char by scalar loads (a vector load's wait here would
    // also wait for the window DMA issued before it)
    {
        v16i r;
        asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(uni_ptr((const uint32_t *)c_amb)) : "memory");
        if (tid == 0) {
#pragma unroll
            for (int i = 0; i < 16; i++) ((uint32_t *)amb)[i] = (uint32_t)r[i];
        }
    }
    const uintptr_t fa = (uintptr_t)d.fill;
    const uint32_t fill0 = (sload1((const uint32_t *)(fa & ~(uintptr_t)3)) >> (8 * (uint32_t)(fa & 3))) & 0xFFu;
    for (uint32_t k = tid; k < 8 * NWP; k += WT) {
        dcnt[k] = 0;
        ncnt[k] = 0;
        ccnt[k] = 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the window landed
    cw0 -= v.o0;
    cw1 -= v.o0;
    lds_sync();
    dense_tile<NWP>(d, v, wl, dcnt, ncnt, ccnt, amb, fill0, Pc, cw0, cw1, t_entry, stl, threadIdx.x, buf);
}


template <int NWP>
int launch(const DenseArgs &a, int64_t n, hipStream_t s) {
    k_tile_dense<NWP><<<(unsigned)n, WT, a.buf_bytes, s>>>(a);
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
    if (dv->n_dense >= ((int64_t)1 << 31)) return s2c_set_error(S2C_ERR_LIMIT, "too many dense tiles");
    DenseArgs a;
    if (!dv->dpc || !dv->dwin) return s2c_set_error(S2C_ERR_ARG, "dense tiles need dwin and dpc (ABI 12)");
    a.rs = dv->rs; a.lp = dv->lp; a.pc = dv->pc; a.dwin = dv->dwin; a.dpc = dv->dpc; a.ops = dv->ops; a.bq = dv->bq; a.bx = dv->bx; a.tiles = dv->tiles; a.items = dv->dense;
    a.thresholds = dv->thresholds; a.tile_stats = dv->tile_stats; a.blk_len = dv->blk_len; a.out = dv->out;
    a.padded_len = (uint32_t)dv->padded_len; a.n_cols = (uint32_t)dv->n_cols; a.n_tiles = (uint32_t)dv->n_tiles;
    a.kwin = (uint32_t)dv->kwin; a.fill_nondash = (uint32_t)dv->fill_nondash;
    a.maxdel_active = dv->maxdel_active ? 1u : 0u;
    a.maxdel = dv->maxdel < 0 ? 0u : (uint32_t)dv->maxdel;
    a.n_items = (uint32_t)dv->n_dense;
    a.word_lo = (uint32_t)dv->word_lo;
    a.ops_end = dv->ops + dv->n_ops;
    a.bq_end = dv->bq + 2 * dv->n_qwords;
    a.n_thr = dv->n_thr; a.min_depth = dv->min_depth;
    a.fill = dv->fill;
    const int64_t n = dv->n_dense;
    // LDS: the largest window of the batch (S2C_DENSE_BYTES, host plan)
    const int64_t lds = dv->dense_lds;
    if (lds <= 0 || lds > S2C_DENSE_LDS || (lds & 15)) return s2c_set_error(S2C_ERR_ARG, "dense_lds outside (0, S2C_DENSE_LDS] or not 16-byte aligned");
    // (the window's LDS doubles as the counters' exchange after the count: at least WPT waves' share)
    // (WPT > 2: the waves' queues may take up to 64·WPT entries past S2C_DENSE_BYTES' share)
    static_assert(WPT * XCH_WAVE_BYTES == S2C_DENSE_MIN_LDS, "s2c.h S2C_DENSE_MIN_LDS (the host's occupancy plan)");
    a.buf_bytes = (uint32_t)std::max<int64_t>(lds + (WPT > 2 ? 256 * WPT : 0), (int64_t)WPT * XCH_WAVE_BYTES);
    if constexpr (WPT <= 2) {   // (≥ 8 words per wave)
        if (dv->tile_max <= 512) return launch<16>(a, n, st);
    }
    if (dv->tile_max <= 1024) return launch<32>(a, n, st);
    return launch<64>(a, n, st);   // tile_max ≤ 2048 (host plan)
}

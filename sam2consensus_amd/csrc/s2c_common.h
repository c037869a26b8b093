// s2c_common.h — device helpers shared by the HIP kernels of libs2c.so (gfx950).
//
// IUPAC table (:317-329), the closed-form vote (:241-251, :359-366), wave reductions,
// LDS-only barriers, and the bit-sliced Harley–Seal counters of the pileup.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/s2c.h"

int s2c_set_error(int code, const std::string &msg);

namespace s2c {

constexpr int WG = 256;
constexpr uint32_t NSYM = S2C_NSYM;
constexpr int VT_TMAX = 4;        // thresholds per epilogue pass (one vote-char word per column)
constexpr int FILL_LDS = 64;      // -f bytes staged in LDS (longer fills read HBM)
constexpr uint32_t FLUSH_RECS = 248;   // records per lane between counter flushes (8-bit counters)

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

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// Scalar loads of uniform read-only words (tile records, layer bounds): s_load through the
// scalar cache, waited here on lgkmcnt — a vector load's wait (vmcnt) would also wait for
// the kernels' own LDS-DMA loads in flight, which the compiler does not see.
__device__ __forceinline__ const uint32_t *uni_ptr(const uint32_t *p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    return (const uint32_t *)(uintptr_t)((uint64_t)uni((uint32_t)v) | ((uint64_t)uni((uint32_t)(v >> 32)) << 32));
}
__device__ __forceinline__ uint32_t sload1(const uint32_t *p) {
    uint32_t r;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(uni_ptr(p)) : "memory");
    return r;
}
__device__ __forceinline__ uint4 sload4(const uint32_t *p) {
    typedef int v4s __attribute__((ext_vector_type(4)));
    v4s r;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(uni_ptr(p)) : "memory");
    return make_uint4((uint32_t)r.x, (uint32_t)r.y, (uint32_t)r.z, (uint32_t)r.w);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for
// its global stores (__syncthreads also drains vmcnt, i.e. waits for every outstanding
// store of the wave).  Global data shared inside a workgroup waits explicitly first.
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// s_waitcnt vmcnt(0) as a real S_WAITCNT (the compiler's wait tracking sees it)
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Diagnostic build S2C_LDS_POISON (`make poison`): at entry every kernel fills all of its
// workgroup's LDS with 0xA5 bytes (then an LDS barrier), so a read of LDS that this workgroup
// did not write sees the same garbage every time instead of whatever an earlier workgroup
// left on that CU — round 5's k_tile keyed stale LDS event slots that way.
#ifdef S2C_LDS_POISON
template <typename T>
__device__ __forceinline__ void lds_poison(T *p, uint32_t bytes) {
    uint32_t *q = (uint32_t *)p;
    for (uint32_t i = threadIdx.x; i < bytes / 4; i += blockDim.x) q[i] = 0xA5A5A5A5u;
}
#define S2C_POISON(p, bytes) lds_poison(p, (uint32_t)(bytes))
#define S2C_POISON_DONE() lds_sync()
#else
#define S2C_POISON(p, bytes) ((void)0)
#define S2C_POISON_DONE() ((void)0)
#endif


// ----------------------------------------------------------------- parsecigar on the device
__device__ __forceinline__ bool op_bases(uint32_t op) { return op == S2C_OP_M || op == S2C_OP_EQ || op == S2C_OP_X; }
__device__ __forceinline__ bool op_dash(uint32_t op) { return op == S2C_OP_D || op == S2C_OP_N || op == S2C_OP_P; }

// The token walk of the reference's parsecigar (:64-81) over one piece (start = query
// index, k = seqout index):
//   M / = / X   take = min(l, len(SEQ) - start) bases (SEQ truncation, :67), k += take
//   D / N / P   l '-' (:70-72), k += l
//   I           event (start_ref, SEQ[start:start+l]) if the slice is non-empty (:73-75)
//   S           start += l (:76-77);  H nothing (:78-79)
// with the maxdel rule (:210): the '-' of a read whose seqout holds more than maxdel of them
// (D/N/P lengths + '-' chars of the bases taken) are not counted.  run(j, gpos, len, kind, q)
// is called for every op word j of the piece (kind S2C_RUN_EMPTY for prefix words, I / S / H
// and parts outside the piece's seqout range); ev(gkey, q, len) for every insertion event of
// an S2C_PF_INS piece keyed at a position ≥ 0 of its reference.  Mem gives op words and base
// plane words (global index): op(j), p0(w), p1(w), x(w).
template <class Mem, class RunFn, class EvFn>
__device__ __forceinline__ void walk_piece(const Mem &m, const uint4 P, uint32_t oend, bool maxdel_active, uint32_t maxdel,
                                           RunFn &&run, EvFn &&ev) {
    const uint32_t slen = P.w & 0xFFFFFFu, fl = P.w >> 24;
    const uint64_t q0 = (uint64_t)P.y * 16;
    uint32_t o = P.z;
    int64_t ka = 0, kb = INT64_MAX;
    if (fl & S2C_PF_RANGE) {
        ka = m.op(o);
        kb = m.op(o + 1);
        run(o, 0u, 0u, S2C_RUN_EMPTY, 0ull);
        run(o + 1, 0u, 0u, S2C_RUN_EMPTY, 0ull);
        o += 2;
    }
    int64_t key0 = 0;
    uint32_t roff = 0;
    const bool ins = (fl & S2C_PF_INS) != 0;
    if (ins) {
        key0 = (int64_t)((uint64_t)m.op(o) | ((uint64_t)m.op(o + 1) << 32));
        roff = m.op(o + 2);
        for (uint32_t j = 0; j < 3; j++) run(o + j, 0u, 0u, S2C_RUN_EMPTY, 0ull);
        o += 3;
    }
    bool drop = false;
    if (maxdel_active) {   // :210
        uint64_t dashes = 0, start = 0;
        for (uint32_t j = o; j < oend; j++) {
            const uint32_t w = m.op(j), op = w & 15u;
            const uint64_t l = w >> 4;
            if (op_bases(op)) {
                uint64_t take = start < slen ? (l < slen - start ? l : slen - start) : 0;
                if (fl & S2C_PF_DASH) {   // '-' chars of SEQ: x = 1, p1 = 0, p0 = 1
                    uint64_t q = q0 + start;
                    while (take) {
                        const uint64_t qw = q >> 5;
                        const uint32_t sh = (uint32_t)(q & 31), n = (uint32_t)(take < 32 - sh ? take : 32 - sh);
                        const uint32_t mask = (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u)) << sh;
                        dashes += (uint32_t)__popc(m.x(qw) & m.p0(qw) & ~m.p1(qw) & mask);
                        q += n;
                        take -= n;
                    }
                }
                start += l;
            } else if (op_dash(op)) {
                dashes += l;
            } else if (op == S2C_OP_I || op == S2C_OP_S) {
                start += l;
            }
        }
        drop = dashes > (uint64_t)maxdel;
    }
    const uint32_t lng = (fl & S2C_PF_LONG) ? S2C_RUN_LONG : 0u;
    const uint32_t bkind = S2C_RUN_BASES | ((fl & S2C_PF_X) ? S2C_RUN_XBIT : 0u) | (drop ? S2C_RUN_DROP : 0u) | lng;
    int64_t k = 0;
    uint64_t start = 0;
    for (uint32_t j = o; j < oend; j++) {
        const uint32_t w = m.op(j), op = w & 15u;
        const uint64_t l = w >> 4;
        uint32_t rg = 0, rl = 0, rk = S2C_RUN_EMPTY;
        uint64_t rq = 0;
        if (op_bases(op) || op_dash(op)) {
            const bool bases = op_bases(op);
            const uint64_t take = bases ? (start < slen ? (l < slen - start ? l : slen - start) : 0) : l;
            const int64_t s = k > ka ? k : ka, e = (k + (int64_t)take) < kb ? k + (int64_t)take : kb;
            if (e > s && (bases || !drop)) {
                rg = P.x + (uint32_t)(s - ka);
                rl = (uint32_t)(e - s);
                rk = bases ? bkind : (S2C_RUN_DASH | lng);
                rq = bases ? q0 + start + (uint64_t)(s - k) : 0ull;
            }
            k += (int64_t)take;
            if (bases) start += l;
        } else if (op == S2C_OP_I) {
            const uint64_t take = start < slen ? (l < slen - start ? l : slen - start) : 0;
            if (ins && take) {
                const int64_t gkey = key0 + k;   // start_ref (:74) = POS-1 + seqout index here
                if (gkey >= (int64_t)roff) ev((uint64_t)gkey, q0 + start, (uint32_t)take);
            }
            start += l;
        } else if (op == S2C_OP_S) {
            start += l;
        }
        run(j, rg, rl, rk, rq);
    }
}

}  // namespace s2c

extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_add_u64(unsigned long long);
extern "C" __device__ __attribute__((const)) unsigned int __ockl_wfred_add_u32(unsigned int);
extern "C" __device__ unsigned int __ockl_wfscan_add_u32(unsigned int, bool);   // (x, inclusive)
extern "C" __device__ unsigned int __ockl_wfred_max_u32(unsigned int);

namespace s2c {

// Sum over the wave's active lanes, every lane gets it (the device library's DPP reduction).
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    if constexpr (sizeof(T) == 8) return (T)__ockl_wfred_add_u64((unsigned long long)v);
    else return (T)__ockl_wfred_add_u32((unsigned int)v);
}

// Closed form of the group-sort vote (proven equal to :241-251 +
// :359-366 in tests/test_oracle.py): symbol i is taken iff c_i != 0 and the sum of the
// counts strictly greater than c_i is < t·cov (fp64 product, exact integer compare).
template <typename T, typename S>
__device__ __forceinline__ void greater_sums(const T (&c)[NSYM], S (&s)[NSYM]) {
#pragma unroll
    for (int i = 0; i < (int)NSYM; i++) {
        S a = 0;
#pragma unroll
        for (int j = 0; j < (int)NSYM; j++) a += (c[j] > c[i]) ? (S)c[j] : (S)0;
        s[i] = a;
    }
}
template <typename T, typename S>
__device__ __forceinline__ uint32_t vote_mask(const T (&c)[NSYM], const S (&s)[NSYM], double tc) {
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < (int)NSYM; i++) m |= ((c[i] != 0) && ((double)s[i] < tc)) ? (1u << i) : 0u;
    return m;
}
// The same mask for non-negative integer sums with one fp64 product x = t·cov per call:
// for an integer S, S < x ⟺ S ≤ lim with lim = ⌈x⌉ − 1 (x > 0; no S ≥ 0 is < x ≤ 0 or
// NaN), so the six tests are u32 compares.  Exact: x is the reference's own product.
__device__ __forceinline__ uint32_t vote_mask_u32(const uint32_t (&c)[NSYM], const uint32_t (&s)[NSYM], double x) {
    if (!(x > 0.0)) return 0u;
    const uint32_t lim = x > 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)(ceil(x) - 1.0);
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < (int)NSYM; i++) m |= ((c[i] != 0) && (s[i] <= lim)) ? (1u << i) : 0u;
    return m;
}

// char of a one-symbol mask, amb[1 << s] = "-ACGNT"[s]
__device__ __forceinline__ uint32_t sym_char(uint32_t s) { return (uint32_t)(0x544E4743412DULL >> (8 * s)) & 0xFFu; }

// The vote shortcut: the largest count m1 is a strict majority (so unique) and
// m1·2^15 ≥ uq·cov with uq = ⌈tmax·2^15⌉ + 1 (per pass; 0 = off: some threshold outside
// (0, 1]).  Then m1 ≥ tmax·cov + cov/2^15 ≥ tmax·cov·(1 + 2^-53) ≥ fl(tmax·cov) — every
// other symbol's greater-sum is ≥ m1 ≥ t·cov for every t of the pass, and the symbol's own
// is 0 < t·cov.  64-bit products: exact for any count.
__device__ __forceinline__ bool majority_fast(uint32_t m1, uint32_t cov, uint32_t uq) {
    return uq && 2ull * m1 > (uint64_t)cov && ((uint64_t)m1 << 15) >= (uint64_t)uq * cov;
}
__host__ __device__ inline uint32_t pass_uq(const double *th, int tn) {
    double tmax = th[0];
    bool ok = true;
    for (int u = 0; u < tn; u++) {
        ok = ok && th[u] > 0.0 && th[u] <= 1.0;
        tmax = th[u] > tmax ? th[u] : tmax;
    }
    return ok ? (uint32_t)ceil(tmax * 32768.0) + 1u : 0u;
}

// ----------------------------------------------------------------- bit-sliced counters
// A counter is 8 bit-planes of 32 positions (bit b of plane i = bit i of the count at
// position b).  Harley–Seal carry-save adds: 16 masks per close, 2 v_bitop3 per CSA.
__device__ __forceinline__ void csa(uint32_t &h, uint32_t &l, uint32_t a, uint32_t b, uint32_t c) {
    uint32_t lo, hi;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(lo) : "v"(a), "v"(b), "v"(c));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(hi) : "v"(a), "v"(b), "v"(c));
    l = lo;
    h = hi;
}
// 8 masks into planes C[0..2]; returns the carry of weight 8
__device__ __forceinline__ uint32_t tree8(uint32_t (&C)[8], const uint32_t (&m)[8]) {
    uint32_t t2a, t2b, t4a, t4b, t8;
    csa(t2a, C[0], C[0], m[0], m[1]);
    csa(t2b, C[0], C[0], m[2], m[3]);
    csa(t4a, C[1], C[1], t2a, t2b);
    csa(t2a, C[0], C[0], m[4], m[5]);
    csa(t2b, C[0], C[0], m[6], m[7]);
    csa(t4b, C[1], C[1], t2a, t2b);
    csa(t8, C[2], C[2], t4a, t4b);
    return t8;
}
// two weight-8 carries into plane C[3], the weight-16 carry rippled into C[4..7]
__device__ __forceinline__ void close16(uint32_t (&C)[8], uint32_t t8a, uint32_t t8b) {
    uint32_t t16;
    csa(t16, C[3], C[3], t8a, t8b);
#pragma unroll
    for (int b = 4; b < 8; b++) {
        const uint32_t t = C[b] & t16;
        C[b] ^= t16;
        t16 = t;
    }
}
// one weight-4 carry into plane C[2], rippled into C[3..7]
__device__ __forceinline__ void close4(uint32_t (&C)[8], uint32_t t4) {
#pragma unroll
    for (int b = 2; b < 8; b++) {
        const uint32_t t = C[b] & t4;
        C[b] ^= t4;
        t4 = t;
    }
}
// one weight-8 carry into plane C[3], rippled into C[4..7]
__device__ __forceinline__ void close8(uint32_t (&C)[8], uint32_t t8) {
#pragma unroll
    for (int b = 3; b < 8; b++) {
        const uint32_t t = C[b] & t8;
        C[b] ^= t8;
        t8 = t;
    }
}
// one mask of weight 1 rippled into all planes (rare masks: '-')
__device__ __forceinline__ void ripple1(uint32_t (&C)[8], uint32_t m) {
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const uint32_t t = C[b] & m;
        C[b] ^= m;
        m = t;
    }
}

// minus one at the positions of mask m (each counted before: no borrow out of plane 7)
__device__ __forceinline__ void ripple_dec(uint32_t (&C)[8], uint32_t m) {
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const uint32_t t = ~C[b] & m;
        C[b] ^= m;
        m = t;
    }
}

// One butterfly of the transpose: the bits of a under m << s and of b under m trade places
// (two shifts and two bit-field inserts, v_bfi_b32).
template <int S, uint32_t M>
__device__ __forceinline__ void tswap(uint32_t &a, uint32_t &b) {
    const uint32_t na = ((b << S) & (M << S)) | (a & ~(M << S));
    b = ((a >> S) & M) | (b & ~M);
    a = na;
}
// 8 bit-planes of one counter → R[r] byte j = count of position 8j + r (8×8 bit transposes
// on 4 byte lanes at once).
__device__ __forceinline__ void transpose8(uint32_t (&R)[8]) {
#pragma unroll
    for (int r = 0; r < 4; r++) tswap<4, 0x0F0F0F0Fu>(R[r], R[r + 4]);
#pragma unroll
    for (int r = 0; r < 8; r++) {
        if (r & 2) continue;
        tswap<2, 0x33333333u>(R[r], R[r + 2]);
    }
#pragma unroll
    for (int r = 0; r < 8; r += 2) tswap<1, 0x55555555u>(R[r], R[r + 1]);
}
// v_bfi_b32: (m & x) | (~m & y), the mask in an SGPR
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(x), "v"(y));
    return r;
}
// tswap with explicit bit-field inserts (two per butterfly), a / b known zero when AZ / BZ
template <int S, uint32_t M, bool AZ, bool BZ>
__device__ __forceinline__ void tswapz(uint32_t &a, uint32_t &b) {
    if constexpr (AZ && BZ) {
        a = 0u;
        b = 0u;
    } else if constexpr (BZ) {
        b = (a >> S) & M;
        a &= ~(M << S);
    } else if constexpr (AZ) {
        a = (b << S) & (M << S);
        b &= ~M;
    } else {
        const uint32_t na = bfi(M << S, b << S, a);
        b = bfi(M, a >> S, b);
        a = na;
    }
}
// transpose8 of planes whose planes NZ .. 7 are zero
template <int NZ>
__device__ __forceinline__ void transpose8z(uint32_t (&R)[8]) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
        if (r >= NZ) R[r] = R[r + 4] = 0u;
        else if (r + 4 >= NZ) tswapz<4, 0x0F0F0F0Fu, false, true>(R[r], R[r + 4]);
        else tswapz<4, 0x0F0F0F0Fu, false, false>(R[r], R[r + 4]);
    }
#pragma unroll
    for (int r = 0; r < 8; r++) {
        if (r & 2) continue;
        tswapz<2, 0x33333333u, false, false>(R[r], R[r + 2]);
    }
#pragma unroll
    for (int r = 0; r < 8; r += 2) tswapz<1, 0x55555555u, false, false>(R[r], R[r + 1]);
}

// ----------------------------------------------------------------- runs (k_reads output)
struct Run {
    uint32_t gpos, len, kind;
    uint64_t q;
};
__device__ __forceinline__ Run run_of(uint4 v) {
    Run r;
    r.gpos = v.x;
    r.len = v.y & ((1u << S2C_RUN_KSHIFT) - 1u);
    r.kind = v.y >> S2C_RUN_KSHIFT;
    r.q = (uint64_t)v.z | ((uint64_t)v.w << 32);
    return r;
}

// The 32-position record of run r at global word W: valid = positions of W the run covers
// (0 if none); the base planes' bits are taken from query base q + (first covered − gpos).
struct RecGeom {
    uint32_t valid, lo;   // covered bits, first covered bit
    uint32_t qs;          // offset into the run of position 32W + lo
};
// 32-bit arithmetic: positions < 2^32, a run's length < 2^27 and the runs a word looks at
// start within 2^31 positions of it
__device__ __forceinline__ RecGeom rec_geom(uint32_t gpos, uint32_t len, uint32_t W) {
    RecGeom g;
    const int32_t s = (int32_t)(gpos - 32u * W), e = s + (int32_t)len;   // run in word-relative coordinates
    const int32_t lo = max(s, 0), hi = min(e, 32), n = hi - lo;
    const uint32_t m = n >= 32 ? 0xFFFFFFFFu : ((1u << (n & 31)) - 1u);
    g.valid = n > 0 ? m << (lo & 31) : 0u;
    g.lo = n > 0 ? (uint32_t)lo : 0u;
    g.qs = n > 0 ? (uint32_t)(lo - s) : 0u;
    return g;
}
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbit(hi, lo, sh);
}

// A run record in LDS (k_tile_dense's window, k_tile's chunks; one per op slot, zero for
// none): x = rs | re << 16, the run's positions [rs, re) relative to its tile's first word,
// biased by REC_BIAS (a window starts ≤ 32·kwin ≤ 1024 positions before its tile and a short
// run ends < 2048 positions after its start, so both fit 16 bits), y = q − rs with q the LDS
// query base (planes) of its first position.  The count takes both ends with one packed
// subtract and the plane word of a 32-position word from y + its biased first position; a
// zero record covers nothing (re = rs).
constexpr int32_t REC_BIAS = 2048;
__device__ __forceinline__ uint2 rec_enc(uint32_t r0, uint32_t len, uint32_t q) {   // r0: tile-relative start
    const uint32_t rs = r0 + (uint32_t)REC_BIAS;
    return make_uint2(rs | ((rs + len) << 16), q - rs);
}
struct Rec {
    uint32_t q, l;   // first query base (window-relative), length
    int32_t r0;      // tile-relative first position
};
__device__ __forceinline__ Rec rec_dec(uint2 v) {
    const uint32_t rs = v.x & 0xFFFFu;
    return Rec{v.y + rs, (v.x >> 16) - rs, (int32_t)rs - REC_BIAS};
}

typedef short v2s __attribute__((ext_vector_type(2)));
typedef unsigned short v2u __attribute__((ext_vector_type(2)));
// The 32-position word at biased tile-relative position wpk (both halves) of record x: the
// covered bits' mask (nb bits from l0) and fx = all ones iff all 32 are covered (v_bfm_b32
// takes widths below 32), from both ends clamped to [0, 32] at once (packed 16-bit: the
// biased ends and wpk are non-negative, so one saturating unsigned subtract clamps at 0).
__device__ __forceinline__ void rec_mask(uint32_t x, v2s wpk, uint32_t &m, uint32_t &fx) {
    const v2u t = __builtin_elementwise_min(
        __builtin_elementwise_sub_sat(__builtin_bit_cast(v2u, x), __builtin_bit_cast(v2u, wpk)), (v2u){32, 32});
    const uint32_t tc = __builtin_bit_cast(uint32_t, t);
    uint32_t nb;   // e - l0 (one SDWA subtract of the halves)
    asm("v_sub_u32_sdwa %0, %1, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0"
        : "=v"(nb) : "v"(tc));
    // nb bits at l0 (v_bfm_b32 reads the offset's low 5 bits: l0 of tc; l0 = 32 only with nb = 0)
    asm("v_bfm_b32 %0, %1, %2" : "=v"(m) : "v"(nb), "v"(tc));
    fx = (uint32_t)__builtin_amdgcn_sbfe((int32_t)nb, 5, 1);
}


}  // namespace s2c

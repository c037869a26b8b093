// s2c_kernels.hip — HIP kernels for gfx950 (MI355X) + their C-ABI launchers.
//
// The reference's hot path (sam2consensus.py) is a per-base Python dict increment
// (:210-218), an insertion motif aggregation (:256-311) and a per-position threshold
// vote (:232-253, :344-389).  Here it is a stream-ordered chain over the packed batch
// built by s2c_host.cpp, whose unit is the TILE (≤2048 positions of one reference):
//
//   k_prep                 zero per-run state (replaces memsets: one launch)
//   k_ins_count            (3) insertion column symbol counts per key (:262-287)
//   k_pileup               (2) bit-sliced counting of the word-major seqout records per
//                          tile (32 positions per VALU op), and (4) for tiles voted in one
//                          work item the vote epilogue: all thresholds, IUPAC, min-depth/
//                          fill, per-(ref,t) stats — counts never reach HBM
//   k_consensus            (4) the same vote for "deep" tiles whose records were split
//                          over several work items (counts summed in HBM)
//   k_ins_vote             (4) insertion columns of called keys (:290-311, :370-385)
//   k_scan / k_assemble    device FASTA body assembly (tile scan + byte scatter)
//
// Everything is integer counting; the single floating-point operation is the
// reference's `cov_nucs < t*coverage` (:362, :376), evaluated as
// (double)S < t * (double)cov — built with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
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

template <typename T>
__device__ __forceinline__ T block_sum(T v, T *sh) {   // 256-thread workgroup sum, all threads get it
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const uint32_t w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    T r = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) r += sh[i];
    return r;
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

// index of the insertion key at position p (p must carry a key): keys before p's word + the
// key bits below p in it
__device__ __forceinline__ uint32_t key_index(const s2c_dev &d, uint32_t p, uint32_t bits) {
    return d.ins_rank[p >> 5] + (uint32_t)__popc(bits & ((1u << (p & 31)) - 1u));
}

// ======================================================================= per-run state
// One launch zeroes everything a run accumulates into: per-(ref,t) stats, flags, the
// insertion bitmap / hash table / column counts, and the count ranges of deep tiles.
constexpr int PREP_BLOCKS = 512;
__global__ __launch_bounds__(WG) void k_prep(const s2c_dev d) {
    if (blockIdx.x < PREP_BLOCKS) {
        const size_t i0 = (size_t)blockIdx.x * WG + threadIdx.x, step = (size_t)PREP_BLOCKS * WG;
        const size_t n_stats = (size_t)d.n_refs * d.n_thr * 4, n_cols = (size_t)d.n_cols * NSYM;
        for (size_t i = i0; i < n_stats; i += step) d.stats[i] = 0;
        for (size_t i = i0; i < 16; i += step) d.scalars[i] = 0;
        for (size_t i = i0; i < n_cols; i += step) d.ins_cols[i] = 0;
        return;
    }
    const uint32_t t = d.deep[blockIdx.x - PREP_BLOCKS];
    const uint32_t a = d.blocks[(size_t)t * S2C_BLOCK_WORDS], n = d.blocks[(size_t)t * S2C_BLOCK_WORDS + 1] - a;
    for (uint32_t c = 0; c < NSYM; c++)
        for (uint32_t i = threadIdx.x; i < n; i += WG) d.counts[(size_t)c * d.padded_len + a + i] = 0;
}

// ======================================================================= (3) insertions
// (:264-271) motif multiplicities and (:284-287) per-column sums are additive: column c of
// key k counts motif[c] over the key's events with len > c.  The host groups events by
// key (sorted) and cuts them into units of ≤ S2C_INS_UNIT events; one thread per unit
// counts every column of its key (columns outer, its events inner) and stores the six
// counts, or adds them when the key is split over several units.  The columns are voted
// (with '-' = cov[key] − Σ column, :294) by k_ins_vote.
__global__ __launch_bounds__(WG) void k_ins_count(const s2c_dev d) {
    const uint32_t u = blockIdx.x * WG + threadIdx.x;
    if (u >= (uint32_t)d.n_units) return;
    const uint32_t k = d.ins_units[2 * u], e0 = d.ins_units[2 * u + 1];
    const uint32_t ke0 = d.ins_koff[k], ke1 = d.ins_koff[k + 1];
    const uint32_t e1 = min(ke1, e0 + (uint32_t)S2C_INS_UNIT);
    const bool whole = e0 == ke0 && e1 == ke1;
    const uint32_t cb = d.ins_kcol[k], ml = d.ins_kcol[k + 1] - cb;
    for (uint32_t c = 0; c < ml; c++) {
        uint32_t cnt[NSYM] = {0, 0, 0, 0, 0, 0};
        for (uint32_t e = e0; e < e1; e++) {
            const uint32_t o0 = d.ins_off[e];
            if (c < d.ins_off[e + 1] - o0) cnt[nibble(d.ins_bases, (uint64_t)o0 + c)]++;
        }
        uint32_t *col = d.ins_cols + (size_t)(cb + c) * NSYM;
#pragma unroll
        for (uint32_t j = 0; j < NSYM; j++) {
            if (whole) col[j] = cnt[j];
            else if (cnt[j]) atomicAdd(&col[j], cnt[j]);
        }
    }
}

// ======================================================================= (4) vote epilogue
// Per position: the closed-form vote for every threshold and the IUPAC char (or fill when
// cov == 0 or cov < min_depth, :356-389).  Per tile: len and sumcov do not depend on the
// threshold (1 per called position or len(fill); cov, :357/:385), the per-threshold
// non-'-' and vote-error counts are wave ballots.  At a position carrying an insertion key
// the key's coverage (0 when not called) is stored for k_ins_vote, which votes the
// insertion columns (:290-311, :370-385) and adds their chars to the same stats.
constexpr int VT_TMAX = 16;   // thresholds per pass over the tile's positions
constexpr int VT_ACC = 2 + 2 * VT_TMAX;   // LDS u64: sumcov, len, {nondash, nerr}[VT_TMAX]

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// acc: LDS [VT_ACC] u64; amb: LDS copy of c_amb.
template <class Fetch>
__device__ __forceinline__ void vote_tile(const s2c_dev &d, uint32_t tile, uint32_t ref, uint32_t a, uint32_t n,
                                          Fetch fetch, unsigned long long *acc, const uint8_t *amb) {
    const int T = d.n_thr;
    const uint32_t lane = threadIdx.x & 63;
    for (int t0 = 0; t0 < T; t0 += VT_TMAX) {
        const int t1 = min(T, t0 + VT_TMAX);
        if (threadIdx.x < (uint32_t)VT_ACC && (t0 == 0 || threadIdx.x >= 2)) acc[threadIdx.x] = 0;
        __syncthreads();
        uint64_t sumcov = 0, len = 0;
        for (uint32_t q0 = 0; q0 < n; q0 += WG) {   // uniform trip count: every lane votes in the ballots
            const uint32_t q = q0 + threadIdx.x, p = a + q;
            const bool in = q < n;
            uint32_t cnt[NSYM];
            uint64_t cov = 0;
#pragma unroll
            for (uint32_t c = 0; c < NSYM; c++) { cnt[c] = in ? fetch(q, c) : 0u; cov += cnt[c]; }
            const bool called = in && cov > 0 && (int64_t)cov >= (int64_t)d.min_depth;   // :359
            if (t0 == 0) {
                sumcov += cov;
                len += called ? 1u : (in ? (uint32_t)d.fill_len : 0u);
                const uint32_t bits = in ? d.ins_bits[p >> 5] : 0u;
                if (bits >> (p & 31) & 1u) d.key_cov[key_index(d, p, bits)] = called ? (uint32_t)cov : 0u;
            }
            int64_t gs[NSYM];
            greater_sums(cnt, gs);
            const uint32_t n_unc = (uint32_t)__popcll(__ballot(in && !called));
            for (int t = t0; t < t1; t++) {
                const double tc = d.thresholds[t] * (double)cov;
                const uint8_t code = called ? amb[vote_mask(cnt, gs, tc)] : (uint8_t)S2C_CODE_FILL;
                if (in) d.codes[(size_t)t * d.padded_len + p] = code;
                const uint32_t nd = (uint32_t)__popcll(__ballot(called && code != '-'));
                const uint32_t ne = (uint32_t)__popcll(__ballot(called && code == 0xFF));
                if (lane == 0) {
                    atomicAdd(&acc[2 + 2 * (t - t0)], (unsigned long long)(nd + (uint64_t)d.fill_nondash * n_unc));
                    if (ne) atomicAdd(&acc[3 + 2 * (t - t0)], (unsigned long long)ne);
                }
            }
        }
        if (t0 == 0) {
            sumcov = wave_sum(sumcov);
            len = wave_sum(len);
            if (lane == 0) {
                atomicAdd(&acc[0], (unsigned long long)sumcov);
                atomicAdd(&acc[1], (unsigned long long)len);
            }
        }
        __syncthreads();
        if (threadIdx.x < 4 * (uint32_t)(t1 - t0)) {   // tile totals → stats[ref][t], blk_len
            const uint32_t t = t0 + threadIdx.x / 4, k = threadIdx.x % 4;
            const unsigned long long v = k < 2 ? acc[k] : acc[2 + 2 * (t - t0) + (k - 2)];
            uint64_t *st = d.stats + ((size_t)ref * T + t) * 4;
            if (v) atomicAdd((unsigned long long *)&st[k], v);
            if (k == 3 && v) atomicOr(&d.scalars[1], 1u);
            if (k == 1) d.blk_len[(size_t)t * d.n_blocks + tile] = v;
        }
        __syncthreads();
    }
}

// Insertion columns of the called keys of one tile (grid = tiles; the tile's keys are the
// contiguous range [rank(a), rank(b)); dynamic LDS [T][4] u64): per column and threshold
// the same vote with '-' = cov[key] − Σ column (:294, signed); '-' results are skipped,
// others emitted after the key's base (:370-385) and added to the tile's len / non-'-' /
// sumcov (cov per emitted char, :385) and block length.
__global__ __launch_bounds__(WG) void k_ins_vote(const s2c_dev d) {
    extern __shared__ unsigned long long iacc[];   // [T][4]
    __shared__ uint32_t em[VT_TMAX][WG];           // emitted chars per (threshold, thread)
    __shared__ uint8_t amb[64];
    const uint32_t tid = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    const uint32_t *blk = d.blocks + (size_t)tile * S2C_BLOCK_WORDS;
    const uint32_t a = uni(blk[0]), b = uni(blk[1]), ref = uni(blk[2]);
    const uint32_t klo = uni(d.ins_rank[a >> 5]), khi = uni(d.ins_rank[(b + 31) >> 5]);
    if (klo == khi) return;
    const int T = d.n_thr;
    for (uint32_t i = tid; i < 4u * (uint32_t)T; i += WG) iacc[i] = 0;
    if (tid < 64) amb[tid] = c_amb[tid];
    __syncthreads();
    const uint32_t *__restrict__ cols = d.ins_cols;
    uint8_t *__restrict__ chr = d.ins_chr;
    for (uint32_t k = klo + tid; k < khi; k += WG) {
        const uint32_t cov = d.key_cov[k];
        if (cov == 0) continue;   // position not called: no insertion chars (:356-358)
        const uint32_t cb = d.ins_kcol[k], ml = d.ins_kcol[k + 1] - cb;
        for (int t0 = 0; t0 < T; t0 += VT_TMAX) {
            const int t1 = min(T, t0 + VT_TMAX);
            for (int t = t0; t < t1; t++) em[t - t0][tid] = 0;
            for (uint32_t c0 = 0; c0 < ml; c0 += 4) {   // 4 columns' loads in flight
                uint32_t cv[4][NSYM];
#pragma unroll
                for (int u = 0; u < 4; u++)
#pragma unroll
                    for (uint32_t j = 0; j < NSYM; j++)
                        cv[u][j] = c0 + u < ml ? cols[(size_t)(cb + c0 + u) * NSYM + j] : 0u;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (c0 + u >= ml) break;
                    int64_t v[NSYM];
                    int64_t tot = 0;
#pragma unroll
                    for (uint32_t j = 0; j < NSYM; j++) { v[j] = cv[u][j]; tot += v[j]; }
                    v[0] = (int64_t)cov - tot;   // :294 (the column's own '-' count is in the sum)
                    int64_t g2[NSYM];
                    greater_sums(v, g2);
                    for (int t = t0; t < t1; t++) {
                        const uint8_t ic = amb[vote_mask(v, g2, d.thresholds[t] * (double)cov)];
                        if (ic == 0xFF) { atomicAdd(&iacc[4 * t + 3], 1ull); continue; }
                        if (ic != '-') chr[(size_t)t * d.n_cols + cb + em[t - t0][tid]++] = ic;
                    }
                }
            }
            for (int t = t0; t < t1; t++) {
                const uint32_t emitted = em[t - t0][tid];
                d.ins_cnt[(size_t)t * d.n_keys + k] = emitted;
                if (emitted) {
                    atomicAdd(&iacc[4 * t + 0], (unsigned long long)cov * emitted);
                    atomicAdd(&iacc[4 * t + 1], (unsigned long long)emitted);
                    atomicAdd(&iacc[4 * t + 2], (unsigned long long)emitted);
                }
            }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < 4u * (uint32_t)T; i += WG) {
        const unsigned long long v = iacc[i];
        if (!v) continue;
        const uint32_t t = i / 4, k = i % 4;
        atomicAdd((unsigned long long *)&d.stats[((size_t)ref * T + t) * 4 + k], v);
        if (k == 3) atomicOr(&d.scalars[1], 1u);
        if (k == 1) atomicAdd((unsigned long long *)&d.blk_len[(size_t)t * d.n_blocks + tile], v);
    }
}

// ======================================================================= (2) pileup
constexpr int TILE_MAX = S2C_TILE_MAX;   // positions per tile (≤ 64 words of 32)
constexpr uint32_t FLUSH_RECS = 248;     // records per lane between flushes: 31 groups of 8 (≤ 255)

// Bit-sliced counting.  A record holds 3 planes of its 32 positions' codes (p2·4+p1·2+p0:
// 0 '-', 1 A, 2 C, 3 G, 4 N, 5 T, 7 = no entry).  Six masks are counted per record, each
// one VALU op from the planes: O = p1|p2 (C,G,N,T,none), A = p0&~O, Y = p1&~p2 (C,G),
// G = Y&p0, Z = p2&~p1 (N,T), T = Z&p0; at the flush '-' = n − O − A, C = Y − G,
// N = Z − T, n = records the lane counted.  A slot past the chunk's end loads the all-zero
// sentinel record recs[n_recs] (no mask set) and is not counted in n.
// Each counter is 8 bit-planes (bit b of the per-position count): ones, twos, fours, eights
// from a Harley–Seal carry-save tree over 16 records (15 CSAs of 2 v_bitop3 each), bits
// 4..7 a ripple counter of the sixteens.  32 positions per VALU op, ≈20 VALU per record.
constexpr int NCTR = 6;
// carry-save adder a + b + c = 2h + l: two v_bitop3_b32 (truth tables 0x96 = xor3, 0xE8 =
// majority; both symmetric, so operand order is free).  Written as asm because the
// compiler shares a^b between the two and spends three ops.
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
// one group of 8 records → the six counters' weight-8 carries
__device__ __forceinline__ void count8(uint32_t (&V)[NCTR][8], const uint32_t (&P)[8][3], uint32_t (&t8)[NCTR]) {
    uint32_t m[8], y[8];
#pragma unroll
    for (int u = 0; u < 8; u++) m[u] = P[u][1] | P[u][2];
    t8[0] = tree8(V[0], m);   // O
#pragma unroll
    for (int u = 0; u < 8; u++) m[u] = P[u][0] & ~(P[u][1] | P[u][2]);
    t8[1] = tree8(V[1], m);   // A
#pragma unroll
    for (int u = 0; u < 8; u++) y[u] = P[u][1] & ~P[u][2];
    t8[2] = tree8(V[2], y);   // Y = C|G
#pragma unroll
    for (int u = 0; u < 8; u++) m[u] = y[u] & P[u][0];
    t8[3] = tree8(V[3], m);   // G
#pragma unroll
    for (int u = 0; u < 8; u++) y[u] = P[u][2] & ~P[u][1];
    t8[4] = tree8(V[4], y);   // Z = N|T
#pragma unroll
    for (int u = 0; u < 8; u++) m[u] = y[u] & P[u][0];
    t8[5] = tree8(V[5], m);   // T
}

// 8 bit-planes of one counter → R[r] byte j = count of position 8j + r (8×8 bit transposes
// on 4 byte lanes at once).
__device__ __forceinline__ void transpose8(uint32_t (&R)[8]) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t t = ((R[r] >> 4) ^ R[r + 4]) & 0x0F0F0F0Fu;
        R[r + 4] ^= t;
        R[r] ^= t << 4;
    }
#pragma unroll
    for (int r = 0; r < 8; r++) {
        if (r & 2) continue;
        const uint32_t t = ((R[r] >> 2) ^ R[r + 2]) & 0x33333333u;
        R[r + 2] ^= t;
        R[r] ^= t << 2;
    }
#pragma unroll
    for (int r = 0; r < 8; r += 2) {
        const uint32_t t = ((R[r] >> 1) ^ R[r + 1]) & 0x55555555u;
        R[r + 1] ^= t;
        R[r] ^= t << 1;
    }
}

// LDS histogram of a tile: u16 counts in pairs, word s = 16·(word of 32) + i holds
// positions i (low half) and i + 16 (high half) of that word; one pad word per 16.
__device__ __forceinline__ uint32_t hslot(uint32_t s) { return s + (s >> 4); }
__device__ __forceinline__ uint32_t hist_get(const uint32_t *h, uint32_t q) {
    return (h[hslot(((q >> 5) << 4) | (q & 15))] >> ((q & 16) ? 16 : 0)) & 0xFFFFu;
}

// One workgroup per work item = (tile [a,b) of ≤ TW = 32·NWP positions, chunk k).  Lane
// L owns 32-position word w = L mod NWP of the tile and lane group g = L / NWP (G = 256/NWP
// lanes per word).  The word's seqout records [wrec[W], wrec[W+1]) are cut into chunks of
// chunk_recs (= 248·G, one flush per lane); the item streams chunk k, lane g taking records
// ≡ g (mod G), 8 at a time with the next 8 in flight (a group's lanes read consecutive
// records: coalesced), counted by count8.  The flush transposes the counters, derives the
// six symbol counts and adds them, two u16 per LDS atomic, into the tile's histogram.  A
// tile voted in one item (not deep) is voted from LDS (vote_tile); a deep tile's chunks add
// their histograms into HBM for k_consensus.
template <int NWP>
__global__ __launch_bounds__(WG) void k_pileup(const s2c_dev d) {
    constexpr int G = WG / NWP, TW = NWP * 32, HP = TW / 2 + TW / 32;
    constexpr uint32_t FB = FLUSH_RECS * G;   // records per word between flushes
    __shared__ uint32_t hist[NSYM][HP];
    __shared__ unsigned long long acc[VT_ACC];
    __shared__ uint8_t amb[64];
    const uint32_t tid = threadIdx.x;
    const uint32_t w = tid % NWP, g = tid / NWP;
    if (tid < 64) amb[tid] = c_amb[tid];   // published by the barrier after the histogram zeroing
    const uint32_t *__restrict__ recs = d.recs;
    const uint32_t CH = (uint32_t)d.chunk_recs;
    const uint32_t nfb = (CH + FB - 1) / FB;
    const uint32_t item = blockIdx.x;   // grid = work items
    const uint32_t *it = d.items + (size_t)item * S2C_ITEM_WORDS;
    const uint32_t a = uni(it[0]), b = uni(it[1]), chunk = uni(it[2]), tile = uni(it[3]);
    const uint32_t *blk = d.blocks + (size_t)tile * S2C_BLOCK_WORDS;
    const uint32_t ref = uni(blk[2]), deep = uni(blk[3]);
    const uint32_t n = b - a;
    for (uint32_t i = tid; i < NSYM * (uint32_t)HP; i += WG) (&hist[0][0])[i] = 0;
    const uint32_t ws = 32u * w;                  // word start, tile-relative
    const bool active = ws < n;
    uint32_t r0 = 0, r1 = 0;   // this word's records in chunk `chunk`
    if (active) {
        const uint32_t W = (a >> 5) + w;
        const uint32_t wb = d.wrec[W], we = d.wrec[W + 1];
        r0 = (uint32_t)min((uint64_t)we, (uint64_t)wb + (uint64_t)chunk * CH);
        r1 = (uint32_t)min((uint64_t)we, (uint64_t)r0 + CH);
    }
    __syncthreads();
    uint32_t V[NCTR][8];
    auto zeroV = [&]() {
#pragma unroll
        for (int c = 0; c < NCTR; c++)
#pragma unroll
            for (int bb = 0; bb < 8; bb++) V[c][bb] = 0;
    };
    const uint32_t sentinel = (uint32_t)d.n_recs;   // all-zero record
    auto load8 = [&](uint32_t (&P)[8][3], uint32_t t, uint32_t e0) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t i = t + u * G < e0 ? t + u * G : sentinel;
            const uint32_t *src = recs + 3 * (size_t)i;
#pragma unroll
            for (int k = 0; k < 3; k++) P[u][k] = src[k];
        }
    };
    uint32_t sink = 0;   // diagnostic ablate&2: loads consumed without counting
    auto sink8 = [&](const uint32_t (&P)[8][3]) {
#pragma unroll
        for (int u = 0; u < 8; u++) sink ^= P[u][0] ^ P[u][1] ^ P[u][2];
    };
    // valid records of the group starting at t
    auto nvalid = [&](uint32_t t, uint32_t e0) -> uint32_t {
        return t < e0 ? min(8u, (e0 - t + G - 1) / G) : 0u;
    };
    // counters of this lane's 32 positions → six symbol counts → LDS histogram
    auto flush = [&](uint32_t nrec) {
        if (active && !(d.ablate & 8)) {
            uint32_t *h0 = &hist[0][0] + 17 * w;
            auto add = [&](uint32_t sym, const uint32_t (&R)[8]) {
                uint32_t *hw = h0 + sym * HP;
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const uint32_t lo = R[r] & 0x00FF00FFu, hi = (R[r] >> 8) & 0x00FF00FFu;
                    if (lo) atomicAdd(hw + r, lo);
                    if (hi) atomicAdd(hw + 8 + r, hi);
                }
            };
            const uint32_t nb = nrec * 0x01010101u;
#pragma unroll
            for (int pr = 0; pr < 3; pr++) {   // (O,A) → '-',A; (Y,G) → C,G; (Z,T) → N,T
                uint32_t X[8], Y[8];
#pragma unroll
                for (int r = 0; r < 8; r++) { X[r] = V[2 * pr][r]; Y[r] = V[2 * pr + 1][r]; }
                transpose8(X);
                transpose8(Y);
#pragma unroll
                for (int r = 0; r < 8; r++) X[r] = pr == 0 ? nb - X[r] - Y[r] : X[r] - Y[r];   // no byte borrows
                add(pr == 0 ? 0 : (pr == 1 ? 2 : 4), X);
                add(pr == 0 ? 1 : (pr == 1 ? 3 : 5), Y);
            }
        }
        zeroV();
    };
    zeroV();
    for (uint32_t fb = 0; fb < ((d.ablate & 1) ? 0u : nfb); fb++) {   // uniform
        const uint32_t s0 = r0 + fb * FB, e0 = min(r1, s0 + FB);
        uint32_t t = s0 + g, nrec = 0;
        if (t < e0) {
            // two groups of 8 per trip (one 16-record carry-save step), the next group
            // always in flight while one is counted.  sched_barrier keeps each group's loads
            // issued ahead of the other group's count (the scheduler otherwise sinks them
            // next to their use to save registers).
            uint32_t P[8][3], Q[8][3], ta[NCTR], tb[NCTR];
            load8(P, t, e0);
            for (; t < e0; t += 16 * G) {
                load8(Q, t + 8 * G, e0);
                __builtin_amdgcn_sched_barrier(0);
                if (d.ablate & 2) sink8(P); else count8(V, P, ta);
                load8(P, t + 16 * G, e0);
                __builtin_amdgcn_sched_barrier(0);
                if (d.ablate & 2) {
                    sink8(Q);
                    continue;
                }
                count8(V, Q, tb);
#pragma unroll
                for (int c = 0; c < NCTR; c++) close16(V[c], ta[c], tb[c]);
                nrec += nvalid(t, e0) + nvalid(t + 8 * G, e0);
            }
        }
        flush(nrec);
    }
    if (sink == 0x9E3779B9u) hist[0][0] = 1;   // keeps the ablation's loads alive
    __syncthreads();
    if (!deep && !(d.ablate & 4)) {   // the tile's whole depth is here: vote it now
        vote_tile(d, tile, ref, a, n, [&](uint32_t q, uint32_t c) { return hist_get(hist[c], q); }, acc, amb);
    } else {
        // deep tile: this chunk's counts → HBM (symbol-major, coalesced atomics); with the
        // diagnostic flag 4 every tile stores its counts instead of voting (parity tests)
        for (uint32_t q = tid; q < n; q += WG)
#pragma unroll
            for (uint32_t c = 0; c < NSYM; c++) {
                uint32_t *dst = d.counts + (size_t)c * d.padded_len + a + q;
                const uint32_t v = hist_get(hist[c], q);
                if (deep) {
                    if (v) atomicAdd(dst, v);
                } else {
                    *dst = v;
                }
            }
    }
}

// Deep tiles: counts summed in HBM by their work items → the same vote epilogue.
__global__ __launch_bounds__(WG) void k_consensus(const s2c_dev d) {
    __shared__ unsigned long long acc[VT_ACC];
    __shared__ uint8_t amb[64];
    if (threadIdx.x < 64) amb[threadIdx.x] = c_amb[threadIdx.x];   // published by vote_tile's first barrier
    const uint32_t tile = d.deep[blockIdx.x];
    const uint32_t *blk = d.blocks + (size_t)tile * S2C_BLOCK_WORDS;
    const uint32_t a = uni(blk[0]), n = uni(blk[1]) - a, ref = uni(blk[2]);
    const uint32_t *cts = d.counts + a;
    const size_t L = d.padded_len;
    vote_tile(d, tile, ref, a, n, [&](uint32_t q, uint32_t c) { return cts[(size_t)c * L + q]; }, acc, amb);
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
template <int ASM_PER>   // consecutive positions per thread (tile_max / 256)
__global__ __launch_bounds__(WG) void k_assemble(const s2c_dev d) {
    __shared__ uint64_t sh[WG / 64];
    const uint32_t bi = blockIdx.x;
    const int t = (int)blockIdx.y;
    const uint32_t *blk = d.blocks + (size_t)bi * S2C_BLOCK_WORDS;
    const uint32_t g0 = uni(blk[0]), g1 = uni(blk[1]);
    const uint64_t base = d.blk_len[(size_t)t * d.n_blocks + bi];
    const uint8_t *codes = d.codes + (size_t)t * d.padded_len;
    const uint32_t p0 = g0 + ASM_PER * threadIdx.x;
    uint32_t lens[ASM_PER], slots[ASM_PER];
    uint64_t my = 0;
#pragma unroll
    for (int j = 0; j < ASM_PER; j++) {
        const uint32_t p = p0 + j;
        lens[j] = 0;
        slots[j] = 0xFFFFFFFFu;
        if (p < g1) {
            const uint8_t c = codes[p];
            if (c == S2C_CODE_FILL) {
                lens[j] = (uint32_t)d.fill_len;
            } else {
                lens[j] = 1;
                const uint32_t bits = d.ins_bits[p >> 5];
                if (bits >> (p & 31) & 1u) {
                    slots[j] = key_index(d, p, bits);
                    lens[j] += d.ins_cnt[(size_t)t * d.n_keys + slots[j]];
                }
            }
        }
        my += lens[j];
    }
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
    for (int j = 0; j < ASM_PER; j++) {
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
                const uint8_t *src = d.ins_chr + (size_t)t * d.n_cols + d.ins_kcol[slots[j]];
                for (uint32_t i = 0; i < ne; i++) d.out[off++] = src[i];
            }
        }
    }
}

inline int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return S2C_OK;
    return s2c_set_error(S2C_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

inline unsigned grid_for(int64_t n, int wg = WG) { return (unsigned)((n + wg - 1) / wg); }

}  // namespace

// ======================================================================= C-ABI
extern "C" int s2c_workspace_sizes(const s2c_batch_info *info, int32_t n_thr, s2c_ws_sizes *o) {
    if (!info || !o || n_thr <= 0) return s2c_set_error(S2C_ERR_ARG, "bad workspace query");
    const int64_t L = info->padded_len, T = n_thr;
    const int64_t nk = std::max<int64_t>(info->n_keys, 1), nc = std::max<int64_t>(info->n_cols, 1);
    o->counts = info->n_deep ? NSYM * L * 4 : 64;   // only deep tiles keep counts in HBM
    o->key_cov = nk * 4;
    o->ins_cols = nc * NSYM * 4;
    o->ins_cnt = T * nk * 4;
    o->ins_chr = T * nc;
    o->scalars = 64;
    o->codes = T * L;
    o->blk_len = (T * info->n_blocks + 1) * 8;
    o->stats = info->n_refs * T * 32;
    return S2C_OK;
}

static int check_dev(const s2c_dev *d) {
    if (!d) return s2c_set_error(S2C_ERR_ARG, "s2c_dev is NULL");
    if (d->n_thr <= 0) return s2c_set_error(S2C_ERR_ARG, "no thresholds");
    if (d->n_thr > 1024) return s2c_set_error(S2C_ERR_LIMIT, "more than 1024 thresholds");
    if (d->tile_max <= 0 || d->tile_max > TILE_MAX) return s2c_set_error(S2C_ERR_ARG, "tile_max out of range");
    if (d->padded_len <= 0 || d->padded_len >= ((int64_t)1 << 32)) return s2c_set_error(S2C_ERR_ARG, "bad padded_len");
    if (d->n_items > 0 && (!d->items || !d->wrec || (d->n_recs > 0 && !d->recs) || d->chunk_recs <= 0))
        return s2c_set_error(S2C_ERR_ARG, "missing pileup buffers");
    {   // one flush per item: the LDS histogram's u16 halves hold ≤ 248·G per position
        int64_t nwp = 8;
        while (nwp * 32 < d->tile_max) nwp *= 2;
        if (d->chunk_recs > (int64_t)FLUSH_RECS * (WG / nwp))
            return s2c_set_error(S2C_ERR_ARG, "chunk_recs exceeds one flush per work item");
    }
    if (d->n_deep > 0 && (!d->deep || !d->counts)) return s2c_set_error(S2C_ERR_ARG, "missing deep-tile buffers");
    if ((d->ablate & 4) && !d->counts) return s2c_set_error(S2C_ERR_ARG, "ablate&4 stores all counts: counts buffer required");
    if (!d->ins_bits || !d->ins_rank) return s2c_set_error(S2C_ERR_ARG, "missing key bitmap/rank");
    if (d->n_keys > 0 && (!d->ins_koff || !d->ins_kcol || !d->ins_off || !d->ins_bases || !d->ins_units ||
                          !d->key_cov || !d->ins_cols || !d->ins_cnt || !d->ins_chr))
        return s2c_set_error(S2C_ERR_ARG, "missing insertion buffers");
    return S2C_OK;
}

// Persistent grid: as many workgroups as fit at once (occupancy query, cached per kernel),
// never more than the items; each pulls items from the ticket.
template <int NWP>
static int launch_pileup(const s2c_dev *d, hipStream_t s) {
    k_pileup<NWP><<<(unsigned)d->n_items, WG, 0, s>>>(*d);
    return hip_check(hipGetLastError(), "k_pileup");
}

// zero per-run state, then the insertion table (must precede the pileup's vote epilogue)
extern "C" int s2c_insertions(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    k_prep<<<(unsigned)(PREP_BLOCKS + d->n_deep), WG, 0, s>>>(*d);
    if (d->n_units) k_ins_count<<<grid_for(d->n_units), WG, 0, s>>>(*d);
    return hip_check(hipGetLastError(), "k_prep/k_ins_count");
}

extern "C" int s2c_pileup(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    if (d->n_items == 0) return S2C_OK;
    hipStream_t s = (hipStream_t)stream;
    if (d->n_items >= ((int64_t)1 << 31)) return s2c_set_error(S2C_ERR_LIMIT, "more than 2^31 work items");
    if (d->tile_max <= 256) return launch_pileup<8>(d, s);
    if (d->tile_max <= 512) return launch_pileup<16>(d, s);
    if (d->tile_max <= 1024) return launch_pileup<32>(d, s);
    return launch_pileup<64>(d, s);
}

extern "C" int s2c_consensus(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (d->n_deep > 0) {
        k_consensus<<<(unsigned)d->n_deep, WG, 0, s>>>(*d);
        if ((rc = hip_check(hipGetLastError(), "k_consensus"))) return rc;
    }
    if (d->n_keys > 0 && d->n_blocks > 0) {
        k_ins_vote<<<(unsigned)d->n_blocks, WG, (size_t)32 * d->n_thr, s>>>(*d);
        if ((rc = hip_check(hipGetLastError(), "k_ins_vote"))) return rc;
    }
    return S2C_OK;
}

extern "C" int s2c_assemble(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int64_t n = (int64_t)d->n_thr * d->n_blocks;
    k_scan<<<1, 1024, 0, s>>>(d->blk_len, n);
    if (d->n_blocks) {
        const dim3 g((unsigned)d->n_blocks, (unsigned)d->n_thr);
        if (d->tile_max <= 256) k_assemble<1><<<g, WG, 0, s>>>(*d);
        else if (d->tile_max <= 512) k_assemble<2><<<g, WG, 0, s>>>(*d);
        else if (d->tile_max <= 1024) k_assemble<4><<<g, WG, 0, s>>>(*d);
        else k_assemble<8><<<g, WG, 0, s>>>(*d);
    }
    return hip_check(hipGetLastError(), "k_assemble");
}

extern "C" int s2c_run(const s2c_dev *d, void *stream) {
    int rc;
    if ((rc = s2c_insertions(d, stream))) return rc;
    if ((rc = s2c_pileup(d, stream))) return rc;
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

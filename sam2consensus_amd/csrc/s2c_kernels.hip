// s2c_kernels.hip — HIP kernels for gfx950 (MI355X) + their C-ABI launchers.
//
// The reference's hot path (sam2consensus.py) is a per-base Python dict increment
// (:210-218), an insertion motif aggregation (:256-311) and a per-position threshold
// vote (:232-253, :344-389).  Here it is a stream-ordered chain over the packed batch
// built by s2c_host.cpp, whose unit is the TILE (≤2048 positions of one reference):
//
//   k_pileup               (2) bit-sliced counting of the word-major seqout records per
//                          tile (32 positions per VALU op), then for a tile whose whole
//                          depth is in one work item the tile epilogue: (3) its insertion
//                          columns (:256-294) and (4) the vote for all thresholds, IUPAC,
//                          min-depth/fill, insertion chars, tile statistics — counts never
//                          reach HBM
//   k_prep / k_consensus   "deep" tiles (records split over several work items): zero their
//                          HBM count range, the items add into it, then the same epilogue
//   k_assemble             device FASTA body assembly: decoupled look-back scan of the
//                          block lengths + byte scatter
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

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for
// its global stores (__syncthreads also drains vmcnt, i.e. waits for every outstanding
// store of the wave — microseconds under load).  Global data shared inside a workgroup
// waits explicitly (s_waitcnt vmcnt(0)) before it.
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ uint32_t nibble(const uint32_t *__restrict__ w, uint64_t idx) {
    return (w[idx >> 3] >> ((idx & 7) * 4)) & 15u;
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


// Diagnostic phase stamps (ablate bit 0x100, k_pileup only): thread 0 of work item i writes
// s_memrealtime (100 MHz) for phase k to ((u64*)counts)[16i + k] (scripts/phases.py).
#define S2C_STAMP(dd, k)                                                                          \
    do {                                                                                          \
        if (((dd).ablate & 0x100) && (dd).n_deep == 0 && threadIdx.x == 0)                       \
            ((uint64_t *)(dd).counts)[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// ======================================================================= per-run state
// Deep tiles add their work items' counts into HBM: their count ranges are zeroed first.
// (Nothing else accumulates across workgroups: tile statistics and lengths are plain
// stores, insertion columns are counted per tile, and the completion counter of the
// epilogues wraps back to zero by itself.)
__global__ __launch_bounds__(WG) void k_prep(const s2c_dev d) {
    const uint32_t t = d.deep[blockIdx.x];
    const uint32_t *blk = d.blocks + (size_t)t * S2C_BLOCK_WORDS;
    if (!(blk[3] & S2C_TILE_DEEP)) return;   // a general tile's item stores all its counts
    const uint32_t a = blk[0], n = blk[1] - a;
    for (uint32_t c = 0; c < NSYM; c++)
        for (uint32_t i = threadIdx.x; i < n; i += WG) d.counts[(size_t)c * d.padded_len + a + i] = 0;
}

// ======================================================================= (3)+(4) tile epilogue
// Runs once per tile, in the workgroup that holds the tile's whole depth (k_pileup for a
// tile voted in one work item, k_consensus for a deep tile), after its counts are complete.
//
// (3) Insertion columns (:256-294).  Motif multiplicities (:264-271) and column sums
// (:284-287) are additive: column c of key k counts motif[c] over the key's events with
// len > c.  The tile's keys, events and columns are contiguous ranges (block words 4-9);
// one thread per event adds its motif's symbols into the tile's column counts [ncol][6] —
// in LDS when ncol ≤ the LDS capacity, else in the tile's own slice of HBM ins_cols.  The
// first 256 event and key records were prefetched into LDS while the counts streamed.
//
// (4) The vote (:344-389).  Per position: the closed-form vote for every threshold and the
// IUPAC char (or fill when cov == 0 or cov < min_depth, :356-359); len and sumcov do not
// depend on the threshold (1 per called position or len(fill); cov, :357/:385), the
// per-threshold non-'-' and vote-error counts are wave ballots.  Then the insertion
// columns of each called key (:290-311, :370-385), thread per key: '-' = cov[key] − Σ
// column (:294, signed), '-' results skipped, others emitted (ins_chr, ins_cnt) and added
// to len / non-'-' / sumcov (cov per emitted char, :385).  The tile's statistics per
// threshold go to tile_stats and its body lengths to blk_len — plain stores.

constexpr int VT_TMAX = 4;                    // thresholds per pass: one vote-char word per column
constexpr int VT_ACC = 1 + 4 * VT_TMAX;       // LDS u64: position sumcov, {nondash, nerr, ins sumcov, ins len}[VT_TMAX]
constexpr uint32_t PF = WG;                   // event / key records prefetched into LDS per tile
constexpr int THR_MAX = WG;                   // thresholds (-c values) supported: all staged in LDS
constexpr int FILL_LDS = 64;                  // -f bytes staged in LDS (longer fills read HBM)
constexpr int TILE_WORDS = S2C_TILE_MAX / 32;

// s_waitcnt vmcnt(0) as a real S_WAITCNT (the compiler's wait tracking sees it): ends the
// rare HBM-reading branches of the epilogue so that no load is "maybe pending" after them —
// a maybe-pending load makes the compiler wait on every later register reuse, and vmcnt is
// in order, i.e. it waits for all the bytes stored meanwhile.
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_add_u64(unsigned long long);
extern "C" __device__ unsigned int __ockl_wfscan_add_u32(unsigned int, bool);   // (x, inclusive)
extern "C" __device__ unsigned int __ockl_wfred_max_u32(unsigned int);
extern "C" __device__ unsigned int __ockl_wfred_min_u32(unsigned int);

// Sum over the wave's active lanes, every lane gets it: the device library's DPP reduction
// (row shifts / broadcasts in the VALU) — a butterfly of __shfl_xor is a dependent chain
// of ds_bpermute round trips through the LDS pipe, ~5x slower.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    if constexpr (sizeof(T) == 8) return (T)__ockl_wfred_add_u64((unsigned long long)v);
    else return (T)__ockl_wfred_add_u32((unsigned int)v);
}

template <bool LDSC>
__device__ __forceinline__ uint32_t col_load(const uint32_t *p) {
    if constexpr (LDSC) return *p;
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // the L2 copy
}

// Vote of one insertion column (:290-311) for up to 4 thresholds th[0..tn): counts v[6] of
// the column's motif symbols, the '-' count replaced by cov − Σ v (:294, signed: the
// column's own '-' count is in the sum); returns the 4 masks packed in bytes.  The group
// sums are computed once; exact in int32 while every count is < 2^28 (always, in
// practice), int64 beyond.
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

// The tile's insertion ranges (block words 4-9) and the LDS of its epilogue.
struct TileIns {
    uint32_t klo, khi, e0, e1, cb0, cb1;
};
__device__ __forceinline__ TileIns tile_ins(const uint32_t *blk) {
    const uint4 v1 = *(const uint4 *)(blk + 4);
    const uint2 v2 = *(const uint2 *)(blk + 8);
    return {uni(v1.x), uni(v1.y), uni(v1.z), uni(v1.w), uni(v2.x), uni(v2.y)};
}
// Everything the epilogue reads lives in LDS (see vm_drain).
template <uint32_t ICOL>   // LDS insertion columns of the kernel variant
struct EpiLds {
    static constexpr bool kEvents = true, kThr = true;
    uint4 ev[PF];                      // event records ins_ev[e0 .. e0+PF)
    uint4 key[PF];                     // key records ins_kinfo[klo .. klo+PF)
    double thr[THR_MAX];               // -c thresholds, CLI order
    unsigned long long acc[VT_ACC];
    uint64_t wsum[VT_TMAX][WG / 64];   // body-length scan: wave totals
    uint32_t kcov[PF];                 // coverage of each key's position if called, else 0
    uint32_t bits[TILE_WORDS];         // key bitmap of the tile's words
    uint32_t wrank[TILE_WORDS];        // keys of the tile before each word
    uint16_t kem[VT_TMAX][PF];         // insertion chars emitted per key (this pass)
    uint16_t colkey[ICOL];             // key slot of each tile column
    uint32_t vchr[ICOL];               // vote chars of each tile column, 4 thresholds per word
    uint8_t fill[FILL_LDS];
    uint8_t amb[64];
};
// LDS of the fast epilogue (k_pileup): no event records (counted from registers in the
// prologue), per-key emitted counts as u16 pairs
template <uint32_t ICOL>
struct FastLds {
    static constexpr bool kEvents = false, kThr = false;   // thresholds: a pass's 4 in SGPRs
    uint4 key[PF];                     // key records ins_kinfo[klo .. klo+PF)
    unsigned long long acc[VT_ACC];
    alignas(16) uint32_t fsum[2][VT_TMAX][WG / 64];   // body-length scan: wave totals (one 16-B read),
                                                      // by chunk parity
    uint32_t bits[TILE_WORDS];         // key bitmap of the tile's words
    uint32_t wrank[TILE_WORDS];        // keys of the tile before each word
    uint32_t kem2[2][PF];              // insertion chars emitted per key: u16 pairs (thresholds 0/2, 1/3)
    uint16_t colkey[ICOL];             // key slot of each tile column
    uint32_t vchr[ICOL];               // vote chars of each tile column, 4 thresholds per word
    uint8_t fill[FILL_LDS];
    uint8_t amb[64];
};
// issue the prefetch loads (registers; stored into LDS by prefetch_store)
struct Prefetch {
    uint4 ev, key;
    double thr;
    uint32_t bits;
    uint8_t fill;
};
template <bool kThr, class D>
__device__ __forceinline__ void prefetch_load(const D &d, uint32_t a, uint32_t n, const TileIns &ti, Prefetch &pf) {
    const uint32_t tid = threadIdx.x;
    pf.ev = make_uint4(0, 0, 0, 0);
    pf.key = make_uint4(0, 0, 0, 0);
    pf.thr = 0.0;
    pf.bits = 0;
    pf.fill = 0;
    if (ti.e0 + tid < ti.e1) pf.ev = ((const uint4 *)d.ins_ev)[ti.e0 + tid];
    if (ti.klo + tid < ti.khi) pf.key = ((const uint4 *)d.ins_kinfo)[ti.klo + tid];
    if (kThr && tid < (uint32_t)d.n_thr) pf.thr = d.thresholds[tid];
    if (tid < (n + 31) / 32) pf.bits = d.ins_bits[(a >> 5) + tid];
    if (tid < (uint32_t)min(d.fill_len, FILL_LDS)) pf.fill = d.fill[tid];
}
template <class D, class EL>
__device__ __forceinline__ void prefetch_store(const D &d, EL &L, uint32_t n, const Prefetch &pf) {
    const uint32_t tid = threadIdx.x;
    if constexpr (EL::kEvents) L.ev[tid] = pf.ev;
    L.key[tid] = pf.key;
    if constexpr (EL::kThr)
        if (tid < (uint32_t)d.n_thr) L.thr[tid] = pf.thr;
    if (tid < (n + 31) / 32) L.bits[tid] = pf.bits;
    if (tid < (uint32_t)min(d.fill_len, FILL_LDS)) L.fill[tid] = pf.fill;
}

// Tile (t, tile)'s body region in `out`: a static slot, so every tile writes its bytes
// without waiting for any other — max(1, len(fill)) bytes per padded position plus one per
// insertion column before it; threshold t's region starts at t·stride.
template <class D>
__device__ __forceinline__ uint64_t body_stride(const D &d) {
    return (uint64_t)max(1, d.fill_len) * (uint64_t)d.padded_len + (uint64_t)d.n_cols;
}
template <class D>
__device__ __forceinline__ uint64_t body_slot(const D &d, uint32_t a, uint32_t cb0) {
    return (uint64_t)max(1, d.fill_len) * a + cb0;
}

// cols: LDS [ICOL][6] (LDSC) or the tile's HBM slice.  fetch(q, c) = count of symbol c at
// tile position q.  Every thread calls (barriers inside).  Per pass of ≤ 4 thresholds:
// (3)/(4) the insertion columns' votes, then per chunk of 512 positions the position vote
// and the tile's FASTA body bytes (a block scan of the per-position lengths gives every
// byte's offset in the tile's slot), then the tile's statistics.
template <bool LDSC, class Fetch, class EL>
__device__ __forceinline__ void tile_epilogue(const s2c_dev &d, uint32_t tile, uint32_t a, uint32_t n,
                                              const TileIns &ti, Fetch fetch, uint32_t *cols, EL &L) {
    const int T = d.n_thr;
    const uint32_t F = (uint32_t)d.fill_len;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t nkeys = ti.khi - ti.klo, ncol = ti.cb1 - ti.cb0;
    const bool no_ins = (d.ablate & 0x200) != 0;   // diagnostic: skip (3)/(4) insertions
    const bool has_ins = ti.khi > ti.klo && !no_ins;
    const bool colpar = LDSC && nkeys <= PF;       // insertion summaries kept in LDS
    if (has_ins) {   // (3) count the tile's insertion columns (uniform branch)
        for (uint32_t i = tid; i < ncol * NSYM; i += WG) cols[i] = 0;
        if constexpr (!LDSC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // zeros in L2 before any atomic
        lds_sync();   // also publishes the prefetched records
        auto add_event = [&](const uint4 r) {
            uint32_t *cc = cols + (size_t)r.x * NSYM;
            for (uint32_t c = 0; c < r.y; c++) {
                uint32_t sym;
                if (c < 8) {
                    sym = (r.w >> (4 * c)) & 15u;
                } else {
                    sym = nibble(d.ins_bases, (uint64_t)r.z + c);   // motifs > 8 bases (rare)
                    vm_drain();
                }
                atomicAdd(&cc[c * NSYM + sym], 1u);
            }
        };
        // the prefetched records from LDS, the rest (tiles with > PF events) from HBM: two
        // loops, so the compiler cannot merge the two sources into one flat load
        if (ti.e0 + tid < ti.e1) add_event(L.ev[tid]);
        for (uint32_t e = ti.e0 + PF + tid; e < ti.e1; e += WG) {
            const uint4 r = ((const uint4 *)d.ins_ev)[e];
            vm_drain();
            add_event(r);
        }
        if constexpr (!LDSC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // atomics done before the reads
    }
    // keys of the tile before each of its words (position → key slot)
    const uint32_t nwords = (n + 31) / 32;
    if (wv == 0) {
        const uint32_t pc = lane < nwords ? (uint32_t)__popc(L.bits[lane]) : 0u;
        const uint32_t inc = __ockl_wfscan_add_u32(pc, true);
        if (lane < nwords) L.wrank[lane] = inc - pc;
    }
    if (has_ins && colpar && tid < nkeys) {   // key coverage (0 if not called) + column → key map
        const uint4 kr = L.key[tid];
        uint32_t cov = 0;
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) cov += fetch(kr.x - a, c);
        L.kcov[tid] = (cov > 0 && (int64_t)cov >= (int64_t)d.min_depth) ? cov : 0u;   // :356-358
        for (uint32_t c = 0; c < kr.z; c++) L.colkey[kr.y - ti.cb0 + c] = (uint16_t)tid;
    }
    S2C_STAMP(d, 3);
    uint8_t *const obase = d.out + body_slot(d, a, ti.cb0);
    const uint64_t ostride = body_stride(d);
    uint4 *cnt_out = (uint4 *)d.ins_cnt;
    for (int t0 = 0; t0 < T; t0 += VT_TMAX) {
        const int tn = min(VT_TMAX, T - t0);
        for (uint32_t i = tid; i < (uint32_t)VT_ACC; i += WG) L.acc[i] = 0;
        lds_sync();
        // ---- (4) insertion columns of the called keys (:290-311, :370-385)
        if (has_ins && colpar) {
            // one thread per column; the tile totals of the emitted chars come from here
            // (Σ over a key's columns = the key's chars): ballot counts, one u64 sum each
            uint64_t cs[VT_TMAX] = {};        // Σ cov over emitted chars (:385)
            uint32_t ec[VT_TMAX] = {}, nc[VT_TMAX] = {};   // emitted / error chars (wave)
            for (uint32_t jb = 0; jb < ncol; jb += WG) {   // uniform trip count (ballots)
                const uint32_t j = jb + tid;
                const uint32_t cov = j < ncol ? L.kcov[L.colkey[j]] : 0u;
                uint32_t word = 0x2D2D2D2Du;   // '-' (not called: never emitted)
                if (cov) {
                    const uint32_t m = column_masks(cols + (size_t)j * NSYM, cov, &L.thr[t0], tn);
                    word = 0;
#pragma unroll
                    for (int u = 0; u < VT_TMAX; u++) word |= (uint32_t)L.amb[(m >> (8 * u)) & 63u] << (8 * u);
                }
                if (j < ncol) L.vchr[j] = word;
#pragma unroll
                for (int u = 0; u < VT_TMAX; u++) {
                    const uint8_t ic = (uint8_t)(word >> (8 * u));
                    const bool em = cov && ic != '-' && ic != 0xFF;
                    ec[u] += (uint32_t)__popcll(__ballot(em));
                    nc[u] += (uint32_t)__popcll(__ballot(cov && ic == 0xFF));
                    cs[u] += em ? cov : 0u;
                }
            }
            if (tid < ((ncol + 63) & ~63u)) {   // waves that held columns
#pragma unroll
                for (int u = 0; u < VT_TMAX; u++) {
                    if (u >= tn) break;
                    const uint64_t scs = wave_sum(cs[u]);
                    if (lane == 0) {
                        unsigned long long *at = L.acc + 1 + 4 * u;
                        if (nc[u]) atomicAdd(&at[1], (unsigned long long)nc[u]);
                        if (ec[u]) {
                            atomicAdd(&at[2], (unsigned long long)scs);
                            atomicAdd(&at[3], (unsigned long long)ec[u]);
                        }
                    }
                }
            }
            lds_sync();
            if (tid < nkeys) {   // per key: chars emitted per threshold
                const uint4 kr = L.key[tid];
                uint32_t em[VT_TMAX] = {};
                if (L.kcov[tid])
                    for (uint32_t c = 0; c < kr.z; c++) {
                        const uint32_t wd = L.vchr[kr.y - ti.cb0 + c];
#pragma unroll
                        for (int u = 0; u < VT_TMAX; u++) {
                            const uint8_t ic = (uint8_t)(wd >> (8 * u));
                            em[u] += (ic != '-' && ic != 0xFF) ? 1u : 0u;
                        }
                    }
#pragma unroll
                for (int u = 0; u < VT_TMAX; u++) L.kem[u][tid] = (uint16_t)min(em[u], 0xFFFFu);
            }
        } else if (has_ins) {
            // general: one thread per key, its columns in turn (> PF keys or HBM columns);
            // the chars go to ins_chr[t][column] and {emitted, first column, columns} to
            // ins_cnt[t][key] in HBM, read back by the body writer below
            auto vote_key = [&](const uint32_t k, const uint4 kr) {
                uint32_t cov = 0;
#pragma unroll
                for (uint32_t c = 0; c < NSYM; c++) cov += fetch(kr.x - a, c);
                const bool called = cov > 0 && (int64_t)cov >= (int64_t)d.min_depth;   // :356-358
                const uint32_t *kcols = cols + (size_t)(kr.y - ti.cb0) * NSYM;
                for (int u = 0; u < tn; u++) {
                    const int t = t0 + u;
                    uint32_t em = 0, ne = 0;
                    for (uint32_t c = 0; called && c < kr.z; c++) {
                        uint32_t v[NSYM];
#pragma unroll
                        for (uint32_t j = 0; j < NSYM; j++) v[j] = col_load<LDSC>(kcols + c * NSYM + j);
                        const uint8_t ic = L.amb[column_masks(v, cov, &L.thr[t], 1) & 63u];
                        em += (ic != '-' && ic != 0xFF) ? 1u : 0u;
                        ne += ic == 0xFF ? 1u : 0u;
                        d.ins_chr[(size_t)t * d.n_cols + kr.y + c] = ic;
                    }
                    cnt_out[(size_t)t * d.n_keys + k] = make_uint4(em, kr.y, kr.z, 0);
                    unsigned long long *at = L.acc + 1 + 4 * u;
                    if (ne) atomicAdd(&at[1], (unsigned long long)ne);
                    if (em) {
                        atomicAdd(&at[2], (unsigned long long)cov * em);
                        atomicAdd(&at[3], (unsigned long long)em);
                    }
                }
            };
            if (tid < nkeys && tid < PF) vote_key(ti.klo + tid, L.key[tid]);
            for (uint32_t k = ti.klo + PF + tid; k < ti.khi; k += WG) {
                const uint4 kr = ((const uint4 *)d.ins_kinfo)[k];
                vm_drain();
                vote_key(k, kr);
            }
            // the summaries / chars are read back from HBM by other threads: stores done,
            // then the barrier below
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        lds_sync();
        S2C_STAMP(d, 4);
        // ---- positions: vote + body bytes, 2 consecutive positions per thread per chunk
        // insertion summary of key slot s for pass threshold u: chars emitted, and the k-th
        // emitted char (LDS in the column-parallel case, else HBM)
        auto body = [&](auto get_em, auto put_chars) {
            uint64_t base[VT_TMAX] = {};   // bytes of the tile's body written so far, per threshold
            uint64_t sumcov = 0;
            for (uint32_t qb = 0; qb < n; qb += 2 * WG) {   // uniform trip count (scans, ballots)
                const uint32_t q0 = qb + 2 * tid;
                // per-position coverage < 2^32 (the batch holds < 2^32 read pieces): u32 sums exact
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
                    const uint32_t bw = in[u] ? L.bits[q >> 5] : 0u;
                    haskey[u] = has_ins && called[u] && ((bw >> (q & 31)) & 1u);
                    slot[u] = in[u] ? L.wrank[q >> 5] + (uint32_t)__popc(bw & ((1u << (q & 31)) - 1u)) : 0u;
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
                        code[u][v] = called[v] ? L.amb[vote_mask_u32(cnt[v], gs[v], th * (double)cov[v])]
                                               : (uint8_t)S2C_CODE_FILL;
                        my[u] += called[v] ? 1u + (haskey[v] ? get_em(u, slot[v]) : 0u) : (in[v] ? F : 0u);
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
                lds_sync();
                S2C_STAMP(d, 5);
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
                            if (F <= (uint32_t)FILL_LDS) {
                                for (uint32_t f = 0; f < F; f++) dst[f] = L.fill[f];
                            } else {   // long -f strings from HBM (rare)
                                for (uint32_t f = 0; f < F; f++) {
                                    const uint8_t b = d.fill[f];
                                    vm_drain();
                                    dst[f] = b;
                                }
                            }
                            dst += F;
                        } else {            // vote char, then the key's insertion chars (:370-385)
                            *dst++ = code[u][v];
                            if (haskey[v]) dst = put_chars(u, slot[v], dst);
                        }
                    }
                    base[u] += tot;
                }
                S2C_STAMP(d, 8);
                lds_sync();   // wsum is rewritten by the next chunk
                S2C_STAMP(d, 9);
            }
            // tile totals per threshold (:352-397): len is the body length itself
            sumcov = wave_sum(sumcov);
            if (lane == 0) atomicAdd(&L.acc[0], (unsigned long long)sumcov);
            lds_sync();
            if (tid < (uint32_t)tn) {
                uint64_t bl = 0;
#pragma unroll
                for (int u = 0; u < VT_TMAX; u++) bl = (uint32_t)u == tid ? base[u] : bl;
                const unsigned long long *at = L.acc + 1 + 4 * tid;
                const size_t j = (size_t)(t0 + tid) * d.n_blocks + tile;
                uint64_t *st = d.tile_stats + j * 4;
                st[0] = L.acc[0] + at[2];   // sumcov: positions + cov per insertion char
                st[1] = bl;                 // len
                st[2] = at[0] + at[3];      // non-'-' chars (insertion chars are never '-')
                st[3] = at[1];              // vote errors (KeyError, :367/:381)
                d.blk_len[j] = bl;
            }
            lds_sync();   // acc is rezeroed by the next pass
        };
        if (!has_ins || colpar) {
            body([&](int u, uint32_t s) -> uint32_t { return L.kem[u][s]; },
                 [&](int u, uint32_t s, uint8_t *dst) -> uint8_t * {
                     const uint4 kr = L.key[s];
                     for (uint32_t c = 0; c < kr.z; c++) {
                         const uint8_t ic = (uint8_t)(L.vchr[kr.y - ti.cb0 + c] >> (8 * u));
                         if (ic != '-' && ic != 0xFF) *dst++ = ic;
                     }
                     return dst;
                 });
        } else {
            body([&](int u, uint32_t s) -> uint32_t {
                     const uint32_t em = cnt_out[(size_t)(t0 + u) * d.n_keys + ti.klo + s].x;
                     vm_drain();
                     return em;
                 },
                 [&](int u, uint32_t s, uint8_t *dst) -> uint8_t * {
                     const uint4 kr = ((const uint4 *)d.ins_kinfo)[ti.klo + s];
                     vm_drain();
                     const uint8_t *src = d.ins_chr + (size_t)(t0 + u) * d.n_cols + kr.y;
                     for (uint32_t c = 0; c < kr.z; c++) {
                         const uint8_t ic = src[c];
                         vm_drain();
                         if (ic != '-' && ic != 0xFF) *dst++ = ic;
                     }
                     return dst;
                 });
        }
    }
    S2C_STAMP(d, 6);
    S2C_STAMP(d, 7);
}

// the epilogue with the column buffer chosen by the tile's column count (uniform)
template <uint32_t ICOL, class Fetch>
__device__ __forceinline__ void tile_finish(const s2c_dev &d, uint32_t tile, uint32_t a, uint32_t n, const TileIns &ti,
                                            Fetch fetch, uint32_t *lds_cols, EpiLds<ICOL> &L) {
    if (ti.cb1 - ti.cb0 <= ICOL) tile_epilogue<true>(d, tile, a, n, ti, fetch, lds_cols, L);
    else tile_epilogue<false>(d, tile, a, n, ti, fetch, d.ins_cols + (size_t)ti.cb0 * NSYM, L);
}

// ======================================================================= (2) pileup
constexpr int TILE_MAX = S2C_TILE_MAX;   // positions per tile (≤ 64 words of 32)
constexpr uint32_t FLUSH_RECS = 248;     // records per lane between flushes: 31 groups of 8 (≤ 255)

// Bit-sliced counting.  A record holds 2 planes of its 32 positions' bases (b1·2+b0: A C G
// T; a position without a base — outside the piece, a '-' / 'N', a dropped '-' — holds A and
// is taken off again by the host's placeholder counts, the '-'/'N' entries added on their
// own).  Three masks are counted per record: X = b0 (C,T), Y = b1 (G,T), Z = b0&b1 (T); at
// the flush T = Z, C = X − Z, G = Y − Z, A = n − X − Y + Z, n = records the lane counted.
// A slot past the lane's range reads zeros (an out-of-range buffer offset) and is not
// counted in n.  Each counter is 8 bit-planes (bit b of the per-position count): ones, twos,
// fours, eights from a Harley–Seal carry-save tree over 16 records (15 CSAs of 2 v_bitop3
// each), bits 4..7 a ripple counter of the sixteens.  32 positions per VALU op, ≈8 VALU per
// record.
constexpr int NCTR = 3;
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
// one weight-8 carry into plane C[3], rippled into C[4..7] (an odd last group of 8)
__device__ __forceinline__ void close8(uint32_t (&C)[8], uint32_t t8) {
#pragma unroll
    for (int b = 3; b < 8; b++) {
        const uint32_t t = C[b] & t8;
        C[b] ^= t8;
        t8 = t;
    }
}
// one group of 8 records → the three counters' weight-8 carries
__device__ __forceinline__ void count8(uint32_t (&V)[NCTR][8], const uint32_t (&P)[8][2], uint32_t (&t8)[NCTR]) {
    uint32_t m[8];
#pragma unroll
    for (int u = 0; u < 8; u++) m[u] = P[u][0];
    t8[0] = tree8(V[0], m);   // X = C|T
#pragma unroll
    for (int u = 0; u < 8; u++) m[u] = P[u][1];
    t8[1] = tree8(V[1], m);   // Y = G|T
#pragma unroll
    for (int u = 0; u < 8; u++) m[u] = P[u][0] & P[u][1];
    t8[2] = tree8(V[2], m);   // Z = T
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
// The histogram layout, HC copies (lane group g adds into copy g mod HC; one copy: the
// same-word lanes of a wave serialize on their LDS atomics, but more copies cost more in
// the epilogue's reads and in occupancy than they save — measured), copy stride CS words.
template <int NWP>
struct Hist {
    static constexpr int HC = 1, HP = 17 * NWP, CS = NSYM * HP + 8;
    // packed u16 pair word s (hslot index) of symbol c, summed over the copies (counts per
    // position ≤ 248·G < 2^16: the halves never carry)
    static __device__ __forceinline__ uint32_t word(const uint32_t *h, uint32_t c, uint32_t s) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < HC; k++) v += h[k * CS + c * HP + s];
        return v;
    }
    static __device__ __forceinline__ uint32_t get(const uint32_t *h, uint32_t c, uint32_t q) {
        return (word(h, c, hslot(((q >> 5) << 4) | (q & 15))) >> ((q & 16) ? 16 : 0)) & 0xFFFFu;
    }
};

// ======================================================================= k_pileup arguments
// What k_pileup reads of s2c_dev, compact (40 SGPRs instead of ≈72: the kernel arguments
// stay in SGPRs for the whole kernel, and the full struct made the compiler spill them to
// VGPR lanes).  Same member names: the device helpers are templates over either struct.
struct PileArgs {
    const uint32_t *items, *iwr, *recs, *fix, *exc;
    const uint32_t *ins_ev, *ins_kinfo, *ins_bases, *ins_bits;
    const double *thresholds;
    const uint8_t *fill;
    uint32_t *counts;
    uint64_t *tile_stats, *blk_len;
    uint8_t *out;
    uint32_t n_recs, padded_len, n_cols, n_blocks;
    int32_t n_thr, min_depth, fill_len, fill_nondash, ablate, n_deep;
};
static PileArgs pile_args(const s2c_dev &d) {
    PileArgs p;
    p.items = d.items; p.iwr = d.iwr; p.recs = d.recs; p.fix = d.fix; p.exc = d.exc;
    p.ins_ev = d.ins_ev; p.ins_kinfo = d.ins_kinfo; p.ins_bases = d.ins_bases; p.ins_bits = d.ins_bits;
    p.thresholds = d.thresholds; p.fill = d.fill; p.counts = d.counts;
    p.tile_stats = d.tile_stats; p.blk_len = d.blk_len; p.out = d.out;
    p.n_recs = (uint32_t)d.n_recs; p.padded_len = (uint32_t)d.padded_len;
    p.n_cols = (uint32_t)d.n_cols; p.n_blocks = (uint32_t)d.n_blocks;
    p.n_thr = d.n_thr; p.min_depth = d.min_depth; p.fill_len = d.fill_len;
    p.fill_nondash = d.fill_nondash; p.ablate = d.ablate; p.n_deep = (int32_t)d.n_deep;
    return p;
}

// ======================================================================= fast tile epilogue
// The common case of k_pileup (columns in LDS, ≤ PF keys, -f ≤ FILL_LDS bytes).  The
// insertion events were already counted into `cols`, the column → key map and the key ranks
// of the tile's words built in the prologue (under the record loads).  After the counts are
// complete, per pass of ≤ 4 thresholds and chunk of 512 positions:
//   A  the column votes (first chunk of a pass) and the position votes;
//   B  each position's body length per threshold (1 + its key's emitted insertion chars,
//      or len(fill)), a packed 16-bit row scan (DPP) per threshold, wave totals, the tile
//      statistics into LDS;
//   C  byte offsets → body bytes; the last chunk writes the tile statistics.
// Barriers: (1) after a pass's column votes, (2) per chunk, (3) between passes.  A thread takes positions q and q + 16 of one
// 32-position word: their u16 counts share a histogram word.  The vote is the closed form
// (S9), evaluated in full only in waves holding a called position whose largest count is
// not unique or is below t·cov of the pass's largest threshold; elsewhere the char is that
// symbol's for every threshold (fl(t·cov) is monotone in t, so m ≥ tmax·cov ⇒ m ≥ t·cov).

// Inclusive prefix sum inside each 16-lane row (DPP row_shr, zeros shifted in).
__device__ __forceinline__ uint32_t row_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    return x;
}

// char of a one-symbol mask, amb[1 << s] = "-ACGNT"[s]
__device__ __forceinline__ uint32_t sym_char(uint32_t s) { return (uint32_t)(0x544E4743412DULL >> (8 * s)) & 0xFFu; }

// One position of the fast epilogue: counts, coverage, called (:356-359), and the vote chars
// of the pass's thresholds (byte u ↔ threshold t0 + u); `slow` = needs the full closed form.
struct Pos {
    uint32_t c[NSYM];
    uint32_t cov, chars;
    uint32_t fl;   // bit 0 in the tile, bit 1 called, bit 2 slow (a VGPR: lane masks held across
                   // the epilogue's phases made the compiler spill SGPRs)
    __device__ __forceinline__ bool in() const { return fl & 1u; }
    __device__ __forceinline__ bool called() const { return fl & 2u; }
    __device__ __forceinline__ bool slow() const { return fl & 4u; }
};
// The shortcut: the largest count m1 is a strict majority (so unique) and m1·2^15 ≥ uq·cov
// with uq = ⌈tmax·2^15⌉ + 1 (per pass; 0 = off: some threshold outside (0, 1]).  Then
// m1 ≥ tmax·cov + cov/2^15 ≥ tmax·cov·(1 + 2^-53) ≥ fl(tmax·cov) — every other symbol's
// greater-sum is ≥ m1 ≥ t·cov for every t of the pass, and the symbol's own is 0 < t·cov.
// Integer-only (counts < 2^17 here: uq·cov < 2^32); a position it misses takes the exact
// closed form.
__device__ __forceinline__ bool majority_fast(uint32_t m1, uint32_t cov, uint32_t uq) {
    return uq && 2 * m1 > cov && (m1 << 15) >= __umul24(uq, cov);
}
__device__ __forceinline__ void pos_vote_fast(Pos &p, bool in, int32_t min_depth, uint32_t uq) {
    p.cov = 0;
#pragma unroll
    for (uint32_t s = 0; s < NSYM; s++) p.cov += p.c[s];
    const bool called = in && p.cov > 0 && (int64_t)p.cov >= (int64_t)min_depth;
    // largest count and its symbol: key = count << 3 | symbol
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

// Prologue part of the fast epilogue, while the first records are in flight: the tile's
// insertion events added into the column counts (cols zeroed before the prologue barrier),
// the column → key slot map and, in wave 0, the keys before each of the tile's words.  The
// records come from the prefetch registers; events beyond PF (rare) from HBM.
template <class D, class EL>
__device__ __forceinline__ void fast_prologue(const D &d, EL &L, uint32_t *cols, const TileIns &ti,
                                              uint32_t n, const Prefetch &pf) {
    const uint32_t tid = threadIdx.x;
    if (ti.khi <= ti.klo || (d.ablate & 0x200)) return;   // uniform
    L.kem2[0][tid] = 0;   // (PF == WG) per-key emitted insertion chars of the first pass
    L.kem2[1][tid] = 0;
    auto add_event = [&](const uint4 r) {   // :264-287 motif symbols into the key's columns
        uint32_t *cc = cols + (size_t)r.x * NSYM;
        for (uint32_t c = 0; c < r.y; c++) {
            uint32_t sym;
            if (c < 8) {
                sym = (r.w >> (4 * c)) & 15u;
            } else {
                sym = nibble(d.ins_bases, (uint64_t)r.z + c);   // motifs > 8 bases (rare)
                vm_drain();
            }
            atomicAdd(&cc[c * NSYM + sym], 1u);
        }
    };
    if (ti.e0 + tid < ti.e1) add_event(pf.ev);
    for (uint32_t e = ti.e0 + PF + tid; e < ti.e1; e += WG) {
        const uint4 r = ((const uint4 *)d.ins_ev)[e];
        vm_drain();
        add_event(r);
    }
    if (ti.klo + tid < ti.khi)
        for (uint32_t c = 0; c < pf.key.z; c++) L.colkey[pf.key.y - ti.cb0 + c] = (uint16_t)tid;
    if (tid < 64) {   // wave 0: exclusive scan of the key counts of the tile's words
        const uint32_t nwords = (n + 31) / 32;
        const uint32_t pc = tid < nwords ? (uint32_t)__popc(pf.bits) : 0u;
        const uint32_t inc = __ockl_wfscan_add_u32(pc, true);
        if (tid < nwords) L.wrank[tid] = inc - pc;
    }
}

// Vote of one insertion column (:290-311) for the pass's thresholds: the '-' count is
// cov − Σ column (:294, signed).  Shortcut as for positions when every count is ≥ 0.
template <class EL>
__device__ __forceinline__ uint32_t column_word(const uint32_t *col, uint32_t cov, const EL &L, const double (&th)[VT_TMAX], int tn,
                                                uint32_t uq) {
    uint32_t v[NSYM], tot = 0;
#pragma unroll
    for (uint32_t c = 0; c < NSYM; c++) { v[c] = col[c]; tot += v[c]; }
    const int64_t dash = (int64_t)cov - (int64_t)tot;   // the column's own '-' count is in the sum
    if (uq && dash >= 0 && cov < (1u << 17)) {
        v[0] = (uint32_t)dash;
        uint32_t kk[NSYM];
#pragma unroll
        for (uint32_t c = 0; c < NSYM; c++) kk[c] = (v[c] << 3) | c;
        const uint32_t mk = max(max(max(kk[0], kk[1]), kk[2]), max(max(kk[3], kk[4]), kk[5]));
        if (majority_fast(mk >> 3, cov, uq)) return sym_char(mk & 7u) * 0x01010101u;
    }
    const uint32_t m = column_masks(col, cov, th, tn);
    uint32_t word = 0;
#pragma unroll
    for (int u = 0; u < VT_TMAX; u++) word |= (uint32_t)L.amb[(m >> (8 * u)) & 63u] << (8 * u);
    return word;
}

// hist: the tile's LDS histogram (Hist<NWP> layout); cols: LDS [ncol][6].
template <int NWP, class D, class EL>
__device__ __forceinline__ void tile_epilogue_fast(const D &d, uint32_t tile, uint32_t a, uint32_t n,
                                                   const TileIns &ti, const uint32_t *hist,
                                                   const uint32_t *cols, EL &L) {
    using H = Hist<NWP>;
    constexpr uint32_t nwp = NWP;
    const int T = d.n_thr;
    const uint32_t F = (uint32_t)d.fill_len;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, row = lane >> 4;
    const uint32_t ncol = ti.cb1 - ti.cb0;
    const bool has_ins = ti.khi > ti.klo && !(d.ablate & 0x200);
    const uint32_t nchunk = (n + 2 * WG - 1) / (2 * WG);
    uint8_t *const obase = d.out + body_slot(d, a, ti.cb0);
    const uint64_t ostride = body_stride(d);
    auto hget = [&](uint32_t q, uint32_t c) { return H::get(hist, c, q); };
    for (int t0 = 0; t0 < T; t0 += VT_TMAX) {
        const int tn = min(VT_TMAX, T - t0);
        double th[VT_TMAX];   // the pass's thresholds (uniform loads)
#pragma unroll
        for (int u = 0; u < VT_TMAX; u++) th[u] = u < tn ? d.thresholds[t0 + u] : 0.0;
        double tmax = th[0];
        bool fastok = true;   // every threshold of the pass in (0, 1] (a lone symbol cannot reach t > 1)
#pragma unroll
        for (int u = 0; u < VT_TMAX; u++)
            if (u < tn) {
                fastok = fastok && th[u] > 0.0 && th[u] <= 1.0;
                tmax = max(tmax, th[u]);
            }
        const uint32_t uq = fastok ? (uint32_t)ceil(tmax * 32768.0) + 1u : 0u;   // majority_fast
        const bool more_pass = t0 + VT_TMAX < T;
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
                        if (e02 | e13) {   // rare: chars of this column are emitted
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
            const bool any_slow = __ballot(P[0].slow() || P[1].slow()) != 0;   // a tie or a split vote
            if (any_slow) {
                pos_vote_slow(P[0], L, th, tn);
                pos_vote_slow(P[1], L, th, tn);
            }
            S2C_STAMP(d, 3);
            if (ch == 0) lds_sync();   // (1) column vote chars, per-key emitted counts, zeroed statistics
            S2C_STAMP(d, 4);
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
                // this row's offset in the wave and its lo-half total: selects, no branches
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
            S2C_STAMP(d, 5);
            lds_sync();   // (2) wave totals, statistics
            S2C_STAMP(d, 8);
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
                        if (F <= (uint32_t)FILL_LDS) {
                            for (uint32_t f = 0; f < F; f++) ob[o + f] = L.fill[f];
                        } else {   // long -f strings from HBM (rare)
                            for (uint32_t f = 0; f < F; f++) ob[o + f] = d.fill[f];
                        }
                    }
                }
                if (multi) {   // insertion chars after the key's char (:370-385)
#pragma unroll
                    for (int v = 0; v < 2; v++) {
                        if (!em_of(em02[v], em13[v], u)) continue;
                        uint32_t o = (v ? o1 : o0) + 1;
                        const uint4 kr = L.key[slot[v]];
                        for (uint32_t c = 0; c < kr.z; c++) {
                            const uint32_t ic = (L.vchr[kr.y - ti.cb0 + c] >> (8 * u)) & 0xFFu;
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
            S2C_STAMP(d, 9);
            if (ch + 1 == nchunk && tid < (uint32_t)tn) {   // tile statistics (:352-397)
                uint64_t bl = 0;
#pragma unroll
                for (int u = 0; u < VT_TMAX; u++) bl = (uint32_t)u == tid ? base[u] : bl;
                const unsigned long long *at = L.acc + 1 + 4 * tid;
                const size_t j = (size_t)(t0 + tid) * d.n_blocks + tile;
                uint64_t *st = d.tile_stats + j * 4;
                st[0] = L.acc[0] + at[2];   // sumcov: positions + cov per insertion char
                st[1] = bl;                 // len
                st[2] = at[0] + at[3];      // non-'-' chars (insertion chars are never '-')
                st[3] = at[1];              // vote errors (KeyError, :367/:381)
                d.blk_len[j] = bl;
            }
            // (3) acc / vchr / kem2 reused by the next pass.  Between chunks no barrier: chunk k+1
            // writes the other fsum half, and chunk k+2's writes come after barrier (2) of k+1,
            // which every wave reaches only after its phase C of chunk k.
            if (ch + 1 == nchunk && more_pass) lds_sync();
        }
    }
    S2C_STAMP(d, 6);
    S2C_STAMP(d, 7);
}

// The host's corrections of a work item's records, added into its LDS histogram during the
// prologue (the additions commute with the flush's: the packed u16 halves may borrow in
// between, the final u32 words are exact), so the item's counts are complete on their own
// (a deep tile's items then add true partial counts into HBM).  A placeholders: fix word
// (w, i) = the count at tile positions 32w+i (low half) and 32w+i+16 (high half), the
// histogram's own pairing, subtracted from A.  '-'/'N' entries: +1 on their symbol.
template <int NWP>
struct Corrections {
    static constexpr int FN = NWP >= 16 ? NWP / 16 : 1;   // fix words per thread (16 per tile word)
    static constexpr int XN = 4;                           // '-'/'N' entries per thread in registers
    uint32_t fx[FN], xe[XN], x0, x1;
    template <class D>
    __device__ __forceinline__ void load(const D &d, uint32_t n, uint32_t fix_off, uint32_t xa, uint32_t xb) {
        const uint32_t tid = threadIdx.x;
        x0 = xa;
        x1 = xb;
        const uint32_t nfix = 16u * ((n + 31) / 32);   // the tile's words
#pragma unroll
        for (int j = 0; j < FN; j++) {
            const uint32_t i = tid + j * WG;
            fx[j] = i < nfix ? d.fix[(size_t)fix_off + i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < XN; j++) {
            const uint32_t i = x0 + tid + j * WG;
            xe[j] = i < x1 ? d.exc[i] : 0xFFFFFFFFu;
        }
    }
    static __device__ __forceinline__ void add_entry(uint32_t *hist, uint32_t e) {
        const uint32_t q = e >> 1, sym = (e & 1) ? 4u : 0u;   // 'N' : '-'
        atomicAdd(hist + sym * (17 * NWP) + hslot(((q >> 5) << 4) | (q & 15)), (q & 16) ? 0x10000u : 1u);
    }
    template <class D>
    __device__ __forceinline__ void apply(uint32_t *hist, const D &d) const {
        const uint32_t tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < FN; j++) {
            const uint32_t i = tid + j * WG;
            if (fx[j]) atomicSub(hist + 17 * NWP + 17 * (i >> 4) + (i & 15), fx[j]);   // symbol A
        }
#pragma unroll
        for (int j = 0; j < XN; j++)
            if (xe[j] != 0xFFFFFFFFu) add_entry(hist, xe[j]);
        for (uint32_t i = x0 + tid + XN * WG; i < x1; i += WG) {   // beyond the registers (rare)
            const uint32_t e = d.exc[i];
            vm_drain();
            add_entry(hist, e);
        }
    }
};

// One workgroup per work item = (tile [a,b) of ≤ TW = 32·NWP positions, chunk k).  Lane
// L owns 32-position word w = L mod NWP of the tile and lane group g = L / NWP (G = 256/NWP
// lanes per word).  The word's seqout records [wrec[W], wrec[W+1]) are cut into chunks of
// chunk_recs (≤ 248·G: one flush per lane); the item streams chunk k, lane g taking records
// ≡ g (mod G), 8 at a time with the next 8 in flight (a group's lanes read consecutive
// records: coalesced), counted by count8.  The flush transposes the counters, derives the
// six symbol counts and adds them, two u16 per LDS atomic, into the tile's histogram.  A
// tile voted in one item (not deep) is finished from LDS by the tile epilogue (insertion
// columns, vote, statistics), its event/key records prefetched under the count stream; a
// deep tile's chunks add their histograms into HBM for k_consensus.
template <int NWP>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4))) void k_pileup(const PileArgs d) {
    constexpr int G = WG / NWP, TW = NWP * 32, HP = TW / 2 + TW / 32;
    using H = Hist<NWP>;
    static_assert(H::HP == HP, "histogram layout");
    // LDS insertion columns: ≤ 40 KB of LDS in all (4 workgroups per CU) at 512 positions
    constexpr uint32_t ICOL = S2C_LDS_COLS(NWP);
    __shared__ __attribute__((aligned(16))) uint32_t hist[H::HC * H::CS];
    __shared__ uint32_t cols[ICOL * NSYM];
    __shared__ FastLds<ICOL> L;
    const uint32_t tid = threadIdx.x;
    // word-major lanes: a wave holds 64/G whole words, so one load instruction reads G
    // consecutive records of each (full memory requests); diagnostic 0x2000: interleaved
    // (a wave holds 64/G lanes of every word)
    const bool wmaj = (d.ablate & 0x2000) == 0;
    const uint32_t w = wmaj ? tid / G : tid % NWP, g = wmaj ? tid % G : tid / NWP;
    if (d.ablate & 0x800) return;   // diagnostic: empty kernel (launch cost)
    S2C_STAMP(d, 0);
    if (tid < 64) L.amb[tid] = c_amb[tid];   // published by the barrier after the histogram zeroing
    const uint32_t *__restrict__ recs = d.recs;
    const uint32_t item = blockIdx.x;   // grid = work items
    // the item descriptor (64 B: its tile's block words and first record copied in) and this
    // lane's word record range: one load round before the records
    const uint4 *iv = (const uint4 *)d.items + 4 * (size_t)item;
    const uint4 itv = iv[0], itc = iv[1], itk = iv[2], itx = iv[3];
    const uint32_t a = uni(itv.x), b = uni(itv.y), chunk = uni(itv.z), tile = uni(itv.w);
    (void)chunk;
    const uint32_t flags = uni(itc.w);
    const bool deep = (flags & S2C_TILE_DEEP) != 0;
    const TileIns ti = {uni(itk.x), uni(itk.y), uni(itk.z), uni(itk.w), uni(itx.x), uni(itx.y)};
    const uint32_t rbase = uni(itx.z);   // the item's first record
    const uint32_t n = b - a;
    const uint32_t ws = 32u * w;                  // word start, tile-relative
    const bool active = ws < n;
    uint32_t r0 = 0, r1 = 0;   // this word's records in this item
    if (active) {
        const uint2 rr = ((const uint2 *)d.iwr)[(size_t)item * NWP + w];
        r0 = rr.x;
        r1 = rr.y;
    }
    // the tile's whole depth is in this item and its insertion keys / columns fit the LDS:
    // finished here by the epilogue (else its counts go to HBM for k_consensus)
    const bool finish = flags == 0 && !(d.ablate & 4);
    const bool fastp = finish;
    Prefetch pf;   // epilogue records, in flight under the count stream
    if (finish) prefetch_load<false>(d, a, n, ti, pf);
    Corrections<NWP> corr;   // A placeholders and '-'/'N' entries of this item's records
    corr.load(d, n, uni(itc.x), uni(itc.y), uni(itc.z));
    uint32_t V[NCTR][8];
    auto zeroV = [&]() {
#pragma unroll
        for (int c = 0; c < NCTR; c++)
#pragma unroll
            for (int bb = 0; bb < 8; bb++) V[c][bb] = 0;
    };
    // The item's records through a buffer resource based at its first word's first record
    // (uniform): a load's address = lane offset (VGPR) + group offset (SGPR) + record slot
    // (immediate); a slot past the lane's range gets an out-of-range offset and the
    // hardware returns zeros (no mask set: nothing counted).
    const uint64_t rbytes = ((uint64_t)d.n_recs - rbase) * 8;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(recs + 2 * (size_t)rbase), (short)0, (int)min(rbytes, (uint64_t)0x7FFF0000u), 0x00020000);
    constexpr uint32_t OOR = 0x80000000u;   // an offset past any record
    const uint32_t e0 = (d.ablate & 1) ? r0 : r1;   // diagnostic 1: no records
    const uint32_t t = r0 + g;                      // the lane's first record
    const uint32_t nrec = t < e0 ? (e0 - t + G - 1) / G : 0u;   // records ≡ g (mod G) in [r0, e0)
    const uint32_t voff = nrec ? (t - rbase) * 8u : OOR;
    const uint32_t ngrp = uni(__ockl_wfred_max_u32((nrec + 7) / 8));   // groups of 8, busiest lane
    auto loadg = [&](uint32_t (&P)[8][2], uint32_t gi) {
        const uint32_t so = gi * 64u * G;   // group gi: records 8·gi·G.. of the lane's stride
#pragma unroll
        for (int u = 0; u < 8; u++) {
            // (the empty asm keeps the offset one register + an immediate: the compiler would
            // otherwise hoist the eight sums out of the loop and spill them)
            uint32_t vo = 8 * gi + u < nrec ? voff : OOR;
            asm volatile("" : "+v"(vo));
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, vo + (uint32_t)(u * 8 * G), so, 0);
            P[u][0] = v[0]; P[u][1] = v[1];
        }
    };
    uint32_t sink = 0;   // diagnostic ablate&2: loads consumed without counting
    auto sink8 = [&](const uint32_t (&P)[8][2]) {
#pragma unroll
        for (int u = 0; u < 8; u++) sink ^= P[u][0] ^ P[u][1];
    };
    zeroV();
    // ---- count this word's records of the chunk (one flush: chunk ≤ 248·G, check_dev) ----
    // the first group is issued before the LDS zeroing and its barrier
    uint32_t P[8][2], Q[8][2];
    S2C_STAMP(d, 10);   // word ranges known (ngrp needs every lane's)
    if (ngrp > 0) loadg(P, 0);
    __builtin_amdgcn_sched_barrier(0);
    S2C_STAMP(d, 11);   // first records issued
    for (uint32_t i = tid; i < (uint32_t)(H::HC * H::CS) / 4; i += WG) ((uint4 *)hist)[i] = make_uint4(0, 0, 0, 0);
    if (fastp)
        for (uint32_t i = tid; i < (ti.cb1 - ti.cb0) * NSYM; i += WG) cols[i] = 0;
    lds_sync();
    S2C_STAMP(d, 1);
    if (finish) prefetch_store(d, L, n, pf);   // their loads were issued before P's
    if (fastp) fast_prologue(d, L, cols, ti, n, pf);
    corr.apply(hist, d);
    {
        // two groups of 8 per trip (one 16-record carry-save step), the next group always
        // in flight while one is counted; an odd last group closes alone.  sched_barrier
        // keeps each group's loads issued ahead of the other group's count (the scheduler
        // otherwise sinks them next to their use to save registers).
        uint32_t ta[NCTR], tb[NCTR];
        for (uint32_t gi = 0; gi < ngrp; gi += 2) {   // uniform trip count
            loadg(Q, gi + 1);
            __builtin_amdgcn_sched_barrier(0);
            if (d.ablate & 2) sink8(P); else count8(V, P, ta);
            loadg(P, gi + 2);
            __builtin_amdgcn_sched_barrier(0);
            if (d.ablate & 2) {
                sink8(Q);
                continue;
            }
            count8(V, Q, tb);
#pragma unroll
            for (int c = 0; c < NCTR; c++) close16(V[c], ta[c], tb[c]);
        }
    }
    // ---- flush: counters → four symbol counts → LDS histogram ----
    {
        // X = C|T, Y = G|T, Z = T → T, C = X − Z, G = Y − Z, A = n − X − Y + Z (no byte
        // borrows: every difference is a count)
        uint32_t X[8], Y[8], Z[8];
#pragma unroll
        for (int r = 0; r < 8; r++) { X[r] = V[0][r]; Y[r] = V[1][r]; Z[r] = V[2][r]; }
        transpose8(X);
        transpose8(Y);
        transpose8(Z);
        // The G lanes of a word sit side by side (word-major): add pairs, then quads of them
        // with DPP row shifts while a byte cannot carry (≤ 255), so that one lane in `red`
        // adds into the histogram — the lanes of a word hit the same LDS words, and those
        // atomics serialize.  Whole words are active or not, and G ≥ 4: no sum mixes words.
        uint32_t nsum = nrec, red = 1;
        auto shr1 = [](uint32_t &v) { v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true); };
        auto shr2 = [](uint32_t &v) { v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true); };
        if (wmaj) {
            const uint32_t nmax = uni(__ockl_wfred_max_u32(nrec));
            if (nmax < 128) {   // pair sums ≤ 254
                red = 2;
                shr1(nsum);
#pragma unroll
                for (int r = 0; r < 8; r++) { shr1(X[r]); shr1(Y[r]); shr1(Z[r]); }
                if (nmax < 64) {   // quad sums ≤ 252
                    red = 4;
                    shr2(nsum);
#pragma unroll
                    for (int r = 0; r < 8; r++) { shr2(X[r]); shr2(Y[r]); shr2(Z[r]); }
                }
            }
        }
        if (active && (g % red) == red - 1 && !(d.ablate & 8)) {
        uint32_t *h0 = hist + (g % H::HC) * H::CS + 17 * w;   // this lane group's copy
        auto add = [&](uint32_t sym, const uint32_t (&R)[8]) {
            uint32_t *hw = h0 + sym * HP;
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const uint32_t lo = R[r] & 0x00FF00FFu, hi = (R[r] >> 8) & 0x00FF00FFu;
                atomicAdd(hw + r, lo);
                atomicAdd(hw + 8 + r, hi);
            }
        };
        const uint32_t nb = nsum * 0x01010101u;
        add(5, Z);
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const uint32_t a1 = nb - X[r] - Y[r] + Z[r];
            X[r] -= Z[r];
            Y[r] -= Z[r];
            Z[r] = a1;
        }
        add(2, X);
        add(3, Y);
        add(1, Z);
        }
    }
    if (sink == 0x9E3779B9u) hist[0] = 1;   // keeps the ablation's loads alive
    // the count loop's last prefetch group is never consumed: drain it here (long landed),
    // or every later reuse of its registers would wait behind the epilogue's stores
    vm_drain();
    lds_sync();
    S2C_STAMP(d, 2);
    if (finish) {   // the tile's whole depth is here: finish it now
        // diagnostic 0x1000: the same epilogue code runs twice (phase stamps of the warm run)
        const int reps = (d.ablate & 0x1000) ? 2 : 1;
#pragma nounroll
        for (int rep = 0; rep < reps; rep++) tile_epilogue_fast<NWP>(d, tile, a, n, ti, hist, cols, L);
    } else {
        // deep tile: this chunk's counts → HBM (symbol-major, coalesced atomics); a general
        // tile's (and, with the diagnostic flag 4, every tile's) counts: plain stores
        for (uint32_t q = tid; q < n; q += WG)
#pragma unroll
            for (uint32_t c = 0; c < NSYM; c++) {
                uint32_t *dst = d.counts + (size_t)c * d.padded_len + a + q;
                const uint32_t v = H::get(hist, c, q);
                if (deep) {
                    if (v) atomicAdd(dst, v);
                } else {
                    *dst = v;
                }
            }
    }
}

// Deep tiles: counts summed in HBM by their work items → the same epilogue.
__global__ __launch_bounds__(WG) void k_consensus(const s2c_dev d) {
    constexpr uint32_t ICOL = 1024;
    __shared__ uint32_t cols[ICOL * NSYM];
    __shared__ EpiLds<ICOL> L;
    if (threadIdx.x < 64) L.amb[threadIdx.x] = c_amb[threadIdx.x];   // published by the epilogue's first barrier
    const uint32_t tile = d.deep[blockIdx.x];
    const uint32_t *blk = d.blocks + (size_t)tile * S2C_BLOCK_WORDS;
    const uint32_t a = uni(blk[0]), n = uni(blk[1]) - a;
    const TileIns ti = tile_ins(blk);
    Prefetch pf;
    prefetch_load<true>(d, a, n, ti, pf);
    prefetch_store(d, L, n, pf);
    const uint32_t *cts = d.counts + a;
    const size_t Lp = d.padded_len;
    tile_finish<ICOL>(d, tile, a, n, ti, [&](uint32_t q, uint32_t c) { return cts[(size_t)c * Lp + q]; }, cols, L);
}

inline int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return S2C_OK;
    return s2c_set_error(S2C_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// ======================================================================= C-ABI
extern "C" int s2c_workspace_sizes(const s2c_batch_info *info, int32_t n_thr, s2c_ws_sizes *o) {
    if (!info || !o || n_thr <= 0) return s2c_set_error(S2C_ERR_ARG, "bad workspace query");
    const int64_t L = info->padded_len, T = n_thr, NB = T * info->n_blocks;
    const int64_t nk = std::max<int64_t>(info->n_keys, 1), nc = std::max<int64_t>(info->n_cols, 1);
    o->counts = info->n_deep ? NSYM * L * 4 : 64;   // only deep tiles keep counts in HBM
    o->ins_cols = nc * NSYM * 4;
    o->ins_cnt = T * nk * 16;
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
    if (d->tile_max <= 0 || d->tile_max > TILE_MAX) return s2c_set_error(S2C_ERR_ARG, "tile_max out of range");
    if (d->padded_len <= 0 || d->padded_len >= ((int64_t)1 << 32)) return s2c_set_error(S2C_ERR_ARG, "bad padded_len");
    if (d->n_blocks >= ((int64_t)1 << 31) || (int64_t)d->n_thr * d->n_blocks >= ((int64_t)1 << 40))
        return s2c_set_error(S2C_ERR_LIMIT, "too many (threshold, tile) blocks");
    if (d->n_items > 0 && (!d->items || !d->iwr || !d->recs || !d->fix || d->chunk_recs <= 0))
        return s2c_set_error(S2C_ERR_ARG, "missing pileup buffers");
    if (d->n_exc > 0 && !d->exc) return s2c_set_error(S2C_ERR_ARG, "missing '-'/'N' entries");
    {   // one flush per item: the LDS histogram's u16 halves hold ≤ 248·G per position
        int64_t nwp = 8;
        while (nwp * 32 < d->tile_max) nwp *= 2;
        if (d->chunk_recs > (int64_t)FLUSH_RECS * (WG / nwp))
            return s2c_set_error(S2C_ERR_ARG, "chunk_recs exceeds one flush per work item");
    }
    if (d->n_deep > 0 && (!d->deep || !d->counts)) return s2c_set_error(S2C_ERR_ARG, "missing deep-tile buffers");
    if ((d->ablate & 0x104) && !d->counts) return s2c_set_error(S2C_ERR_ARG, "ablate&0x104 writes `counts`: counts buffer required");
    if (!d->ins_bits) return s2c_set_error(S2C_ERR_ARG, "missing key bitmap");
    if (d->n_keys > 0 && (!d->ins_ev || !d->ins_kinfo || !d->ins_bases || !d->ins_cols || !d->ins_cnt || !d->ins_chr))
        return s2c_set_error(S2C_ERR_ARG, "missing insertion buffers");
    if (d->n_blocks > 0 && (!d->blocks || !d->blk_len || !d->tile_stats || !d->out))
        return s2c_set_error(S2C_ERR_ARG, "missing vote/body buffers");
    if (d->fill_len < 0 || (d->fill_len > 0 && !d->fill)) return s2c_set_error(S2C_ERR_ARG, "bad fill");
    {   // every tile's body slot must fit: T regions of max(1, len(fill))·L + n_cols bytes
        const int64_t need = (int64_t)d->n_thr * ((int64_t)std::max(1, d->fill_len) * d->padded_len + d->n_cols);
        if (d->out_cap < need) return s2c_set_error(S2C_ERR_ARG, "out buffer smaller than the body slots");
    }
    return S2C_OK;
}

template <int NWP>
static int launch_pileup(const s2c_dev *d, hipStream_t s) {
    k_pileup<NWP><<<(unsigned)d->n_items, WG, 0, s>>>(pile_args(*d));
    return hip_check(hipGetLastError(), "k_pileup");
}

extern "C" int s2c_pileup(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (d->n_deep > 0) {
        k_prep<<<(unsigned)d->n_deep, WG, 0, s>>>(*d);
        if ((rc = hip_check(hipGetLastError(), "k_prep"))) return rc;
    }
    if (d->n_items == 0) return S2C_OK;
    if (d->n_items >= ((int64_t)1 << 31)) return s2c_set_error(S2C_ERR_LIMIT, "more than 2^31 work items");
    if (d->tile_max <= 256) return launch_pileup<8>(d, s);
    if (d->tile_max <= 512) return launch_pileup<16>(d, s);
    if (d->tile_max <= 1024) return launch_pileup<32>(d, s);
    return launch_pileup<64>(d, s);
}

extern "C" int s2c_consensus(const s2c_dev *d, void *stream) {
    int rc = check_dev(d);
    if (rc) return rc;
    if (d->n_deep > 0) {
        k_consensus<<<(unsigned)d->n_deep, WG, 0, (hipStream_t)stream>>>(*d);
        return hip_check(hipGetLastError(), "k_consensus");
    }
    return S2C_OK;
}

extern "C" int s2c_run(const s2c_dev *d, void *stream) {
    int rc;
    if ((rc = s2c_pileup(d, stream))) return rc;
    return s2c_consensus(d, stream);
}

/*
 * s2c.h — C-ABI of libs2c.so, the MI355X (gfx950) pileup-and-vote engine behind
 * the sam2consensus.py drop-in CLI.
 *
 * The reference (zoujiayun/sam2consensus v2.1) is ONE Python-2 script; its hot path
 * is inline in main().  Each entry point below names the reference region it
 * replaces (sam2consensus.py:LINE).  A Python host binds these with ctypes
 * (sam2consensus_amd/_lib.py); INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every function returns int: S2C_OK (0) or a negative S2C_ERR_* code;
 *     s2c_last_error() gives the message (thread-local).
 *   - error codes S2C_ERR_KEY..S2C_ERR_OVERFLOW are the Python exception classes the
 *     reference dies with on the same input (SURVEY.md §5 "Failure detection");
 *     the host raises that class, exits non-zero and writes no FASTA.
 *   - no torch / HIP C++ types in signatures: device buffers are plain pointers
 *     owned by the caller (torch tensors in the Python host); the stream is a
 *     hipStream_t passed as void*.
 */
#ifndef S2C_H
#define S2C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define S2C_ABI_VERSION 4

/* ---- status codes ---------------------------------------------------------------- */
#define S2C_OK            0
#define S2C_ERR_KEY      -1   /* KeyError:   unknown RNAME (:212,:221), base not in -ACGNT (:212,:287), vote key (:367,:381) */
#define S2C_ERR_INDEX    -2   /* IndexError: <6 / <10 fields (:195,:206), empty RNAME (:200), pos out of range (:212), insertion key (:294) */
#define S2C_ERR_VALUE    -3   /* ValueError: non-int POS (:201) or LN (:164); int(nan*100) (:394) */
#define S2C_ERR_ZERODIV  -4   /* ZeroDivisionError: zero-length record (:395, e.g. -f "") */
#define S2C_ERR_OVERFLOW -5   /* OverflowError: int(inf*100) (:394) */
#define S2C_ERR_IO      -10   /* file / gzip I/O */
#define S2C_ERR_HIP     -11   /* HIP runtime failure */
#define S2C_ERR_ARG     -12   /* bad argument / shape check failed before a launch */
#define S2C_ERR_LIMIT   -13   /* input beyond this build's limits (e.g. > 2^32 positions) */

const char *s2c_last_error(void);
int s2c_abi_version(void);
/* ABI self-check for FFI mirrors: fills out[0..n) with sizeof/offsetof values of the
 * structs below (order documented in sam2consensus_amd/_lib.py); returns the count. */
int s2c_layout(int64_t *out, int n);

/* ---- constants shared with the kernels -------------------------------------------- */
#define S2C_NSYM          6    /* symbols '-','A','C','G','N','T' — sorted() order (:367) */
#define S2C_POS_ALIGN    64    /* each reference starts at a multiple of this global coordinate */
#define S2C_ITEM_WORDS   16    /* u32 words per pileup work item {a, b, chunk, tile, fix_off, x0, x1,
                                  flags, klo, khi, e0, e1, cb0, cb1, rbase, 0} */
#define S2C_BLOCK_WORDS  12    /* u32 words per tile {a, b, ref, flags, klo, khi, e0, e1, cb0, cb1, 0, 0} */
#define S2C_TILE_DEEP     1    /* flags: the tile's records take several work items (HBM counts) */
#define S2C_TILE_GENERAL  2    /* flags: more insertion columns / keys than k_pileup's LDS holds:
                                  its counts go to HBM and k_consensus votes it */
#define S2C_EPI_KEYS    256    /* keys per tile the k_pileup epilogue holds in LDS */
/* insertion columns per tile the k_pileup epilogue holds in LDS, by words per tile */
#define S2C_LDS_COLS(nwp) ((nwp) <= 16 ? 640 : ((nwp) == 32 ? 448 : 192))
#define S2C_CODE_FILL     0    /* internal vote char of a fill position */
#define S2C_CODE_ERR   0xFF    /* vote char where the vote hit a missing amb key (:367) */
#define S2C_TILE_MAX   2048    /* positions per tile */

/* ======================================================================================
 * Host side: SAM/SAM.gz parser → packed read batch          (replaces :147-228, :256-294)
 * ======================================================================================
 * The parser reproduces the reference's record handling exactly (header pass :149-172,
 * record filter :195, RNAME/POS :200-201, parsecigar :46-82, maxdel rule :210, error
 * classes in file order) and emits the packed batch: every read's seqout (:64-81) cut
 * at the global 32-position grid into word-major records of 3 bit-planes, insertion
 * events, the pileup / consensus work plan, and a host-side read-piece table.
 */
typedef struct s2c_parser s2c_parser;
typedef struct s2c_batch  s2c_batch;

/* maxdel_active = 0 reproduces Python 2's `int <= str` when -d is given (:102,:210). */
int  s2c_parser_new(int maxdel_active, int64_t maxdel, s2c_parser **out);
/* Feed raw SAM text (any chunking; lines may straddle calls). */
int  s2c_parser_feed(s2c_parser *p, const char *buf, size_t len);
/* Parse a whole file; ".gz" suffix → zlib (:111-114). */
int  s2c_parser_feed_file(s2c_parser *p, const char *path);
/* End of input: reformat-phase checks (:284-294), global layout and work plan. */
int  s2c_parser_finish(s2c_parser *p, s2c_batch **out);
void s2c_parser_free(s2c_parser *p);

typedef struct {
    int64_t n_refs;            /* @SQ references (:160-169) */
    int64_t total_len;         /* Σ LN over refs (real positions) */
    int64_t padded_len;        /* global coordinate extent (refs aligned to S2C_POS_ALIGN) */
    int64_t header_lines;      /* :158 */
    int64_t lines_total;       /* all lines seen (:194 counts from -header_lines) */
    int64_t reads_mapped;      /* records passing :195 */
    int64_t aligned_bases;     /* A = Σ len(seqout) over mapped reads (the metric's unit) */
    int64_t query_bases;       /* Q = M/=/X + I bases packed (B_alg 0.5·Q) */
    int64_t n_reads;           /* read pieces (after POS=0 wrap splitting, :212) */
    int64_t n_ops;             /* effective op words (B_alg 4·K) */
    int64_t n_recs;            /* (piece, 32-position word) seqout records */
    int64_t chunk_recs;        /* records per word per work item (deep tiles take several) */
    int64_t n_ins;             /* insertion events kept (key in [0, LN), non-empty motif) */
    int64_t n_ins_bases;       /* Σ motif lengths */
    int64_t n_ins_words;       /* u32 words of packed motif bases */
    int64_t n_keys;            /* distinct insertion keys (:262-271 dict keys) */
    int64_t n_cols;            /* insertion columns = Σ over keys of the longest motif (:278-281) */
    int64_t n_items;           /* pileup work items */
    int64_t n_blocks;          /* tiles = consensus/assembly blocks (never straddle a ref) */
    int64_t tile_max;          /* max positions of any tile (≤ 2048) */
    int64_t n_deep;            /* tiles voted by k_consensus: split over several work items
                                  (S2C_TILE_DEEP) or beyond k_pileup's LDS (S2C_TILE_GENERAL) */
    int64_t n_exc;             /* seqout '-' / 'N' entries (kept out of the 2-bit records) */
    int64_t n_fix;             /* u32 words of per-item A-placeholder counts */
    int64_t n_iwr;             /* u32 words of per-item word record ranges (n_items · words · 2) */
} s2c_batch_info;

typedef struct {               /* host pointers into the batch (valid until s2c_batch_free) */
    const int64_t  *ref_len;   /* [n_refs] */
    const int64_t  *ref_off;   /* [n_refs] global coordinate of position 0 */
    const int64_t  *ref_cov_reads; /* [n_refs] pileup records per ref (0 ⇒ Σcov may be 0) */
    const uint32_t *rd_pos;    /* [n_reads]   global coordinate of seqout char 0 (file order) */
    const uint32_t *rd_op;     /* [n_reads+1] op offset (CSR) */
    const uint32_t *rd_span;   /* [n_reads]   seqout length (bits 0-30); bit31 = '-' not counted (maxdel :210) */
    const uint32_t *ops;       /* [n_ops]     (len << 1) | cls, cls 0 = M/=/X, 1 = D/N/P */
    const uint32_t *wrec;      /* [padded_len/32 + 1] CSR: records of global word W = [wrec[W], wrec[W+1]) */
    const uint32_t *recs;      /* [n_recs][2] bit-planes {b0, b1} of the 32 positions' bases
                                  (b1·2+b0: 0 A, 1 C, 2 G, 3 T).  A position without an A/C/G/T
                                  entry — outside the read piece, a '-' of a maxdel-dropped read
                                  (:214-218), or a '-' / 'N' (those are in exc) — holds 0 (A) and
                                  is subtracted again through fix */
    const uint32_t *fix;       /* [n_fix] per work item (from item word 4), 16 u32 per word of its
                                  tile: u32 i of word w = the A placeholders among the item's
                                  records at tile positions 32w+i (low u16) and 32w+i+16 (high) */
    const uint32_t *exc;       /* [n_exc] the counted seqout '-' and 'N' of each work item (item
                                  words 5-6): (position − tile start) << 1 | is_N */
    const uint32_t *ins_key;   /* [n_keys]    global coordinate of each key (:74), ascending */
    const uint32_t *ins_koff;  /* [n_keys+1]  events of key k = [koff[k], koff[k+1]) (file order) */
    const uint32_t *ins_kcol;  /* [n_keys+1]  columns of key k = [kcol[k], kcol[k+1]) */
    const uint32_t *ins_off;   /* [n_ins+1]   nibble offset of each event's motif in ins_bases */
    const uint32_t *ins_bases; /* [n_ins_words] motif symbol codes, 8 nibbles per word */
    const uint32_t *ins_ekey;  /* [n_ins]     key index of each event */
    const uint32_t *ins_ev;    /* [n_ins][4]  {column offset in the key's tile, motif length,
                                                nibble offset, first 8 motif nibbles} */
    const uint32_t *ins_kinfo; /* [n_keys][4] {position, first column, columns, 0} */
    const uint32_t *ins_bits;  /* [padded_len/32] bit p: position p is a key */
    const uint32_t *ins_rank;  /* [padded_len/32+1] keys before 32-position word W */
    const uint32_t *items;     /* [n_items][S2C_ITEM_WORDS] pileup work items {a, b, chunk, tile,
                                  fix_off, x0, x1, flags, klo, khi, e0, e1, cb0, cb1, rbase, 0}:
                                  tile [a, b), records chunk `chunk` of each word, its placeholder
                                  words and '-'/'N' entries [x0, x1), a copy of the tile's block
                                  words 3-9, and wrec[a/32] (the item's first record) */
    const uint32_t *iwr;       /* [n_items][nwp][2] per item and tile word w: its record range
                                  {r0, r1} (nwp = words of the widest tile rounded up to a power
                                  of two ≥ 8; words past the tile: {0, 0}) */
    const uint32_t *blocks;    /* [n_blocks][S2C_BLOCK_WORDS] tiles {g_begin, g_end, ref, flags, then the
                                  tile's keys [klo,khi), events [e0,e1), columns [cb0,cb1)} */
    const uint32_t *deep;      /* [n_deep] indices of the tiles k_consensus votes (flags != 0) */
} s2c_batch_arrays;

int  s2c_batch_info_get(const s2c_batch *b, s2c_batch_info *out);
int  s2c_batch_arrays_get(const s2c_batch *b, s2c_batch_arrays *out);
/* Reference name i (NUL-terminated, owned by the batch). */
const char *s2c_batch_ref_name(const s2c_batch *b, int64_t i);
void s2c_batch_free(s2c_batch *b);

/* parsecigar(cigarstring, seq, pos_ref) (:46-82) for one read, same semantics.
 * seqout: caller buffer of capacity cap (gets NUL); *seqout_len = chars written.
 * Insertions: up to max_ins (ref_pos, seq offset, len) triples into ins[3*k]. */
int  s2c_parsecigar(const char *cigar, size_t cigar_len, const char *seq, size_t seq_len,
                    int64_t pos_ref, char *seqout, size_t cap, size_t *seqout_len,
                    int64_t *ins, size_t max_ins, size_t *n_ins);

/* ======================================================================================
 * Synthetic workloads (BASELINE.json configs C1..C5) — deterministic (splitmix64)
 * ====================================================================================== */
typedef struct {
    int32_t  n_refs;
    int64_t  ref_len;
    double   depth;            /* reads per ref = floor(depth·ref_len / read_len) */
    int32_t  read_len;
    double   ins_frac;         /* fraction of reads with one I of 1..ins_max bases */
    int32_t  ins_max;
    double   del_frac;         /* fraction of reads with one D of 1..del_max bases */
    int32_t  del_max;
    double   long_del_frac;    /* of the D reads, fraction with a D of read_len+1 .. 2·read_len */
    double   sub_rate;         /* substitution rate */
    double   n_rate;           /* N-call rate */
    int32_t  amplicons;        /* >0: starts drawn from this many tiled amplicon starts */
    int32_t  shuffle;          /* 1: record order shuffled (else coordinate-sorted) */
    uint64_t seed;
    const char *ref_prefix;    /* reference names ref_prefix + index (NULL → "gene") */
} s2c_synth_spec;

/* Stream the SAM text of `spec` into parser p (no file), or write it to `path`
 * (gzip if it ends with ".gz").  *n_reads_out gets the record count. */
int s2c_synth_feed(const s2c_synth_spec *spec, s2c_parser *p, int64_t *n_reads_out);
int s2c_synth_write(const s2c_synth_spec *spec, const char *path, int64_t *n_reads_out);

/* ======================================================================================
 * Device side (HIP, gfx950).  All pointers are device pointers; stream = hipStream_t.
 * ====================================================================================== */
typedef struct {
    /* ---- packed batch (device copies of s2c_batch_arrays) ---- */
    const uint32_t *wrec, *recs;   /* word-major seqout records (s2c_batch_arrays) */
    const uint32_t *fix, *exc;     /* A-placeholder counts, '-'/'N' entries (s2c_batch_arrays) */
    const uint32_t *iwr;           /* per-item word record ranges (s2c_batch_arrays) */
    const uint32_t *items, *blocks, *deep;
    const uint32_t *ins_ev, *ins_kinfo, *ins_bases, *ins_bits;   /* (s2c_batch_arrays) */
    int64_t n_recs, chunk_recs, n_items, n_blocks, n_deep, n_keys, n_cols, padded_len, n_exc;
    int32_t tile_max, n_refs;

    /* ---- options (:117-138) ---- */
    const double *thresholds;  /* [T] device copy of -c values, CLI order */
    int32_t  n_thr;
    int32_t  min_depth;        /* -m */
    int32_t  fill_len;         /* len(-f) */
    int32_t  fill_nondash;     /* count of chars != '-' in -f */
    const uint8_t *fill;       /* [fill_len] device copy of -f bytes */

    /* ---- workspace (caller allocates; sizes from s2c_workspace_sizes) ---- */
    uint32_t *counts;          /* [6][padded_len] pileup counts of deep tiles (SoA by symbol) */
    uint32_t *ins_cols;        /* [n_cols][6] column counts of tiles whose columns exceed LDS */
    uint32_t *ins_cnt;         /* [T][n_keys][4] {chars emitted, first column, columns, 0}: tiles
                                  with > 256 keys or HBM columns only */
    uint8_t  *ins_chr;         /* [T][n_cols] column vote chars, same tiles only */

    /* ---- outputs ---- */
    uint64_t *tile_stats;      /* [T][n_blocks][4] {sumcov, len, nondash, vote_errors} per tile
                                  (:352-397; summed per reference by the host) */
    uint64_t *blk_len;         /* [T][n_blocks] FASTA body bytes of (t, tile) */
    uint8_t  *out;             /* FASTA bodies (:350-389): tile (t, tile) at
                                  t·(F·padded_len + n_cols) + F·a + cb0, F = max(1, len(fill)),
                                  a = the tile's first position, cb0 its first insertion column;
                                  blk_len bytes each.  A reference's body for threshold t is its
                                  tiles' pieces in order. */
    int64_t   out_cap;         /* ≥ T·(F·padded_len + n_cols) */

    /* ---- diagnostics, 0 in the product: bit 1 skips counting, bit 2 loads without
     *      counting, bit 8 skips the
     *      histogram flush, 0x200 skips the insertion columns, 0x800 returns at once
     *      (timing ablations, results wrong: scripts/ablate.py); bit 4 makes every tile store
     *      its counts to `counts` (sized 6*padded_len*4) instead of voting (counts parity
     *      tests); 0x100 writes phase timestamps to `counts` (scripts/phases.py) ---- */
    int32_t   ablate;
    int32_t   reserved;
} s2c_dev;

/* Sizes (bytes) of every workspace / output buffer for a batch and T thresholds. */
typedef struct {
    int64_t counts, ins_cols, ins_cnt, ins_chr, blk_len, tile_stats;
    int64_t out_per_fill, out_fixed;   /* out bytes = out_per_fill·max(1, len(fill)) + out_fixed */
} s2c_ws_sizes;
int s2c_workspace_sizes(const s2c_batch_info *info, int32_t n_thr, s2c_ws_sizes *out);

/* Stage order (s2c_run): s2c_pileup → s2c_consensus.
 * (2) pileup per tile; for tiles holding their whole depth in one work item also (3) the
 * insertion columns, (4) the vote (all thresholds, IUPAC, min-depth/fill, insertion
 * chars, tile statistics) and the tile's FASTA body bytes
 *                                          (:206-221, :232-253, :256-311, :344-397) */
int s2c_pileup(const s2c_dev *d, void *stream);
/* (3)+(4) and the bodies for deep tiles (records split over several work items, counts
 * summed in HBM)                                   (:232-253, :256-311, :344-397) */
int s2c_consensus(const s2c_dev *d, void *stream);
/* both, in order, on one stream (graph-capturable: no allocation, no sync) */
int s2c_run(const s2c_dev *d, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* S2C_H */

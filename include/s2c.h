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
 *
 * Split of the work (north_star subsystems):
 *   host   (1) SAM/SAM.gz parse, the reference's error classes in file order, the packed
 *              read batch: CIGAR tokens, 2-bit base planes + a non-ACGT plane in QUERY
 *              order, POS / reference as a global coordinate, pieces bucketed by their
 *              start word (32 positions), and the tile plan (sizes and capacities only).
 *   device (2) k_tile_dense / k_tile: parsecigar (:46-82) + the maxdel rule (:210) of every
 *              piece of the tile's window, staged in LDS (k_tile: layer by layer), its
 *              runs (seqout intervals mapped to query bases or to '-') counted by bit-sliced
 *              counters (:210-218), insertion columns (:276-294), vote for all thresholds
 *              (:232-253, :344-389) and the FASTA body bytes;
 *          (3) k_reads: the insertion events (:73-75, :221) hashed by (position, motif)
 *              into per-tile open-addressing tables with per-entry counts (:262-271), and
 *              the run records of the rare long pieces;
 *          (4) k_consensus: tiles whose depth or insertion layout exceeds one workgroup.
 */
#ifndef S2C_H
#define S2C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define S2C_ABI_VERSION 14

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
#define S2C_TILE_MAX   2048    /* positions per tile */

/* CIGAR token word (ops[]): length << 4 | opcode, opcodes in this order */
#define S2C_OP_M   0
#define S2C_OP_I   1
#define S2C_OP_D   2
#define S2C_OP_N   3
#define S2C_OP_S   4
#define S2C_OP_H   5
#define S2C_OP_P   6
#define S2C_OP_EQ  7
#define S2C_OP_X   8
#define S2C_OP_LEN_MAX 0x0FFFFFFFu

/* piece record pc[i] = {gpos, qh, opoff, slen | flags << 24}:
 *   gpos  global coordinate of seqout char ka (the piece's first position)
 *   qh    the read's first SEQ base = 16·qh in the base planes
 *   opoff the piece's op words are [pc[i].opoff, pc[i+1].opoff): prefix words (flags),
 *         then the read's CIGAR tokens (:58 regex matches, in order)
 *   slen  len(SEQ) (< 2^24)                                                             */
#define S2C_PF_X      0x01   /* SEQ holds non-ACGT chars: read the non-ACGT plane bx      */
#define S2C_PF_RANGE  0x02   /* prefix {ka, kb}: the piece is seqout[ka, kb) (else [0, len(seqout))) */
#define S2C_PF_INS    0x04   /* prefix {key0 lo, key0 hi, ref_off}: this piece emits its read's
                                insertion events; key0 = ref_off + POS-1 (int64), an event at
                                seqout index k has global key key0 + k, used when ≥ ref_off */
#define S2C_PF_LONG   0x08   /* span > the batch's window: reached through the tile long lists */
#define S2C_PF_RUNS   0x10   /* a long piece: k_reads writes its run records (the tile long lists read
                                them; short pieces are walked by the tile kernels themselves) */
#define S2C_PF_DASH   0x20   /* SEQ holds '-' chars (with S2C_PF_X): the maxdel rule (:210) counts
                                them from the planes; without it a read's SEQ adds no '-' */
#define S2C_PF_SIMPLE 0x40   /* one M / = / X token, no prefix words, not long, no '-' in SEQ: its
                                seqout is SEQ[0:take] (:64-69) and slen holds take = min(l, len(SEQ))
                                (every consumer's min(l, slen) is then take) */
#define S2C_PF_XFEW   0x80   /* (with S2C_PF_X) SEQ's non-ACGT chars are at most two 'N' (no '-'), at
                                SEQ offsets < 0xFFFF listed in px[piece] = off0 | off1 << 16 (0xFFFF:
                                none): the kernels take them from there instead of scanning the
                                non-ACGT plane */

/* run record (device-written by k_reads, parallel to ops[]): {gpos, len | kind << 27, qlo, qhi};
   a run (and a read's seqout) is < 2^27 positions: N skips of up to 134 Mb */
#define S2C_RUN_KSHIFT 27
#define S2C_RUN_EMPTY   0u
#define S2C_RUN_BASES   1u   /* seqout [gpos, gpos+len) = query bases [q, q+len) (q = qhi:qlo) */
#define S2C_RUN_DASH    2u   /* seqout '-' (D/N/P, counted: not maxdel-dropped) */
#define S2C_RUN_XBIT   0x04u /* (kind bits) BASES run of a read with non-ACGT chars */
#define S2C_RUN_DROP   0x08u /* (kind bits) the read's '-' are not counted (maxdel, :210) */
#define S2C_RUN_LONG   0x10u /* (kind bits) run of a long piece: skipped by the rs window */

/* tile record tiles[t][S2C_TILE_WORDS] */
#define S2C_TILE_WORDS   24  /* {a, b, ref, flags, boff, bcap, loff, lcap, cb0, ccap, lp0, lp1, nev,
                                 pf0, pf1, o0, o1, qw0, qw1, nl, ly0, 0, 0, 0}: the window's pieces
                                 [pf0, pf1) (short pieces starting in [a/32 - kwin, b/32)), their op
                                 slots [o0, o1) and base plane words [qw0, qw1); nl LAYERS of the
                                 window, copied for k_tile as layers ly0 .. ly0 + nl - 1 of the
                                 layered arrays (lly): layer l holds, from every start word s of the
                                 window, its short pieces [ps[s] + n_s*l/nl, ps[s] + n_s*(l+1)/nl)
                                 (n_s = ps[s+1] - ps[s]), in start-word order — one LDS chunk of
                                 k_tile (S2C_CHUNK_*); ly0 = S2C_LY_MAIN: one layer, the window read in
                                 place from the sorted arrays (pf0 .. qw1) */
#define S2C_LY_MAIN 0xFFFFFFFFu
#define S2C_LY_NONE 0xFFFFFFFEu   /* a dense tile whose layered windows were not built (s2c_batch_layers_mode) */
#define S2C_TILE_DEEP     1  /* several work items: counts summed in HBM, voted by k_consensus */
#define S2C_TILE_GENERAL  2  /* insertion layout beyond k_tile's LDS: voted by k_consensus */
#define S2C_TILE_DENSE    4  /* routed to k_tile_dense (one item, no insertion keys); its long list (lp[lp0, lp1)) holds
                                 piece indices, walked by the kernel; other tiles list run slots (k_reads) */
#define S2C_ITEM_WORDS    4  /* work item {tile, chunk, l0, l1}: the tile's layers [l0, l1) */
#define S2C_DWIN_WORDS   16  /* dense item's window {tile, a, b, cb0, lp0, lp1, pf0, pf1, o0, o1, qw0, qw1, dpc0, 0, 0, 0}:
                                the words of its tile record k_tile_dense needs, in item order (one
                                16-dword scalar load per tile instead of item → tile → record); dpc0 (ABI 12):
                                the first of its window's compact piece records (s2c_batch_arrays.dpc) */
/* k_tile_dense's compact piece records (ABI 12): one per piece of each dense item's window, in
   window order, 3 words {rs | qh' << 12 | nops << 25, oj | len(SEQ) << 13 | flags << 24, px}:
   rs = start position − 32·(first tile word) + 2048 (12 bits), qh' = qh − 2·qw0 (13 bits),
   nops = op slots of the piece (7 bits), oj = op slot − o0 (13 bits), len(SEQ) (11 bits), the
   piece's flags and its px word.  A tile whose window holds a piece beyond these fields
   (len(SEQ) > S2C_DPC_SLEN_MAX, more than S2C_DPC_NOPS_MAX op slots, kwin > 64) is not dense. */
#define S2C_DPC_WORDS     3
#define S2C_DPC_SLEN_MAX  2047
#define S2C_DPC_NOPS_MAX  127
#define S2C_EPI_KEYS    256  /* insertion keys per tile k_tile's epilogue holds in LDS */
/* insertion columns per tile k_tile's epilogue holds in LDS, by words per tile */
#define S2C_LDS_COLS(nwp) ((nwp) <= 16 ? 640 : ((nwp) == 32 ? 448 : 192))
#define S2C_DENSE_LDS 32768  /* bytes of LDS a dense tile's window may take (one wave per tile) */
/* LDS bytes of a dense tile's window of ns op slots and nq base plane words: op words and
   planes {p0, p1} (each 16-byte aligned with 16 bytes of slack: the 16-byte LDS-DMA starts
   at the boundary below the source), run records, the walk's queues (64 entries per wave and
   walk iteration: ≤ pieces + 128).  Device arrays must be
   readable up to their end rounded up to 16 bytes. */
#define S2C_DENSE_BYTES(ns, nq) (((4 * (ns) + 30) & ~15) + ((8 * (nq) + 30) & ~15) + ((12 * (ns) + 1024 + 15) & ~15))
/* the dense kernel's dynamic LDS is at least this: after the count its two waves' counter
   exchange (8,320 bytes each) reuses the window's LDS — the host's occupancy plan counts it */
#define S2C_DENSE_MIN_LDS 16640
#define S2C_DENSE_QW   4096  /* base plane words of a dense tile's window (17-bit query offsets) */
/* k_tile's LDS chunk (one per wave): one layer of a tile window, contiguous in the layered arrays: its
   piece records, op words, base planes
   {p0, p1} through the word after its last base (funnel shift) and non-ACGT words — caps
   per layer — and its run records (= op slots), per 32-position word and counting lane <=
   S2C_CHUNK_LANE_RECS * lanes per word of a wave, 64 / words per tile (8-bit counters).  A work item's run records per
   word are <= S2C_ITEM_RECS (its u16 histogram). */
#define S2C_CHUNK_PIECES     128
#define S2C_CHUNK_QBYTES    4096
/* a layer's base-plane bytes in k_tile<nwp, wq> (nwp: the tile's 32-position words, wq: the
   walk-queue instantiation, s2c_batch_info walk_queue as planned): 4,352 for tiles of <= 512
   positions (against 4,096: fewer layers, each one's DMA round trips and barriers saved; C3
   -2.2 %, C4 -3.4 % at 4,320; 4,608 no better), the base for wider ones; every k_tile<16>
   stays under 53,536 LDS bytes, the largest share measured to keep 3 workgroups per CU.  The
   non-ACGT words of a layer <= half of it.  (wq: kept in the signature — the host cuts the
   layers for the instantiation it plans, and a shard keeps that one.) */
#define S2C_CHUNK_QBYTES_OF(nwp, wq) ((void)(wq), (nwp) <= 16 ? 4352 : S2C_CHUNK_QBYTES)
#define S2C_CHUNK_XBYTES    2048
#define S2C_CHUNK_OBYTES    1024
#define S2C_CHUNK_RECS       192
#define S2C_CHUNK_LANE_RECS  248
#define S2C_CHUNK_SEGS       128
#define S2C_ITEM_RECS      60000
#define S2C_SHORT_MOTIF  16  /* motifs up to this length are hashed inline (3-bit codes) */
#define S2C_CODE_FILL     0  /* internal vote char of a fill position */
#define S2C_CODE_ERR   0xFF  /* vote char where the vote hit a missing amb key (:367) */

/* ======================================================================================
 * Host side: SAM/SAM.gz parser → packed read batch          (replaces :147-228, :284-294)
 * ======================================================================================
 * The parser reproduces the reference's record handling and error classes exactly
 * (header pass :149-172, record filter :195, RNAME/POS :200-201, CIGAR tokens :58-59, the
 * index/symbol checks of :211-218 in file order, insertion checks :284-294) and emits the
 * packed batch.  It does NOT expand CIGARs: runs, '-' and insertion grouping are device
 * work (k_reads).
 */
typedef struct s2c_parser s2c_parser;
typedef struct s2c_batch  s2c_batch;

/* maxdel_active = 0 reproduces Python 2's `int <= str` when -d is given (:102,:210). */
int  s2c_parser_new(int maxdel_active, int64_t maxdel, s2c_parser **out);
/* Feed raw SAM text (any chunking; lines may straddle calls). */
int  s2c_parser_feed(s2c_parser *p, const char *buf, size_t len);
/* The header is over (its lines fed, ending in '\n'): a later '@' line is a body line that
 * the read pass skips (:195), never an @SQ (:149-172) — for parsers fed the header and then
 * a block from the middle of the file (sam2consensus_amd/dparse.py). */
int  s2c_parser_end_header(s2c_parser *p);
/* Parse a whole file; ".gz" suffix → zlib (:111-114).  Read in bounded windows. */
int  s2c_parser_feed_file(s2c_parser *p, const char *path);
/* The same byte source as a stream, for callers that feed blocks (streamed batches): plain,
 * gzip, or BGZF inflated block-parallel on the host threads (:111-114).  read fills dst up to
 * cap bytes (fewer only at the end; *n = 0 once the stream is over). */
typedef struct s2c_reader s2c_reader;
int  s2c_reader_open(const char *path, s2c_reader **out);
int  s2c_reader_read(s2c_reader *r, void *dst, size_t cap, size_t *n);
void s2c_reader_free(s2c_reader *r);
/* End of input: reformat-phase checks (:284-294), global layout, bucketing, tile plan. */
int  s2c_parser_finish(s2c_parser *p, s2c_batch **out);
void s2c_parser_free(s2c_parser *p);

/* Streamed batches over coordinate-sorted input (bounded host memory; the reference reads
 * the whole file first, :185-228, so this has no reference counterpart — its outputs
 * are the same bytes).  A driver (sam2consensus_amd/stream.py) feeds blocks, takes a
 * snapshot, runs the tiles every later read must start after (s2c_batch_shard), and
 * retains only the reads that reach the tiles not yet run.
 *   set_tile_width: the same tiles in every snapshot (0 = plan from depth; else a multiple
 *                   of 64 in [64, 2048]).
 *   snapshot:       the batch of all reads held (no end-of-input flush; the parser goes on).
 *   retain:         drop the reads that change no global position >= gmin.
 *   stream_state:   [0] a read parsed after a retain reaches below its gmin (not sorted:
 *                   the driver falls back to one batch), [1] [2] reference index and POS-1
 *                   of the last mapped read (-1 if none), [3] reads held. */
int  s2c_parser_set_tile_width(s2c_parser *p, int64_t width);
int  s2c_parser_snapshot(s2c_parser *p, s2c_batch **out);
/* (ABI 13) s2c_parser_snapshot planning only the tiles from t_from (a streamed batch's first
 * tile) through the tile of the held reads' last position (info.plan_t0 / plan_t1); the
 * other tiles get no work items.  Needs a tile width. */
int  s2c_parser_snapshot_from(s2c_parser *p, int64_t t_from, s2c_batch **out);
int  s2c_parser_retain(s2c_parser *p, int64_t gmin);
int  s2c_parser_stream_state(const s2c_parser *p, int64_t *state);
/* Pipelined snapshots: detach moves every read held into a new parser *out (the reference
 * table, settings and stream state copied; the partial last line stays in p), so one thread
 * can snapshot / retain *out while another goes on feeding p; attach then puts out's reads
 * (the retained ones) back in front of the reads fed since, takes its stream state and
 * frees it.  Between the two, p and out share no data.  *out takes no input (feed /
 * feed_file / end_header: S2C_ERR_ARG). */
int  s2c_parser_detach(s2c_parser *p, s2c_parser **out);
int  s2c_parser_attach(s2c_parser *p, s2c_parser *det);
/* Unsorted input (counts added to running totals batch by batch, s2c_accumulate): keep
 * only the reads with insertion events, their counted ranges cleared; the last batch
 * (s2c_parser_finish) then holds every insertion event of the file. */
int  s2c_parser_retain_events(s2c_parser *p);

/* Distributed parse for the multi-GPU CLI (sam2consensus_amd/dparse.py; the reference
 * parses on one core, :185-228).  Each rank parses its blocks of the file with its own
 * parser, routes every read to the ranks whose tile range it can change, and plans its
 * sub-batch from the reads it receives.  Each call first parses a pending last line.
 *   pos_weights: w[g >> shift] += len(counted seqout) of each read held, g = the first
 *                global position it can change (n entries).
 *   checks:      per reference r, bad[2r] = an insertion motif base outside -ACGNT (:287),
 *                bad[2r + 1] = an insertion key outside the coverage list (:294).
 *   counters:    {header_lines, lines_total, reads_mapped, aligned_bases} of this parser.
 *   pack:        the reads held that can change a global position in [g0, g1) (tokens,
 *                planes, events; no line counters) into a blob of *len bytes, kept by the
 *                parser until the next pack; blob_copy copies it out.
 *   unpack:      append a blob's reads (read order = order of the unpack calls). */
int  s2c_parser_pos_weights(s2c_parser *p, int64_t shift, int64_t *w, int64_t n);
int  s2c_parser_checks(s2c_parser *p, uint8_t *bad, int64_t n_refs);
int  s2c_parser_counters(s2c_parser *p, int64_t *out);
/* Where the read pass stands, also after a read-pass error (the reference prints its header
   line and progress lines up to the failing line, :182, :224-225, before raising):
   out[5] = {header ended (0/1), references, header lines, lines read (through the failing
   line), error code of the read pass (0: none)}. */
int  s2c_parser_progress(const s2c_parser *p, int64_t *out);

/* (ABI 14) The compute units of the device the batches will run on (the grid shaping of the
 * deep tiles' work items, s2c_parser_finish): 256 (MI355X) until set; a partitioned device
 * mode or another part names its own.  Process-wide; it changes how work is split, never a
 * result. */
int  s2c_plan_set_cus(int64_t cus);

/* FASTA body assembly (:394-418): dst = raw[starts[0] : +lens[0]] ++ raw[starts[1] : +lens[1]]
   ++ ... (n blocks; dst holds their total length), copied on the host threads.  The tiles'
   body slots after the D2H copy of the device output, in [threshold][tile] order.  A block
   outside raw's raw_len bytes is refused (S2C_ERR_ARG) before anything is copied. */
int  s2c_gather_bodies(const uint8_t *raw, int64_t raw_len, const int64_t *starts, const int64_t *lens, int64_t n,
                       uint8_t *dst);
/* n bytes src → dst on the host threads (the host side of a batch's H2D staging). */
int  s2c_copy_bytes(void *dst, const void *src, int64_t n);
int  s2c_parser_pack(s2c_parser *p, int64_t g0, int64_t g1, size_t *len);
int  s2c_parser_blob_copy(const s2c_parser *p, void *dst, size_t cap);
int  s2c_parser_unpack(s2c_parser *p, const void *blob, size_t len);

typedef struct {
    int64_t n_refs;            /* @SQ references (:160-169) */
    int64_t total_len;         /* Σ LN over refs (real positions) */
    int64_t padded_len;        /* global coordinate extent (refs aligned to S2C_POS_ALIGN) */
    int64_t header_lines;      /* :158 */
    int64_t lines_total;       /* all lines seen (:194 counts from -header_lines) */
    int64_t reads_mapped;      /* records passing :195 */
    int64_t aligned_bases;     /* A = Σ len(seqout) over mapped reads (the metric's unit) */
    int64_t query_bases;       /* Q = M/=/X + I bases consumed (B_alg 0.5·Q) */
    int64_t n_pieces;          /* pieces (a read, or its two parts around the POS<=0 wrap, :212) */
    int64_t n_ops;             /* op words (prefix words + CIGAR tokens) = run slots */
    int64_t n_tokens;          /* CIGAR tokens other than S/H (B_alg 4·K) */
    int64_t n_qwords;          /* u32 words per base plane */
    int64_t n_words;           /* padded_len / 32 */
    int64_t n_tiles;           /* tiles (consensus / body blocks, never straddle a reference) */
    int64_t n_items;           /* k_tile work items (non-dense tiles; deep tiles have several) */
    int64_t n_dense;           /* dense tiles (k_tile_dense; k_tile when len(-f) != 1) */
    int64_t n_deep;            /* tiles voted by k_consensus (deep or general) */
    int64_t n_long;            /* long-list entries (tile, run slot of a long piece) */
    int64_t n_rlist;           /* pieces k_reads walks (the counts-only modes) */
    int64_t kwin;              /* window: a short piece spans <= kwin + 1 words */
    int64_t tile_max;          /* max positions of any tile (<= 2048) */
    int64_t chunk;             /* candidate run slots per word per work item */
    int64_t n_ins;             /* insertion events kept (key in [0, LN), non-empty motif) */
    int64_t n_ins_bases;       /* Σ motif lengths */
    int64_t n_bkt;             /* hash-table slots over all tiles (Σ bcap) */
    int64_t n_lng;             /* long-motif event slots over all tiles (Σ lcap) */
    int64_t n_cols;            /* insertion column slots over all tiles (Σ ccap ≥ Σ columns) */
    int64_t runs_max;          /* most run slots any tile's window holds */
    int64_t dense_lds;         /* most LDS bytes any dense tile's window takes (S2C_DENSE_BYTES) */
    int64_t n_layers;          /* layers of the non-dense tiles' windows (lly) */
    int64_t n_lpieces;         /* pieces of the layered arrays (lpc) */
    int64_t n_lops;            /* op words of the layered arrays (lops) */
    int64_t n_lqwords;         /* plane words of the layered arrays (lbq, lbx) */
    int64_t layers_dense;      /* 1: the dense tiles' layered windows are built too (counts-only modes) */
    int64_t layers_built;      /* 1: the layered windows (lly ..., tile word 20) are built (s2c_batch_layers*);
                                  0 for a fresh snapshot or shard */
    int64_t n_dpc;             /* compact piece records of the dense items' windows (ABI 12) */
    int64_t word_lo, word_hi;  /* (ABI 13) the per-word entries any launch reads: rs / ps [word_lo, word_hi],
                                  wtile [word_lo, word_hi) — 0 and n_words for a whole batch, a shard's
                                  own words and its windows' lookback for s2c_batch_shard; the device
                                  copies (s2c_dev rs / ps / wtile) hold only those entries */
    int64_t n_walked;          /* (ABI 13) pieces walked op by op (neither S2C_PF_SIMPLE nor S2C_PF_LONG) */
    int64_t walk_queue;        /* (ABI 13) 1: n_walked >= n_pieces / 32 and tile_max <= 1024 — k_tile queues
                                  those pieces for its walk (a variant of the kernel) */
    int64_t tile_events;       /* (ABI 13) 1 (with walk_queue; S2C_NO_TILE_EVENTS unset): k_tile records its
                                  finish tiles' short-motif insertion events itself — s2c_reads leaves
                                  them (rlist's run prefix n_rlist_run was cut for it) */
    int64_t n_rlist_run;       /* (ABI 13) the first n_rlist_run of rlist: the pieces s2c_reads walks */
    int64_t plan_t0, plan_t1;  /* (ABI 13) the tiles with a window, layers and work items: [0, n_tiles), or
                                  for s2c_parser_snapshot_from(p, t_from) [t_from, the tile of the held
                                  reads' last position] — the others keep bounds and insertion capacities */
} s2c_batch_info;

typedef struct {               /* host pointers into the batch (valid until s2c_batch_free) */
    const int64_t  *ref_len;   /* [n_refs] */
    const int64_t  *ref_off;   /* [n_refs] global coordinate of position 0 */
    const int64_t  *ref_cov_reads; /* [n_refs] pieces with a counted char (0 ⇒ Σcov == 0, :334-341) */
    const uint32_t *pc;        /* [n_pieces+1][4] pieces sorted by start word (+ sentinel {0, qh end, n_ops, 0}):
                                  piece k's planes are query bases [16 qh_k, 16 qh_{k+1}) */
    const uint32_t *ops;       /* [n_ops] op words: prefix words, CIGAR tokens */
    const uint32_t *bq;        /* [n_qwords][2] base planes {p0, p1} of 32 query bases:
                                  A 00, C 01, G 10, T 11 (p1 p0); non-ACGT chars 00 */
    const uint32_t *bx;        /* [n_qwords] 1 = non-ACGT char: 'N' (p0 0) or '-' (p0 1) */
    const uint32_t *rs;        /* [n_words+1] run slots of the pieces starting in words [W0, W1)
                                  are [rs[W0], rs[W1]); a run covering word W belongs to a short
                                  piece starting in [W-kwin, W] or is listed in lp */
    const uint32_t *tiles;     /* [n_tiles][S2C_TILE_WORDS] */
    const uint32_t *items;     /* [n_items][S2C_ITEM_WORDS] */
    const uint32_t *dense;     /* [n_dense][S2C_ITEM_WORDS] items of the dense tiles */
    const uint32_t *deep;      /* [n_deep] tiles k_consensus votes */
    const uint32_t *rlist;     /* [n_rlist] pieces k_reads walks (PF_RUNS or PF_INS) */
    const uint32_t *lp;        /* [n_long] run slots of the long pieces overlapping each tile:
                                  tile t's are lp[tiles[t].lp0 .. tiles[t].lp1) */
    const uint32_t *wtile;     /* [n_words] tile of each 32-position word (0xFFFFFFFF: padding) */
    const uint32_t *ps;        /* [n_words+1] pieces starting in words [W0, W1) are [ps[W0], ps[W1]) */
    /* layered windows of the non-dense tiles (k_tile): tile t's layer l is layer
       tiles[t].ly0 + l; layer L = pieces [lly[L].x, lly[L+1].x) of lpc, op words
       [lly[L].y, lly[L+1].y) of lops, planes from half-word lly[L].z (16-base units) of lbq /
       lbx; a piece record's qh and opoff index these arrays */
    const uint32_t *lly;       /* [n_layers+1][4] {piece, op word, plane half-word, 0} */
    const uint32_t *lpc;       /* [n_lpieces+1][4] */
    const uint32_t *lops;      /* [n_lops] */
    const uint32_t *lbq;       /* [n_lqwords][2] */
    const uint32_t *lbx;       /* [n_lqwords] */
    const uint32_t *px;        /* [n_pieces] the non-ACGT SEQ offsets of S2C_PF_XFEW pieces (else 0xFFFFFFFF) */
    const uint32_t *dwin;      /* [n_dense][S2C_DWIN_WORDS] the dense items' windows */
    const uint32_t *lpx;       /* [n_lpieces] px of the layered pieces (ABI 11: k_tile takes the 'N' of
                                  S2C_PF_XFEW pieces from here instead of scanning the non-ACGT plane) */
    const uint32_t *dpc;       /* [n_dpc][S2C_DPC_WORDS] compact piece records of the dense items' windows (ABI 12) */
} s2c_batch_arrays;

/* Build the batch's layered windows (s2c_batch_arrays lly .. lbx, tile word 20) if not yet
 * built: required before a batch's arrays go to the device; snapshots that are only cut into
 * shards never pay for them (each shard builds its own).  s2c_batch_layers builds them for
 * every tile; s2c_batch_layers_mode(b, 0) skips the dense tiles (k_tile_dense reads their
 * windows in place; tile word 20 = S2C_LY_NONE), which s2c_run needs and the counts-only
 * modes refuse — (b, 1) afterwards rebuilds them all. */
int  s2c_batch_layers(s2c_batch *b);
int  s2c_batch_layers_mode(s2c_batch *b, int with_dense);
int  s2c_batch_info_get(const s2c_batch *b, s2c_batch_info *out);
int  s2c_batch_arrays_get(const s2c_batch *b, s2c_batch_arrays *out);
/* The sub-batch of tiles [t0, t1) for one GPU of a multi-GPU run (positions keep their
 * global coordinates; free it with s2c_batch_free). */
int  s2c_batch_shard(const s2c_batch *b, int64_t t0, int64_t t1, s2c_batch **out);
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
    const uint32_t *pc, *ops, *bq, *bx, *rs;
    const uint32_t *tiles, *items, *dense, *deep, *lp, *wtile, *rlist, *ps;
    const uint32_t *lly, *lpc, *lops, *lbq, *lbx;   /* layered windows (s2c_batch_arrays) */
    int64_t n_pieces, n_ops, n_qwords, n_tiles, n_items, n_dense, n_deep, padded_len, chunk, n_rlist, dense_lds;
    int64_t n_layers, n_lpieces, n_lops, n_lqwords;
    int32_t kwin, tile_max;

    /* ---- options (:102, :117-138) ---- */
    int32_t  maxdel_active;    /* 0 when -d was given (Python 2 int <= str, :210) */
    int32_t  maxdel;           /* 150 (:102) */
    const double *thresholds;  /* [T] device copy of -c values, CLI order */
    int32_t  n_thr;
    int32_t  min_depth;        /* -m */
    int32_t  fill_len;         /* len(-f) */
    int32_t  fill_nondash;     /* count of chars != '-' in -f */
    const uint8_t *fill;       /* [fill_len] device copy of -f bytes */

    /* ---- workspace (caller allocates; sizes from s2c_workspace_sizes) ---- */
    uint32_t *runs;            /* [n_ops][4] run records (k_reads) */
    uint32_t *ibkt;            /* [n_bkt][4] per-tile hash tables {key lo, key hi, count, 0}; zero
                                  before the first run, left zero by every run */
    uint32_t *ilong;           /* [n_lng][4] long-motif events {pos, len, q lo, q hi} */
    uint32_t *ilong_n;         /* [n_tiles] long-motif events per tile (zero, left zero) */
    uint32_t *counts;          /* [6][padded_len] counts of deep / general tiles (SoA by symbol); zero
                                  before the first s2c_run / s2c_pileup, left zero by s2c_consensus
                                  (round 6: no zeroing launch per run) — s2c_pileup_counts leaves
                                  them filled, so zero them again before the next s2c_run */
    uint32_t *ins_cols;        /* [n_cols][6] column counts of general tiles */
    uint8_t  *ins_chr;         /* [T][n_cols] column vote chars of general tiles */
    int64_t   n_cols;

    /* ---- outputs ---- */
    uint64_t *tile_stats;      /* [T][n_tiles][4] {sumcov, len, nondash, vote_errors} per tile
                                  (:352-397; summed per reference by the host) */
    uint64_t *blk_len;         /* [T][n_tiles] FASTA body bytes of (t, tile) */
    uint8_t  *out;             /* FASTA bodies (:350-389): tile (t, tile) at
                                  t·(F·padded_len + n_cols) + F·a + cb0, F = max(1, len(fill)),
                                  a = the tile's first position, cb0 its column slot base;
                                  blk_len bytes each.  A reference's body for threshold t is its
                                  tiles' pieces in order. */
    int64_t   out_cap;         /* ≥ T·(F·padded_len + n_cols) */
    int64_t   layers_dense;    /* the batch's info.layers_dense: s2c_pileup_counts and s2c_accumulate
                                  run dense tiles through k_tile and refuse a batch without them */
    const uint32_t *px;        /* [n_pieces] s2c_batch_arrays.px (ABI 10) */
    int64_t   layers_built;    /* the batch's info.layers_built: every launch with work items refuses 0 */
    const uint32_t *dwin;      /* [n_dense][S2C_DWIN_WORDS] s2c_batch_arrays.dwin, filtered like dense */
    const uint32_t *lpx;       /* [n_lpieces] s2c_batch_arrays.lpx (ABI 11; required with n_layers > 0) */
    const uint32_t *dpc;       /* [n_dpc][S2C_DPC_WORDS] s2c_batch_arrays.dpc (ABI 12; required with n_dense > 0) */
    int64_t   walk_queue;         /* (ABI 13) the batch's info.walk_queue (k_tile's variant) */
    int64_t   tile_events;        /* (ABI 13) the batch's info.tile_events (who records the finish tiles'
                                     events: must match the batch's rlist run prefix) */
    int64_t   n_rlist_run;        /* (ABI 13) the batch's info.n_rlist_run: s2c_reads walks rlist[0, n_rlist_run) */
    int64_t   word_lo, word_hi;   /* (ABI 13) the batch's info.word_lo / word_hi: rs and ps point at entry
                                     word_lo of s2c_batch_arrays rs / ps ([word_lo, word_hi] copied),
                                     wtile at entry word_lo ([word_lo, word_hi) copied) */
} s2c_dev;

/* Sizes (bytes) of every workspace / output buffer for a batch and T thresholds. */
typedef struct {
    int64_t runs, ibkt, ilong, ilong_n, counts, ins_cols, ins_chr, blk_len, tile_stats;
    int64_t out_per_fill, out_fixed;   /* out bytes = out_per_fill·max(1, len(fill)) + out_fixed */
} s2c_ws_sizes;
int s2c_workspace_sizes(const s2c_batch_info *info, int32_t n_thr, s2c_ws_sizes *out);

/* Stage order (s2c_run): s2c_reads → s2c_pileup → s2c_consensus, one stream.
 * (3) insertion events of the pieces that emit them → per-tile hash tables; parsecigar +
 *     maxdel → run records of the long pieces (the tile long lists)
 *                                                           (:46-82, :210, :221, :262-271) */
int s2c_reads(const s2c_dev *d, void *stream);
/* (2)-(4) per tile: parsecigar + maxdel of its window's pieces and pileup of their runs,
 * insertion columns, vote (all thresholds, IUPAC,
 * min-depth/fill), tile statistics and FASTA body bytes; deep / general tiles leave their
 * counts in HBM                         (:210-218, :232-253, :256-311, :344-397) */
int s2c_pileup(const s2c_dev *d, void *stream);
/* (3)+(4) and the bodies of deep / general tiles               (:232-253, :256-311, :344-397) */
int s2c_consensus(const s2c_dev *d, void *stream);
/* all three, in order, on one stream (graph-capturable: no allocation, no sync) */
int s2c_run(const s2c_dev *d, void *stream);

/* (ABI 14) FASTA body assembly on the device (:394-418; replaces the host gather of the
 * output's body slots, s2c_gather_bodies): dst[offs[i], offs[i+1]) = out[starts[i], +len)
 * with len = offs[i+1] - offs[i], for n blocks in [threshold][tile] order — out = s2c_dev.out,
 * starts[i] = the block's slot t·(F·padded_len + n_cols) + F·a + cb0, offs = the exclusive
 * prefix sum of the blocks' blk_len (offs[0] = 0, n + 1 entries).  All pointers are device
 * pointers (int64 arrays); a block reaching past out_len is skipped.  Asynchronous on stream. */
int s2c_gather_bodies_dev(const uint8_t *out, int64_t out_len, const int64_t *starts, const int64_t *offs,
                          int64_t n, uint8_t *dst, void *stream);

/* Diagnostics (tests only, not part of the product path): k_reads over every piece, then
 * every tile's counts stored to d->counts ([6][padded_len] u32) and no vote. */
int s2c_pileup_counts(const s2c_dev *d, void *stream);
/* Streamed batches of unsorted input: run records of every piece, then every tile's counts
 * ADDED to d->counts (the running totals [6][padded_len], zeroed by the caller before the
 * first batch; no k_prep).  keep_tables = 0: the batch's insertion tables are cleared;
 * 1 (the last batch): kept for s2c_consensus, which the caller runs with d->deep listing
 * every tile so all of them are voted from the totals. */
int s2c_accumulate(const s2c_dev *d, int keep_tables, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* S2C_H */

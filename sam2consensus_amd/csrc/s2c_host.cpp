// s2c_host.cpp — host side of libs2c.so: SAM/SAM.gz parser → packed read batch → tile plan.
//
// Reproduces the reference's record handling (zoujiayun/sam2consensus v2.1,
// sam2consensus.py) exactly, including its Python-2 quirks:
//   header pass            :149-172   (leading '@' lines, @SQ SN:/LN: parse)
//   record filter          :195       (line[0] != '@' and field[5] != "*"; FLAG ignored)
//   RNAME / POS            :200-201   (str.split()[0], int() - 1)
//   CIGAR tokens           :58-59     (regex matches; junk skipped)
//   the read pass's errors :195,:200,:201,:206,:212,:217,:221 in file order, and the
//                          reformat phase's :287 / :294 per reference
// and emits north_star subsystem (1), the packed batch: per read its CIGAR tokens and
// its SEQ as 2-bit base planes plus a non-ACGT plane, in QUERY order; pieces (a read,
// or its two parts around the POS<=0 wrap) bucketed by their start word; the tile plan.
// The CIGAR is NOT expanded here: seqout, the maxdel drop (:210) applied to the counts,
// and the insertion motif aggregation (:262-294) are computed on the device (k_reads).
// The host walks the tokens only to raise the reference's errors in file order (which
// needs the seqout length, the '-' count and the counted range) and to size the plan.
#include "../../include/s2c.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <pthread.h>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <string>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;
int s2c_set_error(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
extern "C" const char *s2c_last_error(void) { return g_err.c_str(); }
// No C++ exception crosses the C-ABI: an allocation failure (e.g. a corrupt input's sizes)
// or any other exception becomes an error code.
template <class F>
int s2c_guarded(F &&f) {
    try {
        return f();
    } catch (const std::bad_alloc &) {
        return s2c_set_error(S2C_ERR_LIMIT, "out of host memory");
    } catch (const std::length_error &e) {
        return s2c_set_error(S2C_ERR_LIMIT, std::string("size beyond this build's limits: ") + e.what());
    } catch (const std::exception &e) {
        return s2c_set_error(S2C_ERR_IO, std::string("host exception: ") + e.what());
    }
}
extern "C" int s2c_abi_version(void) { return S2C_ABI_VERSION; }

// ------------------------------------------------------------------ plan knobs
// Overrides of the batch plan's shape (tile widths, deep-tile items, dense / event routing)
// are measurement tools, not options: they are read only when S2C_DEBUG_PLAN is set, so the
// product plan is the same whatever else the environment holds.
static const char *plan_env(const char *name) {
    static const bool debug = getenv("S2C_DEBUG_PLAN") != nullptr;
    return debug ? getenv(name) : nullptr;
}
// The device's compute units (grid shaping of k_tile's launches; s2c_plan_set_cus) — the
// MI355X's 256 until the caller names its device's.
static std::atomic<int64_t> g_plan_cus{256};
extern "C" int s2c_plan_set_cus(int64_t cus) {
    if (cus <= 0 || cus > 4096) return s2c_set_error(S2C_ERR_ARG, "compute units outside (0, 4096]");
    g_plan_cus.store(cus);
    return S2C_OK;
}

// ------------------------------------------------------------------ host worker pools
// Persistent host threads for the parse windows and the plan's parallel loops.  A thread
// made per window (16 per 64 MB block of a streamed file) maps its stack while the other
// threads first-touch their chunks' buffers; those page faults and the mapping serialise on
// the process's memory map, and the last thread of a window started 25-35 ms after the
// first (S2C_HOST_TIMING).  A pool's threads wait on a condition variable between runs.
// One run at a time per pool: a run asked for while the pool is busy (another thread's run,
// or a run nested in one) gets threads of its own, as before.  A forked child makes new pools.
namespace {
class WorkerPool {
  public:
    // f(t) for t in [0, nt): t = 0 on the calling thread, the others on the pool's
    // (an exception of any f(t) is rethrown here once every thread is done with the run)
    template <class F>
    void run(int nt, F &&f) {
        if (nt <= 1) { f(0); return; }
        std::exception_ptr err;
        std::mutex em;
        auto safe = [&](int t) {
            try {
                f(t);
            } catch (...) {
                std::lock_guard<std::mutex> lk(em);
                if (!err) err = std::current_exception();
            }
        };
        // a run nested in this thread's own run of the pool must not try_lock the mutex it
        // holds (undefined behaviour): it is told apart by the owner's thread id
        std::unique_lock<std::mutex> rl;
        if (owner_.load(std::memory_order_relaxed) != std::this_thread::get_id()) rl = std::unique_lock<std::mutex>(run_m_, std::try_to_lock);
        if (!rl.owns_lock()) {   // busy: threads of its own
            std::vector<std::thread> th;
            for (int t = 1; t < nt; t++) th.emplace_back([&safe, t] { safe(t); });
            safe(0);
            for (auto &x : th) x.join();
            if (err) std::rethrow_exception(err);
            return;
        }
        const std::function<void(int)> job = [&safe](int t) { safe(t); };
        owner_.store(std::this_thread::get_id(), std::memory_order_relaxed);
        struct Release {
            std::atomic<std::thread::id> &o;
            ~Release() { o.store(std::thread::id(), std::memory_order_relaxed); }
        } release{owner_};
        {
            std::lock_guard<std::mutex> lk(m_);
            while ((int)n_threads_ < nt - 1) {
                const int t = n_threads_ + 1;
                std::thread([this, t] { loop(t); }).detach();
                n_threads_++;
            }
            job_ = &job;
            want_ = nt;
            left_ = nt - 1;
            gen_++;
        }
        go_.notify_all();
        safe(0);
        {
            std::unique_lock<std::mutex> lk(m_);
            done_.wait(lk, [&] { return left_ == 0; });
            job_ = nullptr;
        }
        if (err) std::rethrow_exception(err);
    }
    // the pool of this process (pools are never destroyed: their threads may outlive main).
    // fork: the registry's mutex is held across the fork (pthread_atfork) and a forked child
    // forgets the parent's pools (their threads do not exist in it) and makes new ones
    static WorkerPool &get(int which) {
        static std::once_flag once;
        std::call_once(once, [] {
            pthread_atfork([] { reg_m().lock(); }, [] { reg_m().unlock(); }, [] {
                for (auto &q : reg()) q = nullptr;
                reg_m().unlock();
            });
        });
        std::lock_guard<std::mutex> lk(reg_m());
        WorkerPool *&q = reg()[which];
        if (!q) q = new WorkerPool();
        return *q;
    }

  private:
    static std::mutex &reg_m() {
        static std::mutex m;
        return m;
    }
    static WorkerPool *(&reg())[3] {
        static WorkerPool *pools[3] = {nullptr, nullptr, nullptr};
        return pools;
    }
    void loop(int t) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            go_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            if (t >= want_) continue;
            const std::function<void(int)> *j = job_;
            lk.unlock();
            (*j)(t);
            lk.lock();
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::mutex run_m_, m_;
    std::atomic<std::thread::id> owner_{};   // the thread running the pool's current run
    std::condition_variable go_, done_;
    const std::function<void(int)> *job_ = nullptr;
    uint64_t gen_ = 0;
    int want_ = 0, left_ = 0, n_threads_ = 0;
};
enum { POOL_PARSE = 0, POOL_PLAN = 1, POOL_IO = 2 };
}  // namespace

// ------------------------------------------------------------------ tables
namespace {
// SEQ char → 3-bit plane code x·4 + p1·2 + p0: A 0, C 1, G 2, T 3, N 4, '-' 5, other 7
constexpr uint8_t Q_N = 4, Q_DASH = 5, Q_BAD = 7;
struct QLut {
    uint8_t v[256];
    QLut() {
        memset(v, Q_BAD, sizeof(v));
        v[(uint8_t)'A'] = 0; v[(uint8_t)'C'] = 1; v[(uint8_t)'G'] = 2; v[(uint8_t)'T'] = 3;
        v[(uint8_t)'N'] = Q_N; v[(uint8_t)'-'] = Q_DASH;
    }
};
const QLut QL;

inline bool py2_ws(char c) {  // Python 2 str.split()/int() whitespace (C locale isspace)
    return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\x0b' || c == '\x0c';
}

// Python 2 int(str): whitespace, sign, decimal digits, whitespace.  Saturates at ±2^62
// (positions that large are out of range anyway and raise IndexError downstream).
bool py2_int(const char *s, size_t n, int64_t *out) {
    size_t i = 0;
    while (i < n && py2_ws(s[i])) i++;
    bool neg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
    size_t d0 = i;
    int64_t v = 0;
    const int64_t CAP = (int64_t)1 << 62;
    while (i < n && s[i] >= '0' && s[i] <= '9') {
        if (v < CAP) v = v * 10 + (s[i] - '0');
        if (v > CAP) v = CAP;
        i++;
    }
    if (i == d0) return false;
    while (i < n && py2_ws(s[i])) i++;
    if (i != n) return false;
    *out = neg ? -v : v;
    return true;
}

// first whitespace-delimited token (Python 2 str.split()[0])
bool py2_first_token(const char *s, size_t n, const char **tb, size_t *tl) {
    size_t i = 0;
    while (i < n && py2_ws(s[i])) i++;
    if (i == n) return false;
    size_t j = i;
    while (j < n && !py2_ws(s[j])) j++;
    *tb = s + i;
    *tl = j - i;
    return true;
}

// str.replace(pat, "") — Python's single left-to-right non-overlapping pass.
std::string py_remove(const char *s, size_t n, const char *pat) {
    size_t m = strlen(pat);
    std::string out;
    out.reserve(n);
    size_t i = 0;
    while (i < n) {
        if (i + m <= n && memcmp(s + i, pat, m) == 0) { i += m; continue; }
        out.push_back(s[i++]);
    }
    return out;
}

inline int opcode_of(char c) {
    switch (c) {
        case 'M': return S2C_OP_M;
        case 'I': return S2C_OP_I;
        case 'D': return S2C_OP_D;
        case 'N': return S2C_OP_N;
        case 'S': return S2C_OP_S;
        case 'H': return S2C_OP_H;
        case 'P': return S2C_OP_P;
        case '=': return S2C_OP_EQ;
        case 'X': return S2C_OP_X;
        default: return -1;
    }
}
inline bool op_bases(uint32_t op) { return op == S2C_OP_M || op == S2C_OP_EQ || op == S2C_OP_X; }
inline bool op_dash(uint32_t op) { return op == S2C_OP_D || op == S2C_OP_N || op == S2C_OP_P; }

// re.findall(r"(\d+)([MIDNSHPX=]{1})", cigar) (:58): a match is a maximal digit run
// immediately followed by an op letter; everything else is skipped.  Appends token words
// (len << 4 | opcode).
template <class V>
int tokenize_cigar(const char *s, size_t n, V &out, uint32_t *ntok) {
    size_t i = 0;
    uint32_t k = 0;
    while (i < n) {
        if (s[i] < '0' || s[i] > '9') { i++; continue; }
        size_t j = i;
        uint64_t v = 0;
        bool big = false;
        while (j < n && s[j] >= '0' && s[j] <= '9') {
            v = v * 10 + (uint64_t)(s[j] - '0');
            if (v > S2C_OP_LEN_MAX) { big = true; v = S2C_OP_LEN_MAX; }
            j++;
        }
        if (j < n) {
            const int oc = opcode_of(s[j]);
            if (oc >= 0) {
                if (big) return s2c_set_error(S2C_ERR_LIMIT, "CIGAR op length >= 2^28 not supported");
                out.push_back((uint32_t)(v << 4) | (uint32_t)oc);
                k++;
                i = j + 1;
                continue;
            }
        }
        i = j;
    }
    *ntok = k;
    return S2C_OK;
}
}  // namespace

// Allocator of the parser's and the batch's big arrays: default-initialising (resize() leaves
// the elements unwritten, so they are first touched by the threads that fill them, not by a
// serial zero-fill) and, from 4 MB on, backed by 2 MB-aligned anonymous mappings advised
// as transparent huge pages (512x fewer page faults for the GB-sized arrays of a batch).
constexpr size_t HUGE_PAGE = (size_t)2 << 20;
inline size_t huge_min() {   // S2C_HUGE_MIN_KB: the smallest array so mapped (default 4 MB)
    static const size_t m = [] { const char *e = getenv("S2C_HUGE_MIN_KB"); return e ? (size_t)atoll(e) << 10 : (size_t)4 << 20; }();
    return m;
}
inline bool huge_pages() {   // S2C_HUGEPAGES=0 turns the advice off
    static const bool on = [] { const char *e = getenv("S2C_HUGEPAGES"); return !e || atoi(e) != 0; }();
    return on;
}
template <class T>
struct uninit_alloc {
    using value_type = T;
    template <class U> struct rebind { using other = uninit_alloc<U>; };
    uninit_alloc() = default;
    template <class U> uninit_alloc(const uninit_alloc<U> &) {}
    static size_t map_len(size_t bytes) { return (bytes + HUGE_PAGE - 1) & ~(HUGE_PAGE - 1); }
    static bool poison() {   // S2C_MAP_POISON=1 (tests): every array starts as 0xA5 bytes, not zero pages
        static const bool on = getenv("S2C_MAP_POISON") != nullptr;
        return on;
    }
    T *allocate(size_t n) {
        T *p = allocate_raw(n);
        if (poison()) memset((void *)p, 0xA5, n * sizeof(T));
        return p;
    }
    T *allocate_raw(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < huge_min()) {
            void *q = ::operator new(bytes);
            return (T *)q;
        }
        const size_t len = map_len(bytes);
        void *raw = mmap(nullptr, len + HUGE_PAGE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (raw == MAP_FAILED) throw std::bad_alloc();
        const uintptr_t r = (uintptr_t)raw, a = (r + HUGE_PAGE - 1) & ~(uintptr_t)(HUGE_PAGE - 1);
        if (a > r) munmap(raw, a - r);                                      // the unaligned head
        if (r + len + HUGE_PAGE > a + len) munmap((void *)(a + len), r + len + HUGE_PAGE - (a + len));   // and tail
        if (huge_pages()) madvise((void *)a, len, MADV_HUGEPAGE);
        return (T *)a;
    }
    void deallocate(T *q, size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < huge_min()) ::operator delete((void *)q);
        else munmap((void *)q, map_len(bytes));
    }
    template <class U> void construct(U *q) noexcept { ::new ((void *)q) U; }
    template <class U, class... A> void construct(U *q, A &&...a) { ::new ((void *)q) U(std::forward<A>(a)...); }
    template <class U> bool operator==(const uninit_alloc<U> &) const { return true; }
    template <class U> bool operator!=(const uninit_alloc<U> &) const { return false; }
};
using u32buf = std::vector<uint32_t, uninit_alloc<uint32_t>>;

// ------------------------------------------------------------------ parser state
// One mapped read as the parser keeps it (file order).  Its tokens, base planes and
// insertion events live in the parse chunk that read it.
struct ReadRec {
    int64_t pos0;           // POS - 1 (:201)
    int64_t klen;           // len(seqout)
    int64_t kc0, kc1;       // counted seqout range [kc0, kc1); kc0 < 0: nothing counted
    uint64_t tok;           // first token (chunk toks)
    uint64_t q;             // first SEQ base (chunk planes, multiple of 16)
    uint32_t ref, ntok, slen, ev0, nev;
    uint8_t has_x, drop;
};
struct Event {              // insertion with a non-empty motif (:73-75), file order
    int64_t key;            // start_ref (:74), reference-relative
    uint64_t q;             // motif's first base (chunk planes)
    uint32_t ref, len, read;
};
struct Chunk {
    std::vector<ReadRec, uninit_alloc<ReadRec>> reads;
    u32buf toks;
    u32buf bq, bx;   // planes [k][2] and [k]; bases [0, nq)
    uint64_t nq = 0;
    uint64_t nz = 0;   // plane words [0, nz) initialised (pack_seq zeroes the words it reaches)
    std::vector<Event> ev;
    int64_t lines_total = 0, reads_mapped = 0, aligned = 0, qbases = 0, ntokens = 0;
    std::vector<uint32_t> sp;       // the current read's SEQ planes (seq_planes: 4 words per 32 chars)
    // an upper bound of its reads' extents (read_extent's hi): reference hb_ref, position
    // hb_pos in it (a read of an earlier reference ends below that reference's offset);
    // hb_pos < 0: no bound (no read yet, or a chunk made by s2c_parser_unpack)
    uint32_t hb_ref = 0;
    int64_t hb_pos = -1;
    void bound(uint32_t ref, int64_t pos0, int64_t klen, int64_t L) {
        const int64_t b = pos0 < 0 ? L : pos0 + klen;   // (a POS <= 0 wrap reaches the reference's end)
        if (hb_pos < 0 || ref > hb_ref) {
            hb_ref = ref;
            hb_pos = b;
        } else if (ref == hb_ref) {
            hb_pos = std::max(hb_pos, b);
        }
    }
};

struct s2c_parser {
    bool maxdel_active = true;
    int64_t maxdel = 150;
    bool in_header = true;
    int64_t header_lines = 0;
    std::vector<std::string> ref_names;
    std::vector<int64_t> ref_len;
    std::unordered_map<std::string, uint32_t> ref_idx;
    std::vector<std::unique_ptr<Chunk>> chunks;   // file order
    std::string carry;              // partial line of the streaming feed
    int err = S2C_OK;
    std::string errmsg;
    std::string last_name;
    int64_t last_ref = -1;
    // streamed batches (s2c_parser_retain): tile width of every reference, the first global
    // position not yet emitted, chunks [0, n_kept) hold the reads kept from earlier batches,
    // and whether a later read reached below the frontier (input not coordinate-sorted)
    int64_t tile_width = 0;
    int64_t frontier = 0;
    int64_t plan_from = -1;   // s2c_parser_snapshot_from: plan the tiles from here only (-1: all)
    size_t n_kept = 0;
    bool late = false;
    bool detached = false;   // made by s2c_parser_detach: snapshot / retain / attach only, no input
    std::vector<uint8_t> blob;   // s2c_parser_pack's output
    // frees the chunks a retain dropped, off the caller's path; one at a time (the next retain
    // joins the previous one first) and joined when the parser is freed
    std::thread freer;
    void free_later(std::vector<std::unique_ptr<Chunk>> v) {
        if (freer.joinable()) freer.join();
        freer = std::thread([](std::vector<std::unique_ptr<Chunk>> w) { w.clear(); }, std::move(v));
    }
    s2c_parser() { chunks.emplace_back(new Chunk()); }
    ~s2c_parser() {
        if (freer.joinable()) freer.join();
    }
};

struct s2c_batch {
    s2c_batch_info info{};
    std::vector<std::string> names;
    std::vector<int64_t> ref_len, ref_off, ref_reads;
    u32buf pc, ops, bq, bx;   // filled entirely by the emitters (resize: no zero-fill)
    std::vector<uint32_t> rs, tiles, items, dense, deep, lp, wtile, rlist, ps;
    std::vector<uint32_t> lly, lpc, lops, lbq, lbx;   // layered windows of the non-dense tiles
    std::vector<uint32_t> lpx;                        // [n_lpieces] px of the layered pieces
    bool layers = false;                               // built (s2c_batch_layers)
    u32buf kmin, kmax;   // host only: global key range of each piece's insertion events
    std::vector<uint8_t> lmot;   // host only: the piece emits a motif > S2C_SHORT_MOTIF bases
    u32buf px;           // [pieces] the non-ACGT SEQ offsets of S2C_PF_XFEW pieces (s2c.h)
    std::vector<uint32_t> dwin;   // [dense][S2C_DWIN_WORDS] the dense items' windows (s2c.h)
    u32buf dpc;                   // [n_dpc][S2C_DPC_WORDS] compact piece records of the dense windows (s2c.h)
};

static int perr(s2c_parser *p, int code, const std::string &msg) {
    p->err = code;
    p->errmsg = msg;
    return s2c_set_error(code, msg);
}

// @SQ line (:160-169): refname = f[1].replace("SN:","").split()[0]; LN = int(f[2].replace("LN:",""))
static int parse_sq(s2c_parser *p, const char *s, size_t n) {
    const char *f[3];
    size_t fl[3];
    int nf = 0;
    const char *cur = s, *end = s + n;
    while (nf < 3) {
        const char *t = (const char *)memchr(cur, '\t', end - cur);
        f[nf] = cur;
        if (!t) { fl[nf++] = end - cur; break; }
        fl[nf++] = t - cur;
        cur = t + 1;
    }
    if (nf < 2) return perr(p, S2C_ERR_INDEX, "IndexError: @SQ line has no field 1 (:163)");
    std::string f1 = py_remove(f[1], fl[1], "SN:");
    const char *tb;
    size_t tl;
    if (!py2_first_token(f1.data(), f1.size(), &tb, &tl))
        return perr(p, S2C_ERR_INDEX, "IndexError: empty @SQ SN (:163)");
    std::string name(tb, tl);
    if (nf < 3) return perr(p, S2C_ERR_INDEX, "IndexError: @SQ line has no field 2 (:164)");
    std::string f2 = py_remove(f[2], fl[2], "LN:");
    int64_t ln;
    if (!py2_int(f2.data(), f2.size(), &ln))
        return perr(p, S2C_ERR_VALUE, "ValueError: invalid @SQ LN '" + f2 + "' (:164)");
    if (ln < 0) ln = 0;  // range(negative) → empty list (:167)
    auto it = p->ref_idx.find(name);
    if (it == p->ref_idx.end()) {
        p->ref_idx.emplace(name, (uint32_t)p->ref_names.size());
        p->ref_names.push_back(name);
        p->ref_len.push_back(ln);
    } else {
        p->ref_len[it->second] = ln;  // duplicate @SQ re-initialises (:167-169)
    }
    return S2C_OK;
}

// Context shared by the record parsers of one parse (read-only reference table).
struct RefView {
    const std::unordered_map<std::string, uint32_t> *idx;
    const std::vector<int64_t> *len;
    bool maxdel_active;
    int64_t maxdel;
};

// SEQ → bit planes, 32 chars per word group {p0, p1, x, bad} (bit j = char 32·w + j; the QL
// code's bits x·4 + p1·2 + p0, and bad = a char outside "-ACGNT"); bits past slen are zero.
static void seq_planes_scalar(const char *seq, size_t slen, uint32_t *o) {
    for (size_t w = 0; w * 32 < slen; w++) {
        const size_t m = std::min<size_t>(slen - 32 * w, 32);
        uint32_t p0 = 0, p1 = 0, x = 0, bad = 0;
        for (size_t j = 0; j < m; j++) {
            const uint32_t v = QL.v[(uint8_t)seq[32 * w + j]];
            p0 |= (v & 1u) << j;
            p1 |= ((v >> 1) & 1u) << j;
            x |= ((v >> 2) & 1u) << j;
            bad |= (v == Q_BAD ? 1u : 0u) << j;
        }
        o[4 * w] = p0; o[4 * w + 1] = p1; o[4 * w + 2] = x; o[4 * w + 3] = bad;
    }
}
#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("avx2"))) static void seq_planes_avx2(const char *seq, size_t slen, uint32_t *o) {
    const __m256i A = _mm256_set1_epi8('A'), Cc = _mm256_set1_epi8('C'), Gg = _mm256_set1_epi8('G');
    const __m256i Tt = _mm256_set1_epi8('T'), Nn = _mm256_set1_epi8('N'), Dd = _mm256_set1_epi8('-');
    size_t w = 0;
    for (; 32 * w + 32 <= slen; w++) {
        const __m256i v = _mm256_loadu_si256((const __m256i *)(seq + 32 * w));
        const uint32_t a = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, A));
        const uint32_t c = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Cc));
        const uint32_t g = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Gg));
        const uint32_t t = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Tt));
        const uint32_t n = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Nn));
        const uint32_t d = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Dd));
        const uint32_t bad = ~(a | c | g | t | n | d);
        o[4 * w] = c | t | d | bad;
        o[4 * w + 1] = g | t | bad;
        o[4 * w + 2] = n | d | bad;
        o[4 * w + 3] = bad;
    }
    if (32 * w < slen) {   // the tail through a 32-byte copy padded with 'A' (all planes 0)
        alignas(32) char t[32];
        memset(t, 'A', sizeof(t));
        memcpy(t, seq + 32 * w, slen - 32 * w);
        const __m256i v = _mm256_load_si256((const __m256i *)t);
        const uint32_t a = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, A));
        const uint32_t c = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Cc));
        const uint32_t g = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Gg));
        const uint32_t tt = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Tt));
        const uint32_t n = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Nn));
        const uint32_t d = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, Dd));
        const uint32_t bad = ~(a | c | g | tt | n | d);
        o[4 * w] = c | tt | d | bad;
        o[4 * w + 1] = g | tt | bad;
        o[4 * w + 2] = n | d | bad;
        o[4 * w + 3] = bad;
    }
}
static const bool HAVE_AVX2 = __builtin_cpu_supports("avx2");
#endif
static void seq_planes(const char *seq, size_t slen, uint32_t *o) {
#if defined(__x86_64__)
    if (HAVE_AVX2) return seq_planes_avx2(seq, slen, o);
#endif
    seq_planes_scalar(seq, slen, o);
}
// the set bits of plane word group k (0 p0, 1 p1, 2 x, 3 bad) in chars [a, b)
static inline uint32_t plane_bits(const uint32_t *sp, int k, size_t a, size_t b, bool any) {
    uint32_t tot = 0;
    for (size_t w = a >> 5; w < ((b + 31) >> 5); w++) {
        uint32_t m = k == 4 ? sp[4 * w + 2] & sp[4 * w] & ~sp[4 * w + 1] : sp[4 * w + k];   // 4: '-' chars
        if (w == (a >> 5)) m &= ~0u << (a & 31);
        if (w == ((b - 1) >> 5) && (b & 31)) m &= ~0u >> (32 - (b & 31));
        if (any && m) return 1;
        tot += (uint32_t)__builtin_popcount(m);
    }
    return tot;
}
// QL code of char i from the planes
static inline uint8_t plane_code(const uint32_t *sp, size_t i) {
    const size_t w = i >> 5, j = i & 31;
    if ((sp[4 * w + 3] >> j) & 1u) return Q_BAD;
    return (uint8_t)(((sp[4 * w] >> j) & 1u) | (((sp[4 * w + 1] >> j) & 1u) << 1) | (((sp[4 * w + 2] >> j) & 1u) << 2));
}

// The read's planes (seq_planes) → the chunk's planes at a 16-base boundary; returns the
// first base index.  *has_x: bit 0 = a non-ACGT char, bit 1 = a '-' char (x = 1, p1 = 0, p0 = 1)
static uint64_t pack_seq(Chunk &c, const uint32_t *sp, size_t slen, uint8_t *has_x) {
    const uint64_t q0 = (c.nq + 15) & ~(uint64_t)15;
    const uint64_t q1 = q0 + slen;
    const size_t need = (size_t)((q1 + 31) >> 5) + 1;
    if (c.bx.size() < need) {   // (grown without a fill: the words are zeroed as reached, below)
        size_t cap = std::max(need, c.bx.size() * 2);
        c.bq.resize(2 * cap);
        c.bx.resize(cap);
    }
    if (c.nz < need) {   // the words first reached by this read (and the funnel word after it)
        memset(&c.bq[2 * c.nz], 0, 8 * (need - c.nz));
        memset(&c.bx[c.nz], 0, 4 * (need - c.nz));
        c.nz = need;
    }
    uint8_t anyx = 0;
    const uint32_t sh = (uint32_t)(q0 & 31);   // 0 or 16
    const uint64_t w0 = q0 >> 5;
    const size_t nw = (slen + 31) / 32;
    for (size_t w = 0; w < nw; w++) {
        const uint32_t p0 = sp[4 * w], p1 = sp[4 * w + 1], x = sp[4 * w + 2];
        anyx |= (x != 0 ? 1 : 0) | ((x & p0 & ~p1) != 0 ? 2 : 0);
        c.bq[2 * (w0 + w)] |= p0 << sh;
        c.bq[2 * (w0 + w) + 1] |= p1 << sh;
        c.bx[w0 + w] |= x << sh;
        if (sh) {
            c.bq[2 * (w0 + w + 1)] |= p0 >> (32 - sh);
            c.bq[2 * (w0 + w + 1) + 1] |= p1 >> (32 - sh);
            c.bx[w0 + w + 1] |= x >> (32 - sh);
        }
    }
    c.nq = q1;
    *has_x = anyx;
    return q0;
}

// The first ten tab-separated fields of line [s, end) (end after its '\n' when present: the
// last field split keeps it, as line.split('\t') does, :191); returns how many.
static int split_fields(const char *s, const char *end, const char **f, size_t *fl, int maxf = 10) {
    int nf = 0;
    const char *cur = s;
    while (nf < maxf) {
        const char *t = (const char *)memchr(cur, '\t', end - cur);
        f[nf] = cur;
        if (!t) { fl[nf++] = end - cur; break; }
        fl[nf++] = t - cur;
        cur = t + 1;
    }
    return nf;
}

// One line of a parse piece [s, lim): its end (after its '\n', else lim) and split_fields of
// it, in one pass — 32 bytes per step compared against '\t' and '\n' at once.
#if defined(__x86_64__)
__attribute__((target("avx2,bmi"))) static const char *scan_line_avx2(const char *s, const char *lim, const char **f,
                                                                     size_t *fl, int *nfo) {
    const __m256i T = _mm256_set1_epi8('\t'), N = _mm256_set1_epi8('\n');
    int nf = 0;
    const char *cur = s, *p = s;
    for (; p + 32 <= lim; p += 32) {
        const __m256i v = _mm256_loadu_si256((const __m256i *)p);
        const uint32_t mn = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, N));
        uint32_t mt = nf < 10 ? (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, T)) : 0u;
        if (mn) mt &= (mn & (0u - mn)) - 1u;   // (the tabs before the line's '\n')
        while (mt && nf < 10) {
            const uint32_t i = (uint32_t)__builtin_ctz(mt);
            mt &= mt - 1;
            f[nf] = cur;
            fl[nf++] = (size_t)(p + i - cur);
            cur = p + i + 1;
        }
        if (mn) {
            const char *e = p + __builtin_ctz(mn) + 1;
            if (nf < 10) {
                f[nf] = cur;
                fl[nf++] = (size_t)(e - cur);
            }
            *nfo = nf;
            return e;
        }
    }
    const char *nl = (const char *)memchr(p, '\n', lim - p);   // (the piece's last < 32 bytes)
    const char *e = nl ? nl + 1 : lim;
    if (nf < 10) nf += split_fields(cur, e, f + nf, fl + nf, 10 - nf);
    *nfo = nf;
    return e;
}
#endif
static const char *scan_line(const char *s, const char *lim, const char **f, size_t *fl, int *nfo) {
#if defined(__x86_64__)
    if (HAVE_AVX2) return scan_line_avx2(s, lim, f, fl, nfo);
#endif
    const char *nl = (const char *)memchr(s, '\n', lim - s);
    const char *e = nl ? nl + 1 : lim;
    *nfo = split_fields(s, e, f, fl);
    return e;
}

static int process_fields(Chunk &c, const RefView &rv, std::string &last_name, int64_t &last_ref, const char **f,
                          const size_t *fl, int nf, std::string &emsg);
// One SAM record line (not a header line), n includes the trailing '\n' when present.
static int process_record(Chunk &c, const RefView &rv, std::string &last_name, int64_t &last_ref,
                          const char *s, size_t n, std::string &emsg) {
    const char *f[10];
    size_t fl[10];
    const int nf = s[0] == '@' ? 0 : split_fields(s, s + n, f, fl);
    return process_fields(c, rv, last_name, last_ref, s[0] == '@' ? nullptr : f, fl, nf, emsg);
}
// The record of fields f (nullptr: a line starting with '@' inside the records, :195).
static int process_fields(Chunk &c, const RefView &rv, std::string &last_name, int64_t &last_ref, const char **f,
                          const size_t *fl, int nf, std::string &emsg) {
    c.lines_total++;
    if (!f) return S2C_OK;                                             // :195
    auto fail = [&](int code, const std::string &m) { emsg = m; return code; };
    if (nf < 6) return fail(S2C_ERR_INDEX, "IndexError: record with < 6 fields (:195)");
    if (fl[5] == 1 && f[5][0] == '*') return S2C_OK;                  // unmapped (:195)
    c.reads_mapped++;
    const char *nb;
    size_t nl;
    if (!py2_first_token(f[2], fl[2], &nb, &nl)) return fail(S2C_ERR_INDEX, "IndexError: empty RNAME (:200)");
    int64_t pos1;
    if (!py2_int(f[3], fl[3], &pos1))
        return fail(S2C_ERR_VALUE, "ValueError: invalid POS '" + std::string(f[3], fl[3]) + "' (:201)");
    const int64_t pos0 = pos1 - 1;
    if (nf < 10) return fail(S2C_ERR_INDEX, "IndexError: record with < 10 fields (:206)");

    // ---- CIGAR tokens (:58-59) ----
    const uint64_t tok0 = c.toks.size();
    uint32_t ntok = 0;
    int rc = tokenize_cigar(f[5], fl[5], c.toks, &ntok);
    if (rc) return fail(rc, s2c_last_error());
    const char *seq = f[9];
    const int64_t slen = (int64_t)fl[9];
    if (slen >= ((int64_t)1 << 24)) return fail(S2C_ERR_LIMIT, "SEQ of 2^24 or more chars not supported");

    // ---- reference lookup: sequences[refname] / insertions[refname] (:212,:217,:221) ----
    int64_t ref;
    if (last_ref >= 0 && last_name.size() == nl && memcmp(last_name.data(), nb, nl) == 0) {
        ref = last_ref;
    } else {
        std::string name(nb, nl);
        auto it = rv.idx->find(name);
        ref = it == rv.idx->end() ? -1 : (int64_t)it->second;
        if (ref >= 0) { last_ref = ref; last_name = name; }
    }

    // ---- the token walk of parsecigar (:64-81): seqout length, its '-' count, the codes of
    //      the bases it takes (validated below), insertion events with non-empty motifs ----
    std::vector<uint32_t> &sp = c.sp;   // SEQ planes (query order)
    if (sp.size() < 4 * (size_t)((slen + 31) / 32)) sp.resize(4 * (size_t)((slen + 31) / 32) + 64);
    seq_planes(seq, (size_t)slen, sp.data());
    int64_t start = 0, start_ref = pos0, klen = 0, dashes = 0, mb = 0;
    bool any_bad = false;
    const uint32_t ev0 = (uint32_t)c.ev.size();
    uint32_t nev = 0;
    for (uint32_t t = 0; t < ntok; t++) {
        const uint32_t w = c.toks[tok0 + t], op = w & 15u;
        const int64_t l = (int64_t)(w >> 4);
        if (op_bases(op)) {
            const int64_t take = start < slen ? std::min(l, slen - start) : 0;
            if (take > 0) {
                dashes += plane_bits(sp.data(), 4, (size_t)start, (size_t)(start + take), false);
                any_bad |= plane_bits(sp.data(), 3, (size_t)start, (size_t)(start + take), true) != 0;
            }
            klen += take;
            mb += take;
            start += l;
            start_ref += l;
        } else if (op_dash(op)) {
            klen += l;
            dashes += l;
            start_ref += l;
        } else if (op == S2C_OP_I) {
            const int64_t take = start < slen ? std::min(l, slen - start) : 0;
            if (take > 0) {   // an empty motif never reaches a column (:280-287)
                c.ev.push_back({start_ref, (uint64_t)start, (uint32_t)std::max<int64_t>(ref, 0), (uint32_t)take,
                                (uint32_t)c.reads.size()});
                nev++;
                c.qbases += take;
            }
            start += l;
        } else if (op == S2C_OP_S) {
            start += l;
        }
        if (op != S2C_OP_S && op != S2C_OP_H) c.ntokens++;
    }
    if (klen >= ((int64_t)1 << S2C_RUN_KSHIFT)) return fail(S2C_ERR_LIMIT, "seqout of 2^27 or more positions not supported");
    c.aligned += klen;
    c.qbases += mb;
    if (ref < 0) return fail(S2C_ERR_KEY, "KeyError: '" + std::string(nb, nl) + "' (:212/:221)");
    const int64_t L = (*rv.len)[ref];

    // ---- maxdel rule (:210) and the checks of :211-218 in seqout order: index, then symbol ----
    const bool drop = rv.maxdel_active && dashes > rv.maxdel;
    const bool in_range = pos0 >= 0 && pos0 + klen <= L;
    int64_t kc0 = -1, kc1 = -1;
    if (!in_range || any_bad || drop) {
        int64_t k = 0, st = 0;
        for (uint32_t t = 0; t < ntok; t++) {
            const uint32_t w = c.toks[tok0 + t], op = w & 15u;
            const int64_t l = (int64_t)(w >> 4);
            int64_t take = 0;
            bool bases = false;
            if (op_bases(op)) { take = st < slen ? std::min(l, slen - st) : 0; bases = true; }
            else if (op_dash(op)) take = l;
            for (int64_t j = 0; j < take; j++, k++) {
                const uint8_t cd = bases ? plane_code(sp.data(), (size_t)(st + j)) : Q_DASH;
                if (drop && cd == Q_DASH) continue;            // '-' skipped (:216)
                const int64_t pp = pos0 + k;
                if (pp < -L || pp >= L) return fail(S2C_ERR_INDEX, "IndexError: list index out of range (:212)");
                if (cd == Q_BAD) return fail(S2C_ERR_KEY, "KeyError: base not in -ACGNT (:212)");
                if (kc0 < 0) kc0 = k;
                kc1 = k + 1;
            }
            if (bases || op == S2C_OP_I || op == S2C_OP_S) st += l;
        }
    } else if (klen > 0) {
        kc0 = 0;
        kc1 = klen;
    }
    for (uint32_t e = ev0; e < ev0 + nev; e++) c.ev[e].ref = (uint32_t)ref;
    ReadRec r;
    r.pos0 = pos0;
    r.klen = klen;
    r.kc0 = kc0;
    r.kc1 = kc1;
    r.tok = tok0;
    r.ref = (uint32_t)ref;
    r.ntok = ntok;
    r.slen = (uint32_t)slen;
    r.ev0 = ev0;
    r.nev = nev;
    r.drop = drop;
    if (kc0 >= 0 || nev > 0) {
        r.q = pack_seq(c, sp.data(), (size_t)slen, &r.has_x);
        for (uint32_t e = ev0; e < ev0 + nev; e++) c.ev[e].q += r.q;
    } else {
        r.q = 0;
        r.has_x = 0;
        c.toks.resize(tok0);   // nothing reaches the device from this read
        r.ntok = 0;
    }
    c.reads.push_back(r);
    c.bound((uint32_t)ref, pos0, klen, L);
    return S2C_OK;
}

// One line of the sequential feed (header lines included).
static int process_line(s2c_parser *p, const char *s, size_t n) {
    if (p->in_header) {
        if (s[0] == '@') {
            p->header_lines++;
            p->chunks.back()->lines_total++;
            if (n >= 3 && s[1] == 'S' && s[2] == 'Q') return parse_sq(p, s, n);
            return S2C_OK;
        }
        p->in_header = false;
    }
    RefView rv{&p->ref_idx, &p->ref_len, p->maxdel_active, p->maxdel};
    std::string emsg;
    int rc = process_record(*p->chunks.back(), rv, p->last_name, p->last_ref, s, n, emsg);
    if (rc) return perr(p, rc, emsg);
    return S2C_OK;
}

static int s2c_parser_new_impl(int maxdel_active, int64_t maxdel, s2c_parser **out) {
    if (!out) return s2c_set_error(S2C_ERR_ARG, "out is NULL");
    s2c_parser *p = new s2c_parser();
    p->maxdel_active = maxdel_active != 0;
    p->maxdel = maxdel;
    *out = p;
    return S2C_OK;
}
extern "C" int s2c_parser_new(int maxdel_active, int64_t maxdel, s2c_parser **out) {
    return s2c_guarded([&] { return s2c_parser_new_impl(maxdel_active, maxdel, out); });
}

extern "C" void s2c_parser_free(s2c_parser *p) { delete p; }

namespace {
int parse_window(s2c_parser *p, const char *s, size_t n);
}

static int s2c_parser_feed_impl(s2c_parser *p, const char *buf, size_t len) {
    if (!p) return s2c_set_error(S2C_ERR_ARG, "parser is NULL");
    if (p->detached) return s2c_set_error(S2C_ERR_ARG, "a detached parser takes no input");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    const char *s = buf, *end = buf + len;
    if (!p->carry.empty()) {
        const char *nl = (const char *)memchr(s, '\n', end - s);
        if (!nl) { p->carry.append(s, len); return S2C_OK; }
        p->carry.append(s, nl + 1 - s);
        int rc = process_line(p, p->carry.data(), p->carry.size());
        p->carry.clear();
        if (rc) return rc;
        s = nl + 1;
    }
    if (end - s >= (ptrdiff_t)(4 << 20)) {   // a large block: its whole lines in parallel pieces
        const char *cut = end;
        while (cut > s && cut[-1] != '\n') cut--;
        if (cut > s) {
            int rc = parse_window(p, s, (size_t)(cut - s));
            if (rc) return rc;
            s = cut;
        }
        if (s < end) p->carry.assign(s, end - s);
        return S2C_OK;
    }
    while (s < end) {
        const char *nl = (const char *)memchr(s, '\n', end - s);
        if (!nl) { p->carry.assign(s, end - s); break; }
        int rc = process_line(p, s, nl + 1 - s);
        if (rc) return rc;
        s = nl + 1;
    }
    return S2C_OK;
}
extern "C" int s2c_parser_feed(s2c_parser *p, const char *buf, size_t len) {
    return s2c_guarded([&] { return s2c_parser_feed_impl(p, buf, len); });
}

extern "C" int s2c_parser_end_header(s2c_parser *p) {
    if (!p) return s2c_set_error(S2C_ERR_ARG, "parser is NULL");
    if (p->detached) return s2c_set_error(S2C_ERR_ARG, "a detached parser takes no input");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    if (!p->carry.empty()) return s2c_set_error(S2C_ERR_ARG, "header does not end with a newline");
    p->in_header = false;
    return S2C_OK;
}

static int feed_flush(s2c_parser *p) {
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    if (!p->carry.empty()) {   // last line without '\n'
        std::string last;
        last.swap(p->carry);
        int rc = process_line(p, last.data(), last.size());
        if (rc) return rc;
    }
    return S2C_OK;
}

// ------------------------------------------------------------------ parallel file parse
// A file is read in bounded windows (WIN bytes, cut after the last '\n'; the partial last
// line carries into the next window), as the reference reads 50 KB chunks (:185-189).  In
// each window the header lines (:149-172) go first, in order; the record lines are cut
// into pieces at line ends, each parsed by its own thread into its own Chunk (the same
// process_record); chunks are kept in file order.  The first failing record in file order
// decides the error: a chunk stops at its first error, and no later chunk is kept.
namespace {
constexpr size_t WIN = (size_t)64 << 20;

int parse_window(s2c_parser *p, const char *s, size_t n) {
    size_t i = 0;
    while (i < n && p->in_header) {
        if (s[i] != '@') { p->in_header = false; break; }
        const char *nl = (const char *)memchr(s + i, '\n', n - i);
        const size_t e = nl ? (size_t)(nl - s) + 1 : n;
        int rc = process_line(p, s + i, e - i);
        if (rc) return rc;
        i = e;
    }
    if (i == n) return S2C_OK;
    const size_t body = n - i;
    unsigned hw = std::thread::hardware_concurrency();
    int nt = (int)std::min<size_t>(std::min<unsigned>(hw ? hw : 1, 16), std::max<size_t>(1, body >> 22));   // ≥ 4 MB each
    if (const char *e = getenv("S2C_PARSE_THREADS")) nt = std::max(1, std::min(64, atoi(e)));
    // 4 pieces per thread (≥ 1 MB each), taken in turn by the threads: a thread slowed by
    // the others' work (a streamed snapshot planning beside the feed) holds up the window by
    // one piece, not by its fixed share
    const int np = nt == 1 ? 1 : (int)std::min<size_t>((size_t)nt * 4, std::max<size_t>((size_t)nt, body >> 20));
    std::vector<size_t> cut(np + 1, n);
    cut[0] = i;
    for (int k = 1; k < np; k++) {   // piece k starts after the line end nearest to its share
        size_t c = std::max(cut[k - 1], i + body * k / np);
        const char *nl = c < n ? (const char *)memchr(s + c, '\n', n - c) : nullptr;
        cut[k] = nl ? (size_t)(nl - s) + 1 : n;
    }
    std::vector<std::unique_ptr<Chunk>> cs(np);
    std::vector<int> rcs(np, S2C_OK);
    std::vector<std::string> msgs(np);
    RefView rv{&p->ref_idx, &p->ref_len, p->maxdel_active, p->maxdel};
    auto work = [&](int k) {
        cs[k].reset(new Chunk());
        Chunk &c = *cs[k];
        std::string last_name;
        int64_t last_ref = -1;
        const char *b = s + cut[k];
        const size_t m = cut[k + 1] - cut[k];
        c.reads.reserve(m / 150 + 16);   // (SAM lines of ≥ 150 bytes: no regrowth for typical reads)
        c.toks.reserve(m / 100 + 16);
        c.bx.resize(m / 32 + 64);     // SEQ bytes ≤ m: planes of ≤ m bases, 16-base aligned reads
        c.bq.resize(2 * c.bx.size());  // (no fill: pack_seq zeroes the words it reaches)
        size_t j = 0;
        while (j < m) {   // (a last line without '\n' counts, Py2)
            const char *f[10];
            size_t fl[10];
            int nf;
            const size_t e = (size_t)(scan_line(b + j, b + m, f, fl, &nf) - b);
            rcs[k] = process_fields(c, rv, last_name, last_ref, b[j] == '@' ? nullptr : f, fl, nf, msgs[k]);
            if (rcs[k]) return;
            j = e;
        }
    };
    static const bool timing = getenv("S2C_HOST_TIMING") != nullptr;
    std::vector<double> tw(nt, 0.0);
    const auto t0 = std::chrono::steady_clock::now();
    std::atomic<int> next{0};
    std::vector<double> ts(nt, 0.0);
    auto worker = [&](int t) {
        const auto a = std::chrono::steady_clock::now();
        for (int k; (k = next++) < np;) work(k);
        tw[t] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
        ts[t] = std::chrono::duration<double, std::milli>(a - t0).count();
    };
    WorkerPool::get(POOL_PARSE).run(nt, worker);
    if (timing) {   // (S2C_HOST_TIMING: the window's wall time, its threads' longest and mean)
        double mx = 0, sm = 0;
        for (double x : tw) { mx = std::max(mx, x); sm += x; }
        double smax = 0;
        for (double x : ts) smax = std::max(smax, x);
        fprintf(stderr, "[s2c feed] %zu B %d thr %d pieces wall %.2f ms max %.2f mean %.2f last start %.2f\n", n - i, nt, np,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), mx, sm / nt, smax);
    }
    for (int k = 0; k < np; k++) {
        if (!cs[k]->reads.empty() || cs[k]->lines_total) p->chunks.push_back(std::move(cs[k]));
        if (rcs[k]) return perr(p, rcs[k], msgs[k]);
    }
    return S2C_OK;
}

// BGZF (the blocked gzip of samtools / bgzip: members of <= 64 KB, each with a 'BC' extra
// field holding its compressed size) inflated block-parallel: the compressed stream is read
// in 32 MB pieces, the complete blocks of a piece are located by their sizes and inflated on
// all host threads straight into their output offsets (ISIZE from each trailer), CRC-checked.
// A member that is not BGZF-shaped switches the rest of the stream to sequential inflate.
struct Bgzf {
    FILE *f = nullptr;
    std::vector<unsigned char> cb;   // compressed bytes not yet inflated
    std::vector<char> out;           // inflated bytes of the last piece
    size_t opos = 0;
    bool eof = false, seq = false, seq_end = false;
    z_stream z{};
    unsigned nt = 1;
    ~Bgzf() {
        if (seq) inflateEnd(&z);
        if (f) fclose(f);
    }
    static bool block_at(const unsigned char *p, size_t n, size_t *bsize) {   // a BGZF header at p
        if (n < 18 || p[0] != 0x1f || p[1] != 0x8b || p[2] != 8 || !(p[3] & 4)) return false;
        const size_t xlen = p[10] | (p[11] << 8);
        for (size_t k = 12; k + 4 <= 12 + xlen && k + 4 <= n; ) {   // the 'BC' subfield
            const size_t sl = p[k + 2] | (p[k + 3] << 8);
            if (p[k] == 'B' && p[k + 1] == 'C' && sl == 2 && k + 6 <= n) {
                *bsize = (size_t)(p[k + 4] | (p[k + 5] << 8)) + 1;
                return *bsize >= 12 + xlen + 8;
            }
            k += 4 + sl;
        }
        return false;
    }
    bool fill_cb() {   // append up to 32 MB; false at end of file
        const size_t h = cb.size(), want = (size_t)32 << 20;
        cb.resize(h + want);
        const size_t r = fread(cb.data() + h, 1, want, f);
        cb.resize(h + r);
        return r > 0;
    }
    // next piece of output into out; false: no more data (err set on a corrupt stream)
    bool next(bool &err) {
        out.clear();
        opos = 0;
        if (!seq) {
            if (!eof && cb.size() < ((size_t)32 << 20)) eof = !fill_cb();
            std::vector<size_t> off, len, isz;
            size_t k = 0, total = 0;
            while (true) {
                size_t bs;
                if (!block_at(cb.data() + k, cb.size() - k, &bs)) {
                    if (cb.size() - k >= 18 || (eof && cb.size() > k)) seq = true;   // not BGZF from here on
                    break;
                }
                if (k + bs > cb.size()) break;   // partial block: the next piece
                const unsigned char *t = cb.data() + k + bs - 4;
                const size_t is = (size_t)t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
                if (is > 65536) {   // not a BGZF block (≤ 64 KiB inflated): zlib checks the rest sequentially
                    seq = true;
                    break;
                }
                off.push_back(k);
                len.push_back(bs);
                isz.push_back(total);
                total += is;
                k += bs;
            }
            if (!off.empty()) {
                out.resize(total);
                std::atomic<size_t> nextb{0};
                std::atomic<bool> bad{false};
                auto work = [&] {
                    z_stream zz{};
                    if (inflateInit2(&zz, -15) != Z_OK) { bad = true; return; }
                    for (size_t b; (b = nextb++) < off.size();) {
                        const unsigned char *p = cb.data() + off[b];
                        const size_t hl = 12 + (size_t)(p[10] | (p[11] << 8));
                        const size_t dl = len[b] - hl - 8;
                        const size_t ol = (b + 1 < off.size() ? isz[b + 1] : total) - isz[b];
                        inflateReset(&zz);
                        zz.next_in = (Bytef *)(p + hl);
                        zz.avail_in = (uInt)dl;
                        zz.next_out = (Bytef *)out.data() + isz[b];
                        zz.avail_out = (uInt)ol;
                        const int r = inflate(&zz, Z_FINISH);
                        const unsigned char *t = p + len[b] - 8;
                        const uint32_t crc = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
                        if (r != Z_STREAM_END || zz.total_out != ol ||
                            (uint32_t)crc32(0L, (const Bytef *)out.data() + isz[b], (uInt)ol) != crc)
                            bad = true;
                    }
                    inflateEnd(&zz);
                };
                WorkerPool::get(POOL_IO).run((int)std::min<size_t>(nt, off.size()), [&](int) { work(); });
                if (bad) { err = true; return false; }
            }
            cb.erase(cb.begin(), cb.begin() + k);
            if (seq) {
                if (inflateInit2(&z, 31) != Z_OK) { err = true; return false; }
                z.avail_in = 0;
            }
            if (!out.empty()) return true;
            if (!seq) {
                if (eof) {
                    if (!cb.empty()) { err = true; return false; }   // a truncated block
                    return false;
                }
                return next(err);
            }
        }
        // sequential inflate of the rest (gzip members one after the other)
        if (seq_end) return false;
        out.resize((size_t)8 << 20);
        size_t have = 0;
        while (have < out.size()) {
            if (z.avail_in == 0) {
                if (cb.empty()) {
                    if (eof || !fill_cb()) { eof = true; if (cb.empty()) { seq_end = true; break; } }
                }
                z.next_in = cb.data();
                z.avail_in = (uInt)cb.size();
            }
            z.next_out = (Bytef *)out.data() + have;
            z.avail_out = (uInt)(out.size() - have);
            const uInt before = z.avail_in;
            const int r = inflate(&z, Z_NO_FLUSH);
            have = out.size() - z.avail_out;
            const size_t used = before - z.avail_in;
            cb.erase(cb.begin(), cb.begin() + used);
            z.next_in = cb.data();
            z.avail_in = (uInt)cb.size();
            if (r == Z_STREAM_END) {
                if (cb.empty() && eof) { seq_end = true; break; }
                inflateReset(&z);   // the next member
                if (cb.empty() && !fill_cb()) { eof = true; seq_end = true; break; }
                z.next_in = cb.data();
                z.avail_in = (uInt)cb.size();
            } else if (r == Z_BUF_ERROR && cb.empty() && eof) {
                err = true; return false;   // truncated
            } else if (r != Z_OK && r != Z_BUF_ERROR) {
                err = true; return false;
            }
        }
        out.resize(have);
        return have > 0;
    }
    long read(char *dst, size_t n) {
        size_t tot = 0;
        while (tot < n) {
            if (opos == out.size()) {
                bool err = false;
                if (!next(err)) {
                    if (err) return -1;
                    break;
                }
            }
            const size_t k = std::min(n - tot, out.size() - opos);
            memcpy(dst + tot, out.data() + opos, k);
            opos += k;
            tot += k;
        }
        return (long)tot;
    }
};

struct Reader {   // plain, gzip or BGZF (:111-114) byte source
    FILE *f = nullptr;
    gzFile g = nullptr;
    std::unique_ptr<Bgzf> bz;
    int fd = -1;        // plain file: read by positioned reads on the host threads
    uint64_t off = 0;   // its next byte
    ~Reader() {
        if (f) fclose(f);
        if (g) gzclose(g);
        if (fd >= 0) close(fd);
    }
    // n bytes (fewer at end of file) of the plain file in parallel pieces of >= 4 MB: one
    // thread's copy out of the page cache was the file parse's bound past 4 parse threads
    long pread_par(char *dst, size_t n) {
        const unsigned hw = std::thread::hardware_concurrency();
        const size_t nt = std::max<size_t>(1, std::min<size_t>({(size_t)std::min(hw ? hw : 1u, 16u), n >> 22}));
        std::vector<size_t> got(nt, 0);
        std::atomic<bool> bad{false};
        auto piece = [&](size_t k) {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            size_t h = 0;
            while (a + h < b) {
                const ssize_t r = pread(fd, dst + a + h, b - a - h, (off_t)(off + a + h));
                if (r < 0) { bad = true; break; }
                if (r == 0) break;   // end of file
                h += (size_t)r;
            }
            got[k] = h;
        };
        WorkerPool::get(POOL_IO).run((int)nt, [&](int k) { piece((size_t)k); });
        if (bad) return -1;
        size_t tot = 0;   // (pieces after a short one are empty: the file ends there)
        for (size_t k = 0; k < nt; k++) {
            tot += got[k];
            if (got[k] < n * (k + 1) / nt - n * k / nt) break;
        }
        off += tot;
        return (long)tot;
    }
    long read(char *dst, size_t n) {
        if (bz) return bz->read(dst, n);
        if (fd >= 0) return pread_par(dst, n);
        if (g) {
            size_t tot = 0;
            while (tot < n) {
                const int r = gzread(g, dst + tot, (unsigned)std::min<size_t>(n - tot, 1u << 30));
                if (r < 0) return -1;
                if (r == 0) break;
                tot += (size_t)r;
            }
            return (long)tot;
        }
        return (long)fread(dst, 1, n, f);
    }
};
}  // namespace

// Open path as the reference reads it (:111-114): ".gz" → gzip (BGZF block-parallel), else plain.
static int reader_open(Reader &rd, const char *path) {
    const size_t n = strlen(path);
    if (n >= 3 && strcmp(path + n - 3, ".gz") == 0) {   // :111
        unsigned char h[18];
        size_t bs = 0, hn = 0;
        if (FILE *t = fopen(path, "rb")) {
            hn = fread(h, 1, sizeof(h), t);
            fclose(t);
        }
        if (Bgzf::block_at(h, hn, &bs)) {   // BGZF: block-parallel inflate
            rd.bz.reset(new Bgzf());
            rd.bz->f = fopen(path, "rb");
            if (!rd.bz->f) return s2c_set_error(S2C_ERR_IO, std::string("cannot open ") + path);
            const unsigned hw = std::thread::hardware_concurrency();
            rd.bz->nt = std::max(1u, std::min(hw ? hw : 1u, 16u));
        } else {
            rd.g = gzopen(path, "rb");
            if (!rd.g) return s2c_set_error(S2C_ERR_IO, std::string("cannot open ") + path);
            gzbuffer(rd.g, 1 << 20);
        }
    } else {
        rd.fd = open(path, O_RDONLY);
        if (rd.fd < 0) return s2c_set_error(S2C_ERR_IO, std::string("cannot open ") + path);
    }
    return S2C_OK;
}

static int s2c_parser_feed_file_impl(s2c_parser *p, const char *path) {
    if (!p || !path) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    if (p->detached) return s2c_set_error(S2C_ERR_ARG, "a detached parser takes no input");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    Reader rd;
    if (const int rc = reader_open(rd, path)) return rc;
    // A reader thread inflates / reads window k + 1 while the workers parse window k (two
    // buffers).  The reader cuts each window after its last '\n' and carries the partial
    // line into the next one.
    struct Slot {
        std::vector<char> buf;
        size_t len = 0;
        bool full = false, eof = false, err = false;
    };
    Slot slots[2];
    std::mutex m;
    std::condition_variable cv;
    bool stop = false;
    std::vector<char> tail(p->carry.begin(), p->carry.end());   // a partial line from s2c_parser_feed
    p->carry.clear();
    std::thread reader([&] {
        for (int k = 0;; k ^= 1) {
            Slot &sl = slots[k];
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return !sl.full || stop; });
                if (stop) return;
            }
            std::vector<char> &buf = sl.buf;
            if (buf.size() < tail.size() + WIN) buf.resize(tail.size() + WIN + (1 << 20));
            if (!tail.empty()) memcpy(buf.data(), tail.data(), tail.size());
            size_t have = tail.size(), cut = 0;
            bool eof = false, err = false;
            for (;;) {
                if (buf.size() - have < WIN / 2) buf.resize(buf.size() + WIN);   // a line longer than a window
                const long r = rd.read(buf.data() + have, buf.size() - have);
                if (r < 0) { err = true; break; }
                have += (size_t)r;
                if (r == 0) { eof = true; cut = have; break; }
                size_t k2 = have;
                while (k2 > 0 && buf[k2 - 1] != '\n') k2--;
                if (k2) { cut = k2; break; }   // else: no complete line yet, read more
            }
            tail.assign(buf.data() + cut, buf.data() + have);
            {
                std::lock_guard<std::mutex> lk(m);
                sl.len = cut;
                sl.eof = eof;
                sl.err = err;
                sl.full = true;
            }
            cv.notify_all();
            if (eof || err) return;
        }
    });
    int rc = S2C_OK;
    for (int k = 0;; k ^= 1) {
        Slot &sl = slots[k];
        {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return sl.full; });
        }
        if (sl.err) {
            rc = perr(p, S2C_ERR_IO, "gzip read error");
            break;
        }
        if (sl.len) rc = parse_window(p, sl.buf.data(), sl.len);
        const bool eof = sl.eof;
        {
            std::lock_guard<std::mutex> lk(m);
            sl.full = false;
            if (rc) stop = true;
        }
        cv.notify_all();
        if (rc || eof) break;
    }
    {
        std::lock_guard<std::mutex> lk(m);
        stop = true;
    }
    cv.notify_all();
    reader.join();
    return rc;
}
extern "C" int s2c_parser_feed_file(s2c_parser *p, const char *path) {
    return s2c_guarded([&] { return s2c_parser_feed_file_impl(p, path); });
}

// The byte source of s2c_parser_feed_file as a stream (streamed batches, stream.py): the
// same plain / gzip / block-parallel BGZF reader, read in caller-sized pieces.
struct s2c_reader {
    Reader rd;
};
extern "C" int s2c_reader_open(const char *path, s2c_reader **out) {
    return s2c_guarded([&] {
        if (!path || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
        std::unique_ptr<s2c_reader> r(new s2c_reader());
        if (const int rc = reader_open(r->rd, path)) return rc;
        *out = r.release();
        return S2C_OK;
    });
}
extern "C" int s2c_reader_read(s2c_reader *r, void *dst, size_t cap, size_t *n) {
    return s2c_guarded([&] {
        if (!r || !n || (cap && !dst)) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
        size_t tot = 0;
        while (tot < cap) {   // (a full buffer unless the stream ends)
            const long k = r->rd.read((char *)dst + tot, cap - tot);
            if (k < 0) return s2c_set_error(S2C_ERR_IO, "gzip read error");
            if (k == 0) break;
            tot += (size_t)k;
        }
        *n = tot;
        return S2C_OK;
    });
}
extern "C" void s2c_reader_free(s2c_reader *r) { delete r; }

// ------------------------------------------------------------------ finish: layout + plan
namespace {
constexpr int64_t TP_MIN = 256, TP_MAX = 2048;      // tile bounds (positions)
static int64_t deep_tile_min() {   // S2C_DEEP_TILE: the narrowest deep tile (positions)
    static const int64_t v = [] {
        const char *e = plan_env("S2C_DEEP_TILE");
        return e ? std::min<int64_t>(std::max<int64_t>(atoll(e), 64), 2048) : (int64_t)512;
    }();
    return v;
}
constexpr double E_TARGET = 262144.0;                // aligned bases per deep tile
// LDS a shallow tile's window is planned to (one wave per tile, ~10 resident per CU; C5's
// 30x gives 1024-position tiles — measured faster than 512, profiles/r02)
constexpr double DENSE_PLAN_BYTES = 16384.0;
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t align_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }
inline uint32_t pow2_at_least(uint64_t v) {
    uint32_t c = 1;
    while (c < v) c <<= 1;
    return c;
}

struct Piece {
    uint64_t gpos;          // global coordinate of seqout char ka
    int64_t ka, kb;         // seqout range
    uint32_t chunk, read;
    uint8_t range, ins, lng;
    uint32_t nslots;        // prefix words + tokens
    uint32_t kmin, kmax;    // global keys of the insertion events it emits (ins)
    uint32_t qlen;          // plane bases: len(SEQ) rounded up to 16
    uint32_t ref;           // reference index
};

// Host threads of the plan: the parse's (≤ 16, S2C_PARSE_THREADS), at most n / grain.
static int plan_threads(int64_t n, int64_t grain) {
    unsigned hw = std::thread::hardware_concurrency();
    int nt = (int)std::min<unsigned>(hw ? hw : 1, 16);
    if (const char *e = getenv("S2C_PARSE_THREADS")) nt = std::max(1, std::min(64, atoi(e)));
    if (const char *e = getenv("S2C_PLAN_THREADS")) nt = std::max(1, std::min(64, atoi(e)));   // (the plan's own)
    return (int)std::max<int64_t>(1, std::min<int64_t>(nt, n / std::max<int64_t>(grain, 1)));
}
// f(t, i0, i1) on nt contiguous ranges of [0, n), thread t on range t
template <class F>
static void par_ranges(int nt, int64_t n, F &&f) {
    if (nt <= 1) { f(0, (int64_t)0, n); return; }
    WorkerPool::get(POOL_PLAN).run(nt, [&f, nt, n](int t) { f(t, n * t / nt, n * (t + 1) / nt); });
}
}  // namespace

// The dense items' windows (S2C_DWIN_WORDS) from the final tile records, and the compact
// piece records of every window (S2C_DPC_WORDS, in window order: a piece of two windows has
// two records, each relative to its own window).
static void build_dwin(s2c_batch *b) {
    const size_t nd = b->dense.size() / S2C_ITEM_WORDS;
    b->dwin.assign(std::max<size_t>(nd, 1) * S2C_DWIN_WORDS, 0u);
    std::vector<uint64_t> base(nd + 1, 0);
    for (size_t i = 0; i < nd; i++) {
        const uint32_t t = b->dense[i * S2C_ITEM_WORDS];
        const uint32_t *tw = &b->tiles[(size_t)t * S2C_TILE_WORDS];
        uint32_t *o = &b->dwin[i * S2C_DWIN_WORDS];
        const uint32_t v[12] = {t, tw[0], tw[1], tw[8], tw[10], tw[11], tw[13], tw[14], tw[15], tw[16], tw[17], tw[18]};
        for (int k = 0; k < 12; k++) o[k] = v[k];
        o[12] = (uint32_t)base[i];
        base[i + 1] = base[i] + (tw[14] - tw[13]);
    }
    if (base[nd] >= ((uint64_t)1 << 32)) throw std::runtime_error("more than 2^32 dense window pieces");
    b->info.n_dpc = (int64_t)base[nd];
    b->dpc.resize(std::max<uint64_t>(base[nd], 1) * S2C_DPC_WORDS);
    if (!base[nd]) b->dpc[0] = b->dpc[1] = b->dpc[2] = 0;
    par_ranges(plan_threads((int64_t)nd, 64), (int64_t)nd, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; i++) {
            const uint32_t *w = &b->dwin[(size_t)i * S2C_DWIN_WORDS];
            const uint32_t T0 = 32 * (w[1] >> 5), o0 = w[8], qw0 = w[10];
            uint32_t *o = &b->dpc[base[i] * S2C_DPC_WORDS];
            for (uint32_t k = w[6]; k < w[7]; k++, o += S2C_DPC_WORDS) {
                const uint32_t *pc = &b->pc[4 * (size_t)k];
                const uint32_t rs = pc[0] - T0 + 2048u, qh = pc[1] - 2 * qw0, nops = pc[6] - pc[2], oj = pc[2] - o0;
                const uint32_t slen = pc[3] & 0xFFFFFFu;
                if (rs >= 4096u || qh >= 8192u || nops > S2C_DPC_NOPS_MAX || oj >= 8192u || slen > S2C_DPC_SLEN_MAX)
                    throw std::runtime_error("dense window piece beyond the compact record's fields");
                o[0] = rs | qh << 12 | nops << 25;
                o[1] = oj | slen << 13 | (pc[3] >> 24) << 24;
                o[2] = b->px[k];
            }
        }
    });
}

// Pieces k_tile_dense's compact records cannot hold (len(SEQ) or op slots beyond their
// fields): prefix counts over the sorted pieces, so a tile window [pf0, pf1) holds one iff
// p[pf1] > p[pf0]; such a tile is not dense.
static std::vector<uint32_t> dpc_bad_prefix(const s2c_batch *b) {
    const int64_t NP = b->info.n_pieces;
    std::vector<uint32_t> p(NP + 1, 0);
    const int nt = plan_threads(NP, 1 << 16);
    std::vector<uint32_t> part(nt + 1, 0);
    auto bad = [&](int64_t k) {
        const uint32_t *pc = &b->pc[4 * (size_t)k];
        return (pc[3] & 0xFFFFFFu) > S2C_DPC_SLEN_MAX || pc[6] - pc[2] > S2C_DPC_NOPS_MAX;
    };
    par_ranges(nt, NP, [&](int t, int64_t k0, int64_t k1) {
        uint32_t c = 0;
        for (int64_t k = k0; k < k1; k++) c += bad(k);
        part[t + 1] = c;
    });
    for (int t = 0; t < nt; t++) part[t + 1] += part[t];
    par_ranges(nt, NP, [&](int t, int64_t k0, int64_t k1) {
        uint32_t c = part[t];
        for (int64_t k = k0; k < k1; k++) p[k + 1] = (c += bad(k));
    });
    return p;
}

// The window of tile [a, b): the short pieces starting in words [a/32 - K, ceil(b/32)) — a
// contiguous range of the bucketed pieces — their op slots and base plane words (+1 word for
// the funnel shift of the last one).  Tile words 13-18.
static void tile_window(const s2c_batch *b, int64_t K, uint64_t a, uint64_t e, uint32_t *tw) {
    const int64_t NP = b->info.n_pieces;
    auto piece_at_word = [&](int64_t w) {   // first piece with start word >= w
        if ((int64_t)b->ps.size() == b->info.n_words + 1 && w <= b->info.n_words) return (int64_t)b->ps[w];
        int64_t lo = 0, hi = NP;
        while (lo < hi) {
            const int64_t m = (lo + hi) / 2;
            if ((int64_t)(b->pc[4 * m] >> 5) < w) lo = m + 1; else hi = m;
        }
        return lo;
    };
    const int64_t pf0 = piece_at_word(std::max<int64_t>((int64_t)(a >> 5) - K, 0)), pf1 = piece_at_word((int64_t)((e + 31) >> 5));
    tw[13] = (uint32_t)pf0;
    tw[14] = (uint32_t)pf1;
    tw[15] = b->pc[4 * pf0 + 2];
    tw[16] = b->pc[4 * pf1 + 2];
    tw[17] = pf1 > pf0 ? (uint32_t)(((uint64_t)b->pc[4 * pf0 + 1] * 16) >> 5) : 0u;
    tw[18] = pf1 > pf0 ? (uint32_t)(((uint64_t)b->pc[4 * (pf1 - 1) + 1] * 16 + (b->pc[4 * (pf1 - 1) + 3] & 0xFFFFFFu) + 31) / 32 + 1)
                       : tw[17];
}

// LDS bytes k_tile_dense keeps a tile's window in (s2c_dense.hip), and whether it fits (with
// query offsets of the window's base planes in 17 bits)
static int64_t dense_bytes(const uint32_t *tw, int64_t) {
    return S2C_DENSE_BYTES((int64_t)(tw[16] - tw[15]), (int64_t)(tw[18] - tw[17]));
}
static bool dense_fits(const uint32_t *tw, int64_t K) {
    return dense_bytes(tw, K) <= S2C_DENSE_LDS && (int64_t)(tw[18] - tw[17]) <= S2C_DENSE_QW;
}

// PF_RUNS on the long pieces (the tile long lists read k_reads' run records of them; the
// tile kernels walk every short piece of their windows themselves), and the list of pieces
// k_reads walks (those, and the pieces emitting insertion events).
// k_tile's walk-queue variant (s2c_batch_info walk_queue): at least 1/32 of the pieces walked
// op by op, tiles of <= 1024 positions (the 2048-position instantiation has no LDS for it).
// It also records its finish tiles' short-motif insertion events (LDS event list, s2c_tile.hip).
static int64_t walk_queue_of(const s2c_batch_info &I) {
    return I.n_walked > 0 && 32 * I.n_walked >= I.n_pieces && I.tile_max <= 1024 ? 1 : 0;
}

// The pieces k_reads walks (rlist): first the ones s2c_run needs (n_rlist_run) — long pieces
// listed by non-dense tiles (k_reads writes their run records) and insertion pieces with an
// event k_tile does not record: a motif > S2C_SHORT_MOTIF bases, a long piece, or a key in a
// tile that is not a finish tile (deep / general: k_consensus votes it) or whose window does
// not hold the piece — then the other insertion pieces (the counts-only modes hash every event).
static void mark_runs(s2c_batch *b) {
    const int64_t NP = b->info.n_pieces, K = b->info.kwin;
    std::vector<uint8_t> need(NP, 0);
    // long pieces listed by run slot (k_tile's tiles: k_reads writes their runs); a dense
    // tile lists its long pieces themselves (k_tile_dense walks them)
    for (int64_t t = 0; t < b->info.n_tiles && b->info.n_long > 0; t++) {
        const uint32_t *tw = &b->tiles[(size_t)t * S2C_TILE_WORDS];
        if (tw[3] & S2C_TILE_DENSE) continue;
        for (uint32_t e = tw[10]; e < tw[11]; e++) {
            const uint32_t slot = b->lp[e];
            int64_t lo = 0, hi = NP - 1;
            while (lo < hi) {
                const int64_t m = (lo + hi + 1) / 2;
                if (b->pc[4 * m + 2] <= slot) lo = m; else hi = m - 1;
            }
            need[lo] = 1;
        }
    }
    // (the layers were cut for the instantiation planned, I.walk_queue: a shard whose parent
    // was planned for the non-queue one keeps it, whose chunk holds more plane bytes)
    b->info.walk_queue = walk_queue_of(b->info) && b->info.walk_queue ? 1 : 0;
    static const bool no_tile_events = plan_env("S2C_NO_TILE_EVENTS") != nullptr;   // (A/B: k_reads hashes every event)
    b->info.tile_events = b->info.walk_queue && !no_tile_events ? 1 : 0;
    const bool rec = b->info.tile_events != 0;
    auto tile_takes_events = [&](int64_t k) {   // every event of insertion piece k recorded by k_tile
        const uint32_t fl = b->pc[4 * k + 3] >> 24;
        if (!rec || (fl & S2C_PF_LONG) || ((size_t)k < b->lmot.size() && b->lmot[k]) || b->kmin[k] == 0xFFFFFFFFu) return false;
        const uint32_t t0 = b->wtile[b->kmin[k] >> 5], t1 = b->wtile[b->kmax[k] >> 5];
        if (t0 == 0xFFFFFFFFu || t1 == 0xFFFFFFFFu) return false;
        const int64_t ws = (int64_t)(b->pc[4 * k] >> 5);
        for (uint32_t t = t0; t <= t1; t++) {
            const uint32_t *tw = &b->tiles[(size_t)t * S2C_TILE_WORDS];
            const int64_t W0 = tw[0] >> 5, W1 = (tw[1] + 31) >> 5;
            if ((tw[3] & (S2C_TILE_DEEP | S2C_TILE_GENERAL | S2C_TILE_DENSE)) || ws < std::max<int64_t>(W0 - K, 0) || ws >= W1)
                return false;
        }
        return true;
    };
    b->rlist.clear();
    const int nt = plan_threads(NP, 1 << 18);
    std::vector<std::vector<uint32_t>> rl(nt), rx(nt);
    par_ranges(nt, NP, [&](int t, int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; k++) {
            uint32_t &w3 = b->pc[4 * k + 3];
            if (need[k]) w3 |= (uint32_t)S2C_PF_RUNS << 24;
            else w3 &= ~((uint32_t)S2C_PF_RUNS << 24);
            const bool ins = ((w3 >> 24) & S2C_PF_INS) != 0;
            if (need[k] || (ins && !tile_takes_events(k))) rl[t].push_back((uint32_t)k);
            else if (ins) rx[t].push_back((uint32_t)k);
        }
    });
    for (int t = 0; t < nt; t++) b->rlist.insert(b->rlist.end(), rl[t].begin(), rl[t].end());
    b->info.n_rlist_run = (int64_t)b->rlist.size();
    for (int t = 0; t < nt; t++) b->rlist.insert(b->rlist.end(), rx[t].begin(), rx[t].end());
    b->info.n_rlist = (int64_t)b->rlist.size();
    if (b->rlist.empty()) b->rlist.push_back(0);
}

// ------------------------------------------------------------------ k_tile's layer plan
// k_tile stages a tile's window in LDS one LAYER at a time: the window's start words
// [S0, S1) (S0 = max(W0 - K, 0)) are its segments, and layer l of nl takes from segment s
// its short pieces among [ps[s] + n_s*l/nl, ps[s] + n_s*(l+1)/nl) — every layer touches
// every word of the tile alike.  The layers are copied contiguously (build_layers), each
// one 16-byte aligned in every array, so a layer is one DMA per array.  A layer must fit
// the chunk (S2C_CHUNK_*): pieces, plane / non-ACGT / op bytes, run records, and per word
// <= S2C_CHUNK_LANE_RECS records per counting lane.
struct PieceBlocks {          // prefix sums over the sorted pieces (mod 2^32: differences exact)
    u32buf n, h, o;   // short pieces, their plane half-words, their op words (filled by the threads: no zero-fill)
};
static inline uint32_t piece_half_words(uint32_t w3) { return ((w3 & 0xFFFFFFu) + 15u) / 16u; }
static void piece_blocks(const s2c_batch *b, PieceBlocks &B) {
    const int64_t NP = b->info.n_pieces;
    B.n.resize(NP + 1);
    B.h.resize(NP + 1);
    B.o.resize(NP + 1);
    B.n[0] = B.h[0] = B.o[0] = 0;
    const int nt = plan_threads(NP, 1 << 18);
    std::vector<uint32_t> sn(nt + 1, 0), sh(nt + 1, 0), so(nt + 1, 0);
    par_ranges(nt, NP, [&](int t, int64_t k0, int64_t k1) {   // range sums (mod 2^32) ...
        uint32_t n = 0, h = 0, o = 0;
        for (int64_t k = k0; k < k1; k++) {
            const uint32_t w3 = b->pc[4 * k + 3];
            const bool s = !((w3 >> 24) & S2C_PF_LONG);
            n += s ? 1u : 0u;
            h += s ? piece_half_words(w3) : 0u;
            o += s ? b->pc[4 * k + 6] - b->pc[4 * k + 2] : 0u;
            B.n[k + 1] = n; B.h[k + 1] = h; B.o[k + 1] = o;
        }
        sn[t + 1] = n; sh[t + 1] = h; so[t + 1] = o;
    });
    for (int t = 0; t < nt; t++) { sn[t + 1] += sn[t]; sh[t + 1] += sh[t]; so[t + 1] += so[t]; }
    par_ranges(nt, NP, [&](int t, int64_t k0, int64_t k1) {   // ... then each range from its base
        for (int64_t k = k0; k < k1; k++) { B.n[k + 1] += sn[t]; B.h[k + 1] += sh[t]; B.o[k + 1] += so[t]; }
    });
}

// Segment s's pieces [p0, p0 + n) cut into nl slices at p0 + floor((n·l + r_s) / nl), the
// rotation r_s = (s · 2654435761) mod nl spreading the segments' rounding (a segment of fewer
// pieces than layers puts them in different layers for different segments, not all in the
// last one).
struct LayerSeg { uint64_t p0, n, s; };
static inline uint64_t layer_rot(uint64_t s, uint64_t nl) { return (s * 2654435761ull) % nl; }
static inline uint64_t layer_lo(const LayerSeg &g, uint64_t l, uint64_t nl) {
    return g.p0 + (g.n * l + layer_rot(g.s, nl)) / nl;
}
// c[l] = layer_lo(g, l, nl) for l = 0..nl with one division (floor((n·l + r) / nl) stepped:
// the remainder grows by n mod nl < nl per layer, so at most one carry per step)
static inline void layer_cuts(const LayerSeg &g, uint64_t nl, uint64_t *c) {
    const uint64_t qn = g.n / nl, rn = g.n % nl;
    uint64_t q = 0, rem = layer_rot(g.s, nl);
    for (uint64_t l = 0; l <= nl; l++) {
        c[l] = g.p0 + q;
        q += qn;
        rem += rn;
        if (rem >= nl) { rem -= nl; q++; }
    }
}
// the cut points of every segment of a tile (segment i's at cuts[i·(nl+1) ..])
static void tile_cuts(const std::vector<LayerSeg> &seg, uint64_t nl, std::vector<uint64_t> &cuts) {
    cuts.resize(seg.size() * (nl + 1));
    for (size_t i = 0; i < seg.size(); i++) layer_cuts(seg[i], nl, &cuts[i * (nl + 1)]);
}

// a layer's plane bytes in k_tile<nwp, wq>'s chunk, nwp = 64 / G (s2c.h S2C_CHUNK_QBYTES_OF)
static inline uint64_t chunk_qbytes(int64_t G, int64_t wq) { return S2C_CHUNK_QBYTES_OF(64 / std::max<int64_t>(G, 1), wq); }

static bool layer_fits(const PieceBlocks &B, size_t NS, const std::vector<uint64_t> &cuts, int64_t S0, int64_t W0,
                       int64_t W1, int64_t K, int64_t G, int64_t wq, uint64_t l, uint64_t nl, std::vector<int64_t> &recs) {
    uint64_t np = 0, nh = 0, rc = 0;
    for (size_t i = 0; i < NS; i++) {
        const uint64_t lo = cuts[i * (nl + 1) + l], hi = cuts[i * (nl + 1) + l + 1];
        recs[i] = (int64_t)(uint32_t)(B.o[hi] - B.o[lo]);
        np += (uint32_t)(B.n[hi] - B.n[lo]);
        nh += (uint32_t)(B.h[hi] - B.h[lo]);
        rc += (uint64_t)recs[i];
    }
    // (planes: 8 B per 2 half-words, + the funnel word, rounded to 16 B; non-ACGT: half)
    const uint64_t qb = chunk_qbytes(G, wq);
    if (np > S2C_CHUNK_PIECES || 4 * nh + 32 > qb || 2 * nh + 32 > qb / 2 ||
        4 * rc + 32 > S2C_CHUNK_OBYTES || rc > S2C_CHUNK_RECS)
        return false;
    for (int64_t W = W0; W < W1; W++) {
        int64_t r = 0;
        for (int64_t s = std::max(W - K, S0); s <= W; s++) r += recs[s - S0];
        if (r > (int64_t)S2C_CHUNK_LANE_RECS * G) return false;
    }
    return true;
}

// nl of tile [a, e) (0: a layer cannot fit, i.e. one piece alone exceeds the chunk)
static int64_t plan_layers(const s2c_batch *b, const PieceBlocks &B, int64_t K, uint64_t a, uint64_t e, int64_t G, int64_t wq) {
    const int64_t W0 = (int64_t)(a >> 5), W1 = (int64_t)((e + 31) >> 5), S0 = std::max<int64_t>(W0 - K, 0);
    std::vector<LayerSeg> seg;
    uint64_t tp = 0, th = 0, tr = 0, maxn = 0;
    for (int64_t s = S0; s < W1; s++) {
        const uint64_t p0 = b->ps[s], n = b->ps[s + 1] - p0;
        seg.push_back({p0, n, (uint64_t)s});
        tp += (uint32_t)(B.n[p0 + n] - B.n[p0]);
        th += (uint32_t)(B.h[p0 + n] - B.h[p0]);
        tr += (uint32_t)(B.o[p0 + n] - B.o[p0]);
        maxn = std::max(maxn, n);
    }
    if (maxn == 0) return 1;
    std::vector<int64_t> recs(seg.size());
    std::vector<uint64_t> cuts;
    // the fewest layers that fit (each layer costs its DMA round trips and barriers whatever
    // it holds: C3 −2.5 %, C4 −1.2 % against a start 10 % above the capacity bound): from the
    // capacity bound up in growing steps, then bisected back to the first fitting count
    uint64_t nl = std::max<uint64_t>({1, tp / S2C_CHUNK_PIECES + 1, (4 * th) / chunk_qbytes(G, wq) + 1,
                                      tr / S2C_CHUNK_RECS + 1});
    // (past maxn layers the rotation still spreads the segments' pieces: up to 4 per piece)
    const uint64_t nlmax = std::max<uint64_t>(maxn, 4 * tp);
    nl = std::min(nl, nlmax);
    auto fits = [&](uint64_t n) {
        tile_cuts(seg, n, cuts);
        bool ok = true;
        for (uint64_t l = 0; l < n && ok; l++) ok = layer_fits(B, seg.size(), cuts, S0, W0, W1, K, G, wq, l, n, recs);
        return ok;
    };
    uint64_t bad = nl - 1;   // (a count known not to fit, or the bound − 1)
    for (;; nl = nl + 1 + nl / 16) {
        if (nl > nlmax) nl = nlmax;
        if (fits(nl)) break;
        if (nl == nlmax) return 0;
        bad = nl;
    }
    while (nl - bad > 1) {   // (bisection: a count that fits is always the one kept, monotone or not)
        const uint64_t mid = bad + (nl - bad) / 2;
        if (fits(mid)) nl = mid;
        else bad = mid;
    }
    return (int64_t)nl;
}

// Whether tile tw's window, read in place from the sorted arrays (one layer: tile word 20 =
// S2C_LY_MAIN), fits k_tile's chunk: its pieces (long ones included: their op words and
// planes are in the range) [pf0, pf1), op words [o0, o1), plane words [qw0, qw1) at their
// arrays' own 16-byte phases.
static bool main_window_fits(const s2c_batch *b, const uint32_t *tw, int64_t K, int64_t G) {
    const uint64_t np = tw[14] - tw[13], no = tw[16] - tw[15], nq = tw[18] - tw[17];
    const uint64_t qb = chunk_qbytes(G, b->info.walk_queue);   // (the instantiation that runs it)
    if (np > S2C_CHUNK_PIECES || no > S2C_CHUNK_RECS || 4 * no + 32 > S2C_CHUNK_OBYTES || 8 * nq + 32 > qb ||
        4 * nq + 32 > qb / 2)
        return false;
    const int64_t W0 = tw[0] >> 5, W1 = (tw[1] + 31) >> 5;
    for (int64_t W = W0; W < W1; W++)
        if ((int64_t)b->rs[W + 1] - (int64_t)b->rs[std::max<int64_t>(W - K, 0)] > (int64_t)S2C_CHUNK_LANE_RECS * G)
            return false;
    return true;
}

// The layered windows (s2c.h, tile words 19-20): for every tile whose window is not read in
// place, its nl layers in order, each a copy of its short pieces (records with re-based qh /
// opoff, op words, base planes and non-ACGT words of SEQ[0:len], len the record's length
// field), contiguous (the kernel's DMA takes each array's 16-byte phase).
static void build_layers(s2c_batch *b, int64_t G, bool with_dense) {
    s2c_batch_info &I = b->info;
    const int64_t NT = I.n_tiles, K = I.kwin;
    std::vector<uint64_t> lyp, lyo, lyh;   // layer starts: pieces, op words, plane half-words
    lyp.push_back(0); lyo.push_back(0); lyh.push_back(0);
    struct TL { int64_t t, ly0, nl; };
    std::vector<TL> tl;
    for (int64_t t = 0; t < NT; t++) {
        uint32_t *tw = &b->tiles[(size_t)t * S2C_TILE_WORDS];
        if ((!with_dense && (tw[3] & S2C_TILE_DENSE)) || tw[19] == 0) {   // (k_tile_dense reads its window in
            tw[20] = S2C_LY_NONE;                                          //  place; a ranged snapshot's unplanned tile)
            continue;
        }
        if (tw[19] == 1 && main_window_fits(b, tw, K, G)) {
            tw[20] = S2C_LY_MAIN;
            continue;
        }
        tl.push_back({t, 0, (int64_t)tw[19]});
    }
    PieceBlocks B;
    if (!tl.empty()) piece_blocks(b, B);
    for (TL &T : tl) {
        uint32_t *tw = &b->tiles[(size_t)T.t * S2C_TILE_WORDS];
        const int64_t nl = T.nl, W0 = tw[0] >> 5, W1 = (tw[1] + 31) >> 5, S0 = std::max<int64_t>(W0 - K, 0);
        T.ly0 = (int64_t)lyp.size() - 1;
        tw[20] = (uint32_t)T.ly0;
        std::vector<LayerSeg> seg;
        for (int64_t s = S0; s < W1; s++) seg.push_back({b->ps[s], (uint64_t)(b->ps[s + 1] - b->ps[s]), (uint64_t)s});
        std::vector<uint64_t> cuts;
        tile_cuts(seg, (uint64_t)nl, cuts);
        for (int64_t l = 0; l < nl; l++) {
            uint64_t np = 0, no = 0, nh = 0;
            for (size_t i = 0; i < seg.size(); i++) {
                const uint64_t lo = cuts[i * (nl + 1) + l], hi = cuts[i * (nl + 1) + l + 1];
                np += (uint32_t)(B.n[hi] - B.n[lo]);
                no += (uint32_t)(B.o[hi] - B.o[lo]);
                nh += (uint32_t)(B.h[hi] - B.h[lo]);
            }
            lyp.push_back(lyp.back() + np);
            lyo.push_back(lyo.back() + no);
            lyh.push_back(lyh.back() + nh);
        }
    }
    const int64_t NL = (int64_t)lyp.size() - 1;
    I.n_layers = NL;
    I.layers_dense = with_dense ? 1 : 0;
    I.n_lpieces = (int64_t)lyp.back();
    I.n_lops = (int64_t)lyo.back();
    I.n_lqwords = (int64_t)(lyh.back() / 2) + 2;   // (+ the funnel word after the last)
    b->lly.assign(4 * (size_t)(NL + 1), 0u);
    for (int64_t L = 0; L <= NL; L++) {
        b->lly[4 * L] = (uint32_t)lyp[L];
        b->lly[4 * L + 1] = (uint32_t)lyo[L];
        b->lly[4 * L + 2] = (uint32_t)lyh[L];
    }
    b->lpc.assign(4 * (size_t)(I.n_lpieces + 1), 0u);
    b->lops.assign(std::max<int64_t>(I.n_lops, 4), 0u);
    b->lbq.assign(2 * (size_t)I.n_lqwords, 0u);
    b->lbx.assign((size_t)I.n_lqwords, 0u);
    b->lpx.assign(std::max<int64_t>(I.n_lpieces, 1), 0xFFFFFFFFu);
    {
        uint32_t *sp = &b->lpc[4 * (size_t)I.n_lpieces];   // sentinel
        sp[1] = (uint32_t)lyh.back();
        sp[2] = (uint32_t)lyo.back();
    }
    auto copy_tiles = [&](size_t i0, size_t i1) {
        const uint16_t *sq = (const uint16_t *)b->bq.data(), *sx = (const uint16_t *)b->bx.data();
        uint16_t *dq = (uint16_t *)b->lbq.data(), *dx = (uint16_t *)b->lbx.data();
        for (size_t i = i0; i < i1; i++) {
            const TL &T = tl[i];
            const uint32_t *tw = &b->tiles[(size_t)T.t * S2C_TILE_WORDS];
            const int64_t W0 = tw[0] >> 5, W1 = (tw[1] + 31) >> 5, S0 = std::max<int64_t>(W0 - K, 0);
            std::vector<LayerSeg> seg;
            for (int64_t s = S0; s < W1; s++) seg.push_back({b->ps[s], (uint64_t)(b->ps[s + 1] - b->ps[s]), (uint64_t)s});
            std::vector<uint64_t> cuts;
            tile_cuts(seg, (uint64_t)T.nl, cuts);
            for (int64_t l = 0; l < T.nl; l++) {
                const int64_t L = T.ly0 + l;
                uint64_t kp = lyp[L], ko = lyo[L], kh = lyh[L];
                for (size_t i = 0; i < seg.size(); i++) {
                    const uint64_t lo = cuts[i * (T.nl + 1) + l], hi = cuts[i * (T.nl + 1) + l + 1];
                    for (uint64_t k = lo; k < hi; k++) {
                        const uint32_t *pr = &b->pc[4 * k];
                        if ((pr[3] >> 24) & S2C_PF_LONG) continue;
                        const uint32_t no = pr[6] - pr[2], nh = piece_half_words(pr[3]);
                        uint32_t *dp = &b->lpc[4 * kp];
                        dp[0] = pr[0];
                        dp[1] = (uint32_t)kh;
                        dp[2] = (uint32_t)ko;
                        dp[3] = pr[3];
                        b->lpx[kp] = b->px[k];
                        memcpy(&b->lops[ko], &b->ops[pr[2]], 4 * (size_t)no);
                        for (uint32_t h = 0; h < nh; h++) {
                            const uint64_t a = (uint64_t)pr[1] + h, d = kh + h;
                            dq[(d >> 1) * 4 + (d & 1)] = sq[(a >> 1) * 4 + (a & 1)];
                            dq[(d >> 1) * 4 + 2 + (d & 1)] = sq[(a >> 1) * 4 + 2 + (a & 1)];
                            dx[d] = sx[a];
                        }
                        kp++;
                        ko += no;
                        kh += nh;
                    }
                }
            }
        }
    };
    const size_t NTL = tl.size();
    unsigned hw = std::thread::hardware_concurrency();
    const int nt = (int)std::max<size_t>(1, std::min<size_t>(std::min<unsigned>(hw ? hw : 1, 16), NTL / 64));
    par_ranges(nt, (int64_t)NTL, [&](int, int64_t k0, int64_t k1) { copy_tiles((size_t)k0, (size_t)k1); });
}

// Work items of a tile of nl layers: {tile, c, l0, l1}, enough that each one's run records
// per word stay <= S2C_ITEM_RECS (its u16 histogram) and, past 2·IL layers, an item takes
// <= IL (parallelism for the deep tiles: C4's 16.5 kb at 100,000x); IL = 64 per-wave layers
// (16 per wave), S2C_ITEM_LAYERS overrides.
static int64_t item_layers() {
    static const int64_t il = [] {
        const char *e = plan_env("S2C_ITEM_LAYERS");
        return e ? std::max<int64_t>(4, atoll(e)) : (int64_t)64;
    }();
    return il;
}
static int64_t plan_items(const s2c_batch *b, int64_t K, uint64_t a, uint64_t e, int64_t nl, int64_t IL) {
    if (nl <= 1) return 1;   // (one layer: one item whatever its records)
    const int64_t W0 = (int64_t)(a >> 5), W1 = (int64_t)((e + 31) >> 5), S0 = std::max<int64_t>(W0 - K, 0);
    std::vector<LayerSeg> seg;
    for (int64_t s = S0; s < W1; s++) seg.push_back({b->ps[s], (uint64_t)(b->ps[s + 1] - b->ps[s]), (uint64_t)s});
    std::vector<uint64_t> cuts;
    tile_cuts(seg, (uint64_t)nl, cuts);
    // op slot of each cut (the records between two cuts: their difference)
    for (uint64_t &c : cuts) c = b->pc[4 * c + 2];
    const uint64_t stride = (uint64_t)nl + 1;
    int64_t nch = nl > 2 * IL ? (nl + IL - 1) / IL : 1;
    for (;; nch++) {
        bool ok = true;
        for (int64_t c = 0; c < nch && ok; c++) {
            const uint64_t l0 = (uint64_t)(c * nl / nch), l1 = (uint64_t)((c + 1) * nl / nch);
            for (int64_t W = W0; W < W1 && ok; W++) {
                int64_t r = 0;
                for (int64_t s = std::max(W - K, S0); s <= W; s++) {
                    const uint64_t *cs = &cuts[(uint64_t)(s - S0) * stride];
                    r += (uint32_t)(cs[l1] - cs[l0]);
                }
                ok = r <= S2C_ITEM_RECS;
            }
        }
        if (ok || nch >= nl) return nch;
    }
}

// Global coordinate of each reference's position 0 (header order, S2C_POS_ALIGN-aligned).
static std::vector<int64_t> ref_offsets(const s2c_parser *p, int64_t *padded) {
    std::vector<int64_t> off(p->ref_len.size());
    int64_t g = 0;
    for (size_t r = 0; r < off.size(); r++) {
        off[r] = g;
        g = (g + p->ref_len[r] + S2C_POS_ALIGN - 1) / S2C_POS_ALIGN * S2C_POS_ALIGN;
    }
    if (padded) *padded = g;
    return off;
}

// Global positions a read can change: its counted chars (the POS<=0 wrap puts the leading
// part at the reference's end, :212) and its emitted insertion keys.  false: none.
static bool read_extent(const Chunk &c, const ReadRec &r, int64_t off, int64_t L, int64_t *lo, int64_t *hi) {
    int64_t a = INT64_MAX, b = INT64_MIN;
    if (r.kc0 >= 0) {
        const int64_t pa = r.pos0 + r.kc0, pb = r.pos0 + r.kc1;   // [pa, pb) reference-relative
        if (pa < 0) {
            a = std::min(a, off + L + pa);
            b = std::max(b, off + L + std::min<int64_t>(pb, 0) - 1);
            if (pb > 0) { a = off; b = std::max(b, off + pb - 1); }
        } else {
            a = off + pa;
            b = off + pb - 1;
        }
    }
    for (uint32_t e = r.ev0; e < r.ev0 + r.nev; e++)
        if (c.ev[e].key >= 0) {
            a = std::min(a, off + c.ev[e].key);
            b = std::max(b, off + c.ev[e].key);
        }
    *lo = a;
    *hi = b;
    return a <= b;
}

// host phase times on stderr (S2C_HOST_TIMING=1)
struct PhaseClock {
    bool on = getenv("S2C_HOST_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char *what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "[s2c host] %-18s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

static int build_batch(s2c_parser *p, s2c_batch **out);

// pred(chunk, read, ref_off) of every read held in chunks [c0, end), on the host threads (the
// streamed batches' per-read tests: a few ms per million reads instead of tens): flags in
// chunk-then-read order
template <class Pred, class ChunkPred>
static std::vector<uint8_t> read_flags(const s2c_parser *p, size_t c0, const std::vector<int64_t> &off, Pred &&pred,
                                       ChunkPred &&chunk_may) {
    const size_t nc = p->chunks.size() > c0 ? p->chunks.size() - c0 : 0;
    std::vector<int64_t> base(nc + 1, 0);
    std::vector<uint8_t> may(nc, 1);   // (chunk_may false: every flag of the chunk is 0, no read looked at)
    for (size_t i = 0; i < nc; i++) {
        may[i] = chunk_may(*p->chunks[c0 + i]) ? 1 : 0;
        base[i + 1] = base[i] + (may[i] ? (int64_t)p->chunks[c0 + i]->reads.size() : 0);
    }
    const int64_t n = base[nc];
    std::vector<uint8_t> g((size_t)n, 0);
    par_ranges(plan_threads(n, 1 << 15), n, [&](int, int64_t i0, int64_t i1) {
        if (i0 >= i1) return;
        size_t ci = (size_t)(std::upper_bound(base.begin(), base.end(), i0) - base.begin()) - 1;
        for (int64_t i = i0; i < i1; i++) {
            while (i >= base[ci + 1]) ci++;
            const Chunk &c = *p->chunks[c0 + ci];
            const ReadRec &r = c.reads[(size_t)(i - base[ci])];
            g[(size_t)i] = pred(c, r, off[r.ref]) ? 1 : 0;
        }
    });
    // the flags of every read, chunk by chunk (0 for the chunks skipped)
    std::vector<uint8_t> f;
    f.reserve(n);
    for (size_t i = 0; i < nc; i++) {
        if (may[i]) f.insert(f.end(), g.begin() + base[i], g.begin() + base[i + 1]);
        else f.insert(f.end(), p->chunks[c0 + i]->reads.size(), (uint8_t)0);
    }
    return f;
}

// Whether a read parsed since the last retain reaches below its frontier.
static void check_late(s2c_parser *p) {
    if (p->frontier <= 0 || p->late) return;
    const std::vector<int64_t> off = ref_offsets(p, nullptr);
    const std::vector<uint8_t> f = read_flags(p, p->n_kept, off, [&](const Chunk &c, const ReadRec &r, int64_t o) {
        int64_t lo, hi;
        return read_extent(c, r, o, p->ref_len[r.ref], &lo, &hi) && lo < p->frontier;
    }, [](const Chunk &) { return true; });
    p->late = std::find(f.begin(), f.end(), (uint8_t)1) != f.end();
}

static int s2c_parser_finish_impl(s2c_parser *p, s2c_batch **out) {
    if (!p || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    int rc = feed_flush(p);
    if (rc) return rc;
    check_late(p);
    return build_batch(p, out);
}
extern "C" int s2c_parser_finish(s2c_parser *p, s2c_batch **out) {
    return s2c_guarded([&] { return s2c_parser_finish_impl(p, out); });
}

static int s2c_parser_set_tile_width_impl(s2c_parser *p, int64_t width) {
    if (!p) return s2c_set_error(S2C_ERR_ARG, "parser is NULL");
    if (width != 0 && (width < S2C_POS_ALIGN || width > 2048 || width % S2C_POS_ALIGN))
        return s2c_set_error(S2C_ERR_ARG, "tile width must be 0 or a multiple of 64 in [64, 2048]");
    p->tile_width = width;
    return S2C_OK;
}
extern "C" int s2c_parser_set_tile_width(s2c_parser *p, int64_t width) {
    return s2c_guarded([&] { return s2c_parser_set_tile_width_impl(p, width); });
}

// The batch of everything parsed so far (the partial last line stays unparsed); the
// parser keeps going.  With t_from >= 0 (s2c_parser_snapshot_from) only the tiles a streamed
// batch can run are planned: from t_from through the tile of the reads' last position.
static int s2c_parser_snapshot_impl(s2c_parser *p, int64_t t_from, s2c_batch **out) {
    if (!p || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    if (t_from >= 0 && p->tile_width <= 0) return s2c_set_error(S2C_ERR_ARG, "a ranged snapshot needs a tile width");
    check_late(p);
    p->plan_from = t_from;
    const int rc = build_batch(p, out);
    p->plan_from = -1;
    return rc;
}
extern "C" int s2c_parser_snapshot(s2c_parser *p, s2c_batch **out) {
    return s2c_guarded([&] { return s2c_parser_snapshot_impl(p, -1, out); });
}
extern "C" int s2c_parser_snapshot_from(s2c_parser *p, int64_t t_from, s2c_batch **out) {
    if (t_from < 0) return s2c_set_error(S2C_ERR_ARG, "t_from < 0");
    return s2c_guarded([&] { return s2c_parser_snapshot_impl(p, t_from, out); });
}

// Move the reads `keep` selects into one chunk (their tokens, planes and events; no line
// counted again); with events_only they keep only their insertion events (counted range
// cleared: their counts are already in the running totals).
// Append read r of chunk c to chunk d (its tokens, planes and events; no line counted
// again); with events_only it keeps only its insertion events (counted range cleared).
static void append_read(Chunk &d, const Chunk &c, const ReadRec &r, bool events_only) {
    ReadRec n = r;
    if (events_only) n.kc0 = n.kc1 = -1;
    n.tok = d.toks.size();
    d.toks.insert(d.toks.end(), c.toks.begin() + r.tok, c.toks.begin() + r.tok + r.ntok);
    n.ev0 = (uint32_t)d.ev.size();
    if (r.kc0 >= 0 || r.nev > 0) {   // its planes, 16 bases at a time
        const uint64_t q0 = (d.nq + 15) & ~(uint64_t)15, q1 = q0 + r.slen;
        const size_t need = (size_t)((q1 + 31) >> 5) + 1;
        if (d.bx.size() < need) {
            const size_t cap = std::max(need, d.bx.size() * 2);
            d.bq.resize(2 * cap, 0u);
            d.bx.resize(cap, 0u);
            d.nz = cap;   // (zero-filled)
        }
        const uint16_t *sq = (const uint16_t *)c.bq.data(), *sx = (const uint16_t *)c.bx.data();
        uint16_t *dq = (uint16_t *)d.bq.data(), *dx = (uint16_t *)d.bx.data();
        for (uint64_t h = 0; h < (r.slen + 15) / 16; h++) {
            const uint64_t s = r.q / 16 + h, t = q0 / 16 + h;
            dq[(t >> 1) * 4 + (t & 1)] = sq[(s >> 1) * 4 + (s & 1)];
            dq[(t >> 1) * 4 + 2 + (t & 1)] = sq[(s >> 1) * 4 + 2 + (s & 1)];
            dx[t] = sx[s];
        }
        d.nq = q1;
        n.q = q0;
    }
    for (uint32_t e = r.ev0; e < r.ev0 + r.nev; e++) {
        Event ev = c.ev[e];
        ev.q = ev.q - r.q + n.q;
        ev.read = (uint32_t)d.reads.size();
        d.ev.push_back(ev);
    }
    d.reads.push_back(n);
}

// Move the reads `keep` selects into one chunk; with events_only they keep only their
// insertion events (their counts are already in the running totals).
template <class Keep, class ChunkMay>
static void compact_reads(s2c_parser *p, Keep keep, ChunkMay chunk_may, bool events_only) {
    PhaseClock clk;
    const std::vector<int64_t> off = ref_offsets(p, nullptr);
    // (the tests in parallel — skipping the chunks chunk_may rules out — the copies in order)
    const std::vector<uint8_t> f = read_flags(p, 0, off, keep, [&](const Chunk &c) { return chunk_may(c, off); });
    clk.mark("retain tests");
    std::unique_ptr<Chunk> k(new Chunk());
    size_t i = 0;
    for (auto &cp : p->chunks)
        for (const ReadRec &r : cp->reads)
            if (f[i++]) {
                append_read(*k, *cp, r, events_only);
                k->bound(r.ref, r.pos0, r.klen, p->ref_len[r.ref]);
            }
    clk.mark("retain copies");
    // the dropped chunks' memory goes back on a thread of its own (hundreds of MB of reads:
    // tens of ms of page unmapping off the producer's path)
    p->free_later(std::move(p->chunks));
    p->chunks = std::vector<std::unique_ptr<Chunk>>();
    clk.mark("retain free");
    p->chunks.push_back(std::move(k));
    p->chunks.emplace_back(new Chunk());   // the sequential feed appends here
    p->n_kept = 1;
}

// Drop the reads that cannot change a global position >= gmin (their positions below it
// are emitted).
static int s2c_parser_retain_impl(s2c_parser *p, int64_t gmin) {
    if (!p) return s2c_set_error(S2C_ERR_ARG, "parser is NULL");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    if (gmin < p->frontier) return s2c_set_error(S2C_ERR_ARG, "retain: frontier moves backwards");
    compact_reads(p, [&](const Chunk &c, const ReadRec &r, int64_t off) {
        int64_t lo, hi;
        return read_extent(c, r, off, p->ref_len[r.ref], &lo, &hi) && hi >= gmin;
    }, [&](const Chunk &c, const std::vector<int64_t> &off) {   // (no read of c can reach gmin)
        // (a chunk without bounds — s2c_parser_unpack's — may hold any read: test its reads)
        if (c.hb_pos < 0) return !c.reads.empty();
        return off[c.hb_ref] + c.hb_pos >= gmin;
    }, false);
    p->frontier = gmin;
    return S2C_OK;
}
extern "C" int s2c_parser_retain(s2c_parser *p, int64_t gmin) {
    return s2c_guarded([&] { return s2c_parser_retain_impl(p, gmin); });
}

// Unsorted input: the counts of every read held are in the running totals; keep only the
// reads with insertion events, as event-only reads (their motifs are counted once, by the
// last batch, which holds every event — and the insertion checks of :284-294 see them all).
static int s2c_parser_retain_events_impl(s2c_parser *p) {
    if (!p) return s2c_set_error(S2C_ERR_ARG, "parser is NULL");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    compact_reads(p, [](const Chunk &, const ReadRec &r, int64_t) { return r.nev > 0; },
                  [](const Chunk &c, const std::vector<int64_t> &) { return !c.ev.empty(); }, true);
    return S2C_OK;
}
extern "C" int s2c_parser_retain_events(s2c_parser *p) {
    return s2c_guarded([&] { return s2c_parser_retain_events_impl(p); });
}

// Pipelined snapshots (s2c.h): the reads held move to a new parser with the same reference
// table and stream state; the feeding parser keeps its partial line and starts a new chunk.
static int s2c_parser_detach_impl(s2c_parser *p, s2c_parser **out) {
    if (!p || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    std::unique_ptr<s2c_parser> d(new s2c_parser());
    d->maxdel_active = p->maxdel_active;
    d->maxdel = p->maxdel;
    d->in_header = p->in_header;
    d->header_lines = p->header_lines;
    d->ref_names = p->ref_names;   // (the name index stays behind: d parses nothing)
    d->ref_len = p->ref_len;
    d->detached = true;
    d->last_name = p->last_name;
    d->last_ref = p->last_ref;
    d->tile_width = p->tile_width;
    d->frontier = p->frontier;
    d->n_kept = p->n_kept;
    d->late = p->late;
    d->chunks = std::move(p->chunks);
    p->chunks.clear();
    p->chunks.emplace_back(new Chunk());   // the sequential feed appends here
    p->n_kept = 0;
    *out = d.release();
    return S2C_OK;
}
extern "C" int s2c_parser_detach(s2c_parser *p, s2c_parser **out) {
    return s2c_guarded([&] { return s2c_parser_detach_impl(p, out); });
}
static int s2c_parser_attach_impl(s2c_parser *p, s2c_parser *det) {
    if (!p || !det) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    std::unique_ptr<s2c_parser> d(det);
    if (d->err && !p->err) {   // (an error of the detached reads comes first in file order)
        p->err = d->err;
        p->errmsg = d->errmsg;
    }
    std::vector<std::unique_ptr<Chunk>> cs = std::move(d->chunks);
    const size_t kept = cs.size();
    for (auto &c : p->chunks) cs.push_back(std::move(c));
    p->chunks = std::move(cs);
    // the detached parser's retained chunks are the kept ones; the reads fed since follow
    p->n_kept = kept;
    p->frontier = std::max(p->frontier, d->frontier);
    p->late = p->late || d->late;
    return S2C_OK;
}
extern "C" int s2c_parser_attach(s2c_parser *p, s2c_parser *det) {
    return s2c_guarded([&] { return s2c_parser_attach_impl(p, det); });
}

// state[0] = 1 if a read parsed after a retain reached below its frontier; state[1..2] =
// (reference index, POS - 1) of the last mapped read in file order (-1, 0: none yet);
// state[3] = reads held.
extern "C" int s2c_parser_stream_state(const s2c_parser *p, int64_t *state) {
    if (!p || !state) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    state[0] = p->late ? 1 : 0;
    state[1] = -1;
    state[2] = 0;
    state[3] = 0;
    for (auto it = p->chunks.rbegin(); it != p->chunks.rend(); ++it)
        if (!(*it)->reads.empty() && state[1] < 0) {
            state[1] = (*it)->reads.back().ref;
            state[2] = (*it)->reads.back().pos0;
        }
    for (auto &cp : p->chunks) state[3] += (int64_t)cp->reads.size();
    return S2C_OK;
}

// The insertion checks of the reformat phase (:284-294) over the reads held, per reference:
// a motif base outside -ACGNT (:287), a key outside the coverage list (:294).
static void insertion_checks(const s2c_parser *p, std::vector<uint8_t> &bad_sym, std::vector<uint8_t> &bad_key) {
    const size_t R = p->ref_names.size();
    bad_sym.assign(R, 0);
    bad_key.assign(R, 0);
    for (auto &cp : p->chunks) {
        const Chunk &c = *cp;
        for (const Event &e : c.ev) {
            const int64_t L = p->ref_len[e.ref];
            for (uint32_t j = 0; j < e.len; j++) {
                const uint64_t b = e.q + j;
                const uint32_t x = (c.bx[b >> 5] >> (b & 31)) & 1u, p1 = (c.bq[2 * (b >> 5) + 1] >> (b & 31)) & 1u;
                if (x && p1) { bad_sym[e.ref] = 1; break; }   // code 7: not in -ACGNT
            }
            if (e.key < -L || e.key >= L) bad_key[e.ref] = 1;
        }
    }
}

// ------------------------------------------------------------------ distributed parse
// Multi-GPU CLI (sam2consensus_amd/dparse.py): every rank parses its blocks of the file;
// each read goes to the ranks whose position range it can change (read_extent, as the
// streamed retain); a rank plans its sub-batch from the reads it receives.

static int s2c_parser_pos_weights_impl(s2c_parser *p, int64_t shift, int64_t *w, int64_t n) {
    if (!p || (!w && n > 0) || shift < 0 || shift > 40) return s2c_set_error(S2C_ERR_ARG, "bad argument");
    int rc = feed_flush(p);
    if (rc) return rc;
    const std::vector<int64_t> off = ref_offsets(p, nullptr);
    for (auto &cp : p->chunks)
        for (const ReadRec &r : cp->reads) {
            int64_t lo, hi;
            if (!read_extent(*cp, r, off[r.ref], p->ref_len[r.ref], &lo, &hi)) continue;
            const int64_t k = lo >> shift;
            if (k >= 0 && k < n) w[k] += r.kc0 >= 0 ? r.kc1 - r.kc0 : 1;
        }
    return S2C_OK;
}
extern "C" int s2c_parser_pos_weights(s2c_parser *p, int64_t shift, int64_t *w, int64_t n) {
    return s2c_guarded([&] { return s2c_parser_pos_weights_impl(p, shift, w, n); });
}

static int s2c_parser_checks_impl(s2c_parser *p, uint8_t *bad, int64_t n_refs) {
    if (!p || (!bad && n_refs > 0)) return s2c_set_error(S2C_ERR_ARG, "bad argument");
    if (n_refs != (int64_t)p->ref_names.size()) return s2c_set_error(S2C_ERR_ARG, "n_refs differs from the header's");
    int rc = feed_flush(p);
    if (rc) return rc;
    std::vector<uint8_t> bs, bk;
    insertion_checks(p, bs, bk);
    for (int64_t r = 0; r < n_refs; r++) {
        bad[2 * r] = bs[r];
        bad[2 * r + 1] = bk[r];
    }
    return S2C_OK;
}
extern "C" int s2c_parser_checks(s2c_parser *p, uint8_t *bad, int64_t n_refs) {
    return s2c_guarded([&] { return s2c_parser_checks_impl(p, bad, n_refs); });
}

// FASTA body assembly (:394-418): the tiles' body slots, concatenated in [threshold][tile]
// order (n blocks: raw[starts[i], starts[i] + lens[i]) → dst at the running offset), on the
// host threads for large outputs.  Every block must lie inside raw's raw_len bytes (the
// lengths come from the device: a block past the end is refused, never read).
static int s2c_gather_bodies_impl(const uint8_t *raw, int64_t raw_len, const int64_t *starts, const int64_t *lens,
                                  int64_t n, uint8_t *dst) {
    if (n < 0 || raw_len < 0 || (n > 0 && (!starts || !lens))) return s2c_set_error(S2C_ERR_ARG, "bad gather arguments");
    std::vector<int64_t> off(n + 1, 0);
    for (int64_t i = 0; i < n; i++) {
        if (lens[i] < 0 || starts[i] < 0) return s2c_set_error(S2C_ERR_ARG, "negative block");
        if (lens[i] > raw_len || starts[i] > raw_len - lens[i])
            return s2c_set_error(S2C_ERR_ARG, "body block past the end of the device output");
        off[i + 1] = off[i] + lens[i];
    }
    if (off[n] > 0 && (!raw || !dst)) return s2c_set_error(S2C_ERR_ARG, "bad gather arguments");
    par_ranges(plan_threads(off[n], (int64_t)1 << 22), n, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; i++) memcpy(dst + off[i], raw + starts[i], (size_t)lens[i]);
    });
    return S2C_OK;
}
extern "C" int s2c_gather_bodies(const uint8_t *raw, int64_t raw_len, const int64_t *starts, const int64_t *lens,
                                 int64_t n, uint8_t *dst) {
    return s2c_guarded([&] { return s2c_gather_bodies_impl(raw, raw_len, starts, lens, n, dst); });
}

// n bytes src → dst on the host threads (staging a batch into pinned buffers for its H2D:
// one thread's memcpy runs at a fraction of the memory bandwidth)
static int s2c_copy_bytes_impl(void *dst, const void *src, int64_t n) {
    if (n < 0 || (n > 0 && (!dst || !src))) return s2c_set_error(S2C_ERR_ARG, "bad copy arguments");
    const int64_t pieces = std::max<int64_t>(1, n >> 20);   // 1 MB pieces
    par_ranges(plan_threads(n, (int64_t)1 << 21), pieces, [&](int, int64_t i0, int64_t i1) {
        const int64_t a = n * i0 / pieces, b = n * i1 / pieces;
        memcpy((char *)dst + a, (const char *)src + a, (size_t)(b - a));
    });
    return S2C_OK;
}
extern "C" int s2c_copy_bytes(void *dst, const void *src, int64_t n) {
    return s2c_guarded([&] { return s2c_copy_bytes_impl(dst, src, n); });
}

extern "C" int s2c_parser_progress(const s2c_parser *p, int64_t *out) {
    if (!p || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    out[0] = p->in_header ? 0 : 1;
    out[1] = (int64_t)p->ref_names.size();
    out[2] = p->header_lines;
    out[3] = 0;
    for (auto &cp : p->chunks) out[3] += cp->lines_total;
    out[4] = p->err;
    return S2C_OK;
}

extern "C" int s2c_parser_counters(s2c_parser *p, int64_t *out) {
    if (!p || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    int rc = feed_flush(p);
    if (rc) return rc;
    out[0] = p->header_lines;
    out[1] = out[2] = out[3] = 0;
    for (auto &cp : p->chunks) {
        out[1] += cp->lines_total;
        out[2] += cp->reads_mapped;
        out[3] += cp->aligned;
    }
    return S2C_OK;
}

namespace {
struct BlobHdr {
    uint32_t magic, version;
    uint64_t n_reads, n_toks, nq, n_qw, n_ev;
};
constexpr uint32_t BLOB_MAGIC = 0x42433253u;   // "S2CB"
}  // namespace

static int s2c_parser_pack_impl(s2c_parser *p, int64_t g0, int64_t g1, size_t *len) {
    if (!p || !len) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    int rc = feed_flush(p);
    if (rc) return rc;
    const std::vector<int64_t> off = ref_offsets(p, nullptr);
    Chunk d;
    for (auto &cp : p->chunks)
        for (const ReadRec &r : cp->reads) {
            int64_t lo, hi;
            if (read_extent(*cp, r, off[r.ref], p->ref_len[r.ref], &lo, &hi) && lo < g1 && hi >= g0)
                append_read(d, *cp, r, false);
        }
    BlobHdr h{BLOB_MAGIC, (uint32_t)S2C_ABI_VERSION, d.reads.size(), d.toks.size(), d.nq, d.bx.size(), d.ev.size()};
    const size_t bytes = sizeof(h) + h.n_reads * sizeof(ReadRec) + 4 * h.n_toks + 12 * h.n_qw + h.n_ev * sizeof(Event);
    p->blob.resize(bytes);
    uint8_t *o = p->blob.data();
    auto put = [&](const void *src, size_t n) {
        if (n) memcpy(o, src, n);
        o += n;
    };
    put(&h, sizeof(h));
    put(d.reads.data(), h.n_reads * sizeof(ReadRec));
    put(d.toks.data(), 4 * h.n_toks);
    put(d.bq.data(), 8 * h.n_qw);
    put(d.bx.data(), 4 * h.n_qw);
    put(d.ev.data(), h.n_ev * sizeof(Event));
    *len = bytes;
    return S2C_OK;
}
extern "C" int s2c_parser_pack(s2c_parser *p, int64_t g0, int64_t g1, size_t *len) {
    return s2c_guarded([&] { return s2c_parser_pack_impl(p, g0, g1, len); });
}

extern "C" int s2c_parser_blob_copy(const s2c_parser *p, void *dst, size_t cap) {
    if (!p || (!dst && !p->blob.empty())) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    if (cap < p->blob.size()) return s2c_set_error(S2C_ERR_ARG, "blob larger than the buffer");
    if (!p->blob.empty()) memcpy(dst, p->blob.data(), p->blob.size());
    return S2C_OK;
}

static int s2c_parser_unpack_impl(s2c_parser *p, const void *blob, size_t len) {
    if (!p || (!blob && len)) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    int rc = feed_flush(p);
    if (rc) return rc;
    BlobHdr h;
    if (len < sizeof(h)) return s2c_set_error(S2C_ERR_ARG, "blob too short");
    memcpy(&h, blob, sizeof(h));
    if (h.magic != BLOB_MAGIC || h.version != (uint32_t)S2C_ABI_VERSION)
        return s2c_set_error(S2C_ERR_ARG, "not a blob of this library version");
    const uint64_t lim = (uint64_t)len;
    if (h.n_reads > lim || h.n_toks > lim || h.n_qw > lim || h.n_ev > lim ||
        sizeof(h) + h.n_reads * sizeof(ReadRec) + 4 * h.n_toks + 12 * h.n_qw + h.n_ev * sizeof(Event) != len ||
        (h.nq + 31) / 32 + 1 > h.n_qw + (h.n_qw == 0 ? 1 : 0))
        return s2c_set_error(S2C_ERR_ARG, "blob size does not match its header");
    std::unique_ptr<Chunk> c(new Chunk());
    const uint8_t *in = (const uint8_t *)blob + sizeof(h);
    auto get = [&](auto &vec, size_t n) {
        vec.resize(n);
        const size_t nb = n * sizeof(vec[0]);
        if (nb) memcpy(vec.data(), in, nb);
        in += nb;
    };
    get(c->reads, h.n_reads);
    get(c->toks, h.n_toks);
    get(c->bq, 2 * h.n_qw);
    get(c->bx, h.n_qw);
    get(c->ev, h.n_ev);
    c->nq = h.nq;
    c->nz = h.n_qw;
    const size_t R = p->ref_names.size();
    for (const ReadRec &r : c->reads)   // indices into this chunk and the header's references
        if (r.ref >= R || r.tok + r.ntok > h.n_toks || (uint64_t)r.ev0 + r.nev > h.n_ev ||
            ((r.kc0 >= 0 || r.nev > 0) && r.q + r.slen > 32 * h.n_qw))
            return s2c_set_error(S2C_ERR_ARG, "blob read out of range");
    for (const Event &e : c->ev)
        if (e.ref >= R || e.read >= h.n_reads || e.q + e.len > 32 * h.n_qw)
            return s2c_set_error(S2C_ERR_ARG, "blob event out of range");
    p->chunks.push_back(std::move(c));
    p->chunks.emplace_back(new Chunk());   // the sequential feed appends here
    return S2C_OK;
}
extern "C" int s2c_parser_unpack(s2c_parser *p, const void *blob, size_t len) {
    return s2c_guarded([&] { return s2c_parser_unpack_impl(p, blob, len); });
}

// Opt-in phase clock of the host plan (S2C_HOST_TIMING=1: one line per phase on stderr).

// px of a piece of read r (s2c.h S2C_PF_XFEW): the SEQ offsets of its first two non-ACGT
// chars when they are all 'N' (no '-': the maxdel rule never needs the plane scan), at most
// two and below 0xFFFF; sets S2C_PF_XFEW in fl.  0xFFFFFFFF otherwise.
static uint32_t xfew_offsets(const Chunk &c, const ReadRec &r, uint32_t &fl) {
    if (!(r.has_x & 1) || (r.has_x & 2)) return 0xFFFFFFFFu;
    const uint16_t *sx = (const uint16_t *)c.bx.data();
    uint32_t off[2] = {0xFFFFu, 0xFFFFu}, nf = 0;
    for (uint64_t h = 0; h < ((uint64_t)r.slen + 15) / 16; h++) {
        uint32_t m = sx[r.q / 16 + h];
        while (m) {
            const uint64_t o = 16 * h + (uint64_t)__builtin_ctz(m);
            m &= m - 1;
            if (o >= r.slen) break;
            if (nf == 2 || o >= 0xFFFFu) return 0xFFFFFFFFu;
            off[nf++] = (uint32_t)o;
        }
    }
    if (nf == 0) return 0xFFFFFFFFu;
    fl |= S2C_PF_XFEW;
    return off[0] | off[1] << 16;
}

static int build_batch(s2c_parser *p, s2c_batch **out) {
    PhaseClock clk;
    const int64_t R = (int64_t)p->ref_names.size();
    auto &CH = p->chunks;

    // ---- reformat-phase checks (:284-294), refs in header order: motif symbols (KeyError,
    //      :287) are checked for every key before any key's coverage lookup (IndexError, :294)
    {
        std::vector<uint8_t> bad_sym, bad_key;
        insertion_checks(p, bad_sym, bad_key);
        for (int64_t r = 0; r < R; r++) {
            if (bad_sym[r]) return s2c_set_error(S2C_ERR_KEY, "KeyError: insertion base not in -ACGNT (:287)");
            if (bad_key[r]) return s2c_set_error(S2C_ERR_INDEX, "IndexError: insertion key out of range (:294)");
        }
    }

    clk.mark("checks");
    s2c_batch *b = new s2c_batch();
    std::unique_ptr<s2c_batch> guard(b);
    s2c_batch_info &I = b->info;
    b->names = p->ref_names;
    b->ref_len = p->ref_len;
    b->ref_off.resize(R);
    b->ref_reads.assign(R, 0);
    int64_t g = 0;
    for (int64_t r = 0; r < R; r++) {
        b->ref_off[r] = g;
        g = align_up(g + p->ref_len[r], S2C_POS_ALIGN);
    }
    const int64_t Lpad = std::max<int64_t>(g, S2C_POS_ALIGN);
    if (Lpad >= ((int64_t)1 << 32) - 4096) return s2c_set_error(S2C_ERR_LIMIT, "more than 2^32 reference positions");
    const int64_t NW = Lpad / 32;
    I.n_refs = R;
    I.padded_len = Lpad;
    I.n_words = NW;
    I.word_lo = 0;
    I.word_hi = NW;
    for (int64_t r = 0; r < R; r++) I.total_len += p->ref_len[r];
    I.header_lines = p->header_lines;
    for (auto &cp : CH) {
        I.lines_total += cp->lines_total;
        I.reads_mapped += cp->reads_mapped;
        I.aligned_bases += cp->aligned;
        I.query_bases += cp->qbases;
        I.n_tokens += cp->ntokens;
    }

    // ---- pieces: the counted range of each read, split at the POS<=0 wrap (:212), plus a
    //      zero-span piece for a read whose insertion events have nothing counted; in file
    //      order (chunk by chunk), counted and then written by the host threads ----
    const int64_t NC = (int64_t)CH.size();
    // the pieces of read ri of chunk ci into dst (nullptr: count only); returns how many
    auto read_pieces = [&](uint32_t ci, uint32_t ri, Piece *dst, int64_t *span, int64_t *nrd) -> int {
        const Chunk &c = *CH[ci];
        const ReadRec &r = c.reads[ri];
        const int64_t L = p->ref_len[r.ref], off = b->ref_off[r.ref];
        bool any_key = false;   // an event the consensus can emit (key >= 0)
        uint64_t kmin = ~0ull, kmax = 0;
        for (uint32_t e = r.ev0; e < r.ev0 + r.nev; e++)
            if (c.ev[e].key >= 0) {
                any_key = true;
                kmin = std::min<uint64_t>(kmin, (uint64_t)(off + c.ev[e].key));
                kmax = std::max<uint64_t>(kmax, (uint64_t)(off + c.ev[e].key));
            }
        Piece tmp[2];
        int n = 0;
        if (r.kc0 >= 0) {
            const int64_t pa = r.pos0 + r.kc0;
            if (pa < 0) {
                const int64_t kb = std::min(r.kc1, -r.pos0);
                tmp[n++] = {(uint64_t)(off + L + pa), r.kc0, kb, ci, ri, 1, 0, 0, 0, 0, 0, 0, 0};
                if (r.kc1 > -r.pos0) tmp[n++] = {(uint64_t)off, -r.pos0, r.kc1, ci, ri, 1, 0, 0, 0, 0, 0, 0, 0};
            } else {
                const bool whole = r.kc0 == 0 && r.kc1 == r.klen;
                tmp[n++] = {(uint64_t)(off + pa), r.kc0, r.kc1, ci, ri, (uint8_t)!whole, 0, 0, 0, 0, 0, 0, 0};
            }
            nrd[r.ref] += n;
        }
        if (any_key) {   // (a read with events but nothing counted: a zero-span piece at its first key)
            if (n == 0) tmp[n++] = {kmin, 0, 0, ci, ri, 1, 0, 0, 0, 0, 0, 0, 0};
            tmp[0].ins = 1;
            tmp[0].kmin = (uint32_t)kmin;
            tmp[0].kmax = (uint32_t)kmax;
        }
        for (int k = 0; k < n; k++) {
            span[r.ref] += tmp[k].kb - tmp[k].ka;
            tmp[k].nslots = r.ntok + (tmp[k].range ? 2u : 0u) + (tmp[k].ins ? 3u : 0u);
            tmp[k].qlen = (uint32_t)align_up(r.slen, 16);
            tmp[k].ref = r.ref;
            if (dst) dst[k] = tmp[k];
        }
        return n;
    };
    std::vector<int64_t> chof(NC + 1, 0);
    const int ntp = plan_threads(NC, 1);
    std::vector<std::vector<int64_t>> tspan(ntp, std::vector<int64_t>(R, 0)), treads(ntp, std::vector<int64_t>(R, 0));
    {
        std::atomic<int64_t> nextc{0};
        par_ranges(ntp, ntp, [&](int t, int64_t, int64_t) {   // pass 1: pieces per chunk
            std::vector<int64_t> sp(R, 0), rd(R, 0);
            for (int64_t ci; (ci = nextc++) < NC;) {
                int64_t n = 0;
                for (uint32_t ri = 0; ri < (uint32_t)CH[ci]->reads.size(); ri++) n += read_pieces((uint32_t)ci, ri, nullptr, sp.data(), rd.data());
                chof[ci + 1] = n;
            }
            (void)t;
        });
    }
    for (int64_t ci = 0; ci < NC; ci++) chof[ci + 1] += chof[ci];
    std::vector<Piece, uninit_alloc<Piece>> pcs((size_t)chof[NC]);
    {
        std::atomic<int64_t> nextc{0};
        par_ranges(ntp, ntp, [&](int t, int64_t, int64_t) {   // pass 2: written in place
            for (int64_t ci; (ci = nextc++) < NC;) {
                Piece *dst = pcs.data() + chof[ci];
                for (uint32_t ri = 0; ri < (uint32_t)CH[ci]->reads.size(); ri++)
                    dst += read_pieces((uint32_t)ci, ri, dst, tspan[t].data(), treads[t].data());
            }
        });
    }
    std::vector<int64_t> ref_span(R, 0);
    for (int t = 0; t < ntp; t++)
        for (int64_t r = 0; r < R; r++) {
            ref_span[r] += tspan[t][r];
            b->ref_reads[r] += treads[t][r];
        }
    clk.mark("pieces");
    const int64_t NP = (int64_t)pcs.size();
    if (NP >= ((int64_t)1 << 32) - 2) return s2c_set_error(S2C_ERR_LIMIT, "more than 2^32 pieces (split the input)");
    I.n_pieces = NP;

    // ---- window: pieces up to S positions are short (reached from the run-slot CSR of the
    //      kwin + 1 words before a word); the rare longer ones go to the tile long lists ----
    int64_t S = 64;
    const int ntw = plan_threads(NP, 1 << 18);
    {
        std::vector<std::vector<int64_t>> th(ntw, std::vector<int64_t>(4097, 0));
        par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
            for (int64_t k = k0; k < k1; k++) th[t][std::min<int64_t>(pcs[k].kb - pcs[k].ka, 4096)]++;
        });
        std::vector<int64_t> hist(4097, 0);
        for (int t = 0; t < ntw; t++)
            for (int s = 0; s <= 4096; s++) hist[s] += th[t][s];
        int64_t above = NP, lim = NP / 1000;
        for (int64_t s = 0; s <= 4096; s++) {
            above -= hist[s];
            if (s >= 64 && above <= lim) { S = s; break; }
        }
        S = std::min<int64_t>(S, 1024);
    }
    int64_t K = 0;
    {
        std::vector<int64_t> tk(ntw, 0);
        par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
            int64_t kk = 0;
            for (int64_t k = k0; k < k1; k++) {
                Piece &q = pcs[k];
                const int64_t span = q.kb - q.ka;
                // long: a span past the window, or a piece too big for a quarter of k_tile's
                // per-wave chunk (its runs then come from k_reads through the long lists)
                q.lng = span > S || q.nslots > S2C_CHUNK_RECS / 4 || 4 * (uint64_t)(q.qlen / 16) + 32 > S2C_CHUNK_QBYTES / 4;
                if (!q.lng && span > 0) kk = std::max<int64_t>(kk, (int64_t)(((q.gpos + span - 1) >> 5) - (q.gpos >> 5)));
            }
            tk[t] = kk;
        });
        for (int t = 0; t < ntw; t++) K = std::max(K, tk[t]);
    }
    I.kwin = K;

    clk.mark("window");
    // ---- bucket the pieces by start word (counting sort, stable in file order) ----
    std::vector<uint32_t, uninit_alloc<uint32_t>> order(NP);
    {
        std::atomic<bool> sorted{true};   // (coordinate-sorted input: already in word order)
        par_ranges(ntw, NP, [&](int, int64_t k0, int64_t k1) {
            for (int64_t k = std::max<int64_t>(k0, 1); k < k1 && sorted; k++)
                if ((pcs[k].gpos >> 5) < (pcs[k - 1].gpos >> 5)) sorted = false;
        });
        if (sorted) {
            par_ranges(ntw, NP, [&](int, int64_t k0, int64_t k1) {
                for (int64_t k = k0; k < k1; k++) order[k] = (uint32_t)k;
            });
        } else if ((uint64_t)(NW + 1) * (uint64_t)ntw <= ((uint64_t)1 << 27)) {
            // per-range histograms, word-major offsets, stable scatter (ranges in file order)
            std::vector<std::vector<uint32_t>> cnt(ntw);
            par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
                cnt[t].assign(NW + 1, 0u);
                for (int64_t k = k0; k < k1; k++) cnt[t][pcs[k].gpos >> 5]++;
            });
            uint64_t run = 0;
            for (int64_t w = 0; w <= NW; w++)
                for (int t = 0; t < ntw; t++) {
                    const uint32_t c = cnt[t][w];
                    cnt[t][w] = (uint32_t)run;
                    run += c;
                }
            par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
                for (int64_t k = k0; k < k1; k++) order[cnt[t][pcs[k].gpos >> 5]++] = (uint32_t)k;
            });
        } else {
            std::vector<uint64_t> cnt(NW + 1, 0);
            for (int64_t i = 0; i < NP; i++) cnt[(pcs[i].gpos >> 5) + 1]++;
            for (int64_t w = 0; w < NW; w++) cnt[w + 1] += cnt[w];
            for (int64_t i = 0; i < NP; i++) order[cnt[pcs[i].gpos >> 5]++] = (uint32_t)i;
        }
    }
    // piece CSR by start word: ps[w] = the first sorted piece starting in word ≥ w
    b->ps.resize(NW + 1);
    par_ranges(ntw, NP, [&](int, int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; k++) {
            const int64_t wk = (int64_t)(pcs[order[k]].gpos >> 5), wp = k ? (int64_t)(pcs[order[k - 1]].gpos >> 5) : -1;
            for (int64_t w = wp + 1; w <= wk; w++) b->ps[w] = (uint32_t)k;
        }
    });
    for (int64_t w = NP ? (int64_t)(pcs[order[NP - 1]].gpos >> 5) + 1 : 0; w <= NW; w++) b->ps[w] = (uint32_t)NP;
    clk.mark("bucket");
    // output offsets (ops, bases) in sorted order
    std::vector<uint64_t, uninit_alloc<uint64_t>> ooff(NP + 1), qoff(NP + 1);
    ooff[0] = qoff[0] = 0;
    {   // (range sums, then each range's prefix from its base)
        std::vector<uint64_t> so(ntw + 1, 0), sq(ntw + 1, 0);
        par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
            uint64_t a = 0, q = 0;
            for (int64_t k = k0; k < k1; k++) {
                const Piece &pc = pcs[order[k]];
                a += pc.nslots;
                q += pc.qlen;
                ooff[k + 1] = a;
                qoff[k + 1] = q;
            }
            so[t + 1] = a;
            sq[t + 1] = q;
        });
        for (int t = 0; t < ntw; t++) { so[t + 1] += so[t]; sq[t + 1] += sq[t]; }
        par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
            for (int64_t k = k0; k < k1; k++) { ooff[k + 1] += so[t]; qoff[k + 1] += sq[t]; }
        });
    }
    clk.mark("offsets");
    const uint64_t NOPS = ooff[NP], NQ = qoff[NP];
    // the kernels address run records and base planes with 32-bit buffer offsets (< 3.5 GB)
    if (16 * NOPS >= 0xE0000000ull) return s2c_set_error(S2C_ERR_LIMIT, "more than 2^28 op words (split the input)");
    if (NQ / 4 >= 0xE0000000ull) return s2c_set_error(S2C_ERR_LIMIT, "more than 14 G query bases (split the input)");
    I.n_ops = (int64_t)NOPS;
    I.n_qwords = (int64_t)((NQ + 31) / 32) + 2;
    b->pc.resize(4 * (size_t)(NP + 1));
    b->kmin.resize(NP);
    b->kmax.resize(NP);
    b->lmot.resize(NP);
    b->px.resize(std::max<int64_t>(NP, 1));
    b->ops.resize(std::max<uint64_t>(NOPS, 1));
    b->bq.resize(2 * (size_t)I.n_qwords);
    b->bx.resize((size_t)I.n_qwords);
    {   // the words the pieces do not cover: from the half-word after the last piece's bases on
        const uint64_t h0 = NQ / 16, nh = 2 * (uint64_t)I.n_qwords;
        uint16_t *dq = (uint16_t *)b->bq.data(), *dx = (uint16_t *)b->bx.data();
        for (uint64_t d = h0; d < nh; d++) {
            dq[(d >> 1) * 4 + (d & 1)] = 0;
            dq[(d >> 1) * 4 + 2 + (d & 1)] = 0;
            dx[d] = 0;
        }
        b->ops[0] = 0;
        for (int j = 0; j < 4; j++) b->pc[4 * (size_t)NP + j] = 0;
    }
    clk.mark("alloc");
    {   // emit in parallel over ranges of sorted pieces (each thread first-touches its range)
        const int nt = plan_threads(NP, 65536);
        auto emit = [&](int64_t k0, int64_t k1) {
            uint16_t *dq = (uint16_t *)b->bq.data();   // half-words: [k][plane][2 halves]
            uint16_t *dx = (uint16_t *)b->bx.data();
            for (int64_t k = k0; k < k1; k++) {
                const Piece &q = pcs[order[k]];
                const Chunk &c = *CH[q.chunk];
                const ReadRec &r = c.reads[q.read];
                uint32_t *o = &b->ops[ooff[k]];
                uint32_t fl = (r.has_x ? S2C_PF_X : 0u) | ((r.has_x & 2) ? S2C_PF_DASH : 0u);
                if (q.range) { fl |= S2C_PF_RANGE; *o++ = (uint32_t)q.ka; *o++ = (uint32_t)q.kb; }
                b->kmin[k] = 0xFFFFFFFFu;
                b->kmax[k] = 0u;
                b->lmot[k] = 0;
                if (q.ins) {
                    fl |= S2C_PF_INS;
                    b->kmin[k] = q.kmin;
                    b->kmax[k] = q.kmax;
                    for (uint32_t e = r.ev0; e < r.ev0 + r.nev; e++)
                        if (c.ev[e].key >= 0 && c.ev[e].len > S2C_SHORT_MOTIF) b->lmot[k] = 1;
                    const int64_t off = b->ref_off[r.ref], key0 = off + r.pos0;
                    *o++ = (uint32_t)(uint64_t)key0;
                    *o++ = (uint32_t)((uint64_t)key0 >> 32);
                    *o++ = (uint32_t)off;
                }
                if (q.lng) fl |= S2C_PF_LONG;
                memcpy(o, &c.toks[r.tok], 4 * (size_t)r.ntok);
                b->px[k] = xfew_offsets(c, r, fl);
                uint32_t slen = r.slen;
                if (!q.range && !q.ins && !q.lng && r.ntok == 1 && op_bases(c.toks[r.tok] & 15u) && !(fl & S2C_PF_DASH)) {
                    fl |= S2C_PF_SIMPLE;   // seqout = SEQ[0:take]: the field holds take (s2c.h)
                    slen = std::min<uint32_t>(c.toks[r.tok] >> 4, r.slen);
                }
                uint32_t *pr = &b->pc[4 * (size_t)k];
                pr[0] = (uint32_t)q.gpos;
                pr[1] = (uint32_t)(qoff[k] / 16);
                pr[2] = (uint32_t)ooff[k];
                pr[3] = slen | (fl << 24);
                // the read's planes, 16 bases at a time (both sides start at multiples of 16)
                const uint16_t *sq = (const uint16_t *)c.bq.data(), *sx = (const uint16_t *)c.bx.data();
                for (uint64_t h = 0; h < (r.slen + 15) / 16; h++) {
                    const uint64_t s = r.q / 16 + h, d = qoff[k] / 16 + h;
                    dq[(d >> 1) * 4 + (d & 1)] = sq[(s >> 1) * 4 + (s & 1)];           // p0
                    dq[(d >> 1) * 4 + 2 + (d & 1)] = sq[(s >> 1) * 4 + 2 + (s & 1)];   // p1
                    dx[d] = sx[s];
                }
            }
        };
        par_ranges(nt, NP, [&](int, int64_t k0, int64_t k1) { emit(k0, k1); });
    clk.mark("emit threads");
        uint32_t *pr = &b->pc[4 * (size_t)NP];   // sentinel
        pr[1] = (uint32_t)(NQ / 16);
        pr[2] = (uint32_t)NOPS;
        // run-slot CSR by start word: the op slots before the first piece of word w
        b->rs.resize(NW + 1);
        par_ranges(plan_threads(NW + 1, 1 << 16), NW + 1, [&](int, int64_t w0, int64_t w1) {
            for (int64_t w = w0; w < w1; w++) b->rs[w] = (uint32_t)ooff[b->ps[w]];
        });
    }

    {   // pieces walked op by op (neither one token nor long): k_tile's walk queue pays for them
        std::atomic<int64_t> nw{0};
        par_ranges(plan_threads(NP, 1 << 18), NP, [&](int, int64_t k0, int64_t k1) {
            int64_t m = 0;
            for (int64_t k = k0; k < k1; k++) m += !((b->pc[4 * k + 3] >> 24) & (S2C_PF_SIMPLE | S2C_PF_LONG));
            nw += m;
        });
        I.n_walked = nw;
    }
    clk.mark("emit");
    // ---- tiles: width from depth; a shallow tile keeps its window's runs in LDS ----
    struct Tile { int64_t a, b, ref; };
    std::vector<Tile> tiles;
    int64_t tile_max = S2C_POS_ALIGN;
    int64_t tile_force = 0;   // diagnostic override (S2C_TILE_POS, a multiple of 64 in [64, 2048])
    const bool no_dense = plan_env("S2C_NO_DENSE") != nullptr;   // diagnostic: every tile through k_tile
    if (const char *e = plan_env("S2C_TILE_POS"))
        tile_force = align_up(std::min<int64_t>(std::max<int64_t>(atoll(e), 64), TP_MAX), S2C_POS_ALIGN);
    if (p->tile_width > 0) tile_force = p->tile_width;   // streamed batches: the same tiles every time
    std::vector<int64_t> ref_slots(R, 0), ref_np(R, 0), ref_qw(R, 0);
    std::vector<int64_t> longs;   // sorted indices of the long pieces
    {
        std::vector<std::vector<int64_t>> ts(ntw, std::vector<int64_t>(3 * R, 0)), tl(ntw);
        par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
            int64_t *a = ts[t].data();
            for (int64_t k = k0; k < k1; k++) {   // (a piece's reference from its start position)
                const Piece &q = pcs[order[k]];
                const uint32_t ref = q.ref;
                a[3 * ref] += q.nslots;
                a[3 * ref + 1]++;
                a[3 * ref + 2] += q.qlen;
                if (q.lng) tl[t].push_back(k);
            }
        });
        for (int t = 0; t < ntw; t++) {
            for (int64_t r = 0; r < R; r++) {
                ref_slots[r] += ts[t][3 * r];
                ref_np[r] += ts[t][3 * r + 1];
                ref_qw[r] += ts[t][3 * r + 2];
            }
            longs.insert(longs.end(), tl[t].begin(), tl[t].end());
        }
    }
    for (int64_t r = 0; r < R; r++) {
        const int64_t L = p->ref_len[r], off = b->ref_off[r];
        if (L == 0) continue;
        const double depth = (double)ref_span[r] / (double)L, spp = (double)ref_slots[r] / (double)L;
        // deep: ≈ E_TARGET aligned bases per tile, a power of two of words (every counting lane
        // of k_tile's waves busy) and at least S2C_DEEP_TILE positions (default 512: measured
        // against 256 / 320 on C3 and 256 on C4, profiles/r03/)
        int64_t tp = TP_MAX;
        if (depth > 0) {
            const double want = std::max(64.0, std::ceil(E_TARGET / depth));
            tp = (int64_t)1 << (int64_t)std::llround(std::log2(want));
            tp = std::max<int64_t>(tp, deep_tile_min());
        }
        const double win = 32.0 * (double)(K + 1) * spp;    // run slots per word's window
        if (win <= 200.0 && spp > 0) {
            // shallow: the widest tile whose window (12 B per op slot and 12 B per base plane word
            // in LDS, plane words below S2C_DENSE_QW; with a margin for the depth's spread) fits
            // the dense kernel
            const double qpp = ((double)ref_qw[r] / 32.0 + 0.25 * (double)ref_np[r]) / (double)L;
            const double bpp = (16.0 * (double)ref_slots[r] / (double)L) + 8.0 * qpp;   // S2C_DENSE_BYTES per position
            tp = TP_MAX;
            while (tp > TP_MIN && (((double)tp + 32.0 * (double)(K + 1)) * bpp + 1024.0 > DENSE_PLAN_BYTES ||
                                   ((double)tp + 32.0 * (double)(K + 1)) * qpp > 0.8 * S2C_DENSE_QW))
                tp /= 2;
        }
        tp = std::min(std::max(tp, TP_MIN), TP_MAX);
        if (tile_force > 0) tp = tile_force;
        const int64_t nt = ceil_div(L, tp);
        const int64_t step = align_up(ceil_div(L, nt), S2C_POS_ALIGN);
        for (int64_t a = off; a < off + L; a += step) {
            tiles.push_back({a, std::min(a + step, off + L), r});
            tile_max = std::max(tile_max, tiles.back().b - a);
        }
    }
    // A ranged snapshot (s2c_parser_snapshot_from) plans tiles [P0, P1) only: from the first
    // tile its streamed batch runs through the tile of the held reads' last position (the
    // pieces' ends, the last read's POS: the stream driver's bound); the other tiles keep
    // their bounds and insertion capacities but get no window, layers or work items
    int64_t P0 = 0, P1 = INT64_MAX;   // (a whole batch: every tile, after any split below)
    if (p->plan_from >= 0) {   // (a fixed tile width: no split)
        const int64_t NT0 = (int64_t)tiles.size();
        std::vector<int64_t> tmax(ntw, -1);
        par_ranges(ntw, NP, [&](int t, int64_t k0, int64_t k1) {
            int64_t m = -1;
            for (int64_t k = k0; k < k1; k++)
                if (pcs[k].kb > pcs[k].ka) m = std::max<int64_t>(m, (int64_t)pcs[k].gpos + (pcs[k].kb - pcs[k].ka) - 1);
            tmax[t] = m;
        });
        int64_t gmax = *std::max_element(tmax.begin(), tmax.end());
        for (auto it = p->chunks.rbegin(); it != p->chunks.rend(); ++it)
            if (!(*it)->reads.empty()) {
                const ReadRec &r = (*it)->reads.back();
                const int64_t L = p->ref_len[r.ref];
                if (L > 0) gmax = std::max<int64_t>(gmax, b->ref_off[r.ref] + std::min<int64_t>(std::max<int64_t>(r.pos0, 0), L - 1));
                break;
            }
        P0 = std::min<int64_t>(p->plan_from, NT0);
        int64_t tl = P0;   // first tile past gmax
        if (gmax >= 0) {
            int64_t lo = 0, hi = NT0;   // first tile with a > gmax
            while (lo < hi) {
                const int64_t m = (lo + hi) / 2;
                if (tiles[m].a > gmax) hi = m; else lo = m + 1;
            }
            tl = lo;
        }
        P1 = std::min<int64_t>(std::max<int64_t>(tl, P0), NT0);
    }
    auto planned = [&](int64_t t) { return t >= P0 && t < P1; };
    // Launch LDS of k_tile_dense = the largest dense window, so one outlier window sets every
    // tile's occupancy: when all but ≤ 0.2 % of the windows fit the share of a CU's 160 KB
    // that lets 8 two-wave tiles reside (4 waves per SIMD, the kernel's register budget), the
    // launch is sized to that share and the few tiles over it are split in two (each half's
    // window fits; C5: 55 of 62,934 tiles), unless the tile width is fixed (streamed batches)
    int64_t dense_cap = S2C_DENSE_LDS;
    {
        const int64_t nwp = tile_max <= 512 ? 16 : tile_max <= 1024 ? 32 : 64;
        // (the kernel's static LDS; its dynamic LDS is never below S2C_DENSE_MIN_LDS, so for
        // 2048-position tiles (cap8 14,208 B) 8 tiles per CU cannot reside whatever the windows:
        // no tile is split for it)
        const int64_t cap8 = 163840 / 8 - (96 * nwp + 128);
        const int64_t n0 = (int64_t)tiles.size();
        std::vector<int64_t> db(n0, -1);
        const int64_t q0 = std::min(P0, n0), q1 = std::min(P1, n0);   // (the planned tiles only: balanced ranges)
        par_ranges(plan_threads(q1 - q0, 64), q1 - q0, [&](int, int64_t i0, int64_t i1) {
            uint32_t tw[S2C_TILE_WORDS];
            for (int64_t t = q0 + i0; t < q0 + i1; t++) {
                tile_window(b, K, (uint64_t)tiles[t].a, (uint64_t)tiles[t].b, tw);
                if (dense_fits(tw, K)) db[t] = dense_bytes(tw, K);
            }
        });
        int64_t nfit = 0, over = 0;
        for (const int64_t x : db)
            if (x >= 0) { nfit++; over += x > cap8; }
        if (over > 0 && over * 500 <= nfit && cap8 >= S2C_DENSE_MIN_LDS) {
            dense_cap = cap8;
            if (tile_force == 0) {
                std::vector<Tile> split;
                split.reserve(n0 + over);
                for (int64_t t = 0; t < n0; t++) {
                    const Tile &T = tiles[t];
                    const int64_t mid = T.a + align_up((T.b - T.a) / 2, S2C_POS_ALIGN);
                    if (db[t] > cap8 && mid < T.b) {
                        split.push_back({T.a, mid, T.ref});
                        split.push_back({mid, T.b, T.ref});
                    } else {
                        split.push_back(T);
                    }
                }
                tiles.swap(split);
            }
        }
    }
    const int64_t NT = (int64_t)tiles.size();
    I.n_tiles = NT;
    I.tile_max = tile_max;
    I.plan_t0 = P0;
    I.plan_t1 = std::min<int64_t>(P1, NT);
    b->wtile.resize(NW);
    par_ranges(plan_threads(NW, 1 << 16), NW, [&](int, int64_t w0, int64_t w1) {
        std::fill(b->wtile.begin() + w0, b->wtile.begin() + w1, 0xFFFFFFFFu);
    });
    par_ranges(plan_threads(NT, 1 << 10), NT, [&](int, int64_t t0, int64_t t1) {   // (tiles hold disjoint words)
        for (int64_t t = t0; t < t1; t++)
            for (int64_t W = tiles[t].a >> 5; W < (tiles[t].b + 31) >> 5; W++) b->wtile[W] = (uint32_t)t;
    });

    clk.mark("tiles");
    // ---- long lists: run slots of long pieces per tile they overlap ----
    std::vector<uint32_t> lcnt(NT + 1, 0);
    auto for_long = [&](auto fn) {
        for (const int64_t k : longs) {
            const Piece &q = pcs[order[k]];
            const uint32_t t0 = b->wtile[q.gpos >> 5], t1 = b->wtile[(q.gpos + (q.kb - q.ka) - 1) >> 5];
            for (uint32_t t = t0; t <= t1; t++) fn(t, k);
        }
    };
    for_long([&](uint32_t t, int64_t k) { lcnt[t + 1] += pcs[order[k]].nslots; });
    for (int64_t t = 0; t < NT; t++) lcnt[t + 1] += lcnt[t];
    b->lp.resize(std::max<uint32_t>(lcnt[NT], 1));
    {
        std::vector<uint32_t> at(lcnt.begin(), lcnt.end() - 1);
        for_long([&](uint32_t t, int64_t k) {
            for (uint64_t s = ooff[k]; s < ooff[k + 1]; s++) b->lp[at[t]++] = (uint32_t)s;
        });
    }
    I.n_long = lcnt[NT];

    clk.mark("long lists");
    // ---- insertion plan: per tile its events' hash-table capacity, long-motif slots and an
    //      upper bound of its columns (Σ motif lengths ≥ Σ over keys of the longest, :278-281)
    std::vector<uint32_t> nshort(NT, 0), nlong(NT, 0), nev(NT, 0);
    std::vector<uint64_t> ccap(NT, 0);
    for (auto &cp : CH)
        for (const Event &e : cp->ev) {
            if (e.key < 0) continue;   // never emitted (:355 walks 0..LN-1)
            const uint64_t gk = (uint64_t)(b->ref_off[e.ref] + e.key);
            const uint32_t t = b->wtile[gk >> 5];
            nev[t]++;
            (e.len <= S2C_SHORT_MOTIF ? nshort : nlong)[t]++;
            ccap[t] += e.len;
            I.n_ins++;
            I.n_ins_bases += e.len;
        }

    clk.mark("ins plan");
    // ---- work items: per tile its layers (k_tile's per-wave LDS chunks; lane groups of G = 64 / nwp
    //      lanes per word) split into items ----
    int64_t nwp = 8;
    while (nwp * 32 < tile_max) nwp *= 2;
    const int64_t G = 64 / nwp;   // (counting lanes per word of one wave: each wave runs its own layers)
    I.chunk = 0;   // (the most layers of any tile)
    PieceBlocks PB;
    piece_blocks(b, PB);
    clk.mark("piece blocks");
    const int64_t lcols = S2C_LDS_COLS(nwp);
    b->tiles.assign((size_t)NT * S2C_TILE_WORDS, 0u);
    uint64_t boff = 0, loff = 0, coff = 0;
    int64_t runs_max = 0;
    // the k_tile instantiation the layers are cut for (its chunk's plane bytes): a shard of this
    // batch keeps the non-queue one when this is planned for it (mark_runs)
    I.walk_queue = walk_queue_of(I);
    const int64_t wq = I.walk_queue;
    // per tile (host threads): its window, the most candidate runs of a word, layers, items
    std::vector<int64_t> t_nl(NT, 0), t_nch(NT, 0), t_maxc(NT, 0), t_wruns(NT, 0);   // (0: an unplanned tile)
    std::atomic<bool> too_big{false};
    const int64_t q0 = std::min(P0, NT), q1 = std::min(P1, NT);   // the planned tiles, in balanced ranges
    par_ranges(plan_threads(q1 - q0, 64), q1 - q0, [&](int, int64_t i0, int64_t i1) {
        for (int64_t t = q0 + i0; t < q0 + i1; t++) {
            const Tile &T = tiles[t];
            const int64_t w0 = T.a >> 5, w1 = (T.b + 31) >> 5;
            const int64_t nlg = lcnt[t + 1] - lcnt[t];
            int64_t maxc = 0;
            for (int64_t W = w0; W < w1; W++)
                maxc = std::max<int64_t>(maxc, (int64_t)b->rs[W + 1] - (int64_t)b->rs[std::max<int64_t>(W - K, 0)] + nlg);
            t_maxc[t] = maxc;
            const int64_t nl = plan_layers(b, PB, K, (uint64_t)T.a, (uint64_t)T.b, G, wq);
            t_nl[t] = nl;
            if (nl <= 0) { too_big = true; continue; }
            t_nch[t] = plan_items(b, K, (uint64_t)T.a, (uint64_t)T.b, nl, item_layers());
            t_wruns[t] = (int64_t)b->rs[w1] - (int64_t)b->rs[std::max<int64_t>(w0 - K, 0)];
            tile_window(b, K, T.a, T.b, &b->tiles[(size_t)t * S2C_TILE_WORDS]);
        }
    });
    clk.mark("tile plans");
    if (too_big) return s2c_set_error(S2C_ERR_LIMIT, "a read whose SEQ or CIGAR exceeds k_tile's LDS chunk");
    // windows k_tile_dense's compact piece records can hold (s2c.h S2C_DPC_*)
    const std::vector<uint32_t> dbad = dpc_bad_prefix(b);
    auto dpc_ok = [&](const uint32_t *tw) { return K <= 64 && dbad[tw[14]] == dbad[tw[13]]; };
    // the dense class, as the loop below decides it (only single-item tiles can be dense)
    auto dense_tile = [&](int64_t t) {
        const uint32_t *tw = &b->tiles[(size_t)t * S2C_TILE_WORDS];
        return t_nch[t] == 1 && nev[t] == 0 && (int64_t)ccap[t] <= lcols && t_maxc[t] <= 255 && !no_dense &&
               dense_fits(tw, K) && dense_bytes(tw, K) <= dense_cap && dpc_ok(tw);
    };
    // Grid shaping for k_tile: work items run in rounds of `slots` workgroups (the device's CUs
    // × k_tile's workgroups per CU); the last round of a launch whose items all take about as
    // long keeps the rest of the device idle.  The multi-item (deep) tiles' items are made
    // smaller (down to half of IL layers) until the launch fills its last round: C4's 2,487
    // items of ≤ 64 layers (3.24 rounds of 768) become 3,0xx of ≤ 52.
    {
        int64_t n_single = 0, n_multi = 0;
        for (int64_t t = P0; t < std::min<int64_t>(P1, NT); t++) {
            if (t_nch[t] > 1) n_multi += t_nch[t];
            else if (!dense_tile(t)) n_single++;
        }
        int64_t slots = g_plan_cus.load() * (nwp <= 16 ? 3 : 2);   // the device's CUs × k_tile<16>'s 3 workgroups per CU by LDS
        if (const char *e = plan_env("S2C_ITEM_SLOTS")) slots = std::max<int64_t>(0, atoll(e));
        const int64_t IL = item_layers();
        if (n_multi > 0 && slots > 0) {
            const int64_t rounds = (n_single + n_multi + slots - 1) / slots;
            int64_t best = IL;
            for (int64_t il = IL - 1; il >= std::max<int64_t>(4, IL / 2); il--) {
                int64_t n = n_single;
                for (int64_t t = 0; t < NT; t++)
                    if (t_nch[t] > 1) n += std::max<int64_t>(t_nch[t], (t_nl[t] + il - 1) / il);
                if (n > rounds * slots) break;
                best = il;
            }
            if (best < IL)
                par_ranges(plan_threads(q1 - q0, 64), q1 - q0, [&](int, int64_t i0, int64_t i1) {
                    for (int64_t t = q0 + i0; t < q0 + i1; t++)
                        if (t_nch[t] > 1)
                            t_nch[t] = std::max<int64_t>(t_nch[t], plan_items(b, K, (uint64_t)tiles[t].a, (uint64_t)tiles[t].b,
                                                                              t_nl[t], best));
                });
        }
    }
    for (int64_t t = 0; t < NT; t++) {
        const Tile &T = tiles[t];
        const int64_t maxc = t_maxc[t], nl = t_nl[t], nch = t_nch[t];
        I.chunk = std::max<int64_t>(I.chunk, nl);
        runs_max = std::max(runs_max, t_wruns[t]);
        uint32_t *tw = &b->tiles[(size_t)t * S2C_TILE_WORDS];
        uint32_t fl = nch > 1 ? S2C_TILE_DEEP : 0u;
        if (nev[t] > S2C_EPI_KEYS || (int64_t)ccap[t] > lcols) fl |= S2C_TILE_GENERAL;
        if (!planned(t)) fl = 0;   // (a ranged snapshot's unplanned tile: no items)
        else if (fl == 0 && nev[t] == 0 && maxc <= 255 && !no_dense && dense_fits(tw, K) &&
            dense_bytes(tw, K) <= dense_cap && dpc_ok(tw))
            fl = S2C_TILE_DENSE;
        const uint32_t bcap = nshort[t] ? pow2_at_least(2 * (uint64_t)nshort[t]) : 0u;
        tw[0] = (uint32_t)T.a; tw[1] = (uint32_t)T.b; tw[2] = (uint32_t)T.ref; tw[3] = fl;
        tw[4] = (uint32_t)boff; tw[5] = bcap; tw[6] = (uint32_t)loff; tw[7] = nlong[t];
        tw[8] = (uint32_t)coff; tw[9] = (uint32_t)ccap[t]; tw[10] = lcnt[t]; tw[11] = lcnt[t + 1];
        tw[12] = nev[t];
        tw[19] = (uint32_t)nl;
        boff += bcap;
        loff += nlong[t];
        coff += ccap[t];
        if (!planned(t)) {
        } else if (fl == S2C_TILE_DENSE) {
            I.dense_lds = std::max<int64_t>(I.dense_lds, dense_bytes(tw, K));
            const uint32_t it[S2C_ITEM_WORDS] = {(uint32_t)t, 0u, 0u, (uint32_t)nl};
            b->dense.insert(b->dense.end(), it, it + S2C_ITEM_WORDS);
        } else {
            for (int64_t c = 0; c < nch; c++) {
                const uint32_t it[S2C_ITEM_WORDS] = {(uint32_t)t, (uint32_t)c, (uint32_t)(c * nl / nch),
                                                     (uint32_t)((c + 1) * nl / nch)};
                b->items.insert(b->items.end(), it, it + S2C_ITEM_WORDS);
            }
        }
        if (fl & (S2C_TILE_DEEP | S2C_TILE_GENERAL)) b->deep.push_back((uint32_t)t);
    }
    clk.mark("items");
    // the long lists once the tiles' kinds are known: a dense tile lists its long pieces
    // (k_tile_dense walks them itself), the others their run slots (k_reads' records)
    if (I.n_long > 0) {
        std::vector<uint32_t> cnt2(NT + 1, 0);
        auto is_dense = [&](uint32_t t) { return (b->tiles[(size_t)t * S2C_TILE_WORDS + 3] & S2C_TILE_DENSE) != 0; };
        for_long([&](uint32_t t, int64_t k) { cnt2[t + 1] += is_dense(t) ? 1u : pcs[order[k]].nslots; });
        for (int64_t t = 0; t < NT; t++) cnt2[t + 1] += cnt2[t];
        std::vector<uint32_t> lp2(std::max<uint32_t>(cnt2[NT], 1), 0u), at(cnt2.begin(), cnt2.end() - 1);
        for_long([&](uint32_t t, int64_t k) {
            if (is_dense(t)) lp2[at[t]++] = (uint32_t)k;
            else
                for (uint64_t sl = ooff[k]; sl < ooff[k + 1]; sl++) lp2[at[t]++] = (uint32_t)sl;
        });
        for (int64_t t = 0; t < NT; t++) {
            b->tiles[(size_t)t * S2C_TILE_WORDS + 10] = cnt2[t];
            b->tiles[(size_t)t * S2C_TILE_WORDS + 11] = cnt2[t + 1];
        }
        b->lp.swap(lp2);
        I.n_long = cnt2[NT];
    }
    if (boff >= (1ull << 32) || loff >= (1ull << 32) || coff >= (1ull << 31))
        return s2c_set_error(S2C_ERR_LIMIT, "insertion tables exceed 2^32 slots (split the input)");
    I.n_items = (int64_t)(b->items.size() / S2C_ITEM_WORDS);
    I.n_dense = (int64_t)(b->dense.size() / S2C_ITEM_WORDS);
    I.n_deep = (int64_t)b->deep.size();
    I.n_bkt = (int64_t)boff;
    I.n_lng = (int64_t)loff;
    I.n_cols = (int64_t)coff;
    I.runs_max = runs_max;
    mark_runs(b);
    clk.mark("mark_runs");
    build_dwin(b);
    clk.mark("dwin");
    *out = guard.release();
    return S2C_OK;
}

// ------------------------------------------------------------------ shards (multi-GPU)
// The sub-batch of tiles [t0, t1): the pieces whose runs can cover those tiles (short ones
// starting up to kwin + 1 words before, the long ones listed for them) or whose insertion
// events are keyed inside them, with their op words and base planes; run slots, long
// lists, hash-table / column slot bases and tile indices re-based.  Positions keep their
// global coordinates; words outside the shard map to no tile (k_reads drops events keyed
// there).  Counts of a position depend only on the runs covering it, so every shard's
// tiles get exactly the unsharded counts — no exchange of counts is needed.
static int s2c_batch_shard_impl(const s2c_batch *b, int64_t t0, int64_t t1, s2c_batch **out) {
    if (!b || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    const s2c_batch_info &I = b->info;
    if (t0 < 0 || t1 > I.n_tiles || t0 > t1) return s2c_set_error(S2C_ERR_ARG, "bad tile range");
    std::unique_ptr<s2c_batch> s(new s2c_batch());
    s2c_batch_info &J = s->info;
    J = I;
    s->names = b->names;
    s->ref_len = b->ref_len;
    s->ref_off = b->ref_off;
    s->ref_reads = b->ref_reads;
    const int64_t NP = I.n_pieces, NW = I.n_words, K = I.kwin;
    const uint32_t *T0 = &b->tiles[(size_t)t0 * S2C_TILE_WORDS];
    const uint64_t A = t1 > t0 ? T0[0] : 0, B = t1 > t0 ? b->tiles[(size_t)(t1 - 1) * S2C_TILE_WORDS + 1] : 0;
    const int64_t W0 = (int64_t)(A >> 5), W1 = (int64_t)((B + 31) >> 5);
    // ---- pieces: the window range, long pieces listed by the tiles, event pieces keyed inside
    std::vector<uint8_t> take(NP, 0);
    auto piece_at_word = [&](int64_t w) {   // first piece with start word >= w
        if ((int64_t)b->ps.size() == b->info.n_words + 1 && w <= b->info.n_words) return (int64_t)b->ps[w];
        int64_t lo = 0, hi = NP;
        while (lo < hi) {
            const int64_t m = (lo + hi) / 2;
            if ((int64_t)(b->pc[4 * m] >> 5) < w) lo = m + 1; else hi = m;
        }
        return lo;
    };
    if (t1 > t0) {
        const int64_t pa = piece_at_word(std::max<int64_t>(W0 - K - 1, 0)), pb = piece_at_word(W1);
        for (int64_t k = pa; k < pb; k++) take[k] = 1;
        auto piece_of_slot = [&](uint32_t slot) {   // piece whose op range holds slot
            int64_t lo = 0, hi = NP - 1;
            while (lo < hi) {
                const int64_t m = (lo + hi + 1) / 2;
                if (b->pc[4 * m + 2] <= slot) lo = m; else hi = m - 1;
            }
            return lo;
        };
        for (int64_t t = t0; t < t1; t++) {
            const uint32_t *tw = &b->tiles[(size_t)t * S2C_TILE_WORDS];
            const bool dl = (tw[3] & S2C_TILE_DENSE) != 0;   // (a dense tile lists pieces, others run slots)
            for (uint32_t e = tw[10]; e < tw[11]; e++) take[dl ? (int64_t)b->lp[e] : piece_of_slot(b->lp[e])] = 1;
        }
        for (int64_t k = 0; k < NP; k++)
            if (b->kmin[k] != 0xFFFFFFFFu && b->kmax[k] >= A && b->kmin[k] < B) take[k] = 1;
    }
    std::vector<int64_t> sel;
    for (int64_t k = 0; k < NP; k++)
        if (take[k]) sel.push_back(k);
    const int64_t NS = (int64_t)sel.size();
    std::vector<uint64_t> ooff(NS + 1, 0), qoff(NS + 1, 0);
    for (int64_t i = 0; i < NS; i++) {
        const int64_t k = sel[i];
        ooff[i + 1] = ooff[i] + (b->pc[4 * (k + 1) + 2] - b->pc[4 * k + 2]);
        qoff[i + 1] = qoff[i] + ((b->pc[4 * k + 3] & 0xFFFFFFu) + 15) / 16 * 16;
    }
    J.n_pieces = NS;
    J.n_ops = (int64_t)ooff[NS];
    J.n_qwords = (int64_t)((qoff[NS] + 31) / 32) + 2;
    s->pc.assign(4 * (size_t)(NS + 1), 0u);
    s->ops.assign(std::max<uint64_t>(ooff[NS], 1), 0u);
    s->bq.assign(2 * (size_t)J.n_qwords, 0u);
    s->bx.assign((size_t)J.n_qwords, 0u);
    s->kmin.assign(NS, 0xFFFFFFFFu);
    s->kmax.assign(NS, 0u);
    s->lmot.assign(NS, 0);
    s->px.assign(std::max<int64_t>(NS, 1), 0xFFFFFFFFu);
    std::unordered_map<uint32_t, uint32_t> slot_new, piece_new;   // old op slot / long piece → new
    {
        const uint16_t *sq = (const uint16_t *)b->bq.data(), *sx = (const uint16_t *)b->bx.data();
        uint16_t *dq = (uint16_t *)s->bq.data(), *dx = (uint16_t *)s->bx.data();
        for (int64_t i = 0; i < NS; i++) {
            const int64_t k = sel[i];
            const uint32_t o0 = b->pc[4 * k + 2], o1 = b->pc[4 * (k + 1) + 2];
            memcpy(&s->ops[ooff[i]], &b->ops[o0], 4 * (size_t)(o1 - o0));
            uint32_t *pr = &s->pc[4 * (size_t)i];
            pr[0] = b->pc[4 * k];
            pr[1] = (uint32_t)(qoff[i] / 16);
            pr[2] = (uint32_t)ooff[i];
            pr[3] = b->pc[4 * k + 3];
            if (pr[3] >> 24 & S2C_PF_LONG) {
                for (uint32_t o = o0; o < o1; o++) slot_new[o] = (uint32_t)(ooff[i] + (o - o0));
                piece_new[(uint32_t)k] = (uint32_t)i;
            }
            s->kmin[i] = b->kmin[k];
            s->kmax[i] = b->kmax[k];
            s->lmot[i] = b->lmot[k];
            s->px[i] = b->px[k];
            const uint32_t slen = b->pc[4 * k + 3] & 0xFFFFFFu;
            for (uint64_t h = 0; h < (slen + 15) / 16; h++) {
                const uint64_t a = (uint64_t)b->pc[4 * k + 1] + h, d = qoff[i] / 16 + h;
                dq[(d >> 1) * 4 + (d & 1)] = sq[(a >> 1) * 4 + (a & 1)];
                dq[(d >> 1) * 4 + 2 + (d & 1)] = sq[(a >> 1) * 4 + 2 + (a & 1)];
                dx[d] = sx[a];
            }
        }
        s->pc[4 * (size_t)NS + 1] = (uint32_t)(qoff[NS] / 16);
        s->pc[4 * (size_t)NS + 2] = (uint32_t)ooff[NS];
    }
    s->rs.assign(NW + 1, 0u);
    s->ps.assign(NW + 1, 0u);
    for (int64_t i = 0; i < NS; i++) {
        s->rs[(s->pc[4 * i] >> 5) + 1] += (uint32_t)(ooff[i + 1] - ooff[i]);
        s->ps[(s->pc[4 * i] >> 5) + 1]++;
    }
    for (int64_t w = 0; w < NW; w++) {
        s->rs[w + 1] += s->rs[w];
        s->ps[w + 1] += s->ps[w];
    }
    // ---- tiles [t0, t1): slot bases re-based, long lists remapped, plan lists re-indexed
    const int64_t NT = t1 - t0;
    J.n_tiles = NT;
    s->tiles.assign(b->tiles.begin() + t0 * S2C_TILE_WORDS, b->tiles.begin() + t1 * S2C_TILE_WORDS);
    const uint32_t boff0 = NT ? T0[4] : 0, loff0 = NT ? T0[6] : 0, coff0 = NT ? T0[8] : 0;
    int64_t nbkt = 0, nlng = 0, ncol = 0;
    for (int64_t t = 0; t < NT; t++) {
        uint32_t *tw = &s->tiles[(size_t)t * S2C_TILE_WORDS];
        tw[4] -= boff0;
        tw[6] -= loff0;
        tw[8] -= coff0;
        nbkt = std::max<int64_t>(nbkt, (int64_t)tw[4] + tw[5]);
        nlng = std::max<int64_t>(nlng, (int64_t)tw[6] + tw[7]);
        ncol = std::max<int64_t>(ncol, (int64_t)tw[8] + tw[9]);
        const uint32_t l0 = (uint32_t)s->lp.size();
        const bool dl = (tw[3] & S2C_TILE_DENSE) != 0;
        for (uint32_t e = tw[10]; e < tw[11]; e++) s->lp.push_back(dl ? piece_new.at(b->lp[e]) : slot_new.at(b->lp[e]));
        tw[10] = l0;
        tw[11] = (uint32_t)s->lp.size();
    }
    J.n_long = (int64_t)s->lp.size();
    if (s->lp.empty()) s->lp.push_back(0);
    J.n_bkt = nbkt;
    J.n_lng = nlng;
    J.n_cols = ncol;
    s->wtile.assign(NW, 0xFFFFFFFFu);
    for (int64_t w = W0; w < W1; w++)
        if (b->wtile[w] != 0xFFFFFFFFu) s->wtile[w] = b->wtile[w] - (uint32_t)t0;
    auto sub_items = [&](const std::vector<uint32_t> &src, std::vector<uint32_t> &dst) {
        for (size_t i = 0; i < src.size(); i += S2C_ITEM_WORDS)
            if (src[i] >= (uint64_t)t0 && src[i] < (uint64_t)t1) {
                dst.insert(dst.end(), &src[i], &src[i] + S2C_ITEM_WORDS);
                dst[dst.size() - S2C_ITEM_WORDS] -= (uint32_t)t0;
            }
    };
    sub_items(b->items, s->items);
    sub_items(b->dense, s->dense);
    for (uint32_t t : b->deep)
        if (t >= (uint64_t)t0 && t < (uint64_t)t1) s->deep.push_back(t - (uint32_t)t0);
    J.n_items = (int64_t)(s->items.size() / S2C_ITEM_WORDS);
    J.n_dense = (int64_t)(s->dense.size() / S2C_ITEM_WORDS);
    J.n_deep = (int64_t)s->deep.size();
    int64_t runs_max = 0, aligned = 0;
    for (int64_t t = 0; t < NT; t++) {
        const uint32_t *tw = &s->tiles[(size_t)t * S2C_TILE_WORDS];
        const int64_t w0 = tw[0] >> 5, w1 = (tw[1] + 31) >> 5;
        runs_max = std::max<int64_t>(runs_max, (int64_t)s->rs[w1] - (int64_t)s->rs[std::max<int64_t>(w0 - K, 0)]);
        aligned += tw[1] - tw[0];
    }
    J.runs_max = runs_max;
    J.dense_lds = 0;
    for (int64_t t = 0; t < NT; t++) {
        uint32_t *tw = &s->tiles[(size_t)t * S2C_TILE_WORDS];
        tile_window(s.get(), K, tw[0], tw[1], tw);
        if (!(tw[3] & S2C_TILE_DENSE)) continue;
        if (!dense_fits(tw, K)) return s2c_set_error(S2C_ERR_LIMIT, "shard window beyond the dense kernel's LDS");
        J.dense_lds = std::max<int64_t>(J.dense_lds, dense_bytes(tw, K));
    }
    // (the shard's own layered windows are built on first use: s2c_batch_layers; until then
    // no tile word 20 names a layer of the parent's and launches with work items refuse it)
    J.n_layers = J.n_lpieces = J.n_lops = J.n_lqwords = 0;
    J.layers_dense = J.layers_built = 0;
    for (int64_t t = 0; t < NT; t++) s->tiles[(size_t)t * S2C_TILE_WORDS + 20] = S2C_LY_NONE;
    {   // the shard's own pieces walked op by op (its k_tile variant: walk_queue_of, mark_runs)
        int64_t nw = 0;
        for (int64_t i = 0; i < NS; i++) nw += !((s->pc[4 * i + 3] >> 24) & (S2C_PF_SIMPLE | S2C_PF_LONG));
        J.n_walked = nw;
    }
    mark_runs(s.get());
    build_dwin(s.get());
    // the shard's share of the workload's aligned bases (by its positions; for reporting)
    // the per-word entries the shard's launches read (s2c_batch_info word_lo / word_hi): its
    // tiles' words, the window lookback of k_tile_dense's run-slot ranges (rs[W - kwin]) and
    // the piece range above; k_reads drops events keyed outside
    J.plan_t0 = 0;   // (every tile of a shard has its plan: tile_window above, items copied)
    J.plan_t1 = NT;
    J.word_lo = t1 > t0 ? std::max<int64_t>(W0 - K - 1, 0) : 0;
    J.word_hi = t1 > t0 ? std::min<int64_t>(W1, NW) : 0;
    J.aligned_bases = I.total_len ? (int64_t)((double)I.aligned_bases * (double)aligned / (double)I.total_len) : 0;
    *out = s.release();
    return S2C_OK;
}
extern "C" int s2c_batch_shard(const s2c_batch *b, int64_t t0, int64_t t1, s2c_batch **out) {
    return s2c_guarded([&] { return s2c_batch_shard_impl(b, t0, t1, out); });
}

static int s2c_batch_layers_impl(s2c_batch *b, bool with_dense) {
    if (!b) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    if (b->layers && (b->info.layers_dense || !with_dense)) return S2C_OK;
    int64_t nwp = 8;
    while (nwp * 32 < b->info.tile_max) nwp *= 2;
    build_layers(b, 64 / nwp, with_dense);
    b->layers = true;
    b->info.layers_built = 1;
    return S2C_OK;
}
extern "C" int s2c_batch_layers(s2c_batch *b) {
    return s2c_guarded([&] { return s2c_batch_layers_impl(b, true); });
}
extern "C" int s2c_batch_layers_mode(s2c_batch *b, int with_dense) {
    return s2c_guarded([&] { return s2c_batch_layers_impl(b, with_dense != 0); });
}

extern "C" int s2c_batch_info_get(const s2c_batch *b, s2c_batch_info *out) {
    if (!b || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    *out = b->info;
    return S2C_OK;
}

extern "C" int s2c_batch_arrays_get(const s2c_batch *b, s2c_batch_arrays *o) {
    if (!b || !o) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    o->ref_len = b->ref_len.data();
    o->ref_off = b->ref_off.data();
    o->ref_cov_reads = b->ref_reads.data();
    o->pc = b->pc.data();
    o->ops = b->ops.data();
    o->bq = b->bq.data();
    o->bx = b->bx.data();
    o->rs = b->rs.data();
    o->tiles = b->tiles.data();
    o->items = b->items.data();
    o->dense = b->dense.data();
    o->deep = b->deep.data();
    o->lp = b->lp.data();
    o->wtile = b->wtile.data();
    o->rlist = b->rlist.data();
    o->px = b->px.data();
    o->dwin = b->dwin.data();
    o->ps = b->ps.data();
    o->lly = b->lly.data();
    o->lpc = b->lpc.data();
    o->lops = b->lops.data();
    o->lbq = b->lbq.data();
    o->lbx = b->lbx.data();
    o->lpx = b->lpx.empty() ? nullptr : b->lpx.data();
    o->dpc = b->dpc.data();
    return S2C_OK;
}

extern "C" const char *s2c_batch_ref_name(const s2c_batch *b, int64_t i) {
    if (!b || i < 0 || i >= (int64_t)b->names.size()) return nullptr;
    return b->names[i].c_str();
}

extern "C" void s2c_batch_free(s2c_batch *b) { delete b; }

// ------------------------------------------------------------------ parsecigar (:46-82)
static int s2c_parsecigar_impl(const char *cigar, size_t cigar_len, const char *seq, size_t seq_len,
                              int64_t pos_ref, char *seqout, size_t cap, size_t *seqout_len,
                              int64_t *ins, size_t max_ins, size_t *n_ins) {
    std::vector<uint32_t> toks;
    uint32_t nt = 0;
    int rc = tokenize_cigar(cigar, cigar_len, toks, &nt);
    if (rc) return rc;
    int64_t start = 0, start_ref = pos_ref;
    const int64_t slen = (int64_t)seq_len;
    size_t o = 0, ni = 0;
    auto put = [&](char c) -> bool {
        if (o + 1 >= cap) return false;
        seqout[o++] = c;
        return true;
    };
    for (uint32_t w : toks) {
        const uint32_t op = w & 15u;
        const int64_t l = (int64_t)(w >> 4);
        if (op_bases(op)) {
            int64_t take = start < slen ? std::min(l, slen - start) : 0;
            for (int64_t j = 0; j < take; j++)
                if (!put(seq[start + j])) return s2c_set_error(S2C_ERR_ARG, "seqout buffer too small");
            start += l;
            start_ref += l;
        } else if (op_dash(op)) {
            for (int64_t j = 0; j < l; j++)
                if (!put('-')) return s2c_set_error(S2C_ERR_ARG, "seqout buffer too small");
            start_ref += l;
        } else if (op == S2C_OP_I) {
            int64_t take = start < slen ? std::min(l, slen - start) : 0;
            if (ni < max_ins) {
                ins[3 * ni] = start_ref;
                ins[3 * ni + 1] = std::min(start, slen);
                ins[3 * ni + 2] = take;
            }
            ni++;
            start += l;
        } else if (op == S2C_OP_S) {
            start += l;
        }
    }
    if (cap) seqout[o] = 0;
    *seqout_len = o;
    *n_ins = ni;
    return ni > max_ins ? s2c_set_error(S2C_ERR_ARG, "insertion buffer too small") : S2C_OK;
}
extern "C" int s2c_parsecigar(const char *cigar, size_t cigar_len, const char *seq, size_t seq_len,
                              int64_t pos_ref, char *seqout, size_t cap, size_t *seqout_len,
                              int64_t *ins, size_t max_ins, size_t *n_ins) {
    return s2c_guarded([&] { return s2c_parsecigar_impl(cigar, cigar_len, seq, seq_len, pos_ref, seqout, cap, seqout_len, ins, max_ins, n_ins); });
}

// ------------------------------------------------------------------ ABI layout self-check
// Lets the ctypes mirror (sam2consensus_amd/_lib.py) verify struct sizes/offsets at load.
#include <cstddef>
extern "C" int s2c_layout(int64_t *out, int n) {
    const int64_t v[] = {
        (int64_t)sizeof(s2c_dev), (int64_t)offsetof(s2c_dev, kwin), (int64_t)offsetof(s2c_dev, thresholds),
        (int64_t)offsetof(s2c_dev, fill), (int64_t)offsetof(s2c_dev, runs), (int64_t)offsetof(s2c_dev, n_cols),
        (int64_t)offsetof(s2c_dev, tile_stats), (int64_t)offsetof(s2c_dev, out_cap),
        (int64_t)sizeof(s2c_synth_spec), (int64_t)offsetof(s2c_synth_spec, seed),
        (int64_t)sizeof(s2c_batch_info), (int64_t)sizeof(s2c_batch_arrays), (int64_t)sizeof(s2c_ws_sizes)};
    const int m = (int)(sizeof(v) / sizeof(v[0]));
    for (int i = 0; i < n && i < m; i++) out[i] = v[i];
    return m;
}

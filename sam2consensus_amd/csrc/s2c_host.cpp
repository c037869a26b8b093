// s2c_host.cpp — host side of libs2c.so: SAM/SAM.gz parser → packed read batch → work plan.
//
// Reproduces the reference's record handling (zoujiayun/sam2consensus v2.1,
// sam2consensus.py) exactly, including its Python-2 quirks:
//   header pass            :149-172   (leading '@' lines, @SQ SN:/LN: parse)
//   record filter          :195       (line[0] != '@' and field[5] != "*"; FLAG ignored)
//   RNAME / POS            :200-201   (str.split()[0], int() - 1)
//   parsecigar             :46-82     (regex tokens, SEQ truncation, I/S/H/P/N semantics)
//   maxdel rule            :210-218   (total '-' in seqout > maxdel ⇒ '-' not counted)
//   Python negative index  :212       (pos -1 → last base)
//   error classes          :195,:200,:201,:206,:212,:217,:221,:287,:294 in file order
// and emits north_star subsystem (1): the packed batch the HIP kernels consume.
#include "../../include/s2c.h"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
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
extern "C" int s2c_abi_version(void) { return S2C_ABI_VERSION; }

// ------------------------------------------------------------------ tables
namespace {
constexpr uint8_t BAD = 0xFF;
struct CodeLut {
    uint8_t v[256];
    CodeLut() {
        memset(v, BAD, sizeof(v));
        v[(uint8_t)'-'] = 0; v[(uint8_t)'A'] = 1; v[(uint8_t)'C'] = 2;
        v[(uint8_t)'G'] = 3; v[(uint8_t)'N'] = 4; v[(uint8_t)'T'] = 5;
    }
};
const CodeLut LUT;

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

struct Tok { char op; int64_t len; };

// re.findall(r"(\d+)([MIDNSHPX=]{1})", cigar) (:58): a match is a maximal digit run
// immediately followed by an op letter; everything else is skipped.
int tokenize_cigar(const char *s, size_t n, std::vector<Tok> &out) {
    out.clear();
    size_t i = 0;
    while (i < n) {
        if (s[i] < '0' || s[i] > '9') { i++; continue; }
        size_t j = i;
        int64_t v = 0;
        bool big = false;
        while (j < n && s[j] >= '0' && s[j] <= '9') {
            v = v * 10 + (s[j] - '0');
            if (v >= ((int64_t)1 << 31)) { big = true; v = (int64_t)1 << 31; }
            j++;
        }
        if (j < n) {
            char c = s[j];
            if (c == 'M' || c == 'I' || c == 'D' || c == 'N' || c == 'S' || c == 'H' || c == 'P' ||
                c == 'X' || c == '=') {
                if (big) return s2c_set_error(S2C_ERR_LIMIT, "CIGAR op length >= 2^31 not supported");
                out.push_back({c, v});
                i = j + 1;
                continue;
            }
        }
        i = j;
    }
    return S2C_OK;
}
}  // namespace

// ------------------------------------------------------------------ parser state
struct EffOp { uint8_t cls; int64_t len; };   // cls 0 = M (bases), 1 = D (dashes)

struct s2c_parser {
    bool maxdel_active = true;
    int64_t maxdel = 150;
    bool in_header = true;
    int64_t header_lines = 0, lines_total = 0, reads_mapped = 0, aligned = 0, qbases = 0;
    std::vector<std::string> ref_names;
    std::vector<int64_t> ref_len;
    std::unordered_map<std::string, uint32_t> ref_idx;
    // pileup pieces (file order): every position of a piece lies in [0, LN) of its ref
    std::vector<uint32_t> p_ref;
    std::vector<int64_t> p_pos;
    std::vector<uint32_t> p_span;
    std::vector<uint8_t> p_drop;
    std::vector<uint64_t> p_op;     // CSR into ops (size n+1)
    std::vector<uint32_t> ops;      // (len<<1)|cls
    std::vector<uint64_t> p_base;   // CSR (word offsets) into words (size n+1)
    std::vector<uint32_t> words;    // 3 bit-planes per read, word-interleaved
    // insertion events (file order), raw motif bytes (validated at finish, :287)
    std::vector<uint32_t> i_ref;
    std::vector<int64_t> i_key;
    std::vector<uint64_t> i_off;
    std::vector<uint32_t> i_len;
    std::string i_raw;
    // streaming
    std::string carry;
    int err = S2C_OK;
    std::string errmsg;
    // scratch
    std::vector<Tok> toks;
    std::vector<EffOp> eff;
    std::vector<uint8_t> codes, qcodes;
    std::string last_name;
    int64_t last_ref = -1;

    s2c_parser() { p_op.push_back(0); p_base.push_back(0); }
};

struct s2c_batch {
    s2c_batch_info info{};
    std::vector<std::string> names;
    std::vector<int64_t> ref_len, ref_off, ref_reads;
    std::vector<uint32_t> rd_pos, rd_op, rd_span, ops;   // host-side read-piece table
    std::vector<uint32_t> wrec, recs;                     // word-major seqout windows
    std::vector<uint32_t> fix, exc;                       // A placeholders, '-'/'N' entries
    std::vector<uint32_t> iwr;                            // per-item word record ranges
    std::vector<uint32_t> ins_key, ins_koff, ins_kcol, ins_off, ins_bases, ins_ekey, ins_bits, ins_rank;
    std::vector<uint32_t> ins_ev, ins_kinfo;             // device-side event / key records
    std::vector<uint32_t> items, blocks, deep;
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

// Append piece = seqout[ka, kb) of the current read (eff ops + codes) at ref position pos.
// The piece's seqout (:64-81: M/=/X bases, D/N/P as '-' = code 0) is packed as 3
// bit-planes (bit k of each symbol code), word-interleaved: for seqout word i (32
// positions) {plane0[i], plane1[i], plane2[i]}, plus one zero triple at the end so a
// 32-bit window at any offset is a funnel shift of two triples.  The device never walks
// the CIGAR: a read's 32 positions under a word are one window load.  The effective ops
// are kept on the host (planner, CPU model); SIMPLE marks single-M-op pieces.
static void emit_piece(s2c_parser *p, uint32_t ref, int64_t pos, bool drop, int64_t ka, int64_t kb) {
    int64_t k = 0;
    size_t ci = 0;  // index into p->codes (M bases in seqout order)
    uint32_t nops = 0;
    std::vector<uint8_t> &codes = p->codes;
    std::vector<uint8_t> &q = p->qcodes;
    q.clear();
    for (const EffOp &o : p->eff) {
        int64_t a = std::max(k, ka), b = std::min(k + o.len, kb);
        if (b > a) {
            uint32_t w = (uint32_t)(((uint64_t)(b - a) << 1) | o.cls);
            if (nops && (p->ops.back() & 1) == o.cls) {
                p->ops.back() += (uint32_t)((b - a) << 1);   // merge same-class neighbours
            } else {
                p->ops.push_back(w);
                nops++;
            }
            if (o.cls == 0)
                for (int64_t j = a - k; j < b - k; j++) q.push_back(codes[ci + j]);
            else
                q.insert(q.end(), (size_t)(b - a), (uint8_t)0);   // D/N/P: '-' (code 0) in seqout (:71)
        }
        if (o.cls == 0) ci += (size_t)o.len;
        k += o.len;
    }
    const size_t nwq = (q.size() + 31) / 32 + 1;
    const size_t w0 = p->words.size();
    p->words.resize(w0 + 3 * nwq, 0u);
    for (size_t j = 0; j < q.size(); j++) {
        const uint32_t c = q[j], bit = 1u << (j & 31);
        uint32_t *w = &p->words[w0 + 3 * (j >> 5)];
        if (c & 1) w[0] |= bit;
        if (c & 2) w[1] |= bit;
        if (c & 4) w[2] |= bit;
    }
    p->p_ref.push_back(ref);
    p->p_pos.push_back(pos);
    p->p_span.push_back((uint32_t)(kb - ka));
    p->p_drop.push_back(drop ? 1 : 0);
    p->p_op.push_back(p->ops.size());
    p->p_base.push_back(p->words.size());
}

// One SAM line, n includes the trailing '\n' when present (Python 2 line semantics).
static int process_line(s2c_parser *p, const char *s, size_t n) {
    p->lines_total++;
    if (p->in_header) {
        if (s[0] == '@') {
            p->header_lines++;
            if (n >= 3 && s[1] == 'S' && s[2] == 'Q') return parse_sq(p, s, n);
            return S2C_OK;
        }
        p->in_header = false;
    }
    if (s[0] == '@') return S2C_OK;                                   // :195
    const char *f[10];
    size_t fl[10];
    int nf = 0;
    const char *cur = s, *end = s + n;
    while (nf < 10) {
        const char *t = (const char *)memchr(cur, '\t', end - cur);
        f[nf] = cur;
        if (!t) { fl[nf++] = end - cur; break; }
        fl[nf++] = t - cur;
        cur = t + 1;
    }
    if (nf < 6) return perr(p, S2C_ERR_INDEX, "IndexError: record with < 6 fields (:195)");
    if (fl[5] == 1 && f[5][0] == '*') return S2C_OK;                  // unmapped (:195)
    p->reads_mapped++;
    const char *nb;
    size_t nl;
    if (!py2_first_token(f[2], fl[2], &nb, &nl))
        return perr(p, S2C_ERR_INDEX, "IndexError: empty RNAME (:200)");
    int64_t pos1;
    if (!py2_int(f[3], fl[3], &pos1))
        return perr(p, S2C_ERR_VALUE, "ValueError: invalid POS '" + std::string(f[3], fl[3]) + "' (:201)");
    int64_t pos0 = pos1 - 1;
    if (nf < 10) return perr(p, S2C_ERR_INDEX, "IndexError: record with < 10 fields (:206)");

    // ---- parsecigar (:46-82) ----
    int rc = tokenize_cigar(f[5], fl[5], p->toks);
    if (rc) return perr(p, rc, s2c_last_error());
    const char *seq = f[9];
    const int64_t slen = (int64_t)fl[9];
    int64_t start = 0, start_ref = pos0, klen = 0;
    p->eff.clear();
    p->codes.clear();
    size_t ins_first = p->i_ref.size();
    for (const Tok &t : p->toks) {
        int64_t l = t.len;
        switch (t.op) {
            case 'M': case '=': case 'X': {
                int64_t take = start < slen ? std::min(l, slen - start) : 0;
                if (take > 0) {
                    if (!p->eff.empty() && p->eff.back().cls == 0) p->eff.back().len += take;
                    else p->eff.push_back({0, take});
                    for (int64_t j = 0; j < take; j++) p->codes.push_back(LUT.v[(uint8_t)seq[start + j]]);
                    klen += take;
                }
                start += l;
                start_ref += l;
                break;
            }
            case 'D': case 'N': case 'P':
                if (l > 0) {
                    if (!p->eff.empty() && p->eff.back().cls == 1) p->eff.back().len += l;
                    else p->eff.push_back({1, l});
                    klen += l;
                }
                start_ref += l;
                break;
            case 'I': {
                int64_t take = start < slen ? std::min(l, slen - start) : 0;
                if (take > 0) {    // an empty motif never reaches a column (:280-287)
                    p->i_ref.push_back(0);  // fixed below once the ref is known
                    p->i_key.push_back(start_ref);
                    p->i_off.push_back(p->i_raw.size());
                    p->i_len.push_back((uint32_t)take);
                    p->i_raw.append(seq + start, (size_t)take);
                }
                start += l;
                break;
            }
            case 'S':
                start += l;
                break;
            default:  // 'H' (:78-79)
                break;
        }
    }
    if (klen >= ((int64_t)1 << 31)) return perr(p, S2C_ERR_LIMIT, "seqout longer than 2^31");
    p->aligned += klen;

    // ---- reference lookup: sequences[refname] / insertions[refname] (:212,:217,:221) ----
    int64_t ref;
    if (p->last_ref >= 0 && p->last_name.size() == nl && memcmp(p->last_name.data(), nb, nl) == 0) {
        ref = p->last_ref;
    } else {
        std::string name(nb, nl);
        auto it = p->ref_idx.find(name);
        if (it == p->ref_idx.end()) return perr(p, S2C_ERR_KEY, "KeyError: '" + name + "' (:212/:221)");
        ref = it->second;
        p->last_ref = ref;
        p->last_name = name;
    }
    for (size_t i = ins_first; i < p->i_ref.size(); i++) {
        p->i_ref[i] = (uint32_t)ref;
        p->qbases += p->i_len[i];
    }
    const int64_t L = p->ref_len[ref];

    // ---- maxdel rule (:210): '-' count of the whole seqout ----
    int64_t dashes = 0, mbases = 0;
    for (const EffOp &o : p->eff) if (o.cls == 1) dashes += o.len; else mbases += o.len;
    bool any_bad = false;
    for (uint8_t c : p->codes) { dashes += (c == 0); any_bad |= (c == BAD); }
    p->qbases += mbases;
    const bool drop = p->maxdel_active && dashes > p->maxdel;

    // ---- validation in seqout order (:211-218): index check, then symbol check ----
    const bool in_range = pos0 >= 0 && pos0 + klen <= L;
    int64_t kc0 = -1, kc1 = -1;  // first / last counted seqout index
    if (!in_range || any_bad || drop) {
        int64_t k = 0;
        size_t ci = 0;
        for (const EffOp &o : p->eff) {
            for (int64_t j = 0; j < o.len; j++, k++) {
                uint8_t c = o.cls ? 0 : p->codes[ci + j];
                if (drop && c == 0) continue;               // '-' skipped (:216)
                int64_t pp = pos0 + k;
                if (pp < -L || pp >= L)
                    return perr(p, S2C_ERR_INDEX, "IndexError: list index out of range (:212)");
                if (c == BAD) return perr(p, S2C_ERR_KEY, "KeyError: base not in -ACGNT (:212)");
                if (kc0 < 0) kc0 = k;
                kc1 = k + 1;
            }
            if (o.cls == 0) ci += (size_t)o.len;
        }
    } else if (klen > 0) {
        kc0 = 0;
        kc1 = klen;
    }
    if (kc0 < 0) return S2C_OK;   // nothing counted (empty seqout, or all '-' dropped)

    // ---- pieces: Python negative indices wrap (pos -1 → LN-1, :212) ----
    int64_t pa = pos0 + kc0;
    if (pa < 0) {
        int64_t kb = std::min(kc1, -pos0);
        emit_piece(p, (uint32_t)ref, L + pa, drop, kc0, kb);
        if (kc1 > -pos0) emit_piece(p, (uint32_t)ref, 0, drop, -pos0, kc1);
    } else {
        emit_piece(p, (uint32_t)ref, pa, drop, kc0, kc1);
    }
    return S2C_OK;
}

extern "C" int s2c_parser_new(int maxdel_active, int64_t maxdel, s2c_parser **out) {
    if (!out) return s2c_set_error(S2C_ERR_ARG, "out is NULL");
    s2c_parser *p = new s2c_parser();
    p->maxdel_active = maxdel_active != 0;
    p->maxdel = maxdel;
    *out = p;
    return S2C_OK;
}

extern "C" void s2c_parser_free(s2c_parser *p) { delete p; }

extern "C" int s2c_parser_feed(s2c_parser *p, const char *buf, size_t len) {
    if (!p) return s2c_set_error(S2C_ERR_ARG, "parser is NULL");
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
    while (s < end) {
        const char *nl = (const char *)memchr(s, '\n', end - s);
        if (!nl) { p->carry.assign(s, end - s); break; }
        int rc = process_line(p, s, nl + 1 - s);
        if (rc) return rc;
        s = nl + 1;
    }
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
// A whole input file is parsed by worker threads: the header lines (:149-172) first, in
// order; then the record lines, cut into chunks at line ends, each chunk parsed by its own
// parser state (the same process_line) into its own piece / op / plane / insertion arrays;
// the chunks are appended in file order.  The first failing record in file order decides
// the error, as the reference's sequential loop (:188-228) would: a chunk stops at its
// first error, and no later chunk is merged.
namespace {
void append_chunk(s2c_parser *p, const s2c_parser *w) {
    p->lines_total += w->lines_total;
    p->reads_mapped += w->reads_mapped;
    p->aligned += w->aligned;
    p->qbases += w->qbases;
    p->p_ref.insert(p->p_ref.end(), w->p_ref.begin(), w->p_ref.end());
    p->p_pos.insert(p->p_pos.end(), w->p_pos.begin(), w->p_pos.end());
    p->p_span.insert(p->p_span.end(), w->p_span.begin(), w->p_span.end());
    p->p_drop.insert(p->p_drop.end(), w->p_drop.begin(), w->p_drop.end());
    const uint64_t o0 = p->ops.size(), b0 = p->words.size(), r0 = p->i_raw.size();
    for (size_t i = 1; i < w->p_op.size(); i++) p->p_op.push_back(w->p_op[i] + o0);
    for (size_t i = 1; i < w->p_base.size(); i++) p->p_base.push_back(w->p_base[i] + b0);
    p->ops.insert(p->ops.end(), w->ops.begin(), w->ops.end());
    p->words.insert(p->words.end(), w->words.begin(), w->words.end());
    p->i_ref.insert(p->i_ref.end(), w->i_ref.begin(), w->i_ref.end());
    p->i_key.insert(p->i_key.end(), w->i_key.begin(), w->i_key.end());
    p->i_len.insert(p->i_len.end(), w->i_len.begin(), w->i_len.end());
    for (uint64_t o : w->i_off) p->i_off.push_back(o + r0);
    p->i_raw += w->i_raw;
}

int process_lines(s2c_parser *p, const char *s, size_t n) {
    size_t i = 0;
    while (i < n) {
        const char *nl = (const char *)memchr(s + i, '\n', n - i);
        const size_t e = nl ? (size_t)(nl - s) + 1 : n;   // a last line without '\n' counts (Py2)
        int rc = process_line(p, s + i, e - i);
        if (rc) return rc;
        i = e;
    }
    return S2C_OK;
}

int parse_buffer(s2c_parser *p, const char *s, size_t n) {
    size_t i = 0;
    while (i < n && p->in_header && s[i] == '@') {   // header lines, in order
        const char *nl = (const char *)memchr(s + i, '\n', n - i);
        const size_t e = nl ? (size_t)(nl - s) + 1 : n;
        int rc = process_line(p, s + i, e - i);
        if (rc) return rc;
        i = e;
    }
    if (i == n) return S2C_OK;
    p->in_header = false;
    const size_t body = n - i;
    unsigned hw = std::thread::hardware_concurrency();
    int nt = (int)std::min<size_t>(std::min<unsigned>(hw ? hw : 1, 16), std::max<size_t>(1, body >> 23));   // ≥ 8 MB each
    if (const char *e = getenv("S2C_PARSE_THREADS")) nt = std::max(1, std::min(64, atoi(e)));
    if (nt <= 1) return process_lines(p, s + i, body);
    std::vector<size_t> cut(nt + 1, n);
    cut[0] = i;
    for (int k = 1; k < nt; k++) {   // chunk k starts after the line end nearest to its share
        size_t c = std::max(cut[k - 1], i + body * k / nt);
        const char *nl = c < n ? (const char *)memchr(s + c, '\n', n - c) : nullptr;
        cut[k] = nl ? (size_t)(nl - s) + 1 : n;
    }
    std::vector<s2c_parser *> ws(nt);
    std::vector<int> rcs(nt, S2C_OK);
    std::vector<std::thread> th;
    for (int k = 0; k < nt; k++) {
        s2c_parser *w = new s2c_parser();
        w->maxdel_active = p->maxdel_active;
        w->maxdel = p->maxdel;
        w->in_header = false;
        w->ref_names = p->ref_names;
        w->ref_len = p->ref_len;
        w->ref_idx = p->ref_idx;
        ws[k] = w;
        th.emplace_back([&, k] {
            rcs[k] = process_lines(ws[k], s + cut[k], cut[k + 1] - cut[k]);
            if (rcs[k]) ws[k]->errmsg = s2c_last_error();   // thread-local text → the chunk
        });
    }
    for (auto &t : th) t.join();
    int rc = S2C_OK;
    for (int k = 0; k < nt; k++) {
        if (!rc) {
            append_chunk(p, ws[k]);
            if (rcs[k]) rc = perr(p, rcs[k], ws[k]->errmsg);
        }
        delete ws[k];
    }
    return rc;
}
}  // namespace

extern "C" int s2c_parser_feed_file(s2c_parser *p, const char *path) {
    if (!p || !path) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    if (p->err) return s2c_set_error(p->err, p->errmsg);
    size_t n = strlen(path);
    bool gz = n >= 3 && strcmp(path + n - 3, ".gz") == 0;   // :111
    // the whole input in memory (gunzipped), then the parallel parse; a parser that already
    // holds a partial line from s2c_parser_feed continues line by line
    std::string data;
    if (gz) {
        gzFile g = gzopen(path, "rb");
        if (!g) return s2c_set_error(S2C_ERR_IO, std::string("cannot open ") + path);
        gzbuffer(g, 1 << 20);
        std::vector<char> buf(1 << 22);
        for (;;) {
            int r = gzread(g, buf.data(), (unsigned)buf.size());
            if (r < 0) { gzclose(g); return s2c_set_error(S2C_ERR_IO, "gzip read error"); }
            if (r == 0) break;
            data.append(buf.data(), (size_t)r);
        }
        gzclose(g);
    } else {
        FILE *f = fopen(path, "rb");
        if (!f) return s2c_set_error(S2C_ERR_IO, std::string("cannot open ") + path);
        if (fseek(f, 0, SEEK_END) == 0) {
            long sz = ftell(f);
            if (sz > 0) data.reserve((size_t)sz);
            fseek(f, 0, SEEK_SET);
        }
        std::vector<char> buf(1 << 22);
        for (;;) {
            size_t r = fread(buf.data(), 1, buf.size(), f);
            if (r == 0) break;
            data.append(buf.data(), r);
        }
        fclose(f);
    }
    if (!p->carry.empty()) {
        int rc = s2c_parser_feed(p, data.data(), data.size());
        return rc ? rc : feed_flush(p);
    }
    int rc = parse_buffer(p, data.data(), data.size());
    if (rc && !p->err) { p->err = rc; p->errmsg = s2c_last_error(); }
    return rc;
}

// ------------------------------------------------------------------ finish: plan
namespace {
constexpr int64_t TP_MIN = 256, TP_MAX = 2048;      // pileup tile bounds (positions)
constexpr double E_TARGET = 262144.0;                // aligned bases per tile (tile width from depth)
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t align_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }
}  // namespace

extern "C" int s2c_parser_finish(s2c_parser *p, s2c_batch **out) {
    if (!p || !out) return s2c_set_error(S2C_ERR_ARG, "NULL argument");
    int rc = feed_flush(p);
    if (rc) return rc;
    const int64_t R = (int64_t)p->ref_names.size();

    // ---- reformat-phase checks (:284-294), refs in header order: motif symbols (KeyError,
    //      :287) are checked for every key before any key's coverage lookup (IndexError, :294)
    {
        std::vector<uint8_t> bad_sym(R, 0), bad_key(R, 0);
        for (size_t i = 0; i < p->i_ref.size(); i++) {
            uint32_t r = p->i_ref[i];
            const int64_t L = p->ref_len[r];
            for (uint32_t j = 0; j < p->i_len[i]; j++)
                if (LUT.v[(uint8_t)p->i_raw[p->i_off[i] + j]] == BAD) { bad_sym[r] = 1; break; }
            if (p->i_key[i] < -L || p->i_key[i] >= L) bad_key[r] = 1;
        }
        for (int64_t r = 0; r < R; r++) {
            if (bad_sym[r]) return s2c_set_error(S2C_ERR_KEY, "KeyError: insertion base not in -ACGNT (:287)");
            if (bad_key[r]) return s2c_set_error(S2C_ERR_INDEX, "IndexError: insertion key out of range (:294)");
        }
    }

    s2c_batch *b = new s2c_batch();
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
    if (Lpad >= ((int64_t)1 << 32) - 4096) {
        delete b;
        return s2c_set_error(S2C_ERR_LIMIT, "more than 2^32 reference positions");
    }
    I.n_refs = R;
    I.padded_len = Lpad;
    for (int64_t r = 0; r < R; r++) I.total_len += p->ref_len[r];
    I.header_lines = p->header_lines;
    I.lines_total = p->lines_total;
    I.reads_mapped = p->reads_mapped;
    I.aligned_bases = p->aligned;
    I.query_bases = p->qbases;

    // ---- read pieces → global coordinates (host-side read table, file order) ----
    const int64_t NP = (int64_t)p->p_ref.size();
    std::vector<uint64_t> gstart(NP);
    uint64_t nops = 0;
    for (int64_t i = 0; i < NP; i++) {
        gstart[i] = (uint64_t)(b->ref_off[p->p_ref[i]] + p->p_pos[i]);
        b->ref_reads[p->p_ref[i]]++;
        nops += p->p_op[i + 1] - p->p_op[i];
    }
    if (nops >= (1ull << 32) || NP >= ((int64_t)1 << 32) - 1) {
        delete b;
        return s2c_set_error(S2C_ERR_LIMIT, "batch exceeds 2^32 ops or read pieces (split the input)");
    }
    I.n_reads = NP;
    I.n_ops = (int64_t)nops;
    b->rd_pos.resize(NP);
    b->rd_span.resize(NP);
    b->rd_op.resize(NP + 1);
    b->ops.resize(nops);
    {
        uint64_t oo = 0;
        for (int64_t i = 0; i < NP; i++) {
            const uint64_t no = p->p_op[i + 1] - p->p_op[i];
            b->rd_pos[i] = (uint32_t)gstart[i];
            b->rd_span[i] = p->p_span[i] | (p->p_drop[i] ? 0x80000000u : 0u);   // bit31: maxdel drop (:210)
            b->rd_op[i] = (uint32_t)oo;
            memcpy(&b->ops[oo], &p->ops[p->p_op[i]], no * 4);
            oo += no;
        }
        b->rd_op[NP] = (uint32_t)oo;
    }

    // ---- word-major seqout windows: one record per (piece, global 32-position word) ----
    // record = 2 bit-planes {b0, b1} of the word's 32 bases (b1·2+b0: 0 A, 1 C, 2 G, 3 T),
    // grouped by word (CSR wrec), piece order inside.  A position with no A/C/G/T entry in
    // the record — outside the piece, a '-' of a maxdel-dropped read (:214-218, not
    // counted), or a seqout '-' / 'N' — holds 0 (A) and is counted in fix (subtracted from A
    // on the device); a counted '-' / 'N' is also listed in exc (added to its symbol).
    const int64_t NW = Lpad / 32;
    b->wrec.assign(NW + 1, 0);
    uint64_t nrec = 0;
    for (int64_t i = 0; i < NP; i++) {
        const uint64_t span = p->p_span[i];
        if (!span) continue;
        const uint64_t W0 = gstart[i] >> 5, W1 = (gstart[i] + span - 1) >> 5;
        for (uint64_t W = W0; W <= W1; W++) b->wrec[W + 1]++;
        nrec += W1 - W0 + 1;
    }
    if (nrec >= (1ull << 32) - 1) {
        delete b;
        return s2c_set_error(S2C_ERR_LIMIT, "more than 2^32 seqout word records (split the input)");
    }
    for (int64_t W = 0; W < NW; W++) b->wrec[W + 1] += b->wrec[W];
    I.n_recs = (int64_t)nrec;
    // ---- tiles (consensus/assembly blocks) and pileup work items ----
    std::vector<int64_t> ref_events(R, 0);
    for (int64_t i = 0; i < NP; i++) ref_events[p->p_ref[i]] += p->p_span[i];
    struct Tile { int64_t a, b, ref; };
    std::vector<Tile> tiles;
    int64_t tile_max = S2C_POS_ALIGN;
    // diagnostic override of the tile width (S2C_TILE_POS, a multiple of 64 in [64, 2048])
    int64_t tile_force = 0;
    if (const char *e = getenv("S2C_TILE_POS")) {
        tile_force = align_up(std::min<int64_t>(std::max<int64_t>(atoll(e), 64), TP_MAX), S2C_POS_ALIGN);
    }
    for (int64_t r = 0; r < R; r++) {
        const int64_t L = p->ref_len[r], off = b->ref_off[r];
        if (L == 0) continue;
        double depth = (double)ref_events[r] / (double)L;
        int64_t tp = depth > 0 ? align_up((int64_t)std::ceil(E_TARGET / depth), S2C_POS_ALIGN) : TP_MAX;
        tp = std::min(std::max(tp, TP_MIN), TP_MAX);
        if (tile_force > 0) tp = tile_force;
        // spread the ref evenly over ceil(L/tp) tiles, each a multiple of 64
        int64_t nt = ceil_div(L, tp);
        int64_t step = align_up(ceil_div(L, nt), S2C_POS_ALIGN);
        for (int64_t a = off; a < off + L; a += step) {
            tiles.push_back({a, std::min(a + step, off + L), r});
            tile_max = std::max(tile_max, tiles.back().b - a);
        }
    }
    I.tile_max = tile_max;
    // Each tile is also the consensus/assembly block.  k_pileup gives a tile 256 lanes:
    // one 32-position word per lane × G = 256 / words-per-tile lanes per word, each with
    // 8-bit counters (≤248 records per lane between flushes).  A work item takes chunk k of
    // every word's records, [k·chunk, (k+1)·chunk) with chunk = 248·G; a tile whose deepest word
    // needs one chunk is voted in the kernel's epilogue (counts never reach HBM), a deeper
    // ("deep") tile adds its chunks' counts into HBM and is voted by k_consensus.
    int64_t nwp = 8;
    while (nwp * 32 < tile_max) nwp *= 2;
    const int64_t chunk = 248 * (256 / nwp);
    I.chunk_recs = chunk;
    for (size_t t = 0; t < tiles.size(); t++) {
        const Tile &T = tiles[t];
        int64_t maxw = 0;
        for (int64_t W = T.a >> 5; W < (T.b + 31) >> 5; W++)
            maxw = std::max<int64_t>(maxw, (int64_t)(b->wrec[W + 1] - b->wrec[W]));
        // k_pileup addresses a tile's records with 31-bit byte offsets from its first
        if ((int64_t)(b->wrec[(T.b + 31) >> 5] - b->wrec[T.a >> 5]) * 12 >= ((int64_t)1 << 31) - 65536) {
            delete b;
            return s2c_set_error(S2C_ERR_LIMIT, "more than 2 GB of seqout records in one tile");
        }
        const int64_t nch = std::max<int64_t>(1, ceil_div(maxw, chunk));
        for (int64_t c = 0; c < nch; c++) {
            uint32_t it[S2C_ITEM_WORDS] = {(uint32_t)T.a, (uint32_t)T.b, (uint32_t)c, (uint32_t)t};   // 4-6 below
            b->items.insert(b->items.end(), it, it + S2C_ITEM_WORDS);
        }
        uint32_t blk[S2C_BLOCK_WORDS] = {(uint32_t)T.a, (uint32_t)T.b, (uint32_t)T.ref, nch > 1 ? (uint32_t)S2C_TILE_DEEP : 0u};   // words 4-9 below
        b->blocks.insert(b->blocks.end(), blk, blk + S2C_BLOCK_WORDS);
    }
    I.n_items = (int64_t)(b->items.size() / S2C_ITEM_WORDS);
    I.n_blocks = (int64_t)(b->blocks.size() / S2C_BLOCK_WORDS);

    // ---- seqout records, filled per work item: a position without an A/C/G/T entry is
    //      counted in its item's placeholder words (fix) and a '-' / 'N' listed in its
    //      item's entries (exc), so each item's counts are complete on their own (a deep
    //      tile's chunks add into HBM; per-item placeholders fit u16: ≤ chunk_recs) ----
    {
        const int64_t NI = I.n_items;
        std::vector<uint32_t> tile_of_word(NW, 0xFFFFFFFFu), first_item(b->blocks.size() / S2C_BLOCK_WORDS);
        for (int64_t it = NI - 1; it >= 0; it--) first_item[b->items[S2C_ITEM_WORDS * it + 3]] = (uint32_t)it;
        for (size_t t = 0; t < first_item.size(); t++) {
            const uint32_t *blk = &b->blocks[t * S2C_BLOCK_WORDS];
            for (uint32_t W = blk[0] >> 5; W < (blk[1] + 31) >> 5; W++) tile_of_word[W] = (uint32_t)t;
        }
        uint64_t fo = 0;
        for (int64_t it = 0; it < NI; it++) {
            uint32_t *iv = &b->items[S2C_ITEM_WORDS * it];
            iv[4] = (uint32_t)fo;
            fo += 16 * (uint64_t)((iv[1] + 31) / 32 - iv[0] / 32);
        }
        if (fo >= (1ull << 32)) {
            delete b;
            return s2c_set_error(S2C_ERR_LIMIT, "placeholder words exceed 2^32 (split the input)");
        }
        b->recs.resize(2 * nrec);
        b->fix.assign(fo, 0);
        std::vector<uint32_t> xitem;          // item of each '-' / 'N' entry
        std::vector<uint32_t> xent;           // (position − tile start) << 1 | is_N
        std::vector<uint32_t> cur(b->wrec.begin(), b->wrec.end() - 1);
        const uint64_t CH = (uint64_t)I.chunk_recs;
        for (int64_t i = 0; i < NP; i++) {
            const int64_t span = p->p_span[i];
            if (!span) continue;
            const uint32_t *pw = &p->words[p->p_base[i]];   // piece planes + zero pad triple
            const bool drop = p->p_drop[i] != 0;
            const int64_t s0 = (int64_t)gstart[i];
            for (int64_t W = s0 >> 5; W <= (s0 + span - 1) >> 5; W++) {
                const int64_t o = 32 * W - s0;                    // seqout index of the word's first position
                const int64_t qs = std::max<int64_t>(o, 0), bl = std::max<int64_t>(-o, 0);
                const uint32_t *lo = pw + 3 * (qs >> 5), *hi = lo + 3;
                const uint32_t sh = (uint32_t)(qs & 31);
                uint32_t P[3];
                for (int k = 0; k < 3; k++) {
                    const uint64_t v = ((uint64_t)hi[k] << 32 | lo[k]) >> sh;
                    P[k] = (uint32_t)v << bl;
                }
                const int64_t nv = std::min<int64_t>(span - qs, 32 - bl);
                uint32_t valid = (nv >= 32 ? 0xFFFFFFFFu : ((1u << nv) - 1u)) << bl;
                if (drop) valid &= P[0] | P[1] | P[2];
                // 3-bit codes (p2·4+p1·2+p0: 0 '-' 1 A 2 C 3 G 4 N 5 T) → 2-bit bases
                const uint32_t c2 = P[1] & ~P[0] & ~P[2], t5 = P[2] & P[0] & ~P[1], g3 = P[1] & P[0] & ~P[2];
                const uint32_t dash = valid & ~(P[0] | P[1] | P[2]), en = valid & P[2] & ~(P[0] | P[1]);
                const uint64_t ri = cur[W]++;
                uint32_t *r = &b->recs[2 * ri];
                r[0] = valid & (c2 | t5);
                r[1] = valid & (g3 | t5);
                const uint32_t t = tile_of_word[W];
                const uint32_t *blk = &b->blocks[(size_t)t * S2C_BLOCK_WORDS];
                const uint32_t item = first_item[t] + (uint32_t)((ri - b->wrec[W]) / CH);
                const uint32_t *iv = &b->items[S2C_ITEM_WORDS * (size_t)item];
                uint32_t ph = ~valid | dash | en;   // A placeholders
                uint32_t *fw = &b->fix[iv[4] + 16 * (size_t)(W - (iv[0] >> 5))];
                while (ph) {
                    const int j = __builtin_ctz(ph);
                    ph &= ph - 1;
                    fw[j & 15] += (j & 16) ? 0x10000u : 1u;
                }
                uint32_t x = dash | en;
                while (x) {
                    const int j = __builtin_ctz(x);
                    x &= x - 1;
                    xitem.push_back(item);
                    xent.push_back((uint32_t)((32 * W + j - blk[0]) << 1) | ((en >> j) & 1u));
                }
            }
        }
        // '-' / 'N' entries grouped by item (counting sort; item words 5-6 = the range)
        if (xent.size() >= (1ull << 32) - 1) {
            delete b;
            return s2c_set_error(S2C_ERR_LIMIT, "more than 2^32 seqout '-'/'N' entries (split the input)");
        }
        std::vector<uint32_t> xo(NI + 1, 0);
        for (uint32_t it : xitem) xo[it + 1]++;
        for (int64_t it = 0; it < NI; it++) xo[it + 1] += xo[it];
        b->exc.resize(xent.size());
        std::vector<uint32_t> at(xo.begin(), xo.end() - 1);
        for (size_t k = 0; k < xent.size(); k++) b->exc[at[xitem[k]]++] = xent[k];
        for (int64_t it = 0; it < NI; it++) {
            b->items[S2C_ITEM_WORDS * it + 5] = xo[it];
            b->items[S2C_ITEM_WORDS * it + 6] = xo[it + 1];
        }
        I.n_exc = (int64_t)xent.size();
        I.n_fix = (int64_t)fo;
    }

    // ---- insertion events grouped by key (:256-294), keys sorted by position ----
    // Keys in [0, LN) only (negative keys are never emitted, :371).  Per key: its events
    // (file order), a column base (Σ of the keys' longest motif lengths, :278-281), and
    // the key index of each event.  Positions → key index: a bitmap and the
    // number of keys before each 32-position word (rank).
    {
        std::vector<uint32_t> ev;
        ev.reserve(p->i_ref.size());
        for (size_t i = 0; i < p->i_ref.size(); i++)
            if (p->i_key[i] >= 0) ev.push_back((uint32_t)i);
        auto gkey = [&](uint32_t i) { return (uint64_t)(b->ref_off[p->i_ref[i]] + p->i_key[i]); };
        std::stable_sort(ev.begin(), ev.end(), [&](uint32_t x, uint32_t y) { return gkey(x) < gkey(y); });
        uint64_t nb = 0;
        for (uint32_t i : ev) nb += p->i_len[i];
        if (nb >= (1ull << 32) || ev.size() >= (1ull << 31)) {
            delete b;
            return s2c_set_error(S2C_ERR_LIMIT, "insertion events or bases >= 2^31 / 2^32");
        }
        b->ins_off.reserve(ev.size() + 1);
        b->ins_bases.assign((nb + 7) / 8, 0);
        b->ins_bits.assign(NW, 0);
        b->ins_rank.assign(NW + 1, 0);
        b->ins_koff.push_back(0);
        b->ins_kcol.push_back(0);
        uint64_t q = 0, ncol = 0;
        uint32_t maxlen = 0;
        for (size_t j = 0; j < ev.size(); j++) {
            const uint32_t i = ev[j];
            const uint64_t key = gkey(i);
            if (j == 0 || key != b->ins_key.back()) {
                if (j) {                                   // close the previous key
                    ncol += maxlen;
                    b->ins_koff.push_back((uint32_t)j);
                    b->ins_kcol.push_back((uint32_t)ncol);
                }
                b->ins_key.push_back((uint32_t)key);
                b->ins_bits[key >> 5] |= 1u << (key & 31);
                b->ins_rank[(key >> 5) + 1]++;
                maxlen = 0;
            }
            maxlen = std::max(maxlen, p->i_len[i]);
            b->ins_off.push_back((uint32_t)q);
            for (uint32_t c = 0; c < p->i_len[i]; c++, q++)
                b->ins_bases[q >> 3] |= (uint32_t)LUT.v[(uint8_t)p->i_raw[p->i_off[i] + c]] << (4 * (q & 7));
        }
        if (!ev.empty()) {
            ncol += maxlen;
            b->ins_koff.push_back((uint32_t)ev.size());
            b->ins_kcol.push_back((uint32_t)ncol);
        }
        b->ins_off.push_back((uint32_t)q);
        for (int64_t W = 0; W < NW; W++) b->ins_rank[W + 1] += b->ins_rank[W];
        const size_t nk = b->ins_key.size();
        b->ins_ekey.resize(ev.size());
        for (size_t k = 0; k < nk; k++)
            for (uint32_t e = b->ins_koff[k]; e < b->ins_koff[k + 1]; e++) b->ins_ekey[e] = (uint32_t)k;
        // per tile: its keys [klo, khi), events [e0, e1), columns [cb0, cb1) (block words
        // 4-9); per event {column offset in its tile, motif length, nibble offset, first 8
        // nibbles}; per key {position, first column, columns}: one 16-B load each on the device
        b->ins_ev.assign(4 * ev.size(), 0);
        b->ins_kinfo.assign(4 * nk, 0);
        for (size_t k = 0; k < nk; k++) {
            b->ins_kinfo[4 * k] = b->ins_key[k];
            b->ins_kinfo[4 * k + 1] = b->ins_kcol[k];
            b->ins_kinfo[4 * k + 2] = b->ins_kcol[k + 1] - b->ins_kcol[k];
        }
        const size_t ntile = b->blocks.size() / S2C_BLOCK_WORDS;
        for (size_t t = 0; t < ntile; t++) {
            uint32_t *blk = &b->blocks[t * S2C_BLOCK_WORDS];
            const uint32_t klo = nk ? b->ins_rank[blk[0] >> 5] : 0, khi = nk ? b->ins_rank[(blk[1] + 31) >> 5] : 0;
            blk[4] = klo;
            blk[5] = khi;
            blk[6] = nk ? b->ins_koff[klo] : 0;
            blk[7] = nk ? b->ins_koff[khi] : 0;
            blk[8] = nk ? b->ins_kcol[klo] : 0;
            blk[9] = nk ? b->ins_kcol[khi] : 0;
            for (uint32_t e = blk[6]; e < blk[7]; e++) {
                const uint32_t o = b->ins_off[e], len = b->ins_off[e + 1] - o;
                uint32_t w0 = 0;
                for (uint32_t c = 0; c < len && c < 8; c++) w0 |= ((b->ins_bases[(o + c) >> 3] >> (4 * ((o + c) & 7))) & 15u) << (4 * c);
                uint32_t *r = &b->ins_ev[4 * (size_t)e];
                r[0] = b->ins_kcol[b->ins_ekey[e]] - blk[8];
                r[1] = len;
                r[2] = o;
                r[3] = w0;
            }
        }
        I.n_ins = (int64_t)ev.size();
        I.n_ins_bases = (int64_t)nb;
        I.n_ins_words = (int64_t)b->ins_bases.size();
        I.n_keys = (int64_t)nk;
        I.n_cols = (int64_t)ncol;
    }
    {   // tiles k_consensus votes: deep ones, and those whose insertion keys / columns exceed
        // what k_pileup's epilogue holds in LDS (their counts go to HBM)
        const size_t ntile = b->blocks.size() / S2C_BLOCK_WORDS;
        const int64_t lcols = S2C_LDS_COLS(nwp);
        for (size_t t = 0; t < ntile; t++) {
            uint32_t *blk = &b->blocks[t * S2C_BLOCK_WORDS];
            if (blk[5] - blk[4] > S2C_EPI_KEYS || (int64_t)(blk[9] - blk[8]) > lcols) blk[3] |= S2C_TILE_GENERAL;
            if (blk[3]) b->deep.push_back((uint32_t)t);
        }
        I.n_deep = (int64_t)b->deep.size();
    }
    {   // item descriptors: the tile's flags and insertion ranges, the item's first record and,
        // per word, its record range (k_pileup's first load round needs nothing else)
        const int64_t NI = I.n_items;
        const uint64_t CH = (uint64_t)I.chunk_recs;
        b->iwr.assign((size_t)NI * nwp * 2, 0);
        for (int64_t it = 0; it < NI; it++) {
            uint32_t *iv = &b->items[S2C_ITEM_WORDS * it];
            const uint32_t *blk = &b->blocks[(size_t)iv[3] * S2C_BLOCK_WORDS];
            for (int k = 0; k < 7; k++) iv[7 + k] = blk[3 + k];
            iv[14] = b->wrec[iv[0] >> 5];
            for (int64_t w = 0; w < nwp && 32 * w < (int64_t)(iv[1] - iv[0]); w++) {
                const uint64_t W = (iv[0] >> 5) + w, wb = b->wrec[W], we = b->wrec[W + 1];
                const uint64_t r0 = std::min<uint64_t>(we, wb + (uint64_t)iv[2] * CH), r1 = std::min<uint64_t>(we, r0 + CH);
                b->iwr[2 * ((size_t)it * nwp + w)] = (uint32_t)r0;
                b->iwr[2 * ((size_t)it * nwp + w) + 1] = (uint32_t)r1;
            }
        }
        I.n_iwr = (int64_t)b->iwr.size();
    }
    *out = b;
    return S2C_OK;
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
    o->rd_pos = b->rd_pos.data();
    o->rd_op = b->rd_op.data();
    o->rd_span = b->rd_span.data();
    o->ops = b->ops.data();
    o->wrec = b->wrec.data();
    o->recs = b->recs.data();
    o->fix = b->fix.data();
    o->exc = b->exc.data();
    o->iwr = b->iwr.data();
    o->ins_key = b->ins_key.data();
    o->ins_koff = b->ins_koff.data();
    o->ins_kcol = b->ins_kcol.data();
    o->ins_off = b->ins_off.data();
    o->ins_bases = b->ins_bases.data();
    o->ins_ekey = b->ins_ekey.data();
    o->ins_ev = b->ins_ev.data();
    o->ins_kinfo = b->ins_kinfo.data();
    o->ins_bits = b->ins_bits.data();
    o->ins_rank = b->ins_rank.data();
    o->items = b->items.data();
    o->blocks = b->blocks.data();
    o->deep = b->deep.data();
    return S2C_OK;
}

extern "C" const char *s2c_batch_ref_name(const s2c_batch *b, int64_t i) {
    if (!b || i < 0 || i >= (int64_t)b->names.size()) return nullptr;
    return b->names[i].c_str();
}

extern "C" void s2c_batch_free(s2c_batch *b) { delete b; }

// ------------------------------------------------------------------ parsecigar (:46-82)
extern "C" int s2c_parsecigar(const char *cigar, size_t cigar_len, const char *seq, size_t seq_len,
                              int64_t pos_ref, char *seqout, size_t cap, size_t *seqout_len,
                              int64_t *ins, size_t max_ins, size_t *n_ins) {
    std::vector<Tok> toks;
    int rc = tokenize_cigar(cigar, cigar_len, toks);
    if (rc) return rc;
    int64_t start = 0, start_ref = pos_ref;
    const int64_t slen = (int64_t)seq_len;
    size_t o = 0, ni = 0;
    auto put = [&](char c) -> bool {
        if (o + 1 >= cap) return false;
        seqout[o++] = c;
        return true;
    };
    for (const Tok &t : toks) {
        int64_t l = t.len;
        if (t.op == 'M' || t.op == '=' || t.op == 'X') {
            int64_t take = start < slen ? std::min(l, slen - start) : 0;
            for (int64_t j = 0; j < take; j++)
                if (!put(seq[start + j])) return s2c_set_error(S2C_ERR_ARG, "seqout buffer too small");
            start += l;
            start_ref += l;
        } else if (t.op == 'D' || t.op == 'N' || t.op == 'P') {
            for (int64_t j = 0; j < l; j++)
                if (!put('-')) return s2c_set_error(S2C_ERR_ARG, "seqout buffer too small");
            start_ref += l;
        } else if (t.op == 'I') {
            int64_t take = start < slen ? std::min(l, slen - start) : 0;
            if (ni < max_ins) {
                ins[3 * ni] = start_ref;
                ins[3 * ni + 1] = std::min(start, slen);
                ins[3 * ni + 2] = take;
            }
            ni++;
            start += l;
        } else if (t.op == 'S') {
            start += l;
        }
    }
    if (cap) seqout[o] = 0;
    *seqout_len = o;
    *n_ins = ni;
    return ni > max_ins ? s2c_set_error(S2C_ERR_ARG, "insertion buffer too small") : S2C_OK;
}

// ------------------------------------------------------------------ ABI layout self-check
// Lets the ctypes mirror (sam2consensus_amd/_lib.py) verify struct sizes/offsets at load.
#include <cstddef>
extern "C" int s2c_layout(int64_t *out, int n) {
    const int64_t v[] = {
        (int64_t)sizeof(s2c_dev), (int64_t)offsetof(s2c_dev, tile_max), (int64_t)offsetof(s2c_dev, thresholds),
        (int64_t)offsetof(s2c_dev, fill), (int64_t)offsetof(s2c_dev, counts), (int64_t)offsetof(s2c_dev, ins_chr),
        (int64_t)offsetof(s2c_dev, tile_stats), (int64_t)offsetof(s2c_dev, out_cap),
        (int64_t)sizeof(s2c_synth_spec), (int64_t)offsetof(s2c_synth_spec, seed),
        (int64_t)sizeof(s2c_batch_info), (int64_t)sizeof(s2c_batch_arrays), (int64_t)sizeof(s2c_ws_sizes)};
    const int m = (int)(sizeof(v) / sizeof(v[0]));
    for (int i = 0; i < n && i < m; i++) out[i] = v[i];
    return m;
}

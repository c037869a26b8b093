/* s2c_oracle_mc.c — multi-threaded C restatement of sam2consensus.py v2.1 (TEST
 * INFRASTRUCTURE: the multi-core CPU baseline of bench.py and a second checker).
 *
 * Same algorithm as oracle/s2c_oracle.py (which is pinned to the reference's own outputs,
 * tests/golden/), written in plain C with pthreads so the CPU side of the benchmark is a
 * native program on every host core rather than a single Python thread:
 *   header pass            :149-172   (@SQ SN/LN; leading '@' lines)
 *   record pass            :180-228   (split on TAB, CIGAR tokens :58-59, parsecigar :46-82,
 *                                      maxdel :210, counts :211-218, insertions :221)
 *   insertion columns      :262-311   (motif multiplicities per key, '-' = cov - Σ, :294)
 *   consensus              :334-406   (group-sort vote in its closed form, IUPAC :317-329,
 *                                      fill / min depth :355-389, header :394-398)
 *   FASTA files            :411-418   (-n line splitting)
 * Records are split over the threads by byte range (counts added atomically, insertion
 * events kept per thread); each (reference, threshold) body is voted in position chunks in
 * parallel.  The first failure in file order / vote order is reported as the reference's
 * exception class (stdout "status: KeyError", exit 2) and no file is written.
 *
 * Build: make -C oracle (gcc, zlib).  Run: s2c_oracle_mc THREADS -i in.sam [-c ..] [-n ..]
 *        [-o ..] [-p ..] [-m ..] [-f ..] [-d ..]   (the reference's flags, :87-138)
 * Product code never links or runs this file. */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <zlib.h>

/* ------------------------------------------------------------------ small helpers */
typedef struct { char *p; size_t n, cap; } buf_t;
static void buf_put(buf_t *b, const char *s, size_t n) {
    if (b->n + n + 1 > b->cap) {
        size_t c = b->cap ? b->cap : 256;
        while (b->n + n + 1 > c) c *= 2;
        b->p = realloc(b->p, c);
        b->cap = c;
    }
    memcpy(b->p + b->n, s, n);
    b->n += n;
    b->p[b->n] = 0;
}
static void buf_puts(buf_t *b, const char *s) { buf_put(b, s, strlen(s)); }

static const char *ERR_NAMES[] = {"ok", "KeyError", "IndexError", "ValueError", "ZeroDivisionError", "OverflowError"};
enum { E_OK = 0, E_KEY, E_INDEX, E_VALUE, E_ZERO, E_OVERFLOW };

static void fail(int e) {
    printf("status: %s\n", ERR_NAMES[e]);
    exit(2);
}

static int code_of(unsigned char c) {   /* "-ACGNT" index, -1 if none */
    switch (c) {
    case '-': return 0;
    case 'A': return 1;
    case 'C': return 2;
    case 'G': return 3;
    case 'N': return 4;
    case 'T': return 5;
    default: return -1;
    }
}

static int py_ws(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0b || c == 0x0c; }

/* Python 2 int(str): ASCII whitespace, sign, decimal digits (saturating at ±2^62) */
static int py2_int(const char *s, size_t n, int64_t *out) {
    size_t i = 0;
    while (i < n && py_ws((unsigned char)s[i])) i++;
    int neg = 0;
    if (i < n && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
    size_t d0 = i;
    int64_t v = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') {
        if (v < ((int64_t)1 << 58)) v = v * 10 + (s[i] - '0');
        i++;
    }
    if (i == d0) return -1;
    while (i < n && py_ws((unsigned char)s[i])) i++;
    if (i != n) return -1;
    *out = neg ? -v : v;
    return 0;
}

/* ------------------------------------------------------------------ the IUPAC table :317-329 */
static char AMB[64];   /* 0: the reference's amb dict has no key (KeyError) */
static void amb_init(void) {
    const char iupac[16] = {0, 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};
    for (int m = 0; m < 64; m++) {
        const int dash = m & 1, n = (m >> 4) & 1;
        const int b = ((m >> 1) & 1) | (((m >> 2) & 1) << 1) | (((m >> 3) & 1) << 2) | (((m >> 5) & 1) << 3);
        char c = 0;
        if (m == 0) c = 0;
        else if (b == 0) c = (dash && n) ? 'n' : (dash ? '-' : 'N');
        else if (b == 15) c = (n && !dash) ? 0 : 'N';
        else {
            c = iupac[b];
            if (dash || n) c = (char)(c + ('a' - 'A'));
        }
        AMB[m] = c;
    }
}

/* the group-sort vote (:241-251, :298-308, :359-366) literally: the non-zero counts grouped
 * by value, groups taken in descending value order while the running sum is < t·cov
 * (Python int < float: exact here, both below 2^53).  Signed: an insertion column's '-'
 * count (cov - Σ, :294) can be negative. */
static char vote(const int64_t c[6], uint64_t cov, double t, int *err) {
    const double tc = t * (double)cov;
    int m = 0, done = 0;
    int64_t acc = 0, last = INT64_MAX;
    while (!done) {
        int64_t v = INT64_MIN;   /* the largest value below the last group's */
        for (int i = 0; i < 6; i++)
            if (c[i] && c[i] < last && c[i] > v) v = c[i];
        if (v == INT64_MIN) break;
        if (!((double)acc < tc)) break;
        for (int i = 0; i < 6; i++)
            if (c[i] == v) {
                m |= 1 << i;
                acc += v;
            }
        last = v;
    }
    if (!AMB[m]) *err = E_KEY;
    return AMB[m];
}

/* ------------------------------------------------------------------ options :87-138 */
typedef struct {
    const char *filename, *outfolder, *prefix, *fill;
    double thr[256];
    int nthr;
    int64_t n, min_depth;
    int maxdel_active;
    int64_t maxdel;
} opts_t;

/* ------------------------------------------------------------------ references */
typedef struct {
    char *name;
    int64_t len;
    uint32_t *cnt;   /* [len][6] */
} ref_t;
static ref_t *REFS;
static int NREF;

static int ref_find(const char *s, size_t n) {   /* linear probe hash */
    static int *tab;
    static int cap;
    if (!tab) {
        cap = 1;
        while (cap < 4 * NREF + 4) cap <<= 1;
        tab = malloc(sizeof(int) * cap);
        for (int i = 0; i < cap; i++) tab[i] = -1;
        for (int r = 0; r < NREF; r++) {
            uint64_t h = 1469598103934665603ull;
            for (const char *q = REFS[r].name; *q; q++) h = (h ^ (unsigned char)*q) * 1099511628211ull;
            int k = (int)(h & (cap - 1));
            while (tab[k] >= 0) k = (k + 1) & (cap - 1);
            tab[k] = r;
        }
    }
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) h = (h ^ (unsigned char)s[i]) * 1099511628211ull;
    for (int k = (int)(h & (cap - 1));; k = (k + 1) & (cap - 1)) {
        if (tab[k] < 0) return -1;
        const char *nm = REFS[tab[k]].name;
        if (strlen(nm) == n && !memcmp(nm, s, n)) return tab[k];
    }
}

/* ------------------------------------------------------------------ record pass */
typedef struct {
    int ref;
    int64_t key;
    const char *motif;   /* into the input buffer */
    uint32_t len;
} ins_t;

typedef struct {
    const char *a, *b;   /* the chunk's lines */
    const opts_t *o;
    int err;             /* first failure of the chunk */
    ins_t *ins;
    size_t nins, cap;
} chunk_t;

static void ins_push(chunk_t *c, int ref, int64_t key, const char *m, uint32_t len) {
    if (c->nins == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 1024;
        c->ins = realloc(c->ins, sizeof(ins_t) * c->cap);
    }
    c->ins[c->nins++] = (ins_t){ref, key, m, len};
}

#define MAXTOK 4096
static int do_line(chunk_t *c, const char *s, const char *e) {
    if (s[0] == '@') return 0;   /* :195 */
    const char *f[10];
    size_t fl[10];
    int nf = 0;
    const char *p = s;
    while (nf < 10) {
        const char *q = p;
        while (q < e && *q != '\t') q++;
        f[nf] = p;
        fl[nf] = (size_t)(q - p);
        nf++;
        if (q >= e) break;
        p = q + 1;
    }
    if (nf < 6) return E_INDEX;                        /* :195 [5] */
    if (fl[5] == 1 && f[5][0] == '*') return 0;
    const char *rn = f[2], *re = f[2] + fl[2];         /* :200 split()[0] */
    while (rn < re && py_ws((unsigned char)*rn)) rn++;
    if (rn == re) return E_INDEX;
    const char *rq = rn;
    while (rq < re && !py_ws((unsigned char)*rq)) rq++;
    int64_t pos;
    if (py2_int(f[3], fl[3], &pos)) return E_VALUE;    /* :201 */
    pos -= 1;
    if (nf < 10) return E_INDEX;                       /* :206 [9] */
    /* CIGAR tokens (:58-59 regex findall) */
    static __thread int64_t tl[MAXTOK];
    static __thread char top[MAXTOK];
    int nt = 0;
    const char *cg = f[5];
    for (size_t i = 0; i < fl[5];) {
        if (cg[i] >= '0' && cg[i] <= '9') {
            size_t j = i;
            int64_t v = 0;
            while (j < fl[5] && cg[j] >= '0' && cg[j] <= '9') {
                if (v < ((int64_t)1 << 40)) v = v * 10 + (cg[j] - '0');
                j++;
            }
            if (j < fl[5] && strchr("MIDNSHPX=", cg[j]) && cg[j]) {
                if (nt < MAXTOK) {
                    tl[nt] = v;
                    top[nt] = cg[j];
                    nt++;
                }
                i = j + 1;
            } else {
                i = j;
            }
        } else {
            i++;
        }
    }
    const char *seq = f[9];
    const int64_t slen = (int64_t)fl[9];
    const int ref = ref_find(rn, (size_t)(rq - rn));
    /* maxdel (:210): '-' in seqout (D/N/P lengths + '-' chars of SEQ taken) */
    int drop = 0;
    if (c->o->maxdel_active) {
        int64_t dashes = 0, st = 0;
        for (int t = 0; t < nt; t++) {
            const char op = top[t];
            const int64_t l = tl[t];
            if (op == 'M' || op == '=' || op == 'X') {
                const int64_t take = st < slen ? (l < slen - st ? l : slen - st) : 0;
                for (int64_t k = 0; k < take; k++) dashes += seq[st + k] == '-';
                st += l;
            } else if (op == 'D' || op == 'N' || op == 'P') {
                dashes += l;
            } else if (op == 'I' || op == 'S') {
                st += l;
            }
        }
        drop = dashes > c->o->maxdel;
    }
    /* :211-218 (the reference raises KeyError on an unknown RNAME at the first counted char,
       :212/:217, or at :221 when nothing is counted) */
    const int64_t L = ref >= 0 ? REFS[ref].len : 0;
    uint32_t *cr = ref >= 0 ? REFS[ref].cnt : NULL;
    int64_t k = pos, st = 0, key = pos;
    for (int t = 0; t < nt; t++) {
        const char op = top[t];
        const int64_t l = tl[t];
        if (op == 'M' || op == '=' || op == 'X' || op == 'D' || op == 'N' || op == 'P') {
            const int bases = op == 'M' || op == '=' || op == 'X';
            const int64_t take = bases ? (st < slen ? (l < slen - st ? l : slen - st) : 0) : l;
            for (int64_t j = 0; j < take; j++, k++) {
                const unsigned char ch = bases ? (unsigned char)seq[st + j] : '-';
                if (drop && ch == '-') continue;
                if (ref < 0) return E_KEY;
                if (!(-L <= k && k < L)) return E_INDEX;
                const int cd = code_of(ch);
                if (cd < 0) return E_KEY;
                __atomic_fetch_add(&cr[6 * (k < 0 ? k + L : k) + cd], 1u, __ATOMIC_RELAXED);
            }
            if (bases) st += l;
            key += l;   /* start_ref (:69, :72) */
        } else if (op == 'I') {
            const int64_t a = st < slen ? st : slen, b = st + l < slen ? st + l : slen;
            if (ref >= 0) ins_push(c, ref, key, seq + a, (uint32_t)(b > a ? b - a : 0));
            st += l;
        } else if (op == 'S') {
            st += l;
        }
    }
    if (ref < 0) return E_KEY;   /* :221 */
    return 0;
}

static void *chunk_run(void *arg) {
    chunk_t *c = arg;
    const char *p = c->a;
    while (p < c->b) {
        const char *q = memchr(p, '\n', (size_t)(c->b - p));
        const char *e = q ? q : c->b;
        /* a line keeps its '\n' (Py2 iteration): the last field then ends with it */
        const int err = do_line(c, p, q ? q + 1 : c->b);
        (void)e;
        if (err) {
            c->err = err;
            return NULL;
        }
        p = q ? q + 1 : c->b;
    }
    return NULL;
}

/* ------------------------------------------------------------------ insertion columns */
static int ins_cmp(const void *x, const void *y) {
    const ins_t *a = x, *b = y;
    if (a->ref != b->ref) return a->ref < b->ref ? -1 : 1;
    if (a->key != b->key) return a->key < b->key ? -1 : 1;
    return 0;
}

typedef struct {
    int64_t key;
    int ncol;
    int64_t *col;    /* [ncol][6] */
} icol_t;

/* ------------------------------------------------------------------ consensus */
typedef struct {
    const ref_t *r;
    const uint64_t *cov;
    const icol_t *ic;
    int nic;
    double t;
    const opts_t *o;
    int64_t p0, p1;
    buf_t out;
    uint64_t sumcov;
    int err;
} vjob_t;

static void *vote_run(void *arg) {
    vjob_t *j = arg;
    const opts_t *o = j->o;
    const size_t fl = strlen(o->fill);
    /* the first insertion key ≥ p0 */
    int ki = 0;
    while (ki < j->nic && j->ic[ki].key < j->p0) ki++;
    for (int64_t p = j->p0; p < j->p1; p++) {
        const uint64_t c = j->cov[p];
        if (c == 0) {
            buf_put(&j->out, o->fill, fl);
            continue;
        }
        j->sumcov += c;
        if ((int64_t)c >= o->min_depth) {
            int64_t cc[6];
            for (int s = 0; s < 6; s++) cc[s] = j->r->cnt[6 * p + s];
            int err = 0;
            char ch = vote(cc, c, j->t, &err);
            if (err) {
                j->err = err;
                return NULL;
            }
            buf_put(&j->out, &ch, 1);
            while (ki < j->nic && j->ic[ki].key < p) ki++;
            if (ki < j->nic && j->ic[ki].key == p) {
                for (int q = 0; q < j->ic[ki].ncol; q++) {
                    ch = vote(j->ic[ki].col + 6 * q, c, j->t, &err);
                    if (err) {
                        j->err = err;
                        return NULL;
                    }
                    if (ch != '-') {
                        buf_put(&j->out, &ch, 1);
                        j->sumcov += c;
                    }
                }
            }
        } else {
            buf_put(&j->out, o->fill, fl);
        }
    }
    return NULL;
}

/* CPython 2.7 round(x, 2) (correctly rounded, exact binary ties away from zero) */
static double py2_round2(double x) {
    if (x == 0.0 || isnan(x) || isinf(x)) return x;
    char s[512];
    snprintf(s, sizeof s, "%.400f", fabs(x));   /* exact decimal expansion (glibc) */
    char *dot = strchr(s, '.');
    int carry = dot[3] >= '5';                   /* digits after the 2nd decimal: ≥ .005 → up */
    dot[3] = 0;
    /* add one unit of the last place with carry */
    if (carry) {
        char *q = dot + 2;
        for (;;) {
            if (q == dot) q--;
            if (q < s) {
                memmove(s + 1, s, strlen(s) + 1);
                s[0] = '1';
                break;
            }
            if (*q == '9') {
                *q = '0';
                q--;
            } else {
                (*q)++;
                break;
            }
        }
    }
    const double r = strtod(s, NULL);
    return x < 0 ? -r : r;
}

static void py2_str_float(double x, char *out, size_t cap) {
    snprintf(out, cap, "%.12g", x);
    const char *q = out[0] == '-' ? out + 1 : out;
    int digits = *q != 0;
    for (; *q; q++)
        if (*q < '0' || *q > '9') digits = 0;
    if (digits) strncat(out, ".0", cap - strlen(out) - 1);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s THREADS -i in.sam [reference flags]\n", argv[0]);
        return 1;
    }
    int T = atoi(argv[1]);
    if (T < 1) T = 1;
    opts_t o = {0};
    o.outfolder = "./";
    o.prefix = "";
    o.fill = "-";
    o.min_depth = 1;
    o.maxdel_active = 1;
    o.maxdel = 150;
    const char *thr = "0.25";
    for (int i = 2; i < argc; i++) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
        const char *eq = strchr(a, '=');
        char key[64] = {0};
        if (a[0] == '-' && a[1] == '-' && eq) {   /* --opt=value */
            snprintf(key, sizeof key, "%.*s", (int)(eq - a), a);
            v = eq + 1;
            a = key;
        } else {
            i++;
        }
        if (!v) return 1;
        if (!strcmp(a, "-i") || !strcmp(a, "--input")) o.filename = v;
        else if (!strcmp(a, "-c") || !strcmp(a, "--consensus-thresholds")) thr = v;
        else if (!strcmp(a, "-n")) o.n = atoll(v);
        else if (!strcmp(a, "-o") || !strcmp(a, "--outfolder")) o.outfolder = v;
        else if (!strcmp(a, "-p") || !strcmp(a, "--prefix")) o.prefix = v;
        else if (!strcmp(a, "-m") || !strcmp(a, "--min-depth")) o.min_depth = atoll(v);
        else if (!strcmp(a, "-f") || !strcmp(a, "--fill")) o.fill = v;
        else if (!strcmp(a, "-d") || !strcmp(a, "--maxdel")) o.maxdel_active = 0;   /* :102 str → never applied */
        else return 1;
    }
    if (!o.filename) return 1;
    for (const char *p = thr;;) {   /* :117-118 */
        char *end;
        const double d = strtod(p, &end);
        if (end == p || (*end && *end != ',')) fail(E_VALUE);
        o.thr[o.nthr++] = d;
        if (!*end || o.nthr == 256) break;
        p = end + 1;
    }
    char prefix[4096];
    if (!o.prefix[0]) {   /* :121-122 */
        const char *b = strrchr(o.filename, '/');
        b = b ? b + 1 : o.filename;
        snprintf(prefix, sizeof prefix, "%.*s", (int)strcspn(b, "."), b);
        o.prefix = prefix;
    }
    amb_init();
    /* ---- input (gzip or plain) */
    buf_t in = {0};
    {
        gzFile g = gzopen(o.filename, "rb");
        if (!g) return 1;
        char tmp[1 << 16];
        int r;
        while ((r = gzread(g, tmp, sizeof tmp)) > 0) buf_put(&in, tmp, (size_t)r);
        gzclose(g);
    }
    const char *s = in.p ? in.p : "", *e = s + in.n;
    /* ---- header pass :149-172 */
    const char *p = s;
    int cap = 0;
    while (p < e && *p == '@') {
        const char *q = memchr(p, '\n', (size_t)(e - p));
        const char *le = q ? q + 1 : e;
        if (le - p >= 3 && !memcmp(p, "@SQ", 3)) {
            const char *f1 = memchr(p, '\t', (size_t)(le - p));
            if (!f1) fail(E_INDEX);
            f1++;
            const char *f1e = memchr(f1, '\t', (size_t)(le - f1));
            if (!f1e) fail(E_INDEX);
            const char *f2 = f1e + 1, *f2e = memchr(f2, '\t', (size_t)(le - f2));
            if (!f2e) f2e = le;
            /* SN: removed everywhere, split()[0] */
            char nm[4096];
            size_t nn = 0;
            for (const char *x = f1; x < f1e && nn < sizeof nm - 1;) {
                if (f1e - x >= 3 && !memcmp(x, "SN:", 3)) { x += 3; continue; }
                nm[nn++] = *x++;
            }
            nm[nn] = 0;
            char *a0 = nm;
            while (*a0 && py_ws((unsigned char)*a0)) a0++;
            if (!*a0) fail(E_INDEX);
            char *a1 = a0;
            while (*a1 && !py_ws((unsigned char)*a1)) a1++;
            *a1 = 0;
            char ln[256];
            size_t lnn = 0;
            for (const char *x = f2; x < f2e && lnn < sizeof ln - 1;) {
                if (f2e - x >= 3 && !memcmp(x, "LN:", 3)) { x += 3; continue; }
                ln[lnn++] = *x++;
            }
            int64_t L;
            if (py2_int(ln, lnn, &L)) fail(E_VALUE);
            if (L < 0) L = 0;
            int r = -1;
            for (int k = 0; k < NREF; k++)
                if (!strcmp(REFS[k].name, a0)) r = k;
            if (r < 0) {
                if (NREF == cap) {
                    cap = cap ? 2 * cap : 64;
                    REFS = realloc(REFS, sizeof(ref_t) * cap);
                }
                r = NREF++;
                REFS[r].name = strdup(a0);
            }
            REFS[r].len = L;
        }
        p = le;
    }
    for (int r = 0; r < NREF; r++) REFS[r].cnt = calloc((size_t)REFS[r].len * 6 + 6, sizeof(uint32_t));
    ref_find("", 0);   /* builds the name table before the threads read it */
    /* ---- record pass :180-228, T byte ranges at line starts */
    chunk_t *ch = calloc((size_t)T, sizeof(chunk_t));
    pthread_t *th = calloc((size_t)T, sizeof(pthread_t));
    {
        const char *a = s;
        for (int t = 0; t < T; t++) {
            const char *b = t == T - 1 ? e : s + (size_t)((double)in.n * (t + 1) / T);
            if (b < a) b = a;
            if (b < e) {
                const char *q = memchr(b, '\n', (size_t)(e - b));
                b = q ? q + 1 : e;
            }
            ch[t].a = a;
            ch[t].b = b;
            ch[t].o = &o;
            a = b;
        }
        for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, chunk_run, &ch[t]);
        for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
        for (int t = 0; t < T; t++)
            if (ch[t].err) fail(ch[t].err);
    }
    /* ---- insertion events by (ref, key); motif multiplicities → columns :262-311 */
    size_t nins = 0;
    for (int t = 0; t < T; t++) nins += ch[t].nins;
    ins_t *all = malloc(sizeof(ins_t) * (nins + 1));
    for (int t = 0, k = 0; t < T; t++) {
        memcpy(all + k, ch[t].ins, sizeof(ins_t) * ch[t].nins);
        k += (int)ch[t].nins;
    }
    qsort(all, nins, sizeof(ins_t), ins_cmp);
    /* ---- per reference: coverage, columns, then every threshold's body */
    typedef struct { char *name; buf_t body; } file_t;
    file_t *files = calloc((size_t)NREF + 1, sizeof(file_t));
    int nfiles = 0;
    size_t ii = 0;
    for (int r = 0; r < NREF; r++) {
        const ref_t *R = &REFS[r];
        const int64_t L = R->len;
        uint64_t *cov = malloc(sizeof(uint64_t) * (size_t)(L + 1));
        uint64_t tot = 0;
        for (int64_t q = 0; q < L; q++) {
            uint64_t c = 0;
            for (int k = 0; k < 6; k++) c += R->cnt[6 * q + k];
            cov[q] = c;
            tot += c;
        }
        /* columns of this reference's keys (KeyError for every key first, then IndexError) */
        size_t i0 = ii;
        while (ii < nins && all[ii].ref == r) ii++;
        int nic = 0;
        icol_t *ic = NULL;
        for (size_t a = i0; a < ii;) {
            size_t b = a;
            int ncol = 0;
            while (b < ii && all[b].key == all[a].key) {
                if ((int)all[b].len > ncol) ncol = (int)all[b].len;
                b++;
            }
            ic = realloc(ic, sizeof(icol_t) * (size_t)(nic + 1));
            ic[nic].key = all[a].key;
            ic[nic].ncol = ncol;
            ic[nic].col = calloc((size_t)ncol * 6 + 6, sizeof(int64_t));
            for (size_t x = a; x < b; x++)
                for (uint32_t q = 0; q < all[x].len; q++) {
                    const int cd = code_of((unsigned char)all[x].motif[q]);
                    if (cd < 0) fail(E_KEY);
                    ic[nic].col[6 * q + cd]++;
                }
            nic++;
            a = b;
        }
        for (int k = 0; k < nic; k++) {
            if (!ic[k].ncol) continue;
            if (!(-L <= ic[k].key && ic[k].key < L)) fail(E_INDEX);
            const uint64_t cv = cov[ic[k].key < 0 ? ic[k].key + L : ic[k].key];
            for (int q = 0; q < ic[k].ncol; q++) {
                int64_t sum = 0;
                for (int x = 0; x < 6; x++) sum += ic[k].col[6 * q + x];
                ic[k].col[6 * q] = (int64_t)cv - sum;   /* :294 */
            }
        }
        if (tot == 0) {   /* :334-341 */
            free(cov);
            continue;
        }
        for (int ti = 0; ti < o.nthr; ti++) {
            const double t = o.thr[ti];
            vjob_t *jobs = calloc((size_t)T, sizeof(vjob_t));
            for (int k = 0; k < T; k++) {
                jobs[k].r = R;
                jobs[k].cov = cov;
                jobs[k].ic = ic;
                jobs[k].nic = nic;
                jobs[k].t = t;
                jobs[k].o = &o;
                jobs[k].p0 = L * k / T;
                jobs[k].p1 = L * (k + 1) / T;
                pthread_create(&th[k], NULL, vote_run, &jobs[k]);
            }
            for (int k = 0; k < T; k++) pthread_join(th[k], NULL);
            for (int k = 0; k < T; k++)
                if (jobs[k].err) fail(jobs[k].err);
            buf_t seq = {0};
            uint64_t sumcov = 0;
            for (int k = 0; k < T; k++) {
                buf_put(&seq, jobs[k].out.p ? jobs[k].out.p : "", jobs[k].out.n);
                sumcov += jobs[k].sumcov;
                free(jobs[k].out.p);
            }
            free(jobs);
            /* :394-398 */
            const double t100 = t * 100.0;
            if (isnan(t100)) fail(E_VALUE);
            if (isinf(t100)) fail(E_OVERFLOW);
            char tag[400];
            snprintf(tag, sizeof tag, "%.0f", trunc(t100));
            if (!strcmp(tag, "-0")) strcpy(tag, "0");
            if (seq.n == 0) fail(E_ZERO);
            char cs[64];
            py2_str_float(py2_round2((double)sumcov / (double)seq.n), cs, sizeof cs);
            size_t nondash = 0;
            for (size_t q = 0; q < seq.n; q++) nondash += seq.p[q] != '-';
            if (nondash == 0) {
                free(seq.p);
                continue;
            }
            file_t *F = NULL;
            for (int k = 0; k < nfiles; k++)
                if (!strcmp(files[k].name, R->name)) F = &files[k];
            if (!F) {
                F = &files[nfiles++];
                F->name = R->name;
            } else {
                buf_puts(&F->body, "\n");
            }
            char num[32];
            buf_puts(&F->body, ">");
            buf_puts(&F->body, o.prefix);
            buf_puts(&F->body, "|c");
            buf_puts(&F->body, tag);
            buf_puts(&F->body, " reference:");
            buf_puts(&F->body, R->name);
            buf_puts(&F->body, " coverage:");
            buf_puts(&F->body, cs);
            buf_puts(&F->body, " length:");
            snprintf(num, sizeof num, "%zu", nondash);
            buf_puts(&F->body, num);
            buf_puts(&F->body, " consensus_threshold:");
            buf_puts(&F->body, tag);
            buf_puts(&F->body, "%\n");
            if (o.n == 0) {
                buf_put(&F->body, seq.p, seq.n);
            } else if (o.n > 0) {   /* :413-416 */
                for (size_t q = 0; q < seq.n; q += (size_t)o.n) {
                    if (q) buf_puts(&F->body, "\n");
                    buf_put(&F->body, seq.p + q, seq.n - q < (size_t)o.n ? seq.n - q : (size_t)o.n);
                }
            }
            free(seq.p);
        }
        free(cov);
    }
    /* ---- files :411-418 */
    char dir[4096];
    snprintf(dir, sizeof dir, "%s", o.outfolder);
    size_t dl = strlen(dir);
    while (dl > 0 && dir[dl - 1] == '/') dir[--dl] = 0;
    mkdir(dir, 0777);
    for (int k = 0; k < nfiles; k++) {
        char path[8192];
        snprintf(path, sizeof path, "%s/%s__%s.fasta", dir, files[k].name, o.prefix);
        FILE *fh = fopen(path, "wb");
        if (!fh) return 1;
        fwrite(files[k].body.p, 1, files[k].body.n, fh);
        fputs("\n", fh);
        fclose(fh);
    }
    printf("status: ok\nfiles: %d\n", nfiles);
    return 0;
}

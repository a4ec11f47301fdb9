/*
 * tp_regex.c -- tcpprep --regex (src/tcpprep.c:300-335,433-440) for the device.
 *
 * The reference runs regexec(3) (REG_EXTENDED | REG_NOSUB, tcpprep_opts.def:225) over
 * the source address as inet_ntop prints it, per packet.  The strings are short and
 * drawn from 18 characters (hex digits, '.', ':'), so the pattern is compiled here,
 * once, into a DFA over those characters plus two markers (string start / end, which
 * '^' and '$' consume) and the classifier walks it per record on the GPU.
 *
 *   ERE text --parse--> syntax tree --Thompson--> NFA --subsets--> DFA
 *
 * The search is unanchored (regexec finds a match anywhere): every DFA state also holds
 * the NFA start, and a state holding the NFA accept is absorbing.  What this parser
 * does not model (back-references, GNU escapes like \w, equivalence classes) is refused
 * loudly; whatever it accepts is checked against the host's regexec on a probe set
 * before it is used.
 */
#include <arpa/inet.h>
#include <regex.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>

#include "tp_dev_cfg.h"
#include "tp_regex.h"

/* symbols: '0'-'9' 0-9, 'a'-'f' 10-15, '.' 16, ':' 17, start 18, end 19 */
static int sym_of(int c)
{
    if (c >= '0' && c <= '9')
        return c - '0';
    if (c >= 'a' && c <= 'f')
        return 10 + c - 'a';
    if (c == '.')
        return 16;
    if (c == ':')
        return 17;
    return -1;
}
static const char SYM_CHARS[] = "0123456789abcdef.:";
#define ALL_CHARS ((1u << 18) - 1)
#define SYM_BOS (1u << TP_SYM_BOS)
#define SYM_EOS (1u << TP_SYM_EOS)

/* ---- syntax tree ---- */
enum { N_SET, N_CAT, N_ALT, N_REP, N_EMPTY };
typedef struct {
    int type;
    uint32_t set; /* N_SET: symbols it matches */
    int a, b;     /* children */
    int lo, hi;   /* N_REP: {lo,hi}, hi < 0: unbounded */
} node_t;

#define MAX_NODES 2048
#define MAX_NFA 8192
#define MAX_REP 64

typedef struct {
    const char *p;
    node_t n[MAX_NODES];
    int nn;
    char err[160];
} parser_t;

static int mk(parser_t *P, int type, uint32_t set, int a, int b)
{
    if (P->nn >= MAX_NODES) {
        snprintf(P->err, sizeof P->err, "regex too large for the device DFA");
        return -1;
    }
    node_t *x = &P->n[P->nn];
    x->type = type;
    x->set = set;
    x->a = a;
    x->b = b;
    x->lo = x->hi = 0;
    return P->nn++;
}

static int parse_alt(parser_t *P);

/* a bracket expression after '[' (POSIX: ']' first is literal, '\' is literal) */
static int parse_bracket(parser_t *P)
{
    int neg = 0;
    uint32_t set = 0;
    if (*P->p == '^') {
        neg = 1;
        P->p++;
    }
    int first = 1;
    while (*P->p && (first || *P->p != ']')) {
        first = 0;
        if (P->p[0] == '[' && (P->p[1] == ':' || P->p[1] == '=' || P->p[1] == '.')) {
            const char kind = P->p[1];
            const char *end = strchr(P->p + 2, kind);
            if (!end || end[1] != ']') {
                snprintf(P->err, sizeof P->err, "unterminated [%c in a bracket expression", kind);
                return -1;
            }
            if (kind != ':') {
                snprintf(P->err, sizeof P->err, "collating elements / equivalence classes are not supported");
                return -1;
            }
            char name[16] = "";
            const size_t len = (size_t)(end - (P->p + 2));
            if (len >= sizeof name) {
                snprintf(P->err, sizeof P->err, "unknown character class");
                return -1;
            }
            memcpy(name, P->p + 2, len);
            int (*fn)(int) = NULL;
            if (!strcmp(name, "digit")) fn = isdigit;
            else if (!strcmp(name, "xdigit")) fn = isxdigit;
            else if (!strcmp(name, "alpha")) fn = isalpha;
            else if (!strcmp(name, "alnum")) fn = isalnum;
            else if (!strcmp(name, "lower")) fn = islower;
            else if (!strcmp(name, "upper")) fn = isupper;
            else if (!strcmp(name, "punct")) fn = ispunct;
            else if (!strcmp(name, "space")) fn = isspace;
            else if (!strcmp(name, "blank")) fn = isblank;
            else if (!strcmp(name, "cntrl")) fn = iscntrl;
            else if (!strcmp(name, "print")) fn = isprint;
            else if (!strcmp(name, "graph")) fn = isgraph;
            if (!fn) {
                snprintf(P->err, sizeof P->err, "unknown character class [:%s:]", name);
                return -1;
            }
            for (int s = 0; s < 18; s++)
                if (fn((unsigned char)SYM_CHARS[s]))
                    set |= 1u << s;
            P->p = end + 2;
            continue;
        }
        int lo = (unsigned char)*P->p++, hi = lo;
        if (P->p[0] == '-' && P->p[1] && P->p[1] != ']') { /* a range (C locale: by code) */
            hi = (unsigned char)P->p[1];
            P->p += 2;
            if (hi < lo) {
                snprintf(P->err, sizeof P->err, "invalid range end");
                return -1;
            }
        }
        for (int s = 0; s < 18; s++) {
            const int c = (unsigned char)SYM_CHARS[s];
            if (c >= lo && c <= hi)
                set |= 1u << s;
        }
    }
    if (*P->p != ']') {
        snprintf(P->err, sizeof P->err, "unmatched [");
        return -1;
    }
    P->p++;
    return mk(P, N_SET, neg ? (~set & ALL_CHARS) : set, -1, -1);
}

static int parse_atom(parser_t *P)
{
    const char c = *P->p;
    if (c == '(') {
        P->p++;
        const int r = *P->p == ')' ? mk(P, N_EMPTY, 0, -1, -1) : parse_alt(P);
        if (r < 0)
            return -1;
        if (*P->p != ')') {
            snprintf(P->err, sizeof P->err, "unmatched (");
            return -1;
        }
        P->p++;
        return r;
    }
    if (c == '[') {
        P->p++;
        return parse_bracket(P);
    }
    P->p++;
    if (c == '.')
        return mk(P, N_SET, ALL_CHARS, -1, -1);
    if (c == '^')
        return mk(P, N_SET, SYM_BOS, -1, -1);
    if (c == '$')
        return mk(P, N_SET, SYM_EOS, -1, -1);
    if (c == '\\') {
        const char e = *P->p;
        if (!e) {
            snprintf(P->err, sizeof P->err, "trailing backslash");
            return -1;
        }
        if (isalnum((unsigned char)e)) { /* back-references and GNU escapes (\w, \b, \<, ...) */
            snprintf(P->err, sizeof P->err, "escape \\%c is not supported by the device DFA", e);
            return -1;
        }
        P->p++;
        const int s = sym_of(e);
        return mk(P, N_SET, s < 0 ? 0 : 1u << s, -1, -1);
    }
    const int s = sym_of(c);
    return mk(P, N_SET, s < 0 ? 0 : 1u << s, -1, -1); /* a character no address contains: never matches */
}

static int parse_piece(parser_t *P)
{
    int a = parse_atom(P);
    while (a >= 0) {
        int lo, hi;
        const char c = *P->p;
        if (c == '*') {
            lo = 0, hi = -1;
            P->p++;
        } else if (c == '+') {
            lo = 1, hi = -1;
            P->p++;
        } else if (c == '?') {
            lo = 0, hi = 1;
            P->p++;
        } else if (c == '{' && isdigit((unsigned char)P->p[1])) {
            char *end;
            lo = (int)strtol(P->p + 1, &end, 10);
            hi = lo;
            if (*end == ',') {
                end++;
                hi = isdigit((unsigned char)*end) ? (int)strtol(end, &end, 10) : -1;
            }
            if (*end != '}' || (hi >= 0 && hi < lo) || lo > MAX_REP || hi > MAX_REP) {
                snprintf(P->err, sizeof P->err, "invalid or too large interval");
                return -1;
            }
            P->p = end + 1;
        } else {
            break;
        }
        const int r = mk(P, N_REP, 0, a, -1);
        if (r < 0)
            return -1;
        P->n[r].lo = lo;
        P->n[r].hi = hi;
        a = r;
    }
    return a;
}

static int parse_branch(parser_t *P)
{
    int r = -1;
    while (*P->p && *P->p != '|' && *P->p != ')') {
        const int a = parse_piece(P);
        if (a < 0)
            return -1;
        r = r < 0 ? a : mk(P, N_CAT, 0, r, a);
        if (r < 0)
            return -1;
    }
    return r < 0 ? mk(P, N_EMPTY, 0, -1, -1) : r;
}

static int parse_alt(parser_t *P)
{
    int r = parse_branch(P);
    while (r >= 0 && *P->p == '|') {
        P->p++;
        const int b = parse_branch(P);
        if (b < 0)
            return -1;
        r = mk(P, N_ALT, 0, r, b);
    }
    return r;
}

/* ---- NFA (Thompson): a state has a symbol edge or up to two epsilon edges ---- */
typedef struct {
    uint32_t set; /* symbol edge to `to` (0: none) */
    int to, e1, e2;
} nstate_t;

typedef struct {
    nstate_t *s;
    int n;
    char *err;
} nfa_t;

static int ns(nfa_t *A)
{
    if (A->n >= MAX_NFA) {
        snprintf(A->err, 160, "regex too large for the device DFA");
        return -1;
    }
    A->s[A->n].set = 0;
    A->s[A->n].to = A->s[A->n].e1 = A->s[A->n].e2 = -1;
    return A->n++;
}

static void eps(nfa_t *A, int from, int to)
{
    if (A->s[from].e1 < 0)
        A->s[from].e1 = to;
    else
        A->s[from].e2 = to;
}

/* builds node x between fresh states; returns 0 and sets *s / *e */
static int build(const parser_t *P, nfa_t *A, int x, int *s, int *e)
{
    const node_t *nd = &P->n[x];
    if ((*s = ns(A)) < 0 || (*e = ns(A)) < 0)
        return -1;
    switch (nd->type) {
    case N_EMPTY:
        eps(A, *s, *e);
        return 0;
    case N_SET:
        A->s[*s].set = nd->set;
        A->s[*s].to = *e;
        return 0;
    case N_CAT: {
        int as, ae, bs, be;
        if (build(P, A, nd->a, &as, &ae) < 0 || build(P, A, nd->b, &bs, &be) < 0)
            return -1;
        eps(A, *s, as);
        eps(A, ae, bs);
        eps(A, be, *e);
        return 0;
    }
    case N_ALT: {
        int as, ae, bs, be;
        if (build(P, A, nd->a, &as, &ae) < 0 || build(P, A, nd->b, &bs, &be) < 0)
            return -1;
        eps(A, *s, as);
        eps(A, *s, bs);
        eps(A, ae, *e);
        eps(A, be, *e);
        return 0;
    }
    default: { /* N_REP: lo copies, then (hi - lo) optional ones or a star */
        int cur = *s;
        for (int i = 0; i < nd->lo; i++) {
            int as, ae;
            if (build(P, A, nd->a, &as, &ae) < 0)
                return -1;
            eps(A, cur, as);
            cur = ae;
        }
        if (nd->hi < 0) {
            int as, ae, hub;
            if ((hub = ns(A)) < 0 || build(P, A, nd->a, &as, &ae) < 0)
                return -1;
            eps(A, cur, hub);
            eps(A, hub, as);
            eps(A, ae, hub);
            eps(A, hub, *e);
        } else {
            for (int i = nd->lo; i < nd->hi; i++) {
                int as, ae, nx;
                if (build(P, A, nd->a, &as, &ae) < 0 || (nx = ns(A)) < 0)
                    return -1;
                eps(A, cur, as);
                eps(A, cur, nx); /* skip this copy (and the rest) */
                eps(A, ae, nx);
                cur = nx;
            }
            eps(A, cur, *e);
        }
        return 0;
    }
    }
}

/* ---- subset construction ---- */
#define WORDS (MAX_NFA / 64)
typedef struct {
    uint64_t w[WORDS];
} bits_t;

static void closure(const nfa_t *A, bits_t *b, int *stack)
{
    int sp = 0;
    for (int i = 0; i < A->n; i++)
        if (b->w[i >> 6] >> (i & 63) & 1)
            stack[sp++] = i;
    while (sp) {
        const int i = stack[--sp];
        const int t[2] = {A->s[i].e1, A->s[i].e2};
        for (int k = 0; k < 2; k++)
            if (t[k] >= 0 && !(b->w[t[k] >> 6] >> (t[k] & 63) & 1)) {
                b->w[t[k] >> 6] |= 1ull << (t[k] & 63);
                stack[sp++] = t[k];
            }
    }
}

static int tp_regex_build(const char *re, tp_dfa_t *D, char *err, size_t errlen)
{
    parser_t *P = calloc(1, sizeof *P);
    nfa_t A = {calloc(MAX_NFA, sizeof(nstate_t)), 0, NULL};
    bits_t *sets = malloc(sizeof(bits_t) * TP_DFA_MAX);
    int *stack = malloc(sizeof(int) * MAX_NFA * 2);
    int rc = -1;
    if (!P || !A.s || !sets || !stack) {
        snprintf(err, errlen, "out of memory compiling the regex");
        goto done;
    }
    A.err = P->err;
    P->p = re;
    int root = parse_alt(P);
    if (root >= 0 && *P->p) {
        snprintf(P->err, sizeof P->err, "unmatched )");
        root = -1;
    }
    int s0, acc;
    if (root < 0 || build(P, &A, root, &s0, &acc) < 0) {
        snprintf(err, errlen, "%s", P->err[0] ? P->err : "regex not supported by the device DFA");
        goto done;
    }
    /* DFA state 0: the absorbing match state; state 1: the start */
    memset(D, 0, sizeof *D);
    for (int k = 0; k < TP_NSYM; k++)
        D->next[0][k] = 0;
    bits_t start;
    memset(&start, 0, sizeof start);
    start.w[s0 >> 6] |= 1ull << (s0 & 63);
    closure(&A, &start, stack);
    int nd = 0;
    sets[nd++] = start; /* placeholder for state 0 (never looked up) */
    sets[nd++] = start;
    const int start_acc = (int)(start.w[acc >> 6] >> (acc & 63) & 1);
    D->start = start_acc ? 0 : 1;
    for (int d = 1; d < nd; d++) {
        for (int k = 0; k < TP_NSYM; k++) {
            bits_t nx = start; /* unanchored: a match may begin at any symbol */
            for (int i = 0; i < A.n; i++)
                if ((sets[d].w[i >> 6] >> (i & 63) & 1) && (A.s[i].set >> k & 1)) {
                    const int t = A.s[i].to;
                    nx.w[t >> 6] |= 1ull << (t & 63);
                }
            closure(&A, &nx, stack);
            int to;
            if (nx.w[acc >> 6] >> (acc & 63) & 1) {
                to = 0;
            } else {
                for (to = 1; to < nd; to++)
                    if (!memcmp(&sets[to], &nx, sizeof nx))
                        break;
                if (to == nd) {
                    if (nd >= TP_DFA_MAX) {
                        snprintf(err, errlen, "regex needs more than %d DFA states", TP_DFA_MAX);
                        goto done;
                    }
                    sets[nd++] = nx;
                }
            }
            D->next[d][k] = (uint8_t)to;
        }
    }
    D->nstates = nd;
    rc = 0;
done:
    free(P);
    free(A.s);
    free(sets);
    free(stack);
    return rc;
}

int tp_dfa_match(const tp_dfa_t *D, const char *s)
{
    int st = D->next[D->start][TP_SYM_BOS];
    if (D->start == 0)
        return 1;
    for (; *s && st; s++) {
        const int k = sym_of((unsigned char)*s);
        if (k < 0)
            return -1;
        st = D->next[st][k];
    }
    if (st)
        st = D->next[st][TP_SYM_EOS];
    return st == 0;
}

/* the probe set: addresses of every shape inet_ntop prints, random and edge cases */
static int probe(const tp_dfa_t *D, const regex_t *rx, char *err, size_t errlen)
{
    uint64_t x = 0x9e3779b97f4a7c15ull;
    char buf[64];
    for (int i = 0; i < 20000; i++) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        uint8_t a[16];
        for (int k = 0; k < 16; k++)
            a[k] = (uint8_t)(x >> (8 * (k & 7))) ^ (uint8_t)(k * 29 + i);
        const int kind = i % 8;
        if (kind >= 2) { /* sparse IPv6: runs of zero words, v4-mapped / compatible */
            for (int w = 0; w < 8; w++)
                if ((x >> (w + kind)) & 1)
                    a[2 * w] = a[2 * w + 1] = 0;
            if (kind == 6)
                memset(a, 0, 10), a[10] = a[11] = 0xff;
            if (kind == 7)
                memset(a, 0, 12);
        }
        const char *s = kind == 0 ? inet_ntop(AF_INET, a, buf, sizeof buf) : inet_ntop(AF_INET6, a, buf, sizeof buf);
        if (kind == 1) /* small octets / digits the patterns name */
            snprintf(buf, sizeof buf, "%u.%u.%u.%u", (unsigned)(x % 200), (unsigned)(x >> 8) % 256, a[2] % 10, a[3]);
        if (!s)
            continue;
        const int want = regexec(rx, buf, 0, NULL, 0) == 0, got = tp_dfa_match(D, buf);
        if (got != want) {
            snprintf(err, errlen, "regex not supported by the device DFA (it disagrees with regexec on %s)", buf);
            return -1;
        }
    }
    return 0;
}

int tp_regex_compile(const char *re, tp_dfa_t *D, char *err, size_t errlen)
{
    regex_t rx;
    const int e = regcomp(&rx, re, REG_EXTENDED | REG_NOSUB); /* tcpprep_opts.def:225 */
    if (e) {
        char eb[128];
        regerror(e, &rx, eb, sizeof eb);
        snprintf(err, errlen, "Unable to compile regex: %s", eb);
        return -1;
    }
    int rc = tp_regex_build(re, D, err, errlen);
    if (rc == 0)
        rc = probe(D, &rx, err, errlen);
    regfree(&rx);
    return rc;
}

/* diagnostics / tests: the DFA's verdict on one string (-1: the regex is refused) */
int tcpprep_regex_dfa_match(const char *re, const char *s)
{
    tp_dfa_t *D = malloc(sizeof *D);
    char err[200];
    if (!D)
        return -1;
    int r = tp_regex_build(re, D, err, sizeof err) == 0 ? tp_dfa_match(D, s) : -1;
    free(D);
    return r;
}

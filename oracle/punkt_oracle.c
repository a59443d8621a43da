/*
 * Oracle: nltk Punkt sentence segmentation (the reference's `nltk.tokenize.sent_tokenize`,
 * lddl/dask/bert/pretrain.py:86) restated in C over code points.
 *
 * TEST INFRASTRUCTURE ONLY (see lddl_oracle.h). Pinned by tests/golden/punkt.npz, produced by
 * nltk 3.6.5 itself (tests/golden/make_punkt_golden.py). nltk is a third-party dependency of the
 * reference (not vendored under /root/reference); the functions below follow its published
 * algorithm, nltk/tokenize/punkt.py (3.6.5):
 *
 *   PunktSentenceTokenizer.span_tokenize      -> orc_punkt_spans
 *   _slices_from_text (period_context_re finditer + text_contains_sentbreak)
 *   _realign_boundaries (re_boundary_realignment)
 *   PunktBaseClass._tokenize_words / PunktLanguageVars.word_tokenize (_word_tokenize_fmt)
 *   _first_pass_annotation, _second_pass_annotation, _ortho_heuristic
 *   PunktToken: type (_RE_NUMERIC), type_no_period, type_no_sentperiod, first_upper/lower,
 *               is_ellipsis (_RE_ELLIPSIS), is_initial (_RE_INITIAL)
 *
 * Character classes (Python `re` \s, [^\W\d], \d; str.isupper/islower/lower) come from
 * lddl_amd/assets/punkt_props.bin (tools/make_punkt_tables.py records them from Python).
 * Each regular expression is emulated with the backtracking order Python's `re` uses.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lddl_oracle.h"

enum { P_SPACE = 1, P_UPPER = 2, P_LOWER = 4, P_ALNOD = 8, P_DIGIT = 16 };
enum { K_ABBREV = 1, K_STARTER = 2, K_ORTHO = 3, K_COLLOC = 4 };
/* nltk _ORTHO_* flags */
enum { O_BEG_UC = 2, O_MID_UC = 4, O_UNK_UC = 8, O_BEG_LC = 16, O_MID_LC = 32, O_UNK_LC = 64 };
#define O_UC (O_BEG_UC | O_MID_UC | O_UNK_UC)
#define O_LC (O_BEG_LC | O_MID_LC | O_UNK_LC)

typedef struct {
  const uint16_t* l1;
  const uint8_t* pages;
  const int32_t* lower; /* pairs */
  int n_lower;
  /* parameters: records (kind, value, a, b) */
  int n_rec;
  uint8_t* kind;
  uint8_t* value;
  const uint8_t** a;
  int* la;
  const uint8_t** b;
  int* lb;
} Punkt;

struct orc_punkt {
  Punkt p;
  uint8_t* blob;
};

static int props(const Punkt* p, int32_t cp) {
  if (cp < 0 || cp >= 0x110000) return 0;
  return p->pages[(size_t)p->l1[cp >> 8] * 256 + (cp & 255)];
}

/* str.lower() of one code point; returns the number of output code points (1 or 2) */
static int lower_cp(const Punkt* p, int32_t cp, int32_t* out) {
  int lo = 0, hi = p->n_lower - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    int32_t k = p->lower[2 * mid];
    if (k == cp) {
      int32_t v = p->lower[2 * mid + 1];
      if (v < 0) {
        out[0] = 0x69;
        out[1] = 0x307;
        return 2;
      }
      out[0] = v;
      return 1;
    }
    if (k < cp) lo = mid + 1; else hi = mid - 1;
  }
  out[0] = cp;
  return 1;
}

orc_punkt* orc_punkt_create(const uint8_t* table, int64_t table_bytes, const uint8_t* params,
                            int64_t params_bytes) {
  if (table_bytes < 16 || memcmp(table, "LDPK", 4) != 0) return NULL;
  uint32_t hdr[3];
  memcpy(hdr, table + 4, 12);
  orc_punkt* o = (orc_punkt*)calloc(1, sizeof(orc_punkt));
  o->blob = (uint8_t*)malloc((size_t)table_bytes + (size_t)params_bytes + 8);
  memcpy(o->blob, table, (size_t)table_bytes);
  if (params_bytes) memcpy(o->blob + table_bytes, params, (size_t)params_bytes);
  const uint8_t* t = o->blob + 16;
  o->p.l1 = (const uint16_t*)t;
  o->p.pages = t + 0x1100 * 2;
  o->p.lower = (const int32_t*)(o->p.pages + (size_t)hdr[1] * 256);
  o->p.n_lower = (int)hdr[2];
  /* parameter records: u8 kind, u8 value, u16 la, u16 lb, a bytes, b bytes */
  const uint8_t* q = o->blob + table_bytes;
  const uint8_t* end = q + params_bytes;
  int n = 0;
  for (const uint8_t* r = q; r + 6 <= end;) {
    int la = r[2] | (r[3] << 8), lb = r[4] | (r[5] << 8);
    r += 6 + la + lb;
    n++;
  }
  Punkt* p = &o->p;
  p->n_rec = n;
  p->kind = (uint8_t*)calloc(n + 1, 1);
  p->value = (uint8_t*)calloc(n + 1, 1);
  p->a = (const uint8_t**)calloc(n + 1, sizeof(void*));
  p->b = (const uint8_t**)calloc(n + 1, sizeof(void*));
  p->la = (int*)calloc(n + 1, sizeof(int));
  p->lb = (int*)calloc(n + 1, sizeof(int));
  int i = 0;
  for (const uint8_t* r = q; r + 6 <= end; i++) {
    p->kind[i] = r[0];
    p->value[i] = r[1];
    p->la[i] = r[2] | (r[3] << 8);
    p->lb[i] = r[4] | (r[5] << 8);
    p->a[i] = r + 6;
    p->b[i] = r + 6 + p->la[i];
    r += 6 + p->la[i] + p->lb[i];
  }
  return o;
}

void orc_punkt_destroy(orc_punkt* o) {
  if (!o) return;
  free(o->p.kind);
  free(o->p.value);
  free(o->p.a);
  free(o->p.b);
  free(o->p.la);
  free(o->p.lb);
  free(o->blob);
  free(o);
}

/* ---- strings of code points ---------------------------------------------------------------- */

typedef struct {
  int32_t* c;
  int n, cap;
} Str;

static void s_push(Str* s, int32_t c) {
  if (s->n == s->cap) {
    s->cap = s->cap ? 2 * s->cap : 32;
    s->c = (int32_t*)realloc(s->c, sizeof(int32_t) * s->cap);
  }
  s->c[s->n++] = c;
}

static int utf8_encode(const int32_t* c, int n, uint8_t* out) {
  int k = 0;
  for (int i = 0; i < n; i++) {
    int32_t v = c[i];
    if (v < 0x80) {
      out[k++] = (uint8_t)v;
    } else if (v < 0x800) {
      out[k++] = (uint8_t)(0xC0 | (v >> 6));
      out[k++] = (uint8_t)(0x80 | (v & 63));
    } else if (v < 0x10000) {
      out[k++] = (uint8_t)(0xE0 | (v >> 12));
      out[k++] = (uint8_t)(0x80 | ((v >> 6) & 63));
      out[k++] = (uint8_t)(0x80 | (v & 63));
    } else {
      out[k++] = (uint8_t)(0xF0 | (v >> 18));
      out[k++] = (uint8_t)(0x80 | ((v >> 12) & 63));
      out[k++] = (uint8_t)(0x80 | ((v >> 6) & 63));
      out[k++] = (uint8_t)(0x80 | (v & 63));
    }
  }
  return k;
}

/* parameter lookup: record of `kind` whose key equals a (and b for collocations) */
static int find_rec(const Punkt* p, int kind, const Str* a, const Str* b) {
  uint8_t ba[4096], bb[4096];
  if (a->n > 1000 || (b && b->n > 1000)) return -1;
  int na = utf8_encode(a->c, a->n, ba), nb = b ? utf8_encode(b->c, b->n, bb) : 0;
  for (int i = 0; i < p->n_rec; i++) {
    if (p->kind[i] != kind || p->la[i] != na || memcmp(p->a[i], ba, na) != 0) continue;
    if (b && (p->lb[i] != nb || memcmp(p->b[i], bb, nb) != 0)) continue;
    return i;
  }
  return -1;
}

/* ---- PunktToken ------------------------------------------------------------------------------ */

typedef struct {
  const int32_t* t; /* token code points */
  int n;
  Str type;         /* lower() with _RE_NUMERIC -> "##number##" */
  int period_final, sentbreak, abbr, ellipsis;
} Tok;

static int is_ch(int32_t c, const char* set) {
  return c > 0 && c < 128 && strchr(set, (char)c) != NULL;
}

/* _RE_NUMERIC = ^-?[\.,]?\d[\d,\.-]*\.?$ on tok.lower() (lowering never creates or removes
 * the characters involved, so it is tested on the token) */
static int is_numeric(const Punkt* p, const int32_t* t, int n) {
  int i = 0;
  if (i < n && t[i] == '-') i++;
  if (i < n && (t[i] == '.' || t[i] == ',')) i++;
  if (!(i < n && (props(p, t[i]) & P_DIGIT))) return 0;
  i++;
  /* [\d,\.-]* greedy, then \.?$ : backtracking can only give back a final '.', which \.? then
   * takes, so the class run must reach the end */
  while (i < n && ((props(p, t[i]) & P_DIGIT) || t[i] == ',' || t[i] == '.' || t[i] == '-')) i++;
  return i == n;
}

static void tok_init(const Punkt* p, Tok* k, const int32_t* t, int n) {
  memset(k, 0, sizeof(*k));
  k->t = t;
  k->n = n;
  if (is_numeric(p, t, n)) {
    const char* s = "##number##";
    for (int i = 0; s[i]; i++) s_push(&k->type, s[i]);
  } else {
    for (int i = 0; i < n; i++) {
      int32_t o[2];
      int m = lower_cp(p, t[i], o);
      for (int j = 0; j < m; j++) s_push(&k->type, o[j]);
    }
  }
  k->period_final = n > 0 && t[n - 1] == '.';
}

static void tok_free(Tok* k) { free(k->type.c); }

/* type_no_period: the type without a final period, if len(type) > 1 */
static Str type_no_period(const Tok* k) {
  Str s = k->type;
  if (s.n > 1 && s.c[s.n - 1] == '.') s.n--;
  return s;
}

static Str type_no_sentperiod(const Tok* k) { return k->sentbreak ? type_no_period(k) : k->type; }

static int is_ellipsis(const Tok* k) { /* _RE_ELLIPSIS \.\.+$ (re.match) */
  if (k->n < 2) return 0;
  for (int i = 0; i < k->n; i++) if (k->t[i] != '.') return 0;
  return 1;
}

static int is_initial(const Punkt* p, const Tok* k) { /* _RE_INITIAL [^\W\d]\.$ (re.match) */
  return k->n == 2 && (props(p, k->t[0]) & P_ALNOD) && k->t[1] == '.';
}

static void first_pass(const Punkt* p, Tok* k) {
  const int32_t* t = k->t;
  int n = k->n;
  if (n == 1 && is_ch(t[0], ".?!")) {
    k->sentbreak = 1;
  } else if (is_ellipsis(k)) {
    k->ellipsis = 1;
  } else if (k->period_final && !(n >= 2 && t[n - 2] == '.')) {
    /* tok[:-1].lower() in abbrev_types, or its last '-' component */
    Str lo = {0, 0, 0};
    for (int i = 0; i < n - 1; i++) {
      int32_t o[2];
      int m = lower_cp(p, t[i], o);
      for (int j = 0; j < m; j++) s_push(&lo, o[j]);
    }
    int hit = find_rec(p, K_ABBREV, &lo, NULL) >= 0;
    if (!hit) {
      int d = lo.n;
      while (d > 0 && lo.c[d - 1] != '-') d--;
      Str tail = {lo.c + d, lo.n - d, 0};
      hit = find_rec(p, K_ABBREV, &tail, NULL) >= 0;
    }
    free(lo.c);
    if (hit) k->abbr = 1; else k->sentbreak = 1;
  }
}

static int ortho_ctx(const Punkt* p, const Str* typ) {
  int r = find_rec(p, K_ORTHO, typ, NULL);
  return r >= 0 ? p->value[r] : 0;
}

/* _ortho_heuristic: 1 True, 0 False, 2 "unknown" */
static int ortho_heuristic(const Punkt* p, const Tok* k) {
  /* `aug_tok.tok in ";:,.!?"` is a substring test: tokens reaching it are single characters */
  if (k->n == 1 && is_ch(k->t[0], ";:,.!?")) return 0;
  Str ty = type_no_sentperiod(k);
  int oc = ortho_ctx(p, &ty);
  int fu = (props(p, k->t[0]) & P_UPPER) != 0, fl = (props(p, k->t[0]) & P_LOWER) != 0;
  if (fu && (oc & O_LC) && !(oc & O_MID_UC)) return 1;
  if (fl && ((oc & O_UC) || !(oc & O_BEG_LC))) return 0;
  return 2;
}

static void second_pass(const Punkt* p, Tok* a, const Tok* b) {
  if (!a->period_final) return;
  Str typ = type_no_period(a);
  Str next_typ = type_no_sentperiod(b);
  int initial = is_initial(p, a);
  if (find_rec(p, K_COLLOC, &typ, &next_typ) >= 0) {
    a->sentbreak = 0;
    a->abbr = 1;
    return;
  }
  if ((a->abbr || a->ellipsis) && !initial) {
    int h = ortho_heuristic(p, b);
    if (h == 1) {
      a->sentbreak = 1;
      return;
    }
    if ((props(p, b->t[0]) & P_UPPER) && find_rec(p, K_STARTER, &next_typ, NULL) >= 0) {
      a->sentbreak = 1;
      return;
    }
  }
  static const char num[] = "##number##";
  int is_num = typ.n == 10;
  for (int i = 0; is_num && i < 10; i++) is_num = typ.c[i] == num[i];
  if (initial || is_num) {
    int h = ortho_heuristic(p, b);
    if (h == 0) {
      a->sentbreak = 0;
      a->abbr = 1;
      return;
    }
    if (h == 2 && initial && (props(p, b->t[0]) & P_UPPER) && !(ortho_ctx(p, &next_typ) & O_LC)) {
      a->sentbreak = 0;
      a->abbr = 1;
      return;
    }
  }
}

/* ---- word_tokenize (_word_tokenize_fmt, findall) ----------------------------------------------- */

static int is_space(const Punkt* p, int32_t c) { return (props(p, c) & P_SPACE) != 0; }
static int non_word(int32_t c) { return is_ch(c, ")\";}]*:@'({[?!"); }
static int word_start_excl(int32_t c) { return is_ch(c, "(\"`{[:;&#*@)}]-,"); }

/* MultiChar = \-{2,} | \.{2,} | (?:\.\s){2,}\.   -> match length at i, 0 if none */
static int multi_char(const Punkt* p, const int32_t* s, int n, int i) {
  if (i + 1 < n && s[i] == '-' && s[i + 1] == '-') {
    int e = i;
    while (e < n && s[e] == '-') e++;
    return e - i;
  }
  if (i + 1 < n && s[i] == '.' && s[i + 1] == '.') {
    int e = i;
    while (e < n && s[e] == '.') e++;
    return e - i;
  }
  int k = 0, e = i;
  while (e + 1 < n && s[e] == '.' && is_space(p, s[e + 1])) {
    k++;
    e += 2;
  }
  for (; k >= 2; k--) /* backtrack the greedy repetition until a '.' follows */
    if (i + 2 * k < n && s[i + 2 * k] == '.') return 2 * k + 1;
  return 0;
}

/* end-of-word lookahead at e: \s | $ | NonWord | MultiChar | ,(?=$|\s|NonWord|MultiChar) */
static int word_end(const Punkt* p, const int32_t* s, int n, int e) {
  if (e == n) return 1;
  if (is_space(p, s[e]) || non_word(s[e]) || multi_char(p, s, n, e)) return 1;
  if (s[e] == ',') {
    int f = e + 1;
    return f == n || is_space(p, s[f]) || non_word(s[f]) || multi_char(p, s, n, f);
  }
  return 0;
}

/* appends (start, len) of each token of line s[0..n) */
static void word_tokenize(const Punkt* p, const int32_t* s, int n, Str* spans) {
  int i = 0;
  while (i < n) {
    int m = multi_char(p, s, n, i);
    if (m) {
      s_push(spans, i);
      s_push(spans, m);
      i += m;
      continue;
    }
    if (is_space(p, s[i])) {
      i++;
      continue;
    }
    if (!word_start_excl(s[i])) {
      int e = i + 1; /* \S+? : lazily extend until the end lookahead holds */
      while (!word_end(p, s, n, e)) e++;
      s_push(spans, i);
      s_push(spans, e - i);
      i = e;
      continue;
    }
    s_push(spans, i);
    s_push(spans, 1);
    i++;
  }
}

/* text_contains_sentbreak(context): a token marked as a sentence break that has a successor */
static int contains_sentbreak(const Punkt* p, const int32_t* s, int n) {
  Str spans = {0, 0, 0};
  int i = 0; /* _tokenize_words: split on '\n', skip blank lines */
  while (i <= n) {
    int e = i;
    while (e < n && s[e] != '\n') e++;
    int blank = 1;
    for (int j = i; j < e && blank; j++) blank = is_space(p, s[j]);
    if (!blank) {
      int before = spans.n;
      word_tokenize(p, s + i, e - i, &spans);
      for (int j = before; j < spans.n; j += 2) spans.c[j] += i;
    }
    i = e + 1;
  }
  int nt = spans.n / 2, found = 0;
  Tok cur, nxt;
  if (nt > 0) {
    tok_init(p, &cur, s + spans.c[0], spans.c[1]);
    first_pass(p, &cur);
  }
  for (int k = 0; k + 1 < nt && !found; k++) {
    tok_init(p, &nxt, s + spans.c[2 * k + 2], spans.c[2 * k + 3]);
    first_pass(p, &nxt);
    second_pass(p, &cur, &nxt);
    found = cur.sentbreak;
    tok_free(&cur);
    cur = nxt;
  }
  if (nt > 0) tok_free(&cur);
  free(spans.c);
  return found;
}

/* ---- span_tokenize ------------------------------------------------------------------------ */

/* re_boundary_realignment = ["\')\]}]+?(?:\s+|(?=--)|$) (MULTILINE), re.match on s[a..b):
 * returns the match length, -1 if none; *closing = length of the bracket run */
static int realign_match(const Punkt* p, const int32_t* s, int a, int b, int* closing) {
  int i = a;
  while (i < b) {
    if (!is_ch(s[i], "\"')]}")) return -1;
    i++; /* lazy: one more closing char, then try the alternatives */
    if (i < b && is_space(p, s[i])) {
      int e = i;
      while (e < b && is_space(p, s[e])) e++;
      *closing = i - a;
      return e - a;
    }
    if (i + 1 < b && s[i] == '-' && s[i + 1] == '-') {
      *closing = i - a;
      return i - a;
    }
    if (i == b || s[i] == '\n') {
      *closing = i - a;
      return i - a;
    }
  }
  return -1;
}

/* Spans (code-point indices) of one document; returns the count written to out[2*k..]. */
static int punkt_spans_cp(const Punkt* p, const int32_t* s, int n, int64_t* out) {
  int64_t* sl = (int64_t*)malloc(sizeof(int64_t) * (2 * (size_t)n + 4));
  int ns = 0, last_break = 0, pos = 0;
  /* period_context_re finditer: \S* [.?!] (?=(NonWord | \s+ (\S+))) */
  while (pos < n) {
    int found = 0, ms = 0, me = 0, after_end = 0, next_tok = -1;
    for (int st = pos; st < n && !found;) {
      if (is_space(p, s[st])) {
        st++;
        continue;
      }
      int r = st;
      while (r < n && !is_space(p, s[r])) r++;
      for (int q = r - 1; q >= st; q--) { /* greedy \S* backtracking: last end char that fits */
        if (!is_ch(s[q], ".?!")) continue;
        int j = q + 1;
        if (j < n && non_word(s[j])) {
          after_end = j + 1;
          next_tok = -1;
        } else if (j < n && is_space(p, s[j])) {
          int k = j;
          while (k < n && is_space(p, s[k])) k++;
          if (k == n) continue;
          int e = k;
          while (e < n && !is_space(p, s[e])) e++;
          next_tok = k;
          after_end = e;
        } else {
          continue;
        }
        found = 1;
        ms = st;
        me = q + 1;
        break;
      }
      /* no match starting in [st, r): every later start inside the run sees a subset of the
       * same candidates */
      if (!found) st = r;
    }
    if (!found) break;
    /* context = match.group() + match.group("after_tok") = s[ms .. after_end) */
    if (contains_sentbreak(p, s + ms, after_end - ms)) {
      sl[2 * ns] = last_break;
      sl[2 * ns + 1] = me;
      ns++;
      last_break = next_tok >= 0 ? next_tok : me;
    }
    pos = me;
  }
  int rs = n;
  while (rs > 0 && is_space(p, s[rs - 1])) rs--;
  sl[2 * ns] = last_break;
  sl[2 * ns + 1] = rs;
  ns++;
  /* _realign_boundaries */
  int cnt = 0, realign = 0;
  for (int k = 0; k < ns; k++) {
    int64_t a = sl[2 * k] + realign, b = sl[2 * k + 1];
    if (k + 1 == ns) {
      if (b > a) {
        out[2 * cnt] = a;
        out[2 * cnt + 1] = b;
        cnt++;
      }
      continue;
    }
    int closing = 0;
    int m = realign_match(p, s, (int)sl[2 * k + 2], (int)sl[2 * k + 3], &closing);
    if (m >= 0) {
      out[2 * cnt] = a;
      out[2 * cnt + 1] = sl[2 * k + 2] + closing;
      cnt++;
      realign = m;
    } else {
      realign = 0;
      if (b > a) {
        out[2 * cnt] = a;
        out[2 * cnt + 1] = b;
        cnt++;
      }
    }
  }
  free(sl);
  return cnt;
}

static int utf8_decode(const uint8_t* t, int64_t n, int32_t* cp, int64_t* boff) {
  int m = 0;
  for (int64_t i = 0; i < n;) {
    uint8_t c = t[i];
    int len = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
    int32_t v = len == 1 ? c : len == 2 ? (c & 31) : len == 3 ? (c & 15) : (c & 7);
    for (int j = 1; j < len && i + j < n; j++) v = (v << 6) | (t[i + j] & 63);
    boff[m] = i;
    cp[m++] = v;
    i += len;
  }
  boff[m] = n;
  return m;
}

int64_t orc_punkt_spans(orc_punkt* o, const uint8_t* text, const int64_t* doc_off, int64_t n_doc,
                        int64_t* span_start, int64_t* span_end, int64_t* doc_count) {
  int64_t total = 0;
  for (int64_t d = 0; d < n_doc; d++) {
    int64_t b0 = doc_off[d], len = doc_off[d + 1] - b0;
    int32_t* cp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(len + 1));
    int64_t* boff = (int64_t*)malloc(sizeof(int64_t) * (size_t)(len + 2));
    int64_t* sp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(2 * len + 8));
    int m = utf8_decode(text + b0, len, cp, boff);
    int c = punkt_spans_cp(&o->p, cp, m, sp);
    for (int k = 0; k < c; k++) {
      span_start[total + k] = boff[sp[2 * k]];
      span_end[total + k] = boff[sp[2 * k + 1]];
    }
    doc_count[d] = c;
    total += c;
    free(cp);
    free(boff);
    free(sp);
  }
  return total;
}

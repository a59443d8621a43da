/*
 * lddl_oracle — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY (see header).
 *
 * Each function cites the reference (paths relative to /root/reference) or, for code that lives
 * in a third-party dependency of the reference, the dependency and its pinned/installed version.
 */
#include "lddl_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ============================================================================================
 * CPython random (dependency of lddl/dask/bert/pretrain.py:35; Python 3.10.12 in this image).
 * Algorithm: MT19937 (Matsumoto & Nishimura), seeded by init_by_array over the 32-bit limbs of
 * abs(seed); random() = (a*2^26 + b) / 2^53 with a = u32>>5, b = u32>>6; _randbelow(n) draws
 * getrandbits(n.bit_length()) = u32 >> (32-k) until < n; shuffle = Fisher-Yates from the top.
 * ========================================================================================== */
#define MT_N 624
#define MT_M 397

static void mt_init_genrand(orc_mt* s, uint32_t seed) {
  s->mt[0] = seed;
  for (int i = 1; i < MT_N; i++)
    s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
  s->mti = MT_N;
}

void orc_mt_seed_key(orc_mt* s, const uint32_t* key, int key_len) {
  mt_init_genrand(s, 19650218u);
  int i = 1, j = 0;
  for (int k = (MT_N > key_len ? MT_N : key_len); k; k--) {
    s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    i++;
    j++;
    if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
    if (j >= key_len) j = 0;
  }
  for (int k = MT_N - 1; k; k--) {
    s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    i++;
    if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
  }
  s->mt[0] = 0x80000000u;
  s->mti = MT_N;
}

void orc_mt_seed_i64(orc_mt* s, int64_t seed) {
  uint64_t a = seed < 0 ? (uint64_t)(-(seed + 1)) + 1 : (uint64_t)seed;
  uint32_t key[2] = {(uint32_t)a, (uint32_t)(a >> 32)};
  orc_mt_seed_key(s, key, key[1] ? 2 : 1);
}

uint32_t orc_mt_u32(orc_mt* s) {
  static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
  uint32_t y;
  if (s->mti >= MT_N) {
    int kk;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
      y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
      s->mt[kk] = s->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < MT_N - 1; kk++) {
      y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
      s->mt[kk] = s->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (s->mt[MT_N - 1] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
    s->mt[MT_N - 1] = s->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    s->mti = 0;
  }
  y = s->mt[s->mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

double orc_mt_random(orc_mt* s) {
  uint32_t a = orc_mt_u32(s) >> 5, b = orc_mt_u32(s) >> 6;
  return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

uint32_t orc_mt_randbelow(orc_mt* s, uint32_t n) {
  int k = 32 - __builtin_clz(n); /* n.bit_length(); n >= 1 */
  uint32_t r = orc_mt_u32(s) >> (32 - k);
  while (r >= n) r = orc_mt_u32(s) >> (32 - k);
  return r;
}

int64_t orc_mt_randint(orc_mt* s, int64_t a, int64_t b) {
  return a + (int64_t)orc_mt_randbelow(s, (uint32_t)(b - a + 1));
}

void orc_mt_shuffle_i32(orc_mt* s, int32_t* x, int64_t n) {
  for (int64_t i = n - 1; i > 0; i--) {
    int64_t j = orc_mt_randbelow(s, (uint32_t)(i + 1));
    int32_t t = x[i];
    x[i] = x[j];
    x[j] = t;
  }
}

void orc_mt_get_state(const orc_mt* s, uint32_t* st) {
  memcpy(st, s->mt, sizeof(s->mt));
  st[MT_N] = (uint32_t)s->mti;
}

/* ============================================================================================
 * Tokenizer (lddl/dask/bert/pretrain.py:79-80 -> transformers.BertTokenizerFast, i.e. the HF
 * `tokenizers` crate; installed version 0.22.2, reference pins transformers==4.16.2).
 *   1. added special tokens ([PAD] [UNK] [CLS] [SEP] [MASK], normalized=False) are cut out of
 *      the RAW text first, leftmost-longest;
 *   2. every other code point goes through the per-code-point table (tools/make_norm_tables.py):
 *      DROP (clean_text removal, stripped accents), SPACE (word break), ISO (its own word:
 *      punctuation, CJK), WORD (appended to the current word, possibly lowercased/expanded);
 *   3. WordPiece: words longer than 100 chars -> [UNK]; otherwise greedy longest-match with
 *      '##' continuation; any unmatched remainder makes the whole word [UNK];
 *   4. the sentence keeps its first max_pieces pieces (4.16.2 truncation=True, max_length=512).
 * ========================================================================================== */
typedef struct {
  uint64_t h;
  int32_t id, len, off;
  uint8_t cont;
} vent;

struct orc_tok {
  const uint8_t* table; /* header(20) | l1 u16[4352] | pages u32[n][256] | pool */
  const uint16_t* l1;
  const uint32_t* pages;
  const uint8_t* pool;
  char* vblob;
  int32_t vsize;
  int32_t* voff; /* piece i = vblob[voff[i] : voff[i+1]-1] */
  vent* slots;
  uint64_t mask;
  int32_t unk_id;
  int32_t special_id[5];
  const char* special_str[5];
};

static uint64_t fnv(uint8_t cont, const uint8_t* b, int len) {
  uint64_t h = 1469598103934665603ull ^ cont;
  for (int i = 0; i < len; i++) { h ^= b[i]; h *= 1099511628211ull; }
  return h ^ (h >> 29);
}

static int32_t vlookup(const orc_tok* t, uint8_t cont, const uint8_t* b, int len) {
  uint64_t h = fnv(cont, b, len);
  for (uint64_t i = h & t->mask;; i = (i + 1) & t->mask) {
    const vent* e = &t->slots[i];
    if (e->id < 0) return -1;
    if (e->h == h && e->len == len && e->cont == cont && !memcmp(t->vblob + e->off, b, len))
      return e->id;
  }
}

orc_tok* orc_tok_create(const uint8_t* table, int64_t table_len, const char* vocab,
                        int64_t vocab_len) {
  if (table_len < 20 || memcmp(table, "LDNT", 4)) return NULL;
  orc_tok* t = calloc(1, sizeof(orc_tok));
  uint32_t n_pages;
  memcpy(&n_pages, table + 12, 4);
  t->table = table;
  t->l1 = (const uint16_t*)(table + 20);
  t->pages = (const uint32_t*)(table + 20 + 2 * 4352);
  t->pool = table + 20 + 2 * 4352 + 4 * 256 * (int64_t)n_pages;
  t->vblob = malloc(vocab_len + 1);
  memcpy(t->vblob, vocab, vocab_len);
  t->vblob[vocab_len] = '\n';
  int32_t n = 0;
  for (int64_t i = 0; i < vocab_len; i++) n += vocab[i] == '\n';
  if (vocab_len && vocab[vocab_len - 1] != '\n') n++;
  t->vsize = n;
  t->voff = malloc(sizeof(int32_t) * (n + 1));
  int32_t k = 0;
  t->voff[0] = 0;
  for (int64_t i = 0; i < vocab_len + 1 && k < n; i++)
    if (t->vblob[i] == '\n') t->voff[++k] = (int32_t)i + 1;
  uint64_t cap = 1;
  while (cap < 2u * (uint64_t)n + 16) cap <<= 1;
  t->slots = malloc(sizeof(vent) * cap);
  for (uint64_t i = 0; i < cap; i++) t->slots[i].id = -1;
  t->mask = cap - 1;
  for (int32_t id = 0; id < n; id++) {
    const uint8_t* p = (const uint8_t*)t->vblob + t->voff[id];
    int len = t->voff[id + 1] - 1 - t->voff[id];
    if (len > 0 && p[len - 1] == '\r') len--;
    uint8_t cont = 0;
    if (len > 2 && p[0] == '#' && p[1] == '#') { cont = 1; p += 2; len -= 2; }
    uint64_t h = fnv(cont, p, len);
    int dup = 0; /* a duplicated line maps to its LAST id, like HF's vocab HashMap */
    for (uint64_t i = h & t->mask; t->slots[i].id >= 0; i = (i + 1) & t->mask) {
      vent* e = &t->slots[i];
      if (e->h == h && e->len == len && e->cont == cont &&
          !memcmp(t->vblob + e->off, p, len)) { e->id = id; dup = 1; break; }
    }
    if (dup) continue;
    uint64_t i = h & t->mask;
    while (t->slots[i].id >= 0) i = (i + 1) & t->mask;
    t->slots[i] = (vent){h, id, len, (int32_t)(p - (const uint8_t*)t->vblob), cont};
  }
  static const char* specials[5] = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"};
  for (int s = 0; s < 5; s++) {
    t->special_str[s] = specials[s];
    t->special_id[s] = vlookup(t, 0, (const uint8_t*)specials[s], (int)strlen(specials[s]));
  }
  t->unk_id = t->special_id[1];
  return t;
}

void orc_tok_destroy(orc_tok* t) {
  if (!t) return;
  free(t->vblob);
  free(t->voff);
  free(t->slots);
  free(t);
}

int32_t orc_tok_vocab_size(const orc_tok* t) { return t->vsize; }

int32_t orc_tok_token_id(const orc_tok* t, const char* s, int32_t len) {
  uint8_t cont = 0;
  if (len > 2 && s[0] == '#' && s[1] == '#') { cont = 1; s += 2; len -= 2; }
  return vlookup(t, cont, (const uint8_t*)s, len);
}

static uint32_t tab_entry(const orc_tok* t, uint32_t cp) {
  if (cp > 0x10FFFF) return 1u << 30; /* DROP */
  return t->pages[(uint32_t)t->l1[cp >> 8] * 256 + (cp & 255)];
}

/* Decode one UTF-8 code point; invalid sequences decode to U+FFFD (which the table drops). */
static uint32_t utf8_next(const uint8_t* b, int64_t n, int64_t* i) {
  uint8_t c = b[*i];
  if (c < 0x80) { (*i)++; return c; }
  int len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
  if (len == 1 || *i + len > n) { (*i)++; return 0xFFFD; }
  uint32_t cp = c & (0x7F >> len);
  for (int k = 1; k < len; k++) {
    if ((b[*i + k] & 0xC0) != 0x80) { (*i)++; return 0xFFFD; }
    cp = (cp << 6) | (b[*i + k] & 0x3F);
  }
  *i += len;
  return cp;
}

static int put_utf8(uint8_t* o, uint32_t cp) {
  if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
  if (cp < 0x800) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 63); return 2; }
  if (cp < 0x10000) {
    o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 63); o[2] = 0x80 | (cp & 63);
    return 3;
  }
  o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 63); o[2] = 0x80 | ((cp >> 6) & 63);
  o[3] = 0x80 | (cp & 63);
  return 4;
}

typedef struct {
  int32_t* ids;
  int64_t n, cap, limit;
} piece_sink;

static void emit(piece_sink* s, int32_t id) {
  if (s->n < s->limit && s->n < s->cap) s->ids[s->n] = id;
  s->n++;
}

/* WordPiece on one normalised word: bytes w[0..nb), char starts cs[0..nc] (cs[nc] = nb). */
static void wordpiece(const orc_tok* t, const uint8_t* w, int nb, const int* cs, int nc,
                      piece_sink* out) {
  if (nc == 0) return;
  if (nc > 100) { emit(out, t->unk_id); return; }
  int32_t tmp[128];
  int np = 0, start = 0;
  while (start < nc) {
    int found = -1, end;
    for (end = nc; end > start; end--) {
      int32_t id = vlookup(t, start > 0, w + cs[start], cs[end] - cs[start]);
      if (id >= 0) { found = id; break; }
    }
    if (found < 0) { emit(out, t->unk_id); return; }
    tmp[np++] = found;
    start = end;
  }
  for (int i = 0; i < np; i++) emit(out, tmp[i]);
}

static void tokenize_one(const orc_tok* t, const uint8_t* b, int64_t n, piece_sink* out) {
  uint8_t word[512];
  int cs[520];
  int nb = 0, nc = 0, overflow = 0;
#define FLUSH()                                                         \
  do {                                                                  \
    if (nc) {                                                           \
      cs[overflow ? 0 : nc] = nb;                                       \
      if (overflow) emit(out, t->unk_id); else wordpiece(t, word, nb, cs, nc, out); \
    }                                                                   \
    nb = nc = overflow = 0;                                             \
  } while (0)
  int64_t i = 0;
  while (i < n) {
    if (b[i] == '[') { /* raw special-token match (leftmost, longest) */
      int best = -1, blen = 0;
      for (int s = 0; s < 5; s++) {
        int L = (int)strlen(t->special_str[s]);
        if (t->special_id[s] >= 0 && i + L <= n && L > blen &&
            !memcmp(b + i, t->special_str[s], L)) { best = s; blen = L; }
      }
      if (best >= 0) {
        FLUSH();
        emit(out, t->special_id[best]);
        i += blen;
        continue;
      }
    }
    uint32_t cp = utf8_next(b, n, &i);
    uint32_t e = tab_entry(t, cp);
    uint32_t cls = e >> 30;
    if (cls == 1) continue;           /* DROP */
    if (cls == 2) { FLUSH(); continue; } /* SPACE */
    /* output chars of this code point */
    uint8_t ob[16];
    int olen = 0, ochars = 1;
    if (e & (1u << 29)) olen = put_utf8(ob, cp);
    else if (e & (1u << 28)) {
      const uint8_t* p = t->pool + (e & 0xFFFFFF);
      olen = p[0];
      ochars = p[1];
      memcpy(ob, p + 2, olen);
    } else olen = put_utf8(ob, e & 0x1FFFFF);
    if (cls == 3) { /* ISO: its own word */
      FLUSH();
      memcpy(word, ob, olen);
      nb = olen;
      cs[0] = 0;
      nc = 1;
      FLUSH();
      continue;
    }
    /* WORD: append chars (bounded buffer; >100 chars is [UNK] anyway) */
    if (nc + ochars > 100 || nb + olen > 400) { overflow = 1; nc += ochars; continue; }
    if (overflow) { nc += ochars; continue; }
    int k = 0;
    for (int c = 0; c < ochars; c++) {
      cs[nc++] = nb + k;
      uint8_t lead = ob[k];
      k += lead < 0x80 ? 1 : lead >= 0xF0 ? 4 : lead >= 0xE0 ? 3 : 2;
    }
    memcpy(word + nb, ob, olen);
    nb += olen;
  }
  FLUSH();
#undef FLUSH
}

int64_t orc_tokenize(const orc_tok* t, const uint8_t* text, const int64_t* sent_off,
                     int64_t n_sent, int32_t max_pieces, int32_t* ids, int64_t ids_cap,
                     int64_t* out_off) {
  int64_t total = 0;
  out_off[0] = 0;
  for (int64_t s = 0; s < n_sent; s++) {
    piece_sink sink = {ids + total, 0, ids_cap - total, max_pieces};
    tokenize_one(t, text + sent_off[s], sent_off[s + 1] - sent_off[s], &sink);
    int64_t k = sink.n < max_pieces ? sink.n : max_pieces;
    if (total + k > ids_cap) return -1;
    total += k;
    out_off[s + 1] = total;
  }
  return total;
}

/* ============================================================================================
 * Pairs + static masking (lddl/dask/bert/pretrain.py).
 * ========================================================================================== */
typedef struct {
  int32_t* v;
  int64_t n, cap;
} ivec;

static void iv_push(ivec* a, int32_t x) {
  if (a->n == a->cap) {
    a->cap = a->cap ? 2 * a->cap : 256;
    a->v = realloc(a->v, sizeof(int32_t) * a->cap);
  }
  a->v[a->n++] = x;
}

typedef struct {
  int64_t tok_begin; /* into the scratch token store */
  int32_t na, nb, rn, npos;
  int64_t pos_begin;
} pair_rec;

typedef struct {
  pair_rec* r;
  int64_t n, cap;
} pvec;

/* _truncate_seq_pair (pretrain.py:161-176) on [a0,a1) and [b0,b1) views. */
static void truncate_pair(orc_mt* rng, int64_t* a0, int64_t* a1, int64_t* b0, int64_t* b1,
                          int32_t max_num) {
  for (;;) {
    int64_t la = *a1 - *a0, lb = *b1 - *b0;
    if (la + lb <= max_num) break;
    int64_t *lo, *hi;
    if (la > lb) { lo = a0; hi = a1; } else { lo = b0; hi = b1; }
    if (orc_mt_random(rng) < 0.5) (*lo)++;
    else (*hi)--;
  }
}

int64_t orc_partition_pairs(const orc_pair_params* P, int64_t seed, const int64_t* doc_sent,
                            int64_t n_docs, const int64_t* tok_off, const int32_t* ids,
                            int32_t* out_tok, int64_t tok_cap, int64_t* out_tok_off,
                            int32_t* len_a, uint8_t* is_rn, int64_t pair_cap, uint16_t* out_pos,
                            int32_t* out_lab, int64_t pos_cap, int64_t* out_pos_off) {
  orc_mt rng;
  orc_mt_seed_i64(&rng, seed);
  const int32_t max_num = P->seq - 3;
  ivec store = {0}, pstore = {0}, lstore = {0}, A = {0}, B = {0}, cand = {0}, seqv = {0};
  pvec pairs = {0};
  int64_t status = 0;
  for (int d_ = 0; d_ < P->dup; d_++) {
    for (int64_t d = 0; d < n_docs; d++) {
      /* create_pairs_from_document (pretrain.py:241-365) */
      const int64_t s0 = doc_sent[d], ns = doc_sent[d + 1] - doc_sent[d];
      int32_t target = max_num;
      if (orc_mt_random(&rng) < P->short_seq_prob) target = (int32_t)orc_mt_randint(&rng, 2, max_num);
      int64_t chunk0 = 0, chunk_n = 0, cur_len = 0;
      for (int64_t i = 0; i < ns; i++) {
        if (chunk_n == 0) chunk0 = i;
        chunk_n++;
        cur_len += tok_off[s0 + i + 1] - tok_off[s0 + i];
        if (!(i == ns - 1 || cur_len >= target)) continue;
        int64_t a_end = 1;
        if (chunk_n >= 2) a_end = orc_mt_randint(&rng, 1, chunk_n - 1);
        A.n = B.n = 0;
        for (int64_t j = chunk0; j < chunk0 + a_end; j++)
          for (int64_t k = tok_off[s0 + j]; k < tok_off[s0 + j + 1]; k++) iv_push(&A, ids[k]);
        int rn = 0;
        if (chunk_n == 1 || orc_mt_random(&rng) < 0.5) {
          rn = 1;
          int64_t target_b = target - A.n;
          int64_t rd = 0;
          for (int t = 0; t < 10; t++) {
            rd = orc_mt_randint(&rng, 0, n_docs - 1);
            if (rd != d) break;
          }
          if (rd == d) rn = 0;
          const int64_t r0 = doc_sent[rd], rns = doc_sent[rd + 1] - doc_sent[rd];
          int64_t rstart = orc_mt_randint(&rng, 0, rns - 1);
          for (int64_t j = rstart; j < rns; j++) {
            for (int64_t k = tok_off[r0 + j]; k < tok_off[r0 + j + 1]; k++) iv_push(&B, ids[k]);
            if (B.n >= target_b) break;
          }
          i -= chunk_n - a_end; /* put back unused segments */
        } else {
          for (int64_t j = chunk0 + a_end; j < chunk0 + chunk_n; j++)
            for (int64_t k = tok_off[s0 + j]; k < tok_off[s0 + j + 1]; k++) iv_push(&B, ids[k]);
        }
        int64_t a0 = 0, a1 = A.n, b0 = 0, b1 = B.n;
        truncate_pair(&rng, &a0, &a1, &b0, &b1, max_num);
        pair_rec rec = {store.n, (int32_t)(a1 - a0), (int32_t)(b1 - b0), rn, 0, pstore.n};
        /* tokens = [CLS] A [SEP] B [SEP] */
        seqv.n = 0;
        iv_push(&seqv, P->cls_id);
        for (int64_t k = a0; k < a1; k++) iv_push(&seqv, A.v[k]);
        iv_push(&seqv, P->sep_id);
        for (int64_t k = b0; k < b1; k++) iv_push(&seqv, B.v[k]);
        iv_push(&seqv, P->sep_id);
        if (P->masking) {
          /* create_masked_lm_predictions (pretrain.py:182-238) */
          cand.n = 0;
          for (int64_t k = 0; k < seqv.n; k++)
            if (seqv.v[k] != P->cls_id && seqv.v[k] != P->sep_id) iv_push(&cand, (int32_t)k);
          orc_mt_shuffle_i32(&rng, cand.v, cand.n);
          int64_t num = (int64_t)nearbyint((double)seqv.n * P->masked_lm_ratio);
          if (num < 1) num = 1;
          int32_t* orig = malloc(sizeof(int32_t) * seqv.n);
          memcpy(orig, seqv.v, sizeof(int32_t) * seqv.n);
          int64_t nm = 0;
          int32_t* mpos = malloc(sizeof(int32_t) * (cand.n + 1));
          for (int64_t c = 0; c < cand.n && nm < num; c++) {
            int32_t idx = cand.v[c];
            int32_t tokv;
            if (orc_mt_random(&rng) < 0.8) tokv = P->mask_id;
            else if (orc_mt_random(&rng) < 0.5) tokv = orig[idx];
            else tokv = (int32_t)orc_mt_randint(&rng, 0, P->vocab_size - 1);
            seqv.v[idx] = tokv;
            mpos[nm++] = idx;
          }
          /* sort positions ascending (insertion sort: nm is small) */
          for (int64_t x = 1; x < nm; x++) {
            int32_t v = mpos[x];
            int64_t y = x - 1;
            while (y >= 0 && mpos[y] > v) { mpos[y + 1] = mpos[y]; y--; }
            mpos[y + 1] = v;
          }
          for (int64_t x = 0; x < nm; x++) {
            iv_push(&pstore, mpos[x]);
            iv_push(&lstore, orig[mpos[x]]);
          }
          rec.npos = (int32_t)nm;
          free(orig);
          free(mpos);
        }
        for (int64_t k = 1; k < 1 + rec.na; k++) iv_push(&store, seqv.v[k]);
        for (int64_t k = 2 + rec.na; k < 2 + rec.na + rec.nb; k++) iv_push(&store, seqv.v[k]);
        if (pairs.n == pairs.cap) {
          pairs.cap = pairs.cap ? 2 * pairs.cap : 256;
          pairs.r = realloc(pairs.r, sizeof(pair_rec) * pairs.cap);
        }
        pairs.r[pairs.n++] = rec;
        chunk_n = 0;
        cur_len = 0;
      }
    }
  }
  /* random.shuffle(partition_pairs) (pretrain.py:401) */
  int32_t* perm = malloc(sizeof(int32_t) * (pairs.n + 1));
  for (int64_t k = 0; k < pairs.n; k++) perm[k] = (int32_t)k;
  orc_mt_shuffle_i32(&rng, perm, pairs.n);
  if (pairs.n > pair_cap || store.n > tok_cap || pstore.n > pos_cap) {
    status = -1;
  } else {
    int64_t to = 0, po = 0;
    out_tok_off[0] = 0;
    if (out_pos_off) out_pos_off[0] = 0;
    for (int64_t k = 0; k < pairs.n; k++) {
      const pair_rec* r = &pairs.r[perm[k]];
      memcpy(out_tok + to, store.v + r->tok_begin, sizeof(int32_t) * (r->na + r->nb));
      to += r->na + r->nb;
      out_tok_off[k + 1] = to;
      len_a[k] = r->na;
      is_rn[k] = (uint8_t)r->rn;
      if (P->masking) {
        for (int32_t x = 0; x < r->npos; x++) {
          out_pos[po + x] = (uint16_t)pstore.v[r->pos_begin + x];
          out_lab[po + x] = lstore.v[r->pos_begin + x];
        }
        po += r->npos;
        out_pos_off[k + 1] = po;
      }
    }
    status = pairs.n;
  }
  free(perm);
  free(store.v); free(pstore.v); free(lstore.v); free(A.v); free(B.v); free(cand.v);
  free(seqv.v); free(pairs.r);
  return status;
}

/* ============================================================================================
 * Binning (lddl/dask/bert/binning.py:63-93): bin = (num_tokens-1)//bin_size clamped to nbins-1;
 * rows regrouped by bin, stable within a bin.
 * ========================================================================================== */
void orc_bin(const int32_t* num_tokens, int64_t n, int32_t bin_size, int32_t nbins,
             int32_t* bin_id, int64_t* order, int64_t* bin_counts) {
  for (int32_t b = 0; b < nbins; b++) bin_counts[b] = 0;
  for (int64_t i = 0; i < n; i++) {
    int32_t b = (num_tokens[i] - 1) / bin_size;
    if (b > nbins - 1) b = nbins - 1;
    bin_id[i] = b;
    bin_counts[b]++;
  }
  int64_t* start = malloc(sizeof(int64_t) * (nbins + 1));
  start[0] = 0;
  for (int32_t b = 0; b < nbins; b++) start[b + 1] = start[b] + bin_counts[b];
  for (int64_t i = 0; i < n; i++) order[start[bin_id[i]]++] = i;
  free(start);
}

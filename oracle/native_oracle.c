/*
 * native_oracle — CPU restatement of the native-RNG pair path (rng='native', LDDL_RNG_NATIVE).
 * TEST INFRASTRUCTURE ONLY: used by tests/ to check lddl_amd's native planner, masking and
 * partition order bit for bit; never by the product.
 *
 * The algorithm is the reference's (create_pairs_from_document, lddl/dask/bert/pretrain.py:241-365;
 * _truncate_seq_pair 161-176; create_masked_lm_predictions 182-238; the partition shuffle 401),
 * drawing from Philox4x32-10 counter streams instead of one MT19937 per partition (the reference
 * seeds nothing), as lddl_amd/csrc/pairs.hip defines them:
 *   walk of unit r = (duplicate dp, document dl), r = dp * nd + dl: stream (key, r, 1);
 *   masks of the k-th pair the planner made in the partition: sampling (key, k, 2), decisions
 *   (key, k, 4); partition order: a 4-round Feistel permutation keyed by mix64(key ^ 3);
 *   key = mix64(native_seed ^ mix64(part_seed + golden)).
 * Sentences with no tokens are dropped, then documents with no sentences (pretrain.py:89-97).
 */
#include "lddl_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static uint64_t mix64(uint64_t x) { /* splitmix64 finaliser */
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* Philox4x32-10 (Salmon et al., SC'11) */
static void philox(const uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
  uint32_t k0, k1, id0, id1, blk, buf[4];
  int have;
} ctr_rng;

static void rng_init(ctr_rng* g, uint64_t key, int64_t index, uint32_t stream) {
  g->k0 = (uint32_t)key;
  g->k1 = (uint32_t)(key >> 32);
  g->id0 = (uint32_t)index;
  g->id1 = ((uint32_t)((uint64_t)index >> 32) << 4) | stream;
  g->blk = 0;
  g->have = 0;
}

static uint32_t u32(ctr_rng* g) {
  if (g->have == 0) {
    const uint32_t c[4] = {g->blk++, g->id0, g->id1, 0x6C64646Cu};
    philox(c, g->k0, g->k1, g->buf);
    g->have = 4;
  }
  g->have--;
  return g->buf[3 - g->have];
}

static uint64_t rand53(ctr_rng* g) { /* the 53-bit integer behind random() */
  const uint32_t a = u32(g) >> 5, b = u32(g) >> 6;
  return ((uint64_t)a << 26) | b;
}

static int bitlen(uint32_t n) { int k = 0; while (n) { k++; n >>= 1; } return k; }

static uint32_t randbelow(ctr_rng* g, uint32_t n) { /* _randbelow: k-bit draws until < n */
  const int k = bitlen(n);
  uint32_t r = u32(g) >> (32 - k);
  while (r >= n) r = u32(g) >> (32 - k);
  return r;
}

static int64_t randint(ctr_rng* g, int64_t a, int64_t b) { return a + randbelow(g, (uint32_t)(b - a + 1)); }

static int popc(uint32_t x) { int c = 0; while (x) { x &= x - 1; c++; } return c; }

static int32_t heads(ctr_rng* g, int32_t n) { /* heads among n fair coins, 32 per draw */
  int32_t h = 0;
  for (; n >= 32; n -= 32) h += popc(u32(g));
  if (n > 0) h += popc(u32(g) & ((1u << n) - 1u));
  return h;
}

static uint32_t lemire_below(uint32_t x, uint32_t n, ctr_rng* g) { /* uniform in [0, n) */
  uint64_t m = (uint64_t)x * n;
  if ((uint32_t)m < n) {
    const uint32_t t = (0u - n) % n;
    while ((uint32_t)m < t) m = (uint64_t)u32(g) * n;
  }
  return (uint32_t)(m >> 32);
}

/* token o of the run of kept tokens that starts at kept sentence k0 (kept sentences of one
 * document are consecutive, so the run may continue into the next kept sentences) */
static int32_t win_token(const int64_t* ks, const int64_t* pre, const int64_t* tok_off,
                         const int32_t* ids, int64_t k0, int64_t o) {
  const int64_t x = pre[k0] + o;
  int64_t k = k0;
  while (pre[k + 1] <= x) k++;
  return ids[tok_off[ks[k]] + (x - pre[k])];
}

enum { kWalk = 1, kMask = 2, kOrder = 3, kDecide = 4 };
static const uint32_t kNat80 = 3435973837u, kNat90 = 3865470567u; /* ceil(0.8 / 0.9 * 2^32) */

typedef struct {
  int64_t a_ks, b_ks; /* first kept sentence of A / B */
  int32_t a_front, na, b_front, nb, rn;
} npair;

int64_t orc_partition_pairs_native(const orc_pair_params* P, uint64_t native_seed, int64_t part_seed,
                                   const int64_t* doc_sent, int64_t n_docs, const int64_t* tok_off,
                                   const int32_t* ids, int32_t* out_tok, int64_t tok_cap,
                                   int64_t* out_tok_off, int32_t* len_a, uint8_t* is_rn,
                                   int64_t pair_cap, uint16_t* out_pos, int32_t* out_lab,
                                   int64_t pos_cap, int64_t* out_pos_off) {
  /* kept sentences (>= 1 token) and kept documents (>= 1 kept sentence) */
  const int64_t n_sent_all = doc_sent[n_docs] - doc_sent[0];
  int64_t* ks = malloc(sizeof(int64_t) * (n_sent_all + 1)); /* kept sentence -> sentence */
  int64_t* kdoc = malloc(sizeof(int64_t) * (n_docs + 1));   /* kept doc -> first kept sentence */
  int64_t nks = 0, nd = 0;
  for (int64_t d = 0; d < n_docs; d++) {
    const int64_t k0 = nks;
    for (int64_t s = doc_sent[d]; s < doc_sent[d + 1]; s++)
      if (tok_off[s + 1] > tok_off[s]) ks[nks++] = s;
    if (nks > k0) kdoc[nd++] = k0;
  }
  kdoc[nd] = nks;
  int64_t* pre = malloc(sizeof(int64_t) * (nks + 1)); /* cumulative kept lengths */
  pre[0] = 0;
  for (int64_t k = 0; k < nks; k++) pre[k + 1] = pre[k] + (tok_off[ks[k] + 1] - tok_off[ks[k]]);
  /* the token t of the window starting at kept sentence k0, offset `front` */
  #define WIN_TOKEN(k0, front, t) win_token(ks, pre, tok_off, ids, (k0), (int64_t)(front) + (t))
  const uint64_t key = mix64(native_seed ^ mix64((uint64_t)part_seed + 0x9E3779B97F4A7C15ull));
  const int32_t max_num = P->seq - 3;
  uint64_t k_short = 0;
  if (P->short_seq_prob >= 1) k_short = 1ull << 53;
  else if (P->short_seq_prob > 0) k_short = (uint64_t)ceil(ldexp(P->short_seq_prob, 53));
  int64_t cap = 16, n = 0;
  npair* pairs = malloc(sizeof(npair) * cap);
  for (int64_t r = 0; r < (int64_t)P->dup * nd; r++) {
    /* create_pairs_from_document (pretrain.py:241-365) on document dl */
    const int64_t dl = r % nd;
    ctr_rng g;
    rng_init(&g, key, r, kWalk);
    const int64_t s0 = kdoc[dl], ns = kdoc[dl + 1] - s0;
    int32_t target = max_num;
    if (rand53(&g) < k_short) target = (int32_t)randint(&g, 2, max_num);
    int64_t chunk0 = 0, chunk_n = 0, cur = 0;
    for (int64_t i = 0; i < ns; i++) {
      if (chunk_n == 0) chunk0 = i;
      chunk_n++;
      cur += pre[s0 + i + 1] - pre[s0 + i];
      if (!(i == ns - 1 || cur >= target)) continue;
      const int64_t a_end = chunk_n >= 2 ? randint(&g, 1, chunk_n - 1) : 1;
      const int64_t la = pre[s0 + chunk0 + a_end] - pre[s0 + chunk0];
      int64_t lb = 0, b_ks;
      int rn = 0;
      if (chunk_n == 1 || u32(&g) < 0x80000000u) {
        rn = 1;
        const int64_t target_b = target - la;
        int64_t rd = 0;
        for (int t = 0; t < 10; t++) {
          rd = randint(&g, 0, nd - 1);
          if (rd != dl) break;
        }
        if (rd == dl) rn = 0;
        const int64_t r0 = kdoc[rd], rns = kdoc[rd + 1] - r0;
        const int64_t rstart = randint(&g, 0, rns - 1);
        b_ks = r0 + rstart;
        for (int64_t j = rstart; j < rns; j++) {
          lb += pre[r0 + j + 1] - pre[r0 + j];
          if (lb >= target_b) break;
        }
        i -= chunk_n - a_end; /* put back the unused segments (pretrain.py:320-321) */
      } else {
        b_ks = s0 + chunk0 + a_end;
        lb = pre[s0 + chunk0 + chunk_n] - pre[s0 + chunk0 + a_end];
      }
      /* _truncate_seq_pair: each trim removes from the longer side (A on ties -> B: la > lb
       * picks A); front or back is a fair coin, so only the number of front trims matters */
      int32_t na = (int32_t)la, nb = (int32_t)lb, af = 0, bf = 0;
      const int32_t T = na + nb - max_num;
      if (T > 0) {
        const int32_t dd = na - nb, ad = dd < 0 ? -dd : dd;
        const int32_t nA = (dd > 0 ? (dd < T ? dd : T) : 0) + (T > ad ? (T - ad) / 2 : 0);
        af = heads(&g, nA);
        bf = heads(&g, T - nA);
        na -= nA;
        nb -= T - nA;
      }
      if (n == cap) {
        cap *= 2;
        pairs = realloc(pairs, sizeof(npair) * cap);
      }
      pairs[n++] = (npair){s0 + chunk0, b_ks, af, na, bf, nb, rn};
      chunk_n = 0;
      cur = 0;
    }
  }
  /* partition order: output row q takes pair perm(q) (Feistel on [0, 4^h) restricted to [0, n)) */
  const uint64_t okey = mix64(key ^ kOrder);
  int bits = 1;
  while ((1ll << bits) < n) bits++;
  const int h = (bits + 1) >> 1;
  const uint64_t hm = (1ull << h) - 1;
  int64_t status = n, to = 0, po = 0;
  out_tok_off[0] = 0;
  if (out_pos_off) out_pos_off[0] = 0;
  int32_t* tok = malloc(sizeof(int32_t) * (P->seq + 4));
  int32_t* orig = malloc(sizeof(int32_t) * (P->seq + 4));
  int32_t* cand = malloc(sizeof(int32_t) * (P->seq + 4));
  uint8_t* picked = malloc((size_t)P->seq + 4);
  for (int64_t q = 0; q < n && status >= 0; q++) {
    uint64_t x = (uint64_t)q;
    do {
      uint64_t L = x >> h, R = x & hm;
      for (uint64_t rd = 0; rd < 4; rd++) {
        const uint64_t f = mix64(R ^ okey ^ (rd << 56)) & hm;
        const uint64_t nl = R;
        R = L ^ f;
        L = nl;
      }
      x = (L << h) | R;
    } while (x >= (uint64_t)n);
    const npair* pr = &pairs[x];
    const int32_t nt = pr->na + pr->nb;
    if (to + nt > tok_cap || q >= pair_cap) { status = -1; break; }
    for (int32_t t = 0; t < nt; t++)
      tok[t] = t < pr->na ? WIN_TOKEN(pr->a_ks, pr->a_front, t) : WIN_TOKEN(pr->b_ks, pr->b_front, t - pr->na);
    memcpy(orig, tok, sizeof(int32_t) * nt);
    int32_t nm = 0;
    if (P->masking) {
      /* candidates: tokens that are not a literal [CLS]/[SEP] (pretrain.py:190-195) */
      int32_t nc = 0;
      for (int32_t t = 0; t < nt; t++)
        if (tok[t] != P->cls_id && tok[t] != P->sep_id) cand[nc++] = t;
      int32_t num = (int32_t)nearbyint((double)(nt + 3) * P->masked_lm_ratio);
      if (num < 1) num = 1;
      if (num > nc) num = nc;
      /* a uniform num-subset of the candidates (Floyd), then in index order with 80/10/10 */
      ctr_rng gs, gd;
      rng_init(&gs, key, (int64_t)x, kMask);
      rng_init(&gd, key, (int64_t)x, kDecide);
      memset(picked, 0, (size_t)nc);
      for (int32_t s = 0; s < num; s++) {
        const uint32_t j = (uint32_t)(nc - num + s);
        const uint32_t t = lemire_below(u32(&gs), j + 1u, &gs);
        picked[picked[t] ? j : t] = 1;
      }
      if (po + num > pos_cap) { status = -1; break; }
      for (int32_t c = 0; c < nc; c++) {
        if (!picked[c]) continue;
        const uint32_t xd = u32(&gd), yd = u32(&gd);
        const int32_t t = cand[c];
        const int32_t pos = t < pr->na ? t + 1 : t + 2;
        int32_t rep = xd < kNat80 ? P->mask_id : xd < kNat90 ? orig[t]
                                                : (int32_t)lemire_below(yd, (uint32_t)P->vocab_size, &gd);
        out_pos[po + nm] = (uint16_t)pos;
        out_lab[po + nm] = orig[t];
        tok[t] = rep;
        nm++;
      }
      po += nm;
      out_pos_off[q + 1] = po;
    }
    memcpy(out_tok + to, tok, sizeof(int32_t) * nt);
    to += nt;
    out_tok_off[q + 1] = to;
    len_a[q] = pr->na;
    is_rn[q] = (uint8_t)pr->rn;
  }
  free(tok); free(orig); free(cand); free(picked);
  free(pairs); free(ks); free(kdoc); free(pre);
  return status;
}

/*
 * lddl_oracle — CPU restatement of the reference's BERT preprocessing hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / the CPU baseline. The product path
 * (lddl_amd/_lib/liblddl_amd.so) never links or calls it.
 *
 * Parity anchor: pinned by the reference-generated fixtures in tests/golden/ (see
 * tests/golden/make_goldens.py) and checked against them by tests/test_oracle.py.
 */
#ifndef LDDL_ORACLE_H_
#define LDDL_ORACLE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CPython `random` (Modules/_randommodule.c + Lib/random.py, Python 3.10). */
typedef struct {
  uint32_t mt[624];
  int mti;
} orc_mt;
void orc_mt_seed_key(orc_mt* s, const uint32_t* key, int key_len);   /* random.seed(int) */
void orc_mt_seed_i64(orc_mt* s, int64_t seed);
uint32_t orc_mt_u32(orc_mt* s);                                       /* getrandbits(32) */
double orc_mt_random(orc_mt* s);                                      /* random() */
uint32_t orc_mt_randbelow(orc_mt* s, uint32_t n);                     /* _randbelow(n), n>=1 */
int64_t orc_mt_randint(orc_mt* s, int64_t a, int64_t b);              /* randint(a, b) */
void orc_mt_shuffle_i32(orc_mt* s, int32_t* x, int64_t n);            /* shuffle(x) */
void orc_mt_get_state(const orc_mt* s, uint32_t* state625);

/* Tokenizer: BertNormalizer + BertPreTokenizer + WordPiece over a per-code-point table
 * (lddl_amd/assets/bert_norm_*.bin) and a vocab.txt blob. */
typedef struct orc_tok orc_tok;
orc_tok* orc_tok_create(const uint8_t* table, int64_t table_len, const char* vocab,
                        int64_t vocab_len);
void orc_tok_destroy(orc_tok* t);
int32_t orc_tok_vocab_size(const orc_tok* t);
int32_t orc_tok_token_id(const orc_tok* t, const char* s, int32_t len); /* -1 if absent */
/* Tokenize n_sent sentences text[sent_off[i]:sent_off[i+1]], each truncated to max_pieces.
 * ids/out_off as ragged output. Returns total pieces or -1 if ids_cap is too small. */
int64_t orc_tokenize(const orc_tok* t, const uint8_t* text, const int64_t* sent_off,
                     int64_t n_sent, int32_t max_pieces, int32_t* ids, int64_t ids_cap,
                     int64_t* out_off);

/* NSP pair construction + optional static masking for ONE partition, seeded with
 * random.seed(seed) (pretrain.py:386-402 / 241-365 / 161-176 / 182-238).
 * Documents: doc d has sentences [doc_sent[d], doc_sent[d+1]); sentence s has token ids
 * ids[tok_off[s]:tok_off[s+1]].
 * Output (after the final partition shuffle), pair p: post-mask tokens
 * out_tok[out_tok_off[p] : out_tok_off[p] + len_a[p]] = A, then B up to out_tok_off[p+1];
 * is_rn[p]; num_tokens = (out_tok_off[p+1]-out_tok_off[p]) + 3; masked positions / labels
 * ragged by out_pos_off. Returns number of pairs, or -1 on capacity overflow. */
typedef struct {
  int32_t dup, seq, masking, vocab_size, cls_id, sep_id, mask_id;
  double short_seq_prob, masked_lm_ratio;
} orc_pair_params;
int64_t orc_partition_pairs(const orc_pair_params* p, int64_t seed, const int64_t* doc_sent,
                            int64_t n_docs, const int64_t* tok_off, const int32_t* ids,
                            int32_t* out_tok, int64_t tok_cap, int64_t* out_tok_off,
                            int32_t* len_a, uint8_t* is_rn, int64_t pair_cap, uint16_t* out_pos,
                            int32_t* out_lab, int64_t pos_cap, int64_t* out_pos_off);

/* The same partition through lddl_amd's native-RNG mode (oracle/native_oracle.c): the reference's
 * algorithm drawing from Philox4x32-10 streams keyed by (native_seed, part_seed); outputs as
 * orc_partition_pairs. */
int64_t orc_partition_pairs_native(const orc_pair_params* p, uint64_t native_seed, int64_t part_seed,
                                   const int64_t* doc_sent, int64_t n_docs, const int64_t* tok_off,
                                   const int32_t* ids, int32_t* out_tok, int64_t tok_cap,
                                   int64_t* out_tok_off, int32_t* len_a, uint8_t* is_rn,
                                   int64_t pair_cap, uint16_t* out_pos, int32_t* out_lab,
                                   int64_t pos_cap, int64_t* out_pos_off);

/* Binning (binning.py:63-93): bin id per sample and the stable by-bin row order. */
/* nltk Punkt sentence spans (PunktSentenceTokenizer.span_tokenize), oracle/punkt_oracle.c.
 * table = lddl_amd/assets/punkt_props.bin; params = records (u8 kind 1 abbrev / 2 sentence
 * starter / 3 ortho context / 4 collocation, u8 value, u16 len_a, u16 len_b, bytes a, bytes b).
 * Spans are byte offsets relative to each document. */
typedef struct orc_punkt orc_punkt;
orc_punkt* orc_punkt_create(const uint8_t* table, int64_t table_bytes, const uint8_t* params,
                            int64_t params_bytes);
void orc_punkt_destroy(orc_punkt* o);
int64_t orc_punkt_spans(orc_punkt* o, const uint8_t* text, const int64_t* doc_off, int64_t n_doc,
                        int64_t* span_start, int64_t* span_end, int64_t* doc_count);

void orc_bin(const int32_t* num_tokens, int64_t n, int32_t bin_size, int32_t nbins,
             int32_t* bin_id, int64_t* order, int64_t* bin_counts);

#ifdef __cplusplus
}
#endif
#endif

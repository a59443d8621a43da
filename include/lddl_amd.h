/*
 * lddl_amd — C ABI of the MI355X-native BERT preprocessing hot path.
 *
 * The reference (wdykas/LDDL) is pure Python; its hot path calls into the HF `tokenizers` Rust
 * extension, `random`, numpy and CPU torch from Python. Each entry point below replaces one of
 * those call sites and is bound from Python with ctypes (INTEGRATION.md shows the stubs).
 *
 * Conventions
 *   - Plain C types only. `d_*` arguments are DEVICE pointers (HBM, e.g. torch.cuda tensors'
 *     data_ptr()), `h_*` arguments are host pointers. `stream` is a hipStream_t passed as void*
 *     (NULL = the legacy default stream). All device work is asynchronous on `stream`
 *     unless the function says otherwise.
 *   - Return value: 0 on success, negative on error; lddl_last_error() returns a thread-local
 *     message for the last failing call.
 *   - One lddl_ctx per device; a ctx may be shared by host threads only with external locking.
 *     Never create a ctx before fork() in a process whose children touch the GPU.
 */
#ifndef LDDL_AMD_H_
#define LDDL_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lddl_ctx lddl_ctx;

/* ---------------------------------------------------------------------------------------------
 * Errors / version
 * ------------------------------------------------------------------------------------------- */
const char* lddl_last_error(void);
int lddl_version(void);

/* ---------------------------------------------------------------------------------------------
 * Synthetic corpus; host-only, no GPU needed.
 * Generates documents [doc_begin, ...) of the deterministic corpus until >= target_bytes of
 * sentence text. Output: concatenated sentence bytes, sent_off[n_sent+1] (byte offsets),
 * doc_sent_off[n_doc+1] (sentence offsets). Returns the number of text bytes (<0 on overflow).
 * ------------------------------------------------------------------------------------------- */
int64_t lddl_synth_corpus(uint64_t seed, int64_t doc_begin, int64_t target_bytes,
                          double nonascii_frac, uint8_t* text, int64_t text_cap,
                          int64_t* sent_off, int64_t sent_cap, int64_t* doc_sent_off,
                          int64_t doc_cap, int64_t* n_sent_out, int64_t* n_doc_out,
                          int n_threads);

/* ---------------------------------------------------------------------------------------------
 * Context = device-resident tokenizer tables.
 * Replaces `transformers.BertTokenizerFast(vocab_file)` (lddl/dask/bert/pretrain.py:584-587,
 * lddl/torch/bert.py:343-346). `norm_table` is lddl_amd/assets/bert_norm_{uncased,cased}.bin
 * (lowercase=True is the reference default); `vocab` is the raw vocab.txt bytes,
 * token id = line number. special_ids order: [PAD] [UNK] [CLS] [SEP] [MASK] (-1 if absent).
 * ------------------------------------------------------------------------------------------- */
int lddl_ctx_create(int device, const uint8_t* norm_table, int64_t table_len, const char* vocab,
                    int64_t vocab_len, lddl_ctx** out);
int lddl_ctx_destroy(lddl_ctx* ctx);
int lddl_ctx_info(const lddl_ctx* ctx, int32_t* vocab_size, int32_t* special_ids,
                  int32_t* max_piece_bytes);
/* device pointers to the vocab strings (for rendering ' '.join(tokens)): token i is
 * bytes[off[i] .. off[i+1]) */
int lddl_ctx_render_table(const lddl_ctx* ctx, const uint8_t** d_bytes, const int64_t** d_off);

/* ---------------------------------------------------------------------------------------------
 * Tokenize sentences (device in, device out).
 * Replaces `tokenizer.tokenize(s, max_length=512, truncation=True)` per Punkt sentence
 * (lddl/dask/bert/pretrain.py:79-80, 89-92).
 *   d_text[n_bytes], d_sent_off[n_sent+1] (int64 byte offsets; sentence s = text[off[s]:off[s+1]])
 *   -> d_ids[n_bytes] (int32): sentence s's pieces at d_ids[off[s] ...] (pieces <= bytes)
 *   -> d_sent_len[n_sent] (int32): kept piece count (<= max_pieces) | 1<<30 if they contain a
 *      literal [CLS]/[SEP]. A count of 0 means the sentence is dropped (pretrain.py:92).
 * ------------------------------------------------------------------------------------------- */
int lddl_tokenize(lddl_ctx* ctx, void* stream, const uint8_t* d_text, int64_t n_bytes,
                  const int64_t* d_sent_off, int64_t n_sent, int32_t max_pieces, int32_t* d_ids,
                  int32_t* d_sent_len);

#ifdef __cplusplus
}
#endif

#endif /* LDDL_AMD_H_ */

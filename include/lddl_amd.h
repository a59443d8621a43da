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
/* Build identity: the first 16 hex digits of a SHA-256 over this library's sources (csrc/ and
 * include/, as compiled), so that a measurement (bench line, PMC pass) can name the exact build
 * it ran; no reference counterpart. */
const char* lddl_build_id(void);

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
/* The same synthetic documents as raw document text (sentences joined by one space), for the
 * segmentation path: text[doc_off[d] .. doc_off[d+1]). Returns the byte count (< 0: capacity). */
int64_t lddl_synth_doc_text(uint64_t seed, int64_t doc_begin, int64_t target_bytes,
                            double nonascii_frac, uint8_t* text, int64_t text_cap, int64_t* doc_off,
                            int64_t doc_cap, int64_t* n_doc_out, int n_threads);

/* ---------------------------------------------------------------------------------------------
 * Host reader of the preprocessor input (host-only, no GPU): replaces the per-line Python of
 * dask.bag.read_text + random_sample (lddl/dask/readers.py:60-71), split_id_text (readers.py
 * :131-136) and the document shuffle (lddl/dask/bert/pretrain.py:100-111, here per shuffle group
 * with CPython's Random(seed).shuffle) for a batch of blocks, in threads.
 * lddl_read_groups: block i = bytes [starts[i], ends[i]) of file paths[i]; mt_states (may be NULL:
 *   no sampling) holds 625 words per block (the 624-word random_sample state + its index); a line
 *   (block split on '\n', str.strip()ed, empty dropped) is kept iff random() < ratio. Blocks are
 *   grouped into shuffle groups by group_off[n_groups+1]; group g's documents are shuffled by
 *   random.Random(s).shuffle with abs(s) = group_seed_abs[g] and dealt back over its blocks (each
 *   keeps its count). Every block must be valid UTF-8 (dask decodes blocks strictly): else
 *   returns -2 with bad[0] = block, bad[1] = byte offset in the block. On success *n_docs
 *   documents of *n_text bytes (the text after each line's id) are held by *out.
 * lddl_read_fill: text[n_text], doc_off[n_docs+1], block_ndocs[n_blocks] (may be NULL), in block
 *   order. lddl_read_free releases the handle.
 * ------------------------------------------------------------------------------------------- */
typedef struct lddl_reader lddl_reader;
int lddl_read_groups(int64_t n_blocks, const char* const* paths, const int64_t* starts,
                     const int64_t* ends, const uint32_t* mt_states, double ratio, int64_t n_groups,
                     const int64_t* group_off, const uint64_t* group_seed_abs, int n_threads,
                     lddl_reader** out, int64_t* n_docs, int64_t* n_text, int64_t* bad);
int lddl_read_fill(lddl_reader* reader, uint8_t* text, int64_t* doc_off, int64_t* block_ndocs);
/* block_ndocs[n_blocks] and doc_len[n_docs] (text bytes per document), either may be NULL; then
 * lddl_read_fill_range copies documents [d0, d1) only: text[sum of their lengths],
 * doc_off[d1 - d0 + 1] relative to text (a GPU batch at a time). */
int lddl_read_counts(const lddl_reader* reader, int64_t* block_ndocs, int64_t* doc_len);
int lddl_read_fill_range(lddl_reader* reader, int64_t d0, int64_t d1, uint8_t* text,
                         int64_t* doc_off);
int lddl_read_free(lddl_reader* reader);
/* dask 2021.10 `random_state_data_python(n, seed)` (the per-partition MT states of
 * bag.random_sample): n states of 624 words = Random(abs(seed)).randint(0, 2**32) in order, each
 * followed by the index 624 (as setstate stores them: 2**32 becomes 0). out[625 * n]. */
int lddl_random_state_data(int64_t n, uint64_t seed_abs, uint32_t* out);

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
/* Bytes per token id in the pair tables (lddl_pairs_emit tokens and labels, the render inputs):
 * 2 (uint16) when vocab_size <= 65534 (two 16-bit values stay free for the gather's decision
 * table), else 4 (int32). */
int lddl_ctx_id_bytes(const lddl_ctx* ctx);
/* device pointers to the vocab strings (for rendering ' '.join(tokens)): token i is
 * bytes[off[i] .. off[i+1]) */
int lddl_ctx_render_table(const lddl_ctx* ctx, const uint8_t** d_bytes, const int64_t** d_off);

/* Device allocator of the library's per-call temporaries (pair plans, scans, binning scratch).
 * Default: the ctx's own cache of hipMalloc blocks. With callbacks set, every temporary comes
 * from alloc_fn(bytes, stream, user) and goes back through free_fn(p, stream, user) on the
 * stream of its last use — a stream-ordered pool such as PyTorch's caching allocator
 * (lddl_amd/context.py), so one allocator owns HBM. Both NULL restores the default. */
typedef void* (*lddl_alloc_fn)(size_t bytes, void* stream, void* user);
typedef void (*lddl_free_fn)(void* p, void* stream, void* user);
int lddl_ctx_set_allocator(lddl_ctx* ctx, lddl_alloc_fn alloc_fn, lddl_free_fn free_fn,
                           void* user);

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

/* ---------------------------------------------------------------------------------------------
 * UTF-8 validation (the strict decode dask.bag.read_text applies to every input block, readers.py
 * :60-71; the reference raises UnicodeDecodeError on malformed input): *d_first_bad (device int64)
 * = offset of the first byte that does not begin or continue a well-formed sequence (Python's
 * decoder rules: no overlongs, surrogates or > U+10FFFF), or 0x7F7F7F7F7F7F7F7F if all of
 * d_text[0 .. n_bytes) is valid. Asynchronous on `stream`.
 * ------------------------------------------------------------------------------------------- */
int lddl_utf8_check(void* stream, const uint8_t* d_text, int64_t n_bytes, int64_t* d_first_bad);

/* ---------------------------------------------------------------------------------------------
 * Punkt sentence segmentation (device in, device out).
 * Replaces `nltk.tokenize.sent_tokenize(text)` + `strip()` + dropping empty sentences
 * (lddl/dask/bert/pretrain.py:86-88) for every document of a batch: nltk 3.6.5's
 * PunktSentenceTokenizer(params).span_tokenize (nltk/tokenize/punkt.py:1316-1391, realign
 * 1351-1379, annotation 582-630 / 1516-1650), segment.hip.
 * lddl_punkt_set_params: `table` = lddl_amd/assets/punkt_props.bin (Python's character classes),
 *   `records` = the PunktParameters (abbrev_types, sent_starters, ortho_context, collocations)
 *   as records (u8 kind 1/2/3/4, u8 value = ortho flags, u16 len_a, u16 len_b, UTF-8 bytes a, b);
 *   records_bytes = 0 is the untrained PunktSentenceTokenizer(). Keys longer than 255 bytes are
 *   rejected. Must be called once before lddl_segment_count.
 * lddl_segment_count: documents d_text[d_doc_off[d] .. d_doc_off[d+1]) (the text after the
 *   document id, readers.py:131-136; documents contiguous, each < 2 GiB, valid UTF-8, inside
 *   [0, n_bytes)); returns the sentence count
 *   (synchronises the stream). Exactly one lddl_segment_fill must follow on the same ctx.
 * lddl_segment_fill -> d_sent_off[n_sent+1], d_doc_sent_off[n_doc+1]: sentence k of document d
 *   is d_text[sent_off[doc_sent_off[d]+k] .. sent_off[...+1]); it equals the reference's
 *   stripped sentence up to leading/trailing whitespace (sentences are contiguous: whitespace
 *   between sentences is attached to the left one, which the BERT tokenizer ignores), and a
 *   whitespace-only sentence stands for the reference's dropped empty string (0 pieces, dropped
 *   by the pair builder exactly like pretrain.py:92-97). The output feeds lddl_tokenize.
 *   Both outputs NULL cancels the pending segmentation (releases its scratch; the host calls it
 *   when something fails between count and fill).
 * ------------------------------------------------------------------------------------------- */
int lddl_punkt_set_params(lddl_ctx* ctx, const uint8_t* table, int64_t table_bytes,
                          const uint8_t* records, int64_t records_bytes);
int lddl_segment_count(lddl_ctx* ctx, void* stream, const uint8_t* d_text, int64_t n_bytes,
                       const int64_t* d_doc_off, int64_t n_doc, int64_t* n_sent);
int lddl_segment_fill(lddl_ctx* ctx, void* stream, int64_t* d_sent_off, int64_t* d_doc_sent_off);

/* ---------------------------------------------------------------------------------------------
 * NSP pairs + static masking for a batch of partitions (device in, device out).
 * Replaces `_to_partition_pairs` (lddl/dask/bert/pretrain.py:386-402) =
 *   for dup in range(duplicate_factor): for doc: create_pairs_from_document(...)  (241-365)
 *     with _truncate_seq_pair (161-176) and, if masking, create_masked_lm_predictions (182-238)
 *   random.shuffle(partition_pairs)
 * after the empty-sentence / empty-document filtering of _get_documents (89-97).
 * Inputs: the tokenizer output (d_ids, d_sent_len) over d_sent_off[n_sent+1];
 *   d_doc_sent_off[n_doc+1] sentence offsets of documents (doc_sent_off[0]=0,
 *   doc_sent_off[n_doc]=n_sent); d_part_doc_off[n_part+1] document offsets of partitions;
 *   d_part_seed[n_part]: rng=LDDL_RNG_REPLAY reproduces CPython `random` after
 *   random.seed(part_seed[p]) bit for bit (vocab_words in id order).
 * lddl_pairs_plan runs the control plane and returns counts[5] = {pairs, tokens (sum of
 * len(A)+len(B)), masked positions, kept sentences, kept documents}; the caller then allocates
 * outputs and calls lddl_pairs_emit. Output pair q (partition order, then the partition shuffle):
 *   tokens[tok_off[q] : tok_off[q] + len_a[q]] = A (masked), then B up to tok_off[q+1];
 *   num_tokens = len(A)+len(B)+3; is_rn[q]; masked positions (sorted, in [CLS] A [SEP] B [SEP]
 *   coordinates) pos[pos_off[q]:pos_off[q+1]] with original-token labels lab[...].
 * ------------------------------------------------------------------------------------------- */
typedef struct lddl_pairs lddl_pairs;
enum { LDDL_RNG_REPLAY = 0, LDDL_RNG_NATIVE = 1 };
typedef struct {
  int32_t seq;            /* --target-seq-length */
  int32_t dup;            /* --duplicate-factor */
  int32_t masking;        /* --masking */
  int32_t rng;            /* LDDL_RNG_REPLAY | LDDL_RNG_NATIVE */
  double short_seq_prob;  /* --short-seq-prob */
  double masked_lm_ratio; /* --masked-lm-ratio */
  uint64_t native_seed;   /* counter-RNG key for LDDL_RNG_NATIVE */
} lddl_pair_params;
int lddl_pairs_plan(lddl_ctx* ctx, void* stream, const lddl_pair_params* params,
                    const int64_t* d_sent_off, const int32_t* d_ids, const int32_t* d_sent_len,
                    int64_t n_sent, const int64_t* d_doc_sent_off, int64_t n_doc,
                    const int64_t* d_part_doc_off, const int64_t* d_part_seed, int64_t n_part,
                    lddl_pairs** out, int64_t* counts);
int lddl_pairs_emit(lddl_pairs* plan, void* stream, void* d_tokens, int64_t* d_tok_off,
                    int32_t* d_len_a, uint8_t* d_is_rn, uint16_t* d_pos, void* d_lab,
                    int64_t* d_pos_off);
int lddl_pairs_destroy(lddl_pairs* plan, void* stream);
/* d_part_pair_off[n_part + 1]: first output pair of each partition (pairs are emitted in
 * partition order), i.e. the row ranges of the reference's per-partition outputs. */
int lddl_pairs_part_offsets(lddl_pairs* plan, void* stream, int64_t* d_part_pair_off);
/* Device time (ms, HIP events on the plan's stream) of the planner kernel of lddl_pairs_plan. */
int lddl_pairs_plan_ms(const lddl_pairs* plan, float* ms);

/* ---------------------------------------------------------------------------------------------
 * Per-partition sequence-length binning.
 * Replaces _to_dataframe_binned (lddl/dask/bert/binning.py:63-93) applied per partition:
 *   bin_id = min((num_tokens - 1) // bin_size, nbins - 1), rows regrouped by bin, stable.
 * Rows of partition p are d_part_off[p] .. d_part_off[p+1]; row r's num_tokens is d_num_tokens[r],
 * or, with d_num_tokens NULL, d_tok_off[r+1] - d_tok_off[r] + 3 (a lddl_pairs_emit offset table).
 * Outputs (device, every entry written): d_perm[r] = input
 * row of output row r (partition order kept, bins ascending inside a partition), d_bin_id[r] its
 * bin, d_counts[p * nbins + b] = rows of partition p in bin b. nbins <= 8192.
 * ------------------------------------------------------------------------------------------- */
int lddl_bin_partitions(lddl_ctx* ctx, void* stream, const int32_t* d_num_tokens,
                        const int64_t* d_tok_off, int64_t n_rows, const int64_t* d_part_off,
                        int64_t n_part, int32_t bin_size, int32_t nbins, int64_t* d_perm,
                        int64_t* d_bin_id, int64_t* d_counts);

/* The same regroup for ONE large segment (a rank's rows of one batch before the load-balance
 * exchange), spread over many workgroups: d_perm / d_bin_id (may be NULL) as above, d_counts[b]
 * rows per bin. num_tokens of row r = d_num_tokens[r], or, with d_num_tokens NULL, the pair's
 * token count + 3 from a lddl_pairs_emit offset table: d_tok_off[r+1] - d_tok_off[r] + 3. */
int lddl_bin_stable(lddl_ctx* ctx, void* stream, const int32_t* d_num_tokens,
                    const int64_t* d_tok_off, int64_t n_rows, int32_t bin_size, int32_t nbins,
                    int64_t* d_perm, int64_t* d_bin_id, int64_t* d_counts);

/* ---------------------------------------------------------------------------------------------
 * Rendering of the parquet columns (lddl/dask/bert/pretrain.py:345-358):
 *   A, B = ' '.join(tokens), masked_lm_labels = ' '.join(labels) (vocab strings of the ids),
 *   masked_lm_positions = np.save bytes of uint16[k] (lddl/utils.py:98-102; 128 + 2k bytes).
 * Output row r renders pair d_rows[r] (d_rows NULL = identity) of a lddl_pairs_emit table.
 * lddl_render_lengths writes per-row byte lengths; the caller scans them (lddl_scan_i64) into
 * offsets and calls lddl_render_write. Label / position arguments may be NULL (no masking).
 * It also writes the rows' num_tokens (uint16, len(A) + len(B) + 3) and, from d_is_rn,
 * is_random_next in output order (each output pointer may be NULL).
 * ------------------------------------------------------------------------------------------- */
int lddl_render_lengths(lddl_ctx* ctx, void* stream, const void* d_tokens,
                        const int64_t* d_tok_off, const int32_t* d_len_a, const void* d_lab,
                        const int64_t* d_pos_off, const int64_t* d_rows, int64_t n_rows,
                        int64_t* d_a_len, int64_t* d_b_len, int64_t* d_l_len, int64_t* d_npy_len,
                        const uint8_t* d_is_rn, uint16_t* d_num_tokens_out, uint8_t* d_is_rn_out);
int lddl_render_write(lddl_ctx* ctx, void* stream, const void* d_tokens,
                      const int64_t* d_tok_off, const int32_t* d_len_a, const uint16_t* d_pos,
                      const void* d_lab, const int64_t* d_pos_off, const int64_t* d_rows,
                      int64_t n_rows, const int64_t* d_a_off, const int64_t* d_b_off,
                      const int64_t* d_l_off, const int64_t* d_npy_off, uint8_t* d_a_bytes,
                      uint8_t* d_b_bytes, uint8_t* d_l_bytes, uint8_t* d_npy_bytes);

/* ---------------------------------------------------------------------------------------------
 * Row movement of the load balance (lddl_amd/balance.py; replaces the reference's filesystem
 * shuffle, lddl/dask/load_balance.py:84-156). Rows are addressed over TWO sources: row r < n_a is
 * row r of source A, else row r - n_a of source B (B may be NULL when every r < n_a); d_rows NULL
 * = the identity (n_rows <= n_a). elem_bytes in {1, 2, 4, 8}; offsets count elements and are
 * relative to their own source.
 *   lddl_gather_ragged: elements src[off[r] .. off[r+1]) of output row i (r = d_rows[i]) copied to
 *     d_dst[d_dst_off[i] ...].
 *   lddl_take: d_dst[i] = src[r].
 *   lddl_ragged_offsets: d_out[0..n_rows] = exclusive scan of the rows' sizes off[r+1] - off[r].
 *   lddl_expand_segments: segment k covers d_out[seg_off[k] .. seg_off[k+1]); its element t is
 *     v = seg[3k] + t * seg[3k+1], written as v when seg[3k+2] != 0, else as d_src[v]
 *     (the balance plan's strided row runs, expanded on the device).
 *   lddl_pairs_meta_pack: int32[n][4] {len(A)+len(B), len(A), is_random_next, masks} of rows d_rows
 *     of a pair table (d_pos_off NULL: 0 masks); lddl_pairs_meta_unpack splits it into columns
 *     (d_nmask may be NULL).
 * ------------------------------------------------------------------------------------------- */
int lddl_gather_ragged(void* stream, const void* d_src_a, const int64_t* d_off_a, int64_t n_a,
                       const void* d_src_b, const int64_t* d_off_b, int32_t elem_bytes,
                       const int64_t* d_rows, int64_t n_rows, const int64_t* d_dst_off, void* d_dst);
int lddl_take(void* stream, const void* d_a, int64_t n_a, const void* d_b, int32_t elem_bytes,
              const int64_t* d_rows, int64_t n_rows, void* d_dst);
int lddl_ragged_offsets(lddl_ctx* ctx, void* stream, const int64_t* d_off_a, int64_t n_a,
                        const int64_t* d_off_b, const int64_t* d_rows, int64_t n_rows,
                        int64_t* d_out);
int lddl_expand_segments(void* stream, const int64_t* d_src, const int64_t* d_seg,
                         const int64_t* d_seg_off, int64_t n_seg, int64_t total, int64_t* d_out);
int lddl_pairs_meta_pack(void* stream, const int64_t* d_tok_off, const int32_t* d_len_a,
                         const uint8_t* d_is_rn, const int64_t* d_pos_off, const int64_t* d_rows,
                         int64_t n, int32_t* d_meta);
int lddl_pairs_meta_unpack(void* stream, const int32_t* d_meta, int64_t n, int64_t* d_ntok,
                           int32_t* d_len_a, uint8_t* d_is_rn, int64_t* d_nmask);

/* Exclusive prefix sum: d_out[0..n] (d_out[n] = total) of d_in[0..n) (scratch from the ctx). */
int lddl_scan_i64(lddl_ctx* ctx, void* stream, const int64_t* d_in, int64_t n, int64_t* d_out);

/* ---------------------------------------------------------------------------------------------
 * Loader collate (lddl/torch/bert.py:69-149 `_to_encoded_inputs`), one batch, device in/out.
 *   d_bytes: A / B strings of the batch (space-joined tokens, as stored in the parquet shards);
 *   sample b: A = d_bytes[a_off[b], a_off[b+1]), B = d_bytes[b_off[b], b_off[b+1]);
 *   d_na/d_nb: token counts; seq_len = roundup(max(na+nb+3), sequence_length_alignment).
 *   Outputs int64 [batch, seq_len]: input_ids (convert_tokens_to_ids, [UNK] if absent),
 *   token_type_ids, attention_mask, and either special_tokens_mask (dynamic masking) or labels
 *   (static: d_lab_bytes/d_lab_off = masked_lm_labels strings, d_pos/d_pos_off = decoded
 *   masked_lm_positions; unmasked slots = ignore_index). Unused outputs may be NULL.
 *   Token and label writes at positions >= seq_len are dropped (the host refuses such a batch
 *   with IndexError before launching, as the reference's tensor indexing does).
 * ------------------------------------------------------------------------------------------- */
int lddl_collate_encode(lddl_ctx* ctx, void* stream, const uint8_t* d_bytes, const int64_t* d_a_off,
                        const int64_t* d_b_off, const int32_t* d_na, const int32_t* d_nb,
                        int32_t batch, int32_t seq_len, int64_t* d_input_ids,
                        int64_t* d_token_type_ids, int64_t* d_attention_mask,
                        int64_t* d_special_tokens_mask, const uint8_t* d_lab_bytes,
                        const int64_t* d_lab_off, const uint16_t* d_pos, const int64_t* d_pos_off,
                        int64_t* d_labels, int64_t ignore_index);

/* The loader's dynamic-masking collate in one pass (lddl/torch/bert.py:348-365 =
 * _to_encoded_inputs + _mask_tokens): as lddl_collate_encode (dynamic), then the native-RNG
 * masking of lddl_mask_dynamic applied to each slot as it is written; outputs input_ids (masked),
 * token_type_ids, attention_mask, labels. Bit-identical to lddl_collate_encode followed by
 * lddl_mask_dynamic with the same seed / counter. */
int lddl_collate_encode_masked(lddl_ctx* ctx, void* stream, const uint8_t* d_bytes,
                               const int64_t* d_a_off, const int64_t* d_b_off, const int32_t* d_na,
                               const int32_t* d_nb, int32_t batch, int32_t seq_len,
                               int64_t* d_input_ids, int64_t* d_token_type_ids,
                               int64_t* d_attention_mask, int64_t* d_labels, float mlm_probability,
                               int64_t ignore_index, int64_t vocab_len, uint64_t seed,
                               uint64_t counter);

/* ---------------------------------------------------------------------------------------------
 * Dynamic masking (lddl/torch/bert.py:152-196 `_mask_tokens`) in place on d_input_ids
 * [batch, seq_len] int64; writes d_labels. Special slots come from d_special_tokens_mask, or,
 * if NULL, from the lengths (positions 0, na+1 and >= na+nb+2, as _to_encoded_inputs sets them),
 * or, if the lengths are NULL too, from the ids: a slot is special iff its id is one of
 * [PAD] [UNK] [CLS] [SEP] [MASK] (`special_tokens_mask=None`, i.e.
 * tokenizer.get_special_tokens_mask(ids, already_has_special_tokens=True), bert.py:167-172).
 * Native mode: Philox4x32-10 keyed by (seed, counter) — call with a fresh counter per batch.
 * Replay mode (all four d_r_* non-NULL): apply captured torch draws (masked_indices,
 * indices_replaced, indices_random as uint8, random_words int64) bit for bit.
 * ------------------------------------------------------------------------------------------- */
int lddl_mask_dynamic(lddl_ctx* ctx, void* stream, int64_t* d_input_ids, int64_t* d_labels,
                      const int64_t* d_special_tokens_mask, const int32_t* d_na, const int32_t* d_nb,
                      int64_t batch, int64_t seq_len, float mlm_probability, int64_t ignore_index,
                      int64_t vocab_len, uint64_t seed, uint64_t counter,
                      const uint8_t* d_r_masked, const uint8_t* d_r_replaced,
                      const uint8_t* d_r_random, const int64_t* d_r_words);

#ifdef __cplusplus
}
#endif

#endif /* LDDL_AMD_H_ */

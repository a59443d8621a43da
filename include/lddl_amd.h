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

#ifdef __cplusplus
}
#endif

#endif /* LDDL_AMD_H_ */

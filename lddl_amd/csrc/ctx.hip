// lddl_ctx_create / destroy: replaces constructing `transformers.BertTokenizerFast(vocab_file)`
// (lddl/dask/bert/pretrain.py:584-587, lddl/torch/bert.py:343-346) with device-resident tables.
#include <cstring>

#include "common.h"
#include "ctx.h"
#include "lddl_amd.h"

using namespace lddl;

namespace {

template <typename T>
int upload(T** dst, const void* src, size_t bytes) {
  LDDL_HIP(hipMalloc((void**)dst, bytes ? bytes : 16));
  if (bytes) LDDL_HIP(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return 0;
}

uint64_t pack8(const uint8_t* p, int len) {
  uint64_t v = 0;
  for (int i = 0; i < len && i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

}  // namespace

extern "C" int lddl_ctx_create(int device, const uint8_t* norm_table, int64_t table_len,
                               const char* vocab, int64_t vocab_len, lddl_ctx** out) {
  *out = nullptr;
  if (table_len < 20 || memcmp(norm_table, "LDNT", 4) != 0)
    LDDL_FAIL(-1, "bad normaliser table blob");
  uint32_t n_pages, pool_len;
  memcpy(&n_pages, norm_table + 12, 4);
  memcpy(&pool_len, norm_table + 16, 4);
  const int64_t need = 20 + 2 * 4352 + 4 * 256 * (int64_t)n_pages + pool_len;
  if (table_len < need) LDDL_FAIL(-1, "truncated normaliser table (%lld < %lld)",
                                  (long long)table_len, (long long)need);
  LDDL_HIP(hipSetDevice(device));
  // keep stream-ordered allocations (planner / tokenizer temporaries) cached across calls
  // instead of returning them to the driver at every synchronisation
  {
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
      uint64_t thr = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }
  }
  auto* c = new lddl_ctx();
  c->device = device;
  {
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess)
      c->lds_per_block = (size_t)lds;
  }

  // vocab.txt: one token per line, id = line number (BertTokenizerFast / WordPiece.from_file)
  std::string cur;
  for (int64_t i = 0; i < vocab_len; ++i) {
    char ch = vocab[i];
    if (ch == '\n') {
      if (!cur.empty() && cur.back() == '\r') cur.pop_back();
      c->tokens.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  if (!cur.empty()) c->tokens.push_back(cur);
  const int32_t V = (int32_t)c->tokens.size();
  if (V == 0 || V >= (1 << 21)) { delete c; LDDL_FAIL(-1, "vocab size %d unsupported", V); }
  c->vocab_size = V;

  // piece bytes (continuation prefix removed) + render strings
  std::vector<uint8_t> vbytes, render;
  std::vector<int64_t> voff(V + 1), roff(V + 1);
  std::vector<uint8_t> cont(V);
  int max_piece = 1;
  for (int32_t i = 0; i < V; ++i) {
    const std::string& t = c->tokens[i];
    roff[i] = (int64_t)render.size();
    render.insert(render.end(), t.begin(), t.end());
    voff[i] = (int64_t)vbytes.size();
    size_t b = 0;
    if (t.size() > 2 && t[0] == '#' && t[1] == '#') { cont[i] = 1; b = 2; }
    vbytes.insert(vbytes.end(), t.begin() + b, t.end());
    max_piece = std::max(max_piece, (int)(t.size() - b));
  }
  voff[V] = (int64_t)vbytes.size();
  roff[V] = (int64_t)render.size();
  if (max_piece > 255) { delete c; LDDL_FAIL(-1, "vocab piece longer than 255 bytes"); }

  // open-addressing hash, load <= 0.25 (a miss probes ~1.4 slots; 2 MB at 30k pieces stays
  // L2-resident). A duplicated vocab line maps to its LAST id, as the
  // HF WordPiece vocab HashMap built in file order does.
  uint32_t cap = 1;
  while (cap < 4u * (uint32_t)V + 64) cap <<= 1;
  std::vector<VEnt> tab(cap);
  memset(tab.data(), 0, sizeof(VEnt) * cap);
  for (int32_t i = 0; i < V; ++i) {
    const uint8_t* p = vbytes.data() + voff[i];
    const int len = (int)(voff[i + 1] - voff[i]);
    const uint64_t k0 = pack8(p, len);
    const uint32_t k1 = (uint32_t)pack8(p + 8, len > 8 ? std::min(len - 8, 4) : 0);
    const uint32_t meta = kMetaValid | (cont[i] ? kMetaCont : 0) | (len > 12 ? kMetaLong : 0) |
                          ((uint32_t)len << 21) | (uint32_t)i;
    uint64_t h = vhash(k0, k1, len, cont[i]);
    bool dup = false;
    uint32_t s = (uint32_t)h & (cap - 1);
    for (;; s = (s + 1) & (cap - 1)) {
      const VEnt& e = tab[s];
      if (!(e.meta & kMetaValid)) break;
      if (e.k0 == k0 && e.k1 == k1 && ((e.meta ^ meta) & ~0x1FFFFFu) == 0) {
        const int32_t j = meta_id(e.meta);
        if (len <= 12 || memcmp(vbytes.data() + voff[j], p, len) == 0) {
          tab[s].meta = meta;
          dup = true;
          break;
        }
      }
    }
    if (!dup) tab[s] = VEnt{k0, k1, meta};
  }

  // Bloom filter of (continuation, piece bytes) for the tokenizer's longest-match scan
  std::vector<uint32_t> bloom(kBloomWords, 0u);
  for (int32_t i = 0; i < V; ++i) {
    const uint8_t* p = vbytes.data() + voff[i];
    const int len = (int)(voff[i + 1] - voff[i]);
    uint32_t h = 0;
    for (int k = 0; k < len; ++k) h = h * kBloomP + (uint32_t)p[k] + 1u;
    const uint32_t x = bloom_mix(h, (uint32_t)len, cont[i]);
    bloom[bloom_word(x)] |= bloom_bits(x);
  }
  // 32-byte zero-padded copies of the pieces (longer pieces keep only their first 32 bytes: a
  // probe key is at most 32 bytes, so they never reach the tail check)
  std::vector<uint64_t> vlong(4 * (size_t)V, 0ull);
  for (int32_t i = 0; i < V; ++i) {
    const int len = (int)(voff[i + 1] - voff[i]);
    memcpy(reinterpret_cast<uint8_t*>(vlong.data() + 4 * (size_t)i), vbytes.data() + voff[i], std::min(len, 32));
  }
  const uint8_t* l1 = norm_table + 20;
  const uint8_t* pages = l1 + 2 * 4352;
  const uint8_t* pool = pages + 4 * 256 * (int64_t)n_pages;
  int rc = 0;
  if ((rc = upload(&c->d_l1, l1, 2 * 4352)) || (rc = upload(&c->d_pages, pages, 4 * 256 * (size_t)n_pages)) ||
      (rc = upload(&c->d_pool, pool, pool_len)) || (rc = upload(&c->d_vhash, tab.data(), sizeof(VEnt) * cap)) ||
      (rc = upload(&c->d_vbytes, vbytes.data(), vbytes.size())) ||
      (rc = upload(&c->d_voff, voff.data(), sizeof(int64_t) * voff.size())) ||
      (rc = upload(&c->d_render, render.data(), render.size())) ||
      (rc = upload(&c->d_render_off, roff.data(), sizeof(int64_t) * roff.size())) ||
      (rc = upload(&c->d_bloom, bloom.data(), sizeof(uint32_t) * bloom.size())) ||
      (rc = upload(&c->d_vlong, vlong.data(), sizeof(uint64_t) * vlong.size()))) {
    lddl_ctx_destroy(c);
    return rc;
  }
  Tables& T = c->tab;
  T.l1 = c->d_l1;
  T.pages = c->d_pages;
  T.pool = c->d_pool;
  T.vhash = c->d_vhash;
  T.vbytes = c->d_vbytes;
  T.voff = c->d_voff;
  T.vmask = cap - 1;
  T.bloom = c->d_bloom;
  T.vlong = c->d_vlong;
  T.max_piece_bytes = max_piece;
  static const char* kSpecial[kNumSpecial] = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"};
  for (int k = 0; k < kNumSpecial; ++k) {
    T.special_id[k] = -1;
    for (int32_t i = 0; i < V; ++i)
      if (c->tokens[i] == kSpecial[k]) { T.special_id[k] = i; break; }
  }
  // classify the ASCII page for the wave tokenizer's register fast path
  {
    const uint16_t* l1p = reinterpret_cast<const uint16_t*>(l1);
    const uint32_t* pg = reinterpret_cast<const uint32_t*>(pages) + 256 * (size_t)l1p[0];
    bool lower_ok = true, ident_ok = true;
    for (uint32_t cp = 0; cp < 128; ++cp) {
      const uint32_t e = pg[cp];
      if ((e >> 30) != kWord && (e >> 30) != kIso) continue;  // both take the register path
      const uint32_t outc = (e & kIdent) ? cp : (e & kMulti) ? 0xFFFFFFFFu : (e & 0x1FFFFFu);
      const uint32_t want_lower = (cp >= 'A' && cp <= 'Z') ? cp + 32 : cp;
      lower_ok &= outc == want_lower;
      ident_ok &= outc == cp;
    }
    T.ascii_mode = ident_ok ? 2 : lower_ok ? 1 : 0;
  }
  if (T.special_id[kUnk] < 0) { lddl_ctx_destroy(c); LDDL_FAIL(-1, "vocab has no [UNK]"); }
  *out = c;
  return 0;
}

extern "C" int lddl_ctx_destroy(lddl_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  lddl_punkt_release(c);
  for (void* p : {(void*)c->d_l1, (void*)c->d_pages, (void*)c->d_pool, (void*)c->d_vhash,
                  (void*)c->d_vbytes, (void*)c->d_voff, (void*)c->d_render, (void*)c->d_render_off,
                  (void*)c->d_bloom, (void*)c->d_vlong})
    if (p) (void)hipFree(p);
  delete c;
  return 0;
}

extern "C" int lddl_ctx_info(const lddl_ctx* c, int32_t* vocab_size, int32_t* special_ids,
                             int32_t* max_piece_bytes) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (vocab_size) *vocab_size = c->vocab_size;
  if (special_ids)
    for (int k = 0; k < kNumSpecial; ++k) special_ids[k] = c->tab.special_id[k];
  if (max_piece_bytes) *max_piece_bytes = c->tab.max_piece_bytes;
  return 0;
}

extern "C" int lddl_ctx_id_bytes(const lddl_ctx* c) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  return c->id_bytes();
}

extern "C" int lddl_ctx_render_table(const lddl_ctx* c, const uint8_t** d_bytes,
                                     const int64_t** d_off) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  *d_bytes = c->d_render;
  *d_off = c->d_render_off;
  return 0;
}

extern "C" int lddl_ctx_set_allocator(lddl_ctx* c, lddl_alloc_fn alloc_fn, lddl_free_fn free_fn,
                                      void* user) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if ((alloc_fn == nullptr) != (free_fn == nullptr))
    LDDL_FAIL(-1, "set both allocator callbacks or neither");
  c->arena.set_external(alloc_fn, free_fn, user);
  return 0;
}

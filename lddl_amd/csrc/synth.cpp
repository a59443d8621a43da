// Deterministic synthetic English-like corpus (SURVEY.md §8(d) "Synthetic inputs").
//
// The reference reads one document per line, `<doc_id><ws><text>` (lddl/dask/readers.py:131-136,
// lddl/download/wikipedia.py:63), and Punkt-splits each text into sentences
// (lddl/dask/bert/pretrain.py:86). The hot path starts AFTER Punkt, so this generator emits the
// already-segmented form directly: the concatenated bytes of every sentence plus sentence and
// document offset tables. `lddl_synth_write_lines` renders the same corpus in the reference's
// one-document-per-line text format for the CLI path.
//
// Every document is a pure function of (seed, doc index), so the corpus is identical for any
// thread count and any split into batches.
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>
#include <string>
#include <thread>
#include <algorithm>
#include <mutex>

#include "lddl_amd.h"

namespace {

struct Rng {  // splitmix64 -> xoshiro256**
  uint64_t s[4];
  static uint64_t sm(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  explicit Rng(uint64_t seed) { for (auto& v : s) v = sm(seed); }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  double unif() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  int range(int lo, int hi) { return lo + (int)below((uint32_t)(hi - lo + 1)); }  // inclusive
};

const char* kOnsets[] = {"b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t",
                         "v", "w", "z", "br", "cl", "dr", "fl", "gr", "pl", "pr", "sh", "st", "th",
                         "tr", "ch", "qu", "sp", "str", "", ""};
const char* kNuclei[] = {"a", "e", "i", "o", "u", "ai", "ea", "ee", "ie", "oo", "ou", "y", "a", "e",
                         "o", "i"};
const char* kCodas[] = {"", "", "", "n", "r", "s", "t", "l", "m", "nd", "st", "ng", "rt", "ck", "x",
                        "ll", "th", "ss"};
const char* kAccented[] = {"\xc3\xa9", "\xc3\xa8", "\xc3\xaa", "\xc3\xab", "\xc3\xa1", "\xc3\xa0",
                           "\xc3\xa2", "\xc3\xa4", "\xc3\xad", "\xc3\xaf", "\xc3\xb3", "\xc3\xb6",
                           "\xc3\xb4", "\xc3\xba", "\xc3\xbc", "\xc3\xb1", "\xc3\xa7", "\xc3\x89",
                           "\xc3\x9c", "\xc3\x85"};
const char* kGreek[] = {"\xce\xb1", "\xce\xb2", "\xce\xb3", "\xce\xb4", "\xce\xbb", "\xcf\x80",
                        "\xce\xa9", "\xce\xa3"};

template <size_t N> constexpr int count(const char* const (&)[N]) { return (int)N; }

struct Lexicon {
  std::vector<std::string> words;
  std::vector<double> cdf;  // Zipf CDF over ranks
  Lexicon(uint64_t seed, int n, double s) {
    Rng r(seed ^ 0x5EEDF00Dull);
    words.reserve(n);
    for (int i = 0; i < n; ++i) {
      // Frequent ranks get short words (1-2 syllables), rare ranks longer ones.
      int maxsyl = i < 100 ? 1 : (i < 2000 ? 2 : (i < 20000 ? 3 : 4));
      int nsyl = 1 + (int)r.below((uint32_t)maxsyl);
      std::string w;
      for (int k = 0; k < nsyl; ++k) {
        w += kOnsets[r.below(count(kOnsets))];
        w += kNuclei[r.below(count(kNuclei))];
        w += kCodas[r.below(count(kCodas))];
      }
      if (w.empty()) w = "a";
      words.push_back(w);
    }
    cdf.resize(n);
    double acc = 0;
    for (int i = 0; i < n; ++i) { acc += 1.0 / std::pow((double)(i + 1), s); cdf[i] = acc; }
    for (auto& c : cdf) c /= acc;
  }
  const std::string& draw(Rng& r) const {
    double u = r.unif();
    size_t i = std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin();
    if (i >= words.size()) i = words.size() - 1;
    return words[i];
  }
};

void put_utf8(std::string& o, uint32_t cp) {
  if (cp < 0x80) o += (char)cp;
  else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 63)); }
  else if (cp < 0x10000) {
    o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63));
  } else {
    o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 63));
    o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63));
  }
}

// One document: a list of sentences (each already stripped, as Punkt + str.strip() leave them).
void make_doc(const Lexicon& lex, uint64_t seed, int64_t doc, double nonascii,
              std::vector<std::string>& sents) {
  Rng r(seed * 0x100000001B3ull + (uint64_t)doc * 0x9E3779B97F4A7C15ull + 1);
  sents.clear();
  int ns = r.range(3, 60);
  for (int si = 0; si < ns; ++si) {
    std::string s;
    int nw = r.range(6, 32);
    for (int wi = 0; wi < nw; ++wi) {
      if (wi) s += ' ';
      std::string w;
      double u = r.unif();
      if (u < 0.02) {  // number, sometimes with a decimal part
        w = std::to_string(r.range(0, 9999));
        if (r.unif() < 0.2) { w += '.'; w += std::to_string(r.range(0, 99)); }
      } else {
        w = lex.draw(r);
        if (r.unif() < 0.01) { w += '-'; w += lex.draw(r); }
        if (r.unif() < 0.008) { w += "'"; w += (r.unif() < 0.5 ? "s" : "t"); }
        if (wi == 0 || r.unif() < 0.02) w[0] = (char)(w[0] - 'a' + 'A');
        if (r.unif() < nonascii) {
          double v = r.unif();
          if (v < 0.55) {  // accented Latin letter spliced in
            size_t pos = r.below((uint32_t)w.size() + 1);
            w.insert(pos, kAccented[r.below(count(kAccented))]);
          } else if (v < 0.8) {  // CJK run
            w.clear();
            int n = r.range(1, 4);
            for (int k = 0; k < n; ++k) put_utf8(w, 0x4E00 + r.below(0x5000));
          } else if (v < 0.92) {
            w = kGreek[r.below(count(kGreek))] + w;
          } else {  // rare: emoji / symbols / full-width forms
            uint32_t cps[] = {0x1F600, 0x2014, 0x2019, 0xFF21, 0x00B0, 0x20AC, 0x00AD, 0x200B};
            put_utf8(w, cps[r.below(8)]);
          }
        }
      }
      double q = r.unif();
      if (q < 0.006) w = "(" + w + ")";
      else if (q < 0.012) w = "\"" + w + "\"";
      s += w;
      if (wi + 1 < nw && r.unif() < 0.06) s += ',';
    }
    double t = r.unif();
    s += t < 0.9 ? '.' : (t < 0.95 ? '?' : '!');
    sents.push_back(std::move(s));
  }
}

std::mutex g_lex_mu;

const Lexicon& lexicon(uint64_t seed) {  // built once per seed, shared by all threads
  static uint64_t cached_seed = ~0ull;
  static Lexicon* cached = nullptr;
  std::lock_guard<std::mutex> g(g_lex_mu);
  if (!cached || cached_seed != seed) {
    delete cached;
    cached = new Lexicon(seed, 60000, 1.07);
    cached_seed = seed;
  }
  return *cached;
}

}  // namespace

extern "C" int64_t lddl_synth_corpus(uint64_t seed, int64_t doc_begin, int64_t target_bytes,
                                     double nonascii_frac, uint8_t* text, int64_t text_cap,
                                     int64_t* sent_off, int64_t sent_cap, int64_t* doc_sent_off,
                                     int64_t doc_cap, int64_t* n_sent_out, int64_t* n_doc_out,
                                     int n_threads) {
  if (n_threads < 1) n_threads = 1;
  const int64_t kBlock = 256;  // documents per work item
  const Lexicon& lex = lexicon(seed);
  int64_t nbytes = 0, nsent = 0, ndoc = 0;
  sent_off[0] = 0;
  doc_sent_off[0] = 0;
  std::vector<std::vector<std::string>> blocks(n_threads * kBlock);
  int64_t next_doc = doc_begin;
  while (nbytes < target_bytes) {
    std::vector<std::thread> pool;
    for (int t = 0; t < n_threads; ++t)
      pool.emplace_back([&, t]() {
        for (int64_t k = 0; k < kBlock; ++k)
          make_doc(lex, seed, next_doc + t * kBlock + k, nonascii_frac, blocks[t * kBlock + k]);
      });
    for (auto& th : pool) th.join();
    for (auto& doc : blocks) {
      if (nbytes >= target_bytes) break;
      if (ndoc + 1 >= doc_cap || nsent + (int64_t)doc.size() >= sent_cap) return -2;
      for (auto& s : doc) {
        if (nbytes + (int64_t)s.size() > text_cap) return -1;
        std::memcpy(text + nbytes, s.data(), s.size());
        nbytes += (int64_t)s.size();
        sent_off[++nsent] = nbytes;
      }
      doc_sent_off[++ndoc] = nsent;
    }
    next_doc += n_threads * kBlock;
  }
  *n_sent_out = nsent;
  *n_doc_out = ndoc;
  return nbytes;
}

// The same documents as raw document text (what the reference hands to sent_tokenize): each
// document's sentences joined by one space, documents back to back, doc_off[n_doc+1] byte offsets.
extern "C" int64_t lddl_synth_doc_text(uint64_t seed, int64_t doc_begin, int64_t target_bytes,
                                       double nonascii_frac, uint8_t* text, int64_t text_cap,
                                       int64_t* doc_off, int64_t doc_cap, int64_t* n_doc_out,
                                       int n_threads) {
  if (n_threads < 1) n_threads = 1;
  const int64_t kBlock = 256;
  const Lexicon& lex = lexicon(seed);
  int64_t nbytes = 0, ndoc = 0;
  doc_off[0] = 0;
  std::vector<std::vector<std::string>> blocks(n_threads * kBlock);
  int64_t next_doc = doc_begin;
  while (nbytes < target_bytes) {
    std::vector<std::thread> pool;
    for (int t = 0; t < n_threads; ++t)
      pool.emplace_back([&, t]() {
        for (int64_t k = 0; k < kBlock; ++k)
          make_doc(lex, seed, next_doc + t * kBlock + k, nonascii_frac, blocks[t * kBlock + k]);
      });
    for (auto& th : pool) th.join();
    for (auto& doc : blocks) {
      if (nbytes >= target_bytes) break;
      if (ndoc + 1 >= doc_cap) return -2;
      for (size_t k = 0; k < doc.size(); ++k) {
        const std::string& s = doc[k];
        if (nbytes + (int64_t)s.size() + 1 > text_cap) return -1;
        if (k) text[nbytes++] = ' ';
        std::memcpy(text + nbytes, s.data(), s.size());
        nbytes += (int64_t)s.size();
      }
      doc_off[++ndoc] = nbytes;
    }
    next_doc += n_threads * kBlock;
  }
  *n_doc_out = ndoc;
  return nbytes;
}

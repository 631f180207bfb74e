// Row-sharded synthetic CKG builder (host C++) -- SURVEY §8(d) synthetic inputs at the
// C4/C5 sizes, §8(f)3 graph build at 1B edges.
//
// The numpy producer (graph.synthetic_ckg + graph.build_layout) draws the whole graph
// sequentially and sorts every edge on one core: fine at C2 (10M triples, ~10 s), not at
// C5 (500M triples, 1B edges) where each of 8 ranks would hold the whole graph.  Here a
// triple is a pure function of (seed, index): every rank streams all triple indices with
// its threads (counter-based hashes, no shared RNG state), counts the degrees the
// normalisation needs, then keeps only the attentive-matrix entries of ITS rows
// [lo, hi) and coalesces them.  No rank ever materialises another rank's edges.
//
// Triples (same shape as graph.synthetic_ckg): the first 10 % of nodes are users, items
// are the first 10 % of entities; 80 % of the triples are user -> item interactions with
// Zipf(s) item popularity (alias table over popularity ranks, ranks mapped to items by a
// seeded permutation), 20 % are KG triples over the 4 reference relations with uniform
// heads / tails inside the relation's type range.  Repeated triples are dropped and
// redrawn, as SURVEY §8(d) specifies ("duplicate (h, t) are dropped"; graph.synthetic_ckg
// redraws interactions the same way): draw p of a stream is kept iff it is the first
// draw of its triple, and the kept triples are the first M (interactions) / K (KG) kept
// draws in draw order -- a parallel hash pass records each triple's smallest draw index,
// so the result does not depend on the thread count.  Every kept triple is distinct, so
// the attentive matrix holds 2T entries before (row, col) pairs of different blocks are
// coalesced (E ~= 2T, §8(d)).  Repeats that do occur in the layout producer's input are
// still weighted by count (preprocess.py:224-246), and the arithmetic below keeps that rule.
//
// Attentive matrix (preprocess.py:177-246, 628-634): adjacency blocks in the reference
// order  0: user -> item, 1: item -> user (inverse), 2+2r: KG r, 3+2r: KG r inverse;
// block b's entry (row = tail, col = head) = count / outdeg_b(head); entries of one
// (row, col) in several blocks are summed in fp64 in block order, then rounded to fp32
// -- the arithmetic of graph.layout_from_blocks (itself pinned to the reference's own
// Preprocess output by tests/test_host_cpu.py).
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <new>
#include <thread>
#include <vector>

#include "kgat_hip.h"

namespace {

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// independent 64-bit draw `stream` of triple `i`
inline uint64_t draw(uint64_t seed, uint64_t i, uint64_t stream) {
  return mix64(seed ^ mix64(i * 0x9E3779B97F4A7C15ull + stream * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull));
}

inline uint64_t below(uint64_t h, uint64_t n) {  // floor(h * n / 2^64)
  return static_cast<uint64_t>((static_cast<unsigned __int128>(h) * n) >> 64);
}

inline double unit(uint64_t h) { return static_cast<double>(h >> 11) * 0x1.0p-53; }

struct Range {
  int64_t lo = 0, hi = 1;  // [lo, hi) entity ids
  int64_t size() const { return hi - lo; }
};

template <class F>
void parallel_for(int64_t n, int threads, F&& f) {  // f(begin, end, thread)
  threads = std::max(1, std::min<int>(threads, static_cast<int>(std::max<int64_t>(1, n / 4096))));
  if (threads == 1) {
    f(int64_t{0}, n, 0);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(threads);
  for (int t = 0; t < threads; ++t) {
    const int64_t b = n * t / threads, e = n * (t + 1) / threads;
    pool.emplace_back([&f, b, e, t] { f(b, e, t); });
  }
  for (auto& th : pool) th.join();
}

inline void bump(uint32_t* a, int64_t i) { __atomic_fetch_add(a + i, 1u, __ATOMIC_RELAXED); }

inline void atomic_min_u32(uint32_t* a, uint32_t v) {
  uint32_t cur = __atomic_load_n(a, __ATOMIC_RELAXED);
  while (v < cur && !__atomic_compare_exchange_n(a, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
}

// The first `target` distinct keys of a draw stream, in draw order: returns the draw indices p
// (ascending) whose key(p) occurs at no smaller index.  Open-addressing hash of key -> smallest draw
// index (CAS insert + atomic min: the minimum does not depend on thread interleaving), over a
// prefix of P draws, grown by 1.5x until it holds `target` distinct keys or P reaches `limit`
// (a stream with fewer distinct keys than target: all of them are kept).  *draws = the prefix
// length that yields the kept set (index of the last kept draw + 1).
template <class Key>
std::vector<uint32_t> first_distinct(int64_t target, int64_t limit, int threads, Key&& key, int64_t* draws) {
  std::vector<uint32_t> kept;
  *draws = 0;
  if (target <= 0) return kept;
  constexpr uint64_t kEmpty = ~uint64_t{0};
  int64_t P = std::min(limit, target + target / 2 + 4096);
  for (;;) {
    uint64_t S = 1024;
    while (S < static_cast<uint64_t>(P + P / 2)) S <<= 1;
    std::vector<uint64_t> keys(S, kEmpty);
    std::vector<uint32_t> first(S, ~uint32_t{0});
    const uint64_t mask = S - 1;
    auto slot_of = [&](uint64_t k, bool insert) -> uint64_t {
      uint64_t s = mix64(k) & mask;
      for (;;) {
        uint64_t cur = __atomic_load_n(&keys[s], __ATOMIC_RELAXED);
        if (cur == k) return s;
        if (cur == kEmpty) {
          if (!insert) return S;  // not present (cannot happen on the second pass)
          if (__atomic_compare_exchange_n(&keys[s], &cur, k, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED) || cur == k)
            return s;
        }
        s = (s + 1) & mask;
      }
    };
    parallel_for(P, threads, [&](int64_t b, int64_t e, int) {
      for (int64_t p = b; p < e; ++p) atomic_min_u32(&first[slot_of(key(p), true)], static_cast<uint32_t>(p));
    });
    // count, then list, the first occurrences per contiguous chunk (draw order kept)
    const int nt = std::max(1, threads);
    std::vector<int64_t> cnt(nt + 1, 0);
    auto is_first = [&](int64_t p) {
      const uint64_t sl = slot_of(key(p), false);
      return sl < S && first[sl] == static_cast<uint32_t>(p);
    };
    parallel_for(nt, nt, [&](int64_t tb, int64_t te, int) {
      for (int64_t t = tb; t < te; ++t) {
        const int64_t b = P * t / nt, e = P * (t + 1) / nt;
        int64_t c = 0;
        for (int64_t p = b; p < e; ++p) c += is_first(p);
        cnt[t + 1] = c;
      }
    });
    for (int t = 0; t < nt; ++t) cnt[t + 1] += cnt[t];
    if (cnt[nt] >= target || P >= limit) {
      const int64_t take = std::min<int64_t>(target, cnt[nt]);
      kept.assign(static_cast<size_t>(take), 0);
      parallel_for(nt, nt, [&](int64_t tb, int64_t te, int) {
        for (int64_t t = tb; t < te; ++t) {
          int64_t at = cnt[t];
          if (at >= take) continue;
          const int64_t b = P * t / nt, e = P * (t + 1) / nt;
          for (int64_t p = b; p < e && at < take; ++p)
            if (is_first(p)) kept[static_cast<size_t>(at++)] = static_cast<uint32_t>(p);
        }
      });
      *draws = take ? static_cast<int64_t>(kept.back()) + 1 : 0;
      return kept;
    }
    P = std::min(limit, P + P / 2);
  }
}

}  // namespace

struct kgat_synth {
  int64_t n = 0, T = 0, U = 0, E = 0, I = 0, M = 0, K = 0;
  int64_t M_draws = 0, K_draws = 0;  // draws taken to find the M / K distinct triples
  uint64_t seed = 0;
  int threads = 1;
  Range head[4], tail[4];          // per KG relation, entity ids
  std::vector<double> prob;        // alias table over popularity ranks
  std::vector<int32_t> alias;
  std::vector<int32_t> item_perm;  // rank -> item
  std::vector<uint32_t> kept_int, kept_kg;  // kept triple -> its draw index in its stream
  std::vector<uint32_t> deg_user, deg_item, out_r[4], in_r[4];
  // the last built shard
  std::vector<int64_t> rowptr;
  std::vector<int32_t> col;
  std::vector<float> val;

  // interaction draw p of the interaction stream: (user a, item b)
  inline void draw_interaction(int64_t p, int64_t& a, int64_t& b) const {
    a = static_cast<int64_t>(below(draw(seed, p, 0), U));
    const uint64_t k = below(draw(seed, p, 1), I);
    const int64_t rank = unit(draw(seed, p, 2)) < prob[k] ? static_cast<int64_t>(k) : alias[k];
    b = item_perm[rank];
  }
  // KG draw q of the KG stream: (head a, rel, tail b)
  inline void draw_kg(int64_t q, int64_t& a, int32_t& rel, int64_t& b) const {
    rel = static_cast<int32_t>(below(draw(seed, q, 3), 4));
    const Range& h = head[rel];
    a = h.lo + static_cast<int64_t>(below(draw(seed, q, 4), h.size()));
    const Range& t = tail[rel];
    b = std::min<int64_t>(t.lo + static_cast<int64_t>(unit(draw(seed, q, 5)) * static_cast<double>(t.size())), E - 1);
  }
  // distinct keys of the two streams (< 2^63: n < 2^30 is checked at open)
  inline uint64_t interaction_key(int64_t p) const {
    int64_t a, b;
    draw_interaction(p, a, b);
    return static_cast<uint64_t>(a) * static_cast<uint64_t>(I) + static_cast<uint64_t>(b);
  }
  inline uint64_t kg_key(int64_t q) const {
    int64_t a, b;
    int32_t r;
    draw_kg(q, a, r, b);
    return (static_cast<uint64_t>(a) * 4 + static_cast<uint64_t>(r)) * static_cast<uint64_t>(E) + static_cast<uint64_t>(b);
  }

  // kept triple i: (a, rel, b) raw ids -- rel = -1: interaction (user a, item b); else KG (head a, tail b)
  inline void triple(int64_t i, int64_t& a, int32_t& rel, int64_t& b) const {
    if (i < M) {
      draw_interaction(kept_int[i], a, b);
      rel = -1;
      return;
    }
    draw_kg(kept_kg[i - M], a, rel, b);
  }

  // node-id entries of triple i: (row, col, block) x 2
  inline void entries(int64_t i, int64_t* row, int64_t* c, int32_t* blk) const {
    int64_t a, b;
    int32_t r;
    triple(i, a, r, b);
    if (r < 0) {
      row[0] = U + b, c[0] = a, blk[0] = 0;  // user -> item: entry (item, user)
      row[1] = a, c[1] = U + b, blk[1] = 1;  // item -> user
    } else {
      row[0] = U + b, c[0] = U + a, blk[0] = 2 + 2 * r;
      row[1] = U + a, c[1] = U + b, blk[1] = 3 + 2 * r;
    }
  }

  // outdeg of block `blk`'s head node `c` (the entry's column)
  inline uint32_t head_degree(int32_t blk, int64_t c) const {
    if (blk == 0) return deg_user[c];
    if (blk == 1) return deg_item[c - U];
    const int r = (blk - 2) >> 1;
    if ((blk & 1) == 0) return out_r[r][c - U - head[r].lo];
    return in_r[r][c - U - tail[r].lo];
  }

  // pre-coalesce entries of node x's row
  inline int64_t row_entries(int64_t x) const {
    if (x < U) return deg_user[x];
    const int64_t e = x - U;
    int64_t s = e < I ? deg_item[e] : 0;
    for (int r = 0; r < 4; ++r) {
      if (e >= tail[r].lo && e < tail[r].hi) s += in_r[r][e - tail[r].lo];
      if (e >= head[r].lo && e < head[r].hi) s += out_r[r][e - head[r].lo];
    }
    return s;
  }
};

extern "C" {

int kgat_synth_open(int64_t n_nodes, int64_t n_triples, uint64_t seed, double zipf_s, int n_threads,
                    kgat_synth** out) {
  if (!out || n_nodes < 2 || n_triples < 0 || n_nodes >= (int64_t{1} << 30)) return KGAT_ERR_INVALID;
  *out = nullptr;
  kgat_synth* g = new (std::nothrow) kgat_synth();
  if (!g) return KGAT_ERR_INVALID;
  try {
    g->n = n_nodes, g->T = n_triples, g->seed = mix64(seed + 0x51ED2701ull), g->threads = std::max(1, n_threads);
    // sizes as graph.synthetic_ckg
    g->U = std::max<int64_t>(1, static_cast<int64_t>(static_cast<double>(n_nodes) * 0.1));
    g->E = n_nodes - g->U;
    g->I = std::max<int64_t>(1, static_cast<int64_t>(static_cast<double>(g->E) * 0.1));
    g->M = static_cast<int64_t>(static_cast<double>(n_triples) * 0.8);
    g->K = n_triples - g->M;
    const int64_t rest = std::max<int64_t>(4, g->E - g->I);
    int64_t bnd[5];
    for (int k = 0; k < 5; ++k) bnd[k] = g->I + rest * k / 4;
    for (int r = 0; r < 4; ++r) {
      // tails: [bnd[r], bnd[r+1]) clipped to E-1; heads: items, or (r = 3) the IN_CONTEST tail range
      g->tail[r].lo = std::min(bnd[r], g->E - 1);
      g->tail[r].hi = std::max(g->tail[r].lo + 1, std::min(bnd[r + 1], g->E));
      if (r < 3) {
        g->head[r] = Range{0, g->I};
      } else {
        g->head[r].lo = bnd[2];
        g->head[r].hi = std::max(bnd[2] + 1, bnd[3]);
      }
      if (g->head[r].hi > g->E) return delete g, KGAT_ERR_INVALID;  // graph too small for the type ranges
    }
    // Zipf(s) over popularity ranks 1..I: Vose alias table (fp64, deterministic)
    const int64_t I = g->I;
    std::vector<double> w(I);
    double tot = 0.0;
    for (int64_t k = 0; k < I; ++k) tot += (w[k] = std::pow(static_cast<double>(k + 1), -zipf_s));
    g->prob.assign(I, 0.0);
    g->alias.assign(I, 0);
    std::vector<int64_t> small, large;
    for (int64_t k = 0; k < I; ++k) {
      w[k] = w[k] * static_cast<double>(I) / tot;
      (w[k] < 1.0 ? small : large).push_back(k);
    }
    while (!small.empty() && !large.empty()) {
      const int64_t s = small.back(), l = large.back();
      small.pop_back();
      g->prob[s] = w[s];
      g->alias[s] = static_cast<int32_t>(l);
      w[l] = (w[l] + w[s]) - 1.0;
      if (w[l] < 1.0) {
        large.pop_back();
        small.push_back(l);
      }
    }
    for (int64_t k : large) g->prob[k] = 1.0;
    for (int64_t k : small) g->prob[k] = 1.0;
    // rank -> item: Fisher-Yates under a counter hash
    g->item_perm.resize(I);
    for (int64_t k = 0; k < I; ++k) g->item_perm[k] = static_cast<int32_t>(k);
    for (int64_t k = I - 1; k > 0; --k)
      std::swap(g->item_perm[k], g->item_perm[below(draw(g->seed, k, 7), static_cast<uint64_t>(k + 1))]);
    // distinct triples: the first M interaction draws / K KG draws of distinct keys (draw indices
    // are uint32: at most 2^32 - 1 draws per stream)
    const int64_t lim_m = std::min<int64_t>(int64_t{0xFFFFFFFF}, 64 * g->M + 4096);
    const int64_t lim_k = std::min<int64_t>(int64_t{0xFFFFFFFF}, 64 * g->K + 4096);
    g->kept_int = first_distinct(g->M, lim_m, g->threads, [g](int64_t p) { return g->interaction_key(p); },
                                 &g->M_draws);
    g->kept_kg = first_distinct(g->K, lim_k, g->threads, [g](int64_t q) { return g->kg_key(q); }, &g->K_draws);
    g->M = static_cast<int64_t>(g->kept_int.size());
    g->K = static_cast<int64_t>(g->kept_kg.size());
    g->T = g->M + g->K;
    // degrees (pass 1 over every kept triple)
    g->deg_user.assign(g->U, 0);
    g->deg_item.assign(I, 0);
    for (int r = 0; r < 4; ++r) {
      g->out_r[r].assign(g->head[r].size(), 0);
      g->in_r[r].assign(g->tail[r].size(), 0);
    }
    parallel_for(g->T, g->threads, [g](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; ++i) {
        int64_t a, c;
        int32_t r;
        g->triple(i, a, r, c);
        if (r < 0) {
          bump(g->deg_user.data(), a);
          bump(g->deg_item.data(), c);
        } else {
          bump(g->out_r[r].data(), a - g->head[r].lo);
          bump(g->in_r[r].data(), c - g->tail[r].lo);
        }
      }
    });
  } catch (...) {
    delete g;
    return KGAT_ERR_INVALID;
  }
  *out = g;
  return KGAT_OK;
}

void kgat_synth_close(kgat_synth* g) { delete g; }

int kgat_synth_info(const kgat_synth* g, int64_t* info) {
  if (!g || !info) return KGAT_ERR_INVALID;
  const int64_t v[8] = {g->n, g->T, g->U, g->E, g->I, g->M, g->K, g->M_draws + g->K_draws};
  for (int k = 0; k < 8; ++k) info[k] = v[k];
  return KGAT_OK;
}

int kgat_synth_row_offsets(const kgat_synth* g, int64_t* offsets) {
  if (!g || !offsets) return KGAT_ERR_INVALID;
  offsets[0] = 0;
  for (int64_t x = 0; x < g->n; ++x) offsets[x + 1] = offsets[x] + g->row_entries(x);
  return KGAT_OK;
}

int kgat_synth_triples(const kgat_synth* g, const int64_t* idx, int64_t count, int64_t* a, int32_t* rel,
                       int64_t* b) {
  if (!g || count < 0 || (count && (!idx || !a || !rel || !b))) return KGAT_ERR_INVALID;
  for (int64_t k = 0; k < count; ++k) {
    if (idx[k] < 0 || idx[k] >= g->T) return KGAT_ERR_INVALID;
    g->triple(idx[k], a[k], rel[k], b[k]);
  }
  return KGAT_OK;
}

int kgat_synth_shard_build(kgat_synth* g, int64_t lo, int64_t hi, int64_t* nnz) {
  return kgat_synth_shard_build_ex(g, lo, hi, 0, nnz);
}

// transpose = 1: rows [lo, hi) of A^T instead -- the entries of A whose COLUMN lies in [lo, hi),
// keyed by that column (the A^T row) with the A row as their column.  The value of an entry is
// A's (count / outdeg of the head, summed over blocks in block order), so these rows are the
// transpose of the layout's A bit for bit.  A node's A^T row has as many pre-coalesce entries as
// its A row (every triple enters A in both directions), so row_entries sizes both.
int kgat_synth_shard_build_ex(kgat_synth* g, int64_t lo, int64_t hi, int32_t transpose, int64_t* nnz) {
  if (!g || !nnz || lo < 0 || hi < lo || hi > g->n) return KGAT_ERR_INVALID;
  try {
    const int64_t rows = hi - lo;
    std::vector<int64_t> start(rows + 1, 0);
    for (int64_t x = 0; x < rows; ++x) start[x + 1] = start[x] + g->row_entries(lo + x);
    // pass 2: place this shard's entries by row (key = col << 4 | block)
    std::vector<uint64_t> keys(static_cast<size_t>(start[rows]));
    std::vector<int64_t> cursor(start.begin(), start.end() - 1);
    parallel_for(g->T, g->threads, [&](int64_t b, int64_t e, int) {
      int64_t row[2], c[2];
      int32_t blk[2];
      for (int64_t i = b; i < e; ++i) {
        g->entries(i, row, c, blk);
        for (int s = 0; s < 2; ++s) {
          // A: entry (row, col); A^T: the same entry as (col, row) -- the block's head is col
          const int64_t r = transpose ? c[s] : row[s], cc = transpose ? row[s] : c[s];
          if (r < lo || r >= hi) continue;
          const int64_t at = __atomic_fetch_add(&cursor[r - lo], 1, __ATOMIC_RELAXED);
          keys[at] = (static_cast<uint64_t>(cc) << 4) | static_cast<uint64_t>(blk[s]);
        }
      }
    });
    // per row: sort (col, block), count repeats, value per block in fp64, sum blocks in order
    std::vector<int64_t> uniq(rows + 1, 0);
    parallel_for(rows, g->threads, [&](int64_t b, int64_t e, int) {
      for (int64_t x = b; x < e; ++x) {
        uint64_t* k0 = keys.data() + start[x];
        uint64_t* k1 = keys.data() + start[x + 1];
        std::sort(k0, k1);
        int64_t u = 0;
        for (uint64_t* p = k0; p < k1; ++p) u += (p == k0 || (*p >> 4) != (p[-1] >> 4));
        uniq[x + 1] = u;
      }
    });
    g->rowptr.assign(rows + 1, 0);
    for (int64_t x = 0; x < rows; ++x) g->rowptr[x + 1] = g->rowptr[x] + uniq[x + 1];
    g->col.assign(static_cast<size_t>(g->rowptr[rows]), 0);
    g->val.assign(static_cast<size_t>(g->rowptr[rows]), 0.0f);
    parallel_for(rows, g->threads, [&](int64_t b, int64_t e, int) {
      for (int64_t x = b; x < e; ++x) {
        const uint64_t* p = keys.data() + start[x];
        const uint64_t* end = keys.data() + start[x + 1];
        int64_t out = g->rowptr[x] - 1;
        int64_t prev_col = -1;
        double sum = 0.0;
        while (p < end) {
          const uint64_t key = *p;
          int64_t cnt = 0;
          while (p < end && *p == key) ++p, ++cnt;
          const int64_t c = static_cast<int64_t>(key >> 4);
          const int32_t blk = static_cast<int32_t>(key & 15);
          // the block's head: A's column (A) or the A^T row itself (transpose)
          const double v = static_cast<double>(cnt) / static_cast<double>(g->head_degree(blk, transpose ? lo + x : c));
          if (c != prev_col) {
            if (out >= g->rowptr[x]) g->val[out] = static_cast<float>(sum);
            ++out;
            g->col[out] = static_cast<int32_t>(c);
            prev_col = c;
            sum = 0.0;
          }
          sum += v;
        }
        if (out >= g->rowptr[x]) g->val[out] = static_cast<float>(sum);
      }
    });
    *nnz = g->rowptr[rows];
  } catch (...) {
    return KGAT_ERR_INVALID;
  }
  return KGAT_OK;
}

int kgat_synth_shard_copy(kgat_synth* g, int64_t* rowptr, int32_t* col, float* val) {
  if (!g || !rowptr || (!g->col.empty() && (!col || !val))) return KGAT_ERR_INVALID;
  std::copy(g->rowptr.begin(), g->rowptr.end(), rowptr);
  std::copy(g->col.begin(), g->col.end(), col);
  std::copy(g->val.begin(), g->val.end(), val);
  std::vector<int64_t>().swap(g->rowptr);
  std::vector<int32_t>().swap(g->col);
  std::vector<float>().swap(g->val);
  return KGAT_OK;
}

}  // extern "C"

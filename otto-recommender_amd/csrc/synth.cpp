// otto-synth: deterministic OTTO-shaped session generator (host C++ / OpenMP).
//
// Test and benchmark input only -- not on the hot path. Every random draw is a
// pure function of (seed, stream, session, event, field) through a counter-based
// mixer, so any session range can be generated independently (per-rank shards,
// per-file slices) and this container and the GPU box produce bit-identical
// events. Parameters follow SURVEY.md §8(d):
//   * session length  clip(round(LogNormal(ln 6, 1.42)), 2, 500)
//     (fitted to model/w2vec_aids.py:226-229 train stats)
//   * event type      iid p = (0.8985, 0.0780, 0.0235)  (clicks / carts / orders)
//   * timestamps      start ~ U[ts0, ts0 + 28 d); gaps: w.p. 0.95 trunc(LogNormal(ln 45 s, 1.5)),
//                     else U[1 h, 7 d]; int32 seconds as in etl/jsonl_to_parquet.py:28
//   * items           Zipf p(r) ∝ (r + 10)^-0.9 over popularity ranks, ids a fixed
//                     random permutation of ranks; w.p. 0.35 revisit an aid already in the session
//   * exact repeats   w.p. p_dup an event repeats the previous event verbatim
//                     (exercises the df.unique() dedup of model/count_co_events.py:92)
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>
#include <algorithm>
#include <omp.h>

#include "../../include/ottosynth.h"

namespace {

inline uint64_t fmix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
// counter-based draw: one 64-bit value per (seed, stream, a, b)
inline uint64_t draw(uint64_t seed, uint64_t stream, uint64_t a, uint64_t b) {
  uint64_t h = fmix64(seed * 0x9E3779B97F4A7C15ULL + stream);
  h = fmix64(h ^ (a * 0xD1B54A32D192ED03ULL));
  h = fmix64(h ^ (b * 0xAEF17502108EF2D9ULL + 0x632BE59BD9B4E019ULL));
  return h;
}
inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
// standard normal by Box-Muller from two independent draws
inline double normal(uint64_t h1, uint64_t h2) {
  double u1 = u01(h1); if (u1 < 1e-300) u1 = 1e-300;
  double u2 = u01(h2);
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

enum : uint64_t { ST_LEN = 1, ST_START, ST_GAP_KIND, ST_GAP_A, ST_GAP_B, ST_TYPE, ST_REVISIT,
                  ST_REVISIT_PICK, ST_ITEM, ST_DUP, ST_PERM, ST_CENTER, ST_CLUSTER, ST_NOISE };

struct ItemTable {
  uint64_t seed = 0; int64_t n = 0; double off = 0, ex = 0;
  std::vector<double> cdf;      // cumulative, normalised to 1
  std::vector<int32_t> perm;    // rank -> aid
};
std::mutex g_mu;
ItemTable* g_tab = nullptr;

const ItemTable* get_table(const otto_synth_params* p) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_tab && g_tab->seed == p->seed && g_tab->n == p->n_items && g_tab->off == p->zipf_offset &&
      g_tab->ex == p->zipf_exponent)
    return g_tab;
  delete g_tab;
  g_tab = new ItemTable();
  ItemTable& t = *g_tab;
  t.seed = p->seed; t.n = p->n_items; t.off = p->zipf_offset; t.ex = p->zipf_exponent;
  t.cdf.resize(t.n);
  double acc = 0.0;
  for (int64_t r = 0; r < t.n; ++r) { acc += std::pow((double)r + t.off, -t.ex); t.cdf[r] = acc; }
  for (int64_t r = 0; r < t.n; ++r) t.cdf[r] /= acc;
  t.cdf[t.n - 1] = 1.0;
  t.perm.resize(t.n);
  for (int64_t r = 0; r < t.n; ++r) t.perm[r] = (int32_t)r;
  for (int64_t r = t.n - 1; r > 0; --r) {  // Fisher-Yates, counter-based
    uint64_t j = draw(p->seed, ST_PERM, (uint64_t)r, 0) % (uint64_t)(r + 1);
    std::swap(t.perm[r], t.perm[j]);
  }
  return g_tab;
}

inline int32_t session_len(const otto_synth_params* p, int64_t s) {
  double z = normal(draw(p->seed, ST_LEN, (uint64_t)s, 0), draw(p->seed, ST_LEN, (uint64_t)s, 1));
  double x = std::exp(p->len_mu + p->len_sigma * z);
  double r = std::nearbyint(x);
  if (!(r >= p->len_min)) r = p->len_min;  // also catches NaN
  if (r > p->len_max) r = p->len_max;
  return (int32_t)r;
}

}  // namespace

extern "C" {

void otto_synth_default_params(otto_synth_params* p) {
  std::memset(p, 0, sizeof(*p));
  p->seed = 0;
  p->n_items = 1855603;
  p->len_mu = std::log(6.0); p->len_sigma = 1.42; p->len_min = 2; p->len_max = 500;
  p->p_type[0] = 0.8985; p->p_type[1] = 0.0780; p->p_type[2] = 0.0235;
  p->ts0 = 1659304800; p->ts_span = 28 * 86400;
  p->gap_mu = std::log(45.0); p->gap_sigma = 1.5;
  p->p_long_gap = 0.05; p->long_gap_min = 3600; p->long_gap_max = 7 * 86400;
  p->zipf_offset = 10.0; p->zipf_exponent = 0.9;
  p->p_revisit = 0.35; p->p_dup = 0.002;
}

int otto_synth_lengths(const otto_synth_params* p, int64_t s0, int64_t n, int32_t* len) {
  if (!p || !len || n < 0 || p->len_min < 1 || p->len_max < p->len_min) return -1;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) len[i] = session_len(p, s0 + i);
  return 0;
}

int64_t otto_synth_sessions_for_events(const otto_synth_params* p, int64_t s0, int64_t target_events,
                                       int64_t* n_events_out) {
  if (!p || target_events < 0) return -1;
  int64_t tot = 0, s = s0;
  while (tot < target_events) { tot += session_len(p, s); ++s; }
  if (n_events_out) *n_events_out = tot;
  return s - s0;
}

int otto_synth_fill(const otto_synth_params* p, int64_t s0, int64_t n, const int64_t* offsets,
                    int32_t* session, int32_t* aid, int32_t* ts, int8_t* type) {
  if (!p || !offsets || !aid || !ts || !type || n < 0) return -1;
  if (p->n_items < 1 || p->n_items > (int64_t)1 << 30) return -2;
  const ItemTable* tab = get_table(p);
  const double* cdf = tab->cdf.data();
  const int32_t* perm = tab->perm.data();
  const int64_t nit = tab->n;
  const double pc = p->p_type[0], pcc = p->p_type[0] + p->p_type[1];
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = s0 + i;
    const uint64_t us = (uint64_t)s;
    const int64_t b = offsets[i] - offsets[0];
    const int32_t L = (int32_t)(offsets[i + 1] - offsets[i]);
    int64_t t = p->ts0 + (int64_t)(u01(draw(p->seed, ST_START, us, 0)) * (double)p->ts_span);
    for (int32_t k = 0; k < L; ++k) {
      const uint64_t uk = (uint64_t)k;
      const int64_t e = b + k;
      if (session) session[e] = (int32_t)s;
      if (k > 0 && u01(draw(p->seed, ST_DUP, us, uk)) < p->p_dup) {  // verbatim repeat
        aid[e] = aid[e - 1]; ts[e] = ts[e - 1]; type[e] = type[e - 1];
        continue;
      }
      if (k > 0) {
        int64_t gap;
        if (u01(draw(p->seed, ST_GAP_KIND, us, uk)) < p->p_long_gap) {
          double u = u01(draw(p->seed, ST_GAP_A, us, uk));
          gap = p->long_gap_min + (int64_t)(u * (double)(p->long_gap_max - p->long_gap_min + 1));
        } else {
          double z = normal(draw(p->seed, ST_GAP_A, us, uk), draw(p->seed, ST_GAP_B, us, uk));
          double g = std::exp(p->gap_mu + p->gap_sigma * z);
          if (g > 1e9) g = 1e9;
          gap = (int64_t)g;  // truncation: ~0.6% zero gaps at (ln 45, 1.5)
        }
        t += gap;
        if (t > 2147483647LL) t = 2147483647LL;
      }
      ts[e] = (int32_t)t;
      double ut = u01(draw(p->seed, ST_TYPE, us, uk));
      type[e] = (int8_t)(ut < pc ? 0 : (ut < pcc ? 1 : 2));
      if (k > 0 && u01(draw(p->seed, ST_REVISIT, us, uk)) < p->p_revisit) {
        uint64_t j = draw(p->seed, ST_REVISIT_PICK, us, uk) % (uint64_t)k;
        aid[e] = aid[b + (int64_t)j];
      } else {
        double u = u01(draw(p->seed, ST_ITEM, us, uk));
        int64_t r = (int64_t)(std::upper_bound(cdf, cdf + nit, u) - cdf);
        if (r >= nit) r = nit - 1;
        aid[e] = perm[r];
      }
    }
  }
  return 0;
}

int otto_synth_embeddings(uint64_t seed, int64_t n, int dim, int n_clusters, float* out) {
  // Item embeddings for config 3: row i = vocabulary rank i (gensim's
  // index_to_key is frequency-sorted, model/w2vec_aids.py:198-199). A mixture of n_clusters
  // Gaussian clusters; the vector norm is 0.5 + 3 (1 - i/n)^2, so rarer items sit closer to
  // the origin (model/w2vec_aids.py:144-148).
  if (!out || n < 1 || dim < 1 || n_clusters < 1) return -1;
  std::vector<float> cen((size_t)n_clusters * dim);
  for (int j = 0; j < n_clusters; ++j)
    for (int d = 0; d < dim; ++d)
      cen[(size_t)j * dim + d] = (float)normal(draw(seed, ST_CENTER, (uint64_t)j, 2 * (uint64_t)d),
                                               draw(seed, ST_CENTER, (uint64_t)j, 2 * (uint64_t)d + 1));
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const int c = (int)(draw(seed, ST_CLUSTER, (uint64_t)i, 0) % (uint64_t)n_clusters);
    float* v = out + i * dim;
    double ss = 0;
    for (int d = 0; d < dim; ++d) {
      const double z = normal(draw(seed, ST_NOISE, (uint64_t)i, 2 * (uint64_t)d),
                              draw(seed, ST_NOISE, (uint64_t)i, 2 * (uint64_t)d + 1));
      const double x = cen[(size_t)c * dim + d] + 0.7 * z;
      v[d] = (float)x;
      ss += x * x;
    }
    const double f = 1.0 - (double)i / (double)n;
    const double scale = (0.5 + 3.0 * f * f) / std::sqrt(ss > 0 ? ss : 1.0);
    for (int d = 0; d < dim; ++d) v[d] = (float)(v[d] * scale);
  }
  return 0;
}

int otto_synth_item_rank(const otto_synth_params* p, int32_t* rank_of_aid) {
  // inverse of the rank -> aid permutation (aid -> popularity rank), used by the
  // embedding generator so that vector norms follow item frequency
  if (!p || !rank_of_aid) return -1;
  const ItemTable* tab = get_table(p);
  for (int64_t r = 0; r < tab->n; ++r) rank_of_aid[tab->perm[r]] = (int32_t)r;
  return 0;
}

}  // extern "C"

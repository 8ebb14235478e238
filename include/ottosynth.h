/* otto-synth: deterministic OTTO-shaped synthetic sessions (host side, test/bench input).
 *
 * Not part of the reference interface: the reference reads real OTTO parquet files
 * (etl/jsonl_to_parquet.py:23-29, schema session:i32, aid:i32, ts:i32 seconds, type:i8).
 * This generator produces the same columns in CSR form so that benchmarks and parity
 * tests can run without the dataset. See SURVEY.md §8(d) for the distribution spec. */
#ifndef OTTOSYNTH_H
#define OTTOSYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t seed;
  int64_t n_items;
  double len_mu, len_sigma;
  int32_t len_min, len_max;
  double p_type[3];
  int64_t ts0, ts_span;
  double gap_mu, gap_sigma;
  double p_long_gap;
  int64_t long_gap_min, long_gap_max;
  double zipf_offset, zipf_exponent;
  double p_revisit;
  double p_dup;
} otto_synth_params;

void otto_synth_default_params(otto_synth_params* p);
/* session lengths of sessions [s0, s0+n) */
int otto_synth_lengths(const otto_synth_params* p, int64_t s0, int64_t n, int32_t* len);
/* number of sessions starting at s0 needed to reach >= target_events events */
int64_t otto_synth_sessions_for_events(const otto_synth_params* p, int64_t s0, int64_t target_events,
                                       int64_t* n_events_out);
/* fill events of sessions [s0, s0+n); offsets[0..n] are CSR offsets (offsets[0] maps to
 * output index 0); session may be NULL */
int otto_synth_fill(const otto_synth_params* p, int64_t s0, int64_t n, const int64_t* offsets,
                    int32_t* session, int32_t* aid, int32_t* ts, int8_t* type);
/* item embeddings [n x dim] fp32, row i = frequency rank i (config 3 of SURVEY.md §8(d)) */
int otto_synth_embeddings(uint64_t seed, int64_t n, int dim, int n_clusters, float* out);
/* aid -> popularity rank (inverse of the generator's rank -> aid permutation) */
int otto_synth_item_rank(const otto_synth_params* p, int32_t* rank_of_aid);

#ifdef __cplusplus
}
#endif
#endif

/* ottohip.h -- C-ABI of libottohip.so, the MI355X (gfx950) co-visitation engine.
 *
 * This is the drop-in boundary for the hot path of nicolaivicol/otto-recommender. The
 * reference has no FFI: its boundary is a set of Python functions on polars DataFrames
 * (SURVEY.md §8b). Each entry point below names the reference function it replaces; the
 * Python host layer (otto-recommender_amd/covis.py) binds them with ctypes and keeps the
 * reference's names, arguments and file contracts. See INTEGRATION.md for the bindings.
 *
 * Conventions
 *   - Buffers are DEVICE pointers unless a field says "host". The caller owns inputs;
 *     the library owns results (ottohip_table) and its workspace (ottohip_ctx).
 *   - Every int-returning call returns 0 on success and a negative OTTOHIP_E* code on
 *     failure; ottohip_last_error() gives a thread-local message.
 *   - One host thread per context; calls are ordered on the given stream (hipStream_t
 *     passed as void*, NULL = default stream). A context is bound to one device.
 */
#ifndef OTTOHIP_H
#define OTTOHIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum {
  OTTOHIP_OK = 0,
  OTTOHIP_EINVAL = -1,    /* bad argument / shape */
  OTTOHIP_ERANGE = -2,    /* aid, type or ts outside the supported range */
  OTTOHIP_ENOMEM = -3,    /* device allocation failed */
  OTTOHIP_EHIP = -4,      /* HIP runtime error */
  OTTOHIP_ELIMIT = -5,    /* input exceeds an engine limit (documented in DESIGN.md) */
};

typedef struct ottohip_ctx ottohip_ctx;
typedef struct ottohip_table ottohip_table;

/* One co-visitation rule: pairs (i, j) of one session with type_i == this_type,
 * type_j in next_type_mask (bit t = type t) and |ts_j - ts_i| <= max_abs_dt.
 * Mirrors config.MAP_NAME_COUNT_TYPE / MAP_MAX_TIME_TO_NEXT (config.py:43-49, 81-88). */
typedef struct {
  int32_t this_type;
  uint32_t next_type_mask;
  int32_t max_abs_dt;
} ottohip_rule;

/* Session-sorted CSR events: session s owns rows [session_offsets[s], session_offsets[s+1])
 * of aid/ts/type; session_offsets[0] == 0. Schema of etl/jsonl_to_parquet.py:23-29.
 * file_session_bounds (HOST, n_files+1 entries) partitions sessions into the reference's
 * parquet files; per-file counts drive the merge rule of count_co_events.py:131-132. */
typedef struct {
  const int64_t* session_offsets;
  int64_t n_sessions;
  const int32_t* aid;
  const int32_t* ts;
  const int8_t* type;
  int64_t n_events;
  const int64_t* file_session_bounds; /* host */
  int32_t n_files;
} ottohip_events;

/* Reference-schema parquet rows -> the CSR above, on the device. Replaces the host-side read of
 * model/count_co_events.py:81,91 (pl.read_parquet of a file written by etl/jsonl_to_parquet.py:59-84,
 * schema :23-29); the caller decodes the parquet columns and uploads them raw (device, n_rows).
 * Rows whose sessions form contiguous runs with distinct ids keep their order (the reference's files):
 * the sessions, and session_ids, are then in FILE order, which need not be ascending (*reordered = 0);
 * otherwise the rows are stably sorted by session id and session_ids ascend (*reordered = 1). Writes session_offsets
 * [n_sessions + 1] = offset_base + row start (so files can be appended into one CSR),
 * session_ids [n_sessions] (may be NULL) and the aid / ts / type columns (may alias the inputs).
 * Capacity: n_rows + 1 offsets, n_rows ids. OTTOHIP_ELIMIT if n_rows >= 2^32. */
int ottohip_events_csr(ottohip_ctx* ctx, const int32_t* session, const int32_t* aid, const int32_t* ts,
                       const int8_t* type, int64_t n_rows, int64_t offset_base, int64_t* session_offsets,
                       int32_t* session_ids, int32_t* aid_out, int32_t* ts_out, int8_t* type_out,
                       int64_t* n_sessions, int* reordered, void* stream);

/* The same over n_files files appended in one table (file f = rows [file_row_starts[f],
 * file_row_starts[f+1]), HOST array of n_files + 1 with file_row_starts[0] == 0): one pass when the
 * run heads ascend strictly over all files (the reference's files), else file by file as above.
 * file_session_bounds (HOST out, n_files + 1) = each file's first session, the last entry the
 * session count: the ottohip_events.file_session_bounds of the result. */
int ottohip_events_csr_files(ottohip_ctx* ctx, const int32_t* session, const int32_t* aid, const int32_t* ts,
                             const int8_t* type, int n_files, const int64_t* file_row_starts,
                             int64_t* session_offsets, int32_t* session_ids, int32_t* aid_out, int32_t* ts_out,
                             int8_t* type_out, int64_t* file_session_bounds, int* reordered, void* stream);

typedef struct {
  int32_t min_dt;   /* config.MIN_TIME_TO_NEXT (-86400), count_co_events.py:33-36 */
  int32_t max_dt;   /* config.MAX_TIME_TO_NEXT (+86400) */
  int32_t n_items;  /* aid range [0, n_items); OTTO: 1855603 */
  int32_t dedup;    /* 1 = df.unique() first (count_co_events.py:92) */
  int32_t sym;      /* ottohip_covis_emit / ottohip_covis_reduce_received only: 1 = a symmetric rule (click_to_click,
                       cart_to_cart, buy_to_buy: count_co_events.py:64-71 with the window symmetric in dt) sends and
                       stores each unordered pair once, its mirror produced by the table's readers; both sides of
                       one exchange must agree, and key cuts (ottohip_file_opts lo / hi) need 0. The other count
                       calls decide this themselves. */
} ottohip_covis_params;

/* per-rule statistics of a count table */
typedef struct {
  int64_t n_rows;          /* distinct (aid, aid_next) over all files */
  int64_t n_pairs;         /* qualifying ordered pairs = sum of counts */
  int64_t file_rows;       /* sum over files of per-file distinct rows (N of :117) */
  int64_t file_rows_ge2;   /* same, per-file rows with count >= 2 (after :131-132) */
} ottohip_rule_stats;

int ottohip_ctx_create(int device, ottohip_ctx** out);
void ottohip_ctx_destroy(ottohip_ctx* ctx);
const char* ottohip_last_error(void);
/* release the context's workspace and spare table buffers (device memory back to the runtime);
 * the next call re-allocates what it needs. Live tables are not affected. */
int ottohip_ctx_trim(ottohip_ctx* ctx);
/* phase timing (HIP events on the call's stream): enable, then read after a call */
int ottohip_ctx_set_timing(ottohip_ctx* ctx, int enable);
int ottohip_ctx_timing(ottohip_ctx* ctx, int idx, const char** name, float* ms, double* bytes);

/* Co-visitation counts for all rules over all files in one pass.
 * Replaces the per-file stage of count_co_events_all_files (model/count_co_events.py:80-100:
 * unique :92 + self_merge_big_df :41-57 + count_co_events :60-77) and the cross-file
 * groupby of concat_files_w_stats (:168). For every (rule, aid, aid_next) the table holds
 *   count     = sum over files of the per-file count          (all rows)
 *   count_ge2 = sum over files of per-file counts that are >= 2 (MIN_COUNT_IN_PART rule)
 * With n_files == 1 the table IS the reference's per-file output of :94. */
int ottohip_covis_count(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules,
                        int n_rules, const ottohip_covis_params* params, ottohip_table** out,
                        void* stream);
/* Per-file options of one rule, for concat_files_w_stats' part-wise branch by rows
 * (model/count_co_events.py:136-158: part i = rows [i * rows_part, (i + 1) * rows_part) of the
 * concatenation of the per-file tables, each file's table in (aid, aid_next) order here):
 *   - a row slice of a boundary file is a key range of its ordered table, key = aid << 32 | aid_next:
 *     the rule's pairs of file lo_file with key < lo_key and of file hi_file with key >= hi_key are
 *     cut before they are counted (-1 = no cut; the file ids of the call: local index, or the
 *     file_ids / global ids of the multi-GPU calls);
 *   - file_rows / file_rows_ge2 (HOST out, n_files entries, n_files <= 1024, may be NULL): per file,
 *     the rule's rows after the cuts and those with per-file count >= 2 (the N of :117 / :131 per file). */
typedef struct {
  int32_t rule;      /* index into the call's rules */
  int32_t lo_file;
  int32_t hi_file;
  int32_t n_files;
  uint64_t lo_key;
  uint64_t hi_key;
  int64_t* file_rows;
  int64_t* file_rows_ge2;
  int32_t keep_words; /* 1: the table keeps the count's emitted pair words and rows (device memory, ~4 B per stored
                         pair; freed with the table) for ottohip_table_count_parts */
} ottohip_file_opts;
int ottohip_covis_count_opts(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules, int n_rules,
                             const ottohip_covis_params* params, const ottohip_file_opts* opts, ottohip_table** out,
                             void* stream);
/* All parts of concat_files_w_stats' branch (2) (model/count_co_events.py:136-166) for ONE rule from
 * ONE count (replaces a count per part with ottohip_file_opts key cuts). Part i is rows
 * [i * rows_part, (i + 1) * rows_part) of the concatenation of the per-file tables, each in (aid,
 * aid_next) order, so a pair of file f with key k = aid << 32 | aid_next belongs to part
 * first_part[f], or first_part[f] + 1 when f holds a cut (cut_file[c] == f) and k >= cut_key[c] (one
 * cut per file; the host falls back to per-part counts otherwise). The table's rows are (part, aid,
 * aid_next) with count / count_ge2 summed over the part's files only; a row's rule index IS its part
 * (ottohip_table_finalize(t, part, ...) orders one part; ottohip_table_stats(t, part) holds the part's
 * rows and pairs). n_rules == 1, n_files <= 1024, n_parts <= 254, n_cuts <= 64, n_items <= 2^24. */
typedef struct {
  int32_t n_files;           /* the call's files */
  int32_t n_parts;
  const int32_t* first_part; /* HOST [n_files] */
  int32_t n_cuts;
  const int32_t* cut_file;   /* HOST [n_cuts] */
  const uint64_t* cut_key;   /* HOST [n_cuts] */
} ottohip_part_opts;
int ottohip_covis_count_parts(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules, int n_rules,
                              const ottohip_covis_params* params, const ottohip_part_opts* parts, ottohip_table** out,
                              void* stream);
/* ottohip_covis_count_parts without counting again: the part-tagged table of `rule` (an index of t's rules) re-folded
 * from the words t kept (ottohip_file_opts.keep_words; the count's file ids, parts as above). A symmetric rule's
 * stored row (a, b), a <= b, yields its mirror (b, a) as an explicit row with the mirror's own part (a cut file's
 * key comparison differs between the two orders): the result is non-symmetric, its slots are not in aid order,
 * and ottohip_table_part_heads takes it as such. Other rules' words in the rule's rows are skipped. */
int ottohip_table_count_parts(ottohip_ctx* ctx, const ottohip_table* t, int rule, const ottohip_part_opts* parts,
                              ottohip_table** out, void* stream);
/* Heads of every part of a ottohip_covis_count_parts table (:155-162 for all parts at once): per part p,
 * among its rows with v >= min_count (v = count_ge2 if use_ge2 else count), the first max_rows_part in
 * (v desc, aid asc, aid_next asc) order, selected by histograms (no sort). Written to out_records
 * (device, cap records of 16 B: {aid, aid_next, v, 0}, the ottohip_table_from_records layout, rule 0) in
 * no particular order; *n_out = records. n_parts <= 32. OTTOHIP_ELIMIT: a part's cut falls on a count
 * >= 65535 (the host orders that part with ottohip_table_finalize instead) or cap is too small. */
int ottohip_table_part_heads(ottohip_ctx* ctx, const ottohip_table* t, int n_parts, int use_ge2, int32_t min_count,
                             int64_t max_rows_part, void* out_records, int64_t cap, int64_t* n_out, void* stream);
/* keys (HOST out [n_idx]) = (aid << 32 | aid_next) of rows idx[i] (HOST) of one rule's rows in
 * (aid, aid_next) order; use_ge2: only rows with per-file count >= 2 (count_ge2 > 0). With a one-file
 * table these are the boundary keys of a row slice (ottohip_file_opts). OTTOHIP_ERANGE: idx >= rows. */
int ottohip_table_keys_at(ottohip_ctx* ctx, const ottohip_table* t, int rule, int use_ge2, const int64_t* idx,
                          int n_idx, uint64_t* keys, void* stream);
/* ottohip_table_keys_at for rules (parts) 0 .. n_parts - 1 of a part-mode table in one pass over its slots (the
 * boundary keys of every boundary file from one ottohip_covis_count_parts table with one part per file,
 * model/count_co_events.py:136-139 / :94): idx (HOST) holds n_idx[0] indices of part 0, then n_idx[1] of part 1,
 * ...; keys (HOST out) likewise. Tables whose parts are symmetric or not in aid order, or n_parts > 16, take
 * ottohip_table_keys_at per part. OTTOHIP_ERANGE: an index >= its part's rows. */
int ottohip_table_keys_at_parts(ottohip_ctx* ctx, const ottohip_table* t, int n_parts, int use_ge2,
                                const int64_t* idx, const int32_t* n_idx, uint64_t* keys, void* stream);
int ottohip_table_stats(const ottohip_table* t, int rule, ottohip_rule_stats* st);
/* copy one rule's rows (unordered) into caller device buffers of n_rows entries;
 * any output pointer may be NULL */
int ottohip_table_copy(const ottohip_table* t, int rule, int32_t* aid, int32_t* aid_next,
                       uint32_t* count, uint32_t* count_ge2, void* stream);
void ottohip_table_free(ottohip_table* t);

/* Final merge of concat_files_w_stats (model/count_co_events.py:103-181) for one rule:
 * pick count or count_ge2 (the per-file filter applies iff click_rule && file_rows > 1e8),
 * keep count >= min_count (MIN_COUNT_TO_SAVE, config.py:56-62), order by count desc with
 * the deterministic tie-break (aid asc, aid_next asc), keep the first max_rows rows
 * (MAX_CO_EVENT_PAIRS_TO_SAVE_DISK). Writes up to max_rows rows; *n_out = rows written.
 * Returns OTTOHIP_ELIMIT if the reference would take its part-wise branch (:135-166) on this
 * table: the host layer runs that branch as whole-file parts (covis.concat_files_w_stats_fused
 * and, sharded, dist.concat_files_w_stats_sharded), each part counted and finalized with this
 * call. OTTOHIP_EINVAL if the per-file filter applies and min_count_in_part != 2 (the table's
 * count_ge2 column is accumulated with the per-file threshold 2 of config.py:63). */
typedef struct {
  int32_t click_rule;        /* 'click_to' in name */
  int32_t min_count_in_part; /* MIN_COUNT_IN_PART (2) */
  int32_t min_count;         /* MIN_COUNT_TO_SAVE[name] */
  int64_t max_rows;          /* MAX_CO_EVENT_PAIRS_TO_SAVE_DISK */
  int64_t filter_rows;       /* 100_000_000 threshold of :131 */
  int64_t max_rows_groupby;  /* MAX_ROWS_POLARS_GROUPBY (3e8) of :135 */
} ottohip_merge_params;
int ottohip_table_finalize(ottohip_ctx* ctx, const ottohip_table* t, int rule,
                           const ottohip_merge_params* mp, int32_t* aid, int32_t* aid_next,
                           int32_t* count, int64_t* n_out, void* stream);

/* concat_files_w_stats (model/count_co_events.py:103-181) over n_tables finished tables given as
 * columns (device; n_rows HOST [n_tables]) concatenated in order: the per-file tables of one
 * folder (files_stats=None, :114) or the two thresholded folder tables of the train+test merge
 * (A7, :218-226, files_stats=[train, test]). With N = total rows:
 *   (1) click_rule && N > filter_rows && !loaded_from_cache: drop rows with count < min_count_in_part;
 *   (2) rows > max_rows_groupby && !loaded_from_cache: ceil(rows / optim_rows) slices of
 *       ceil(rows / n_parts) consecutive rows, each groupby-sum -> count >= min_count_in_part ->
 *       count desc -> head(int(max_rows_groupby / rows * optim_rows)), concatenated;
 *   (3) groupby-sum -> count >= min_count -> count desc -> head(max_rows).
 * Row order inside a table is the caller's (the reference's slices follow file row order);
 * ties at every sort are (aid asc, aid_next asc). Output capacity min(N, max_rows) rows. */
int ottohip_concat_tables(ottohip_ctx* ctx, int n_tables, const int32_t* const* aid, const int32_t* const* aid_next,
                          const uint32_t* const* count, const int64_t* n_rows, int32_t n_items,
                          const ottohip_merge_params* mp, int64_t optim_rows, int loaded_from_cache,
                          int32_t* out_aid, int32_t* out_aid_next, int32_t* out_count, int64_t* n_out, void* stream);
/* Order-independent digest of one rule's rows, for full-size parity checks (out HOST [5], u64
 * wrapping sums over rows): sum mix(key, 1) * count, sum mix(key, 2) * count_ge2, sum count,
 * sum count_ge2, rows; key = rule << 48 | aid << 24 | aid_next, mix = the splitmix64 finaliser of
 * key ^ seed. The CPU oracle computes the first four from per-file tables without a merge
 * (they are linear over files: oracle/covis_oracle.c oracle_count_files_omp). */
int ottohip_table_digest(ottohip_ctx* ctx, const ottohip_table* t, int rule, uint64_t* out, void* stream);
/* Histogram of (x[i] >> shift) & mask over i in [lo, hi) of a device array whose equal keys are
 * contiguous (e.g. the count column of a finalize output, or its aid column inside one count):
 * hist (device, n_bins u64) is overwritten. The sharded finalize all-reduces these to find the
 * global head(max_rows) cut. OTTOHIP_ERANGE if a key >= n_bins. */
int ottohip_run_hist(ottohip_ctx* ctx, const int32_t* x, int64_t lo, int64_t hi, int shift, uint32_t mask,
                     int64_t n_bins, uint64_t* hist, void* stream);

/* R1: per-aid top-first_n of a final co-visitation table with the reference's features
 * (get_df_count_for_co_event_type, model/retrieve.py:18-63). Input: the table in FILE order
 * (device, n rows; row position drives perc_pop). Outputs (device, capacity n): rows with
 * rank <= first_n in (aid asc, rank asc) order; *n_out = rows written.
 *   count_pop = Int16(min((c - min) / (q - min), 1) * 1e4), q = 0.9999 quantile ('nearest')
 *   perc_pop  = Int16(row_nr / n * 1e4), row_nr 1-based file position
 *   rank      = ordinal rank of count desc within aid (ties: file order)
 *   count_rel = Int8(c / max count of the aid * 100) */
int ottohip_topk_per_aid(ottohip_ctx* ctx, const int32_t* aid, const int32_t* aid_next, const int32_t* count,
                         int64_t n, int32_t n_items, int first_n, int32_t* out_aid, int32_t* out_aid_next,
                         int32_t* out_count, int16_t* out_count_pop, int16_t* out_perc_pop, int16_t* out_rank,
                         int8_t* out_count_rel, int64_t* n_out, void* stream);

/* ---- Config-5 candidate generation (R3-R6, R8 order) and recall (R9) ----------------------
 * Candidate columns of retrieve_and_gen_feats (model/retrieve.py:422-657) for every session of
 * a session-sorted event table (raw rows, no dedup: :477 takes the file as read). Sources per
 * aid are CSR lists built with ottohip_lists_build:
 *   q = 0..4 : R1 top-N lists of the 5 co-count tables (CO_EVENTS_TO_COUNT order), rank = R1 rank
 *   q = 5, 6 : kNN lists of the all-types and carts/orders Word2Vec models, rank = rank_w2vec
 * pop_off / pop_aid: per dense cluster index, the aids whose min cl50 rank <= 20 (C3);
 * session_cl: dense cluster index per session (-1 = none). Output per session (CSR): aid_next,
 * ts_order_aid (999 for popularity-only rows) and flags (bit i = i-th of src_self,
 * src_click_to_click, src_click_to_cart_or_buy, src_cart_to_cart, src_cart_to_buy,
 * src_buy_to_buy, src_w2vec_all, src_w2vec_1_2, src_pop_cl50), rows sorted by
 * (ts_order_aid, aid_next). Ordinal-rank ties: aid ascending (deterministic choice). */
typedef struct {
  const uint32_t* off[7];   /* [n_items + 1] or NULL (source absent) */
  const int32_t* nxt[7];
  const int16_t* rank[7];
  int32_t n_items;
  const uint32_t* pop_off;  /* [n_clusters + 1] or NULL */
  const int32_t* pop_aid;
  int32_t n_clusters;
  int32_t max_list_total;   /* max over aids of the summed list lengths (<= 127) */
} ottohip_cand_lists;
typedef struct ottohip_candidates ottohip_candidates;
/* rows (key, nxt, rank) -> CSR by key, stable: out_off [n_keys + 1], out_nxt / out_rank [n] */
int ottohip_lists_build(ottohip_ctx* ctx, const int32_t* key, const int32_t* nxt, const int16_t* rank, int64_t n,
                        int32_t n_keys, uint32_t* out_off, int32_t* out_nxt, int16_t* out_rank, void* stream);
int ottohip_candidates_generate(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions,
                                const int32_t* aid, const int32_t* ts, const int8_t* type,
                                const ottohip_cand_lists* lists, const int32_t* session_cl,
                                ottohip_candidates** out, void* stream);
int ottohip_candidates_info(const ottohip_candidates* c, int64_t* n_sessions, int64_t* n_cand);
int ottohip_candidates_copy(const ottohip_candidates* c, uint64_t* off, int32_t* aid_next, int16_t* ts_order,
                            uint16_t* flags, void* stream);
/* the candidates' own device arrays (valid until ottohip_candidates_free; read-only): a zero-copy view for
 * consumers on the device (R7 reads off / aid_next in place of a ottohip_candidates_copy of 8 B per candidate) */
int ottohip_candidates_view(const ottohip_candidates* c, const uint64_t** off, const int32_t** aid_next,
                            const int16_t** ts_order, const uint16_t** flags);
void ottohip_candidates_free(ottohip_candidates* c);
/* R9 (model/eval_retrieved.py:45-118) for the candidates whose flags intersect src_mask (0 = all):
 * labels per type t as CSR lab_off[t * (n_sessions + 1) + s] into lab_aid (unique per session/type).
 * sums_out[t * 5 + {0..4}] = sum over sessions of min(hit@20, max_k), min(hit@100, max_k),
 * min(hit@200, max_k), min(hit@all, max_k), min(true, max_k). */
/* The label CSR ottohip_candidates_recall reads, built on the device from the label rows (session, aid,
 * type; device, n rows; the test labels model/eval_retrieved.py:59-64 joins): per type t and session
 * s (the index of its id in session_ids, device [n_sessions], any order) the unique aids, ascending.
 * lab_off (device, 3 * (n_sessions + 1)) = global positions in lab_aid (device, capacity n); rows of
 * unknown sessions or types outside {0, 1, 2} are dropped; *n_out = labels kept. */
int ottohip_labels_csr(ottohip_ctx* ctx, const int32_t* session_ids, int64_t n_sessions, const int32_t* session,
                       const int32_t* aid, const int8_t* type, int64_t n, int64_t* lab_off, int32_t* lab_aid,
                       int64_t* n_out, void* stream);
int ottohip_candidates_recall(ottohip_ctx* ctx, const ottohip_candidates* c, const int64_t* lab_off,
                              const int32_t* lab_aid, uint32_t src_mask, int max_k, int64_t* sums_out, void* stream);

/* ---- Pop-cluster source (C1-C3) and session-item similarity (R7) -------------------------
 * C1 compute_sessions_embeddings (model/kmeans_sessions.py:40-86): per session
 *    round6(sum w e_aid / sum w), w = f32(max(0.1, 1 - (max_ts - ts)/259200) * {0.1,0.3,0.6}[type]);
 *    row_of_aid maps an aid to its embedding row (-1 = no embedding: adds 0, keeps its weight).
 *    out: [n_sessions x dim] f32. fp32 accumulation in event order (polars' order is unspecified). */
int ottohip_session_embeddings(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions,
                               const int32_t* aid, const int32_t* ts, const int8_t* type, const int32_t* row_of_aid,
                               int32_t n_aid_map, const float* emb, int dim, float* out, void* stream);
/* C2 KMeans (model/kmeans_sessions.py:140-171): one Lloyd iteration on X [n x dim] with centroids
 * [k x dim] updated in place (empty clusters keep theirs); *shift2 = squared centroid shift (the
 * sklearn / dask-ml convergence quantity). Sums are 2^-24 fixed point: order-independent. k <= 64. */
int ottohip_kmeans_step(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* centroids, int k,
                        int32_t* labels, double* shift2, double* inertia, void* stream);
int ottohip_kmeans_assign(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids, int k,
                          int32_t* labels, double* inertia, void* stream);
/* The Lloyd iteration in parts, for sklearn's _kmeans_single_lloyd (KMeans(init='random',
 * n_init='auto'), model/kmeans_sessions.py:152-159) and for row-sharded KMeans (SURVEY.md §8(e):
 * the host all-reduces sums / counts between partial and update):
 *   partial   E-step on this rank's rows: labels (in: previous, out: nearest centroid, ties to the
 *             lowest index), sums (device k*dim, 2^-24 fixed point) and counts (device k) of the rows
 *             per label (overwritten), *inertia, *n_changed = rows whose label changed;
 *   update    centroids = sums / counts for clusters with counts > 0, *shift2 = squared shift;
 *   farthest  the m rows farthest from their labelled centroid (rows / d2 HOST, distance desc);
 *   relocate  _relocate_empty_clusters_dense on the sums: vector j (vecs, device m*dim) leaves cluster
 *             old_new[2j] and becomes the only member of the empty cluster old_new[2j+1] (HOST);
 *   inertia   sum of |x - centroid[label]|^2 for the given labels. */
int ottohip_kmeans_partial(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids, int k,
                           int32_t* labels, int64_t* sums, int64_t* counts, double* inertia, int64_t* n_changed,
                           void* stream);
int ottohip_kmeans_update(ottohip_ctx* ctx, float* centroids, const int64_t* sums, const int64_t* counts, int k,
                          int dim, double* shift2, void* stream);
/* partial + update of one GPU in a single call with one device->host copy (sklearn 1.2
 * _kmeans_single_lloyd, model/kmeans_sessions.py:152-159): out (HOST double[4]) = inertia, changed
 * labels, shift^2, empty clusters. sums / counts are INCREMENTAL: on entry they hold the exact
 * fixed-point sums / counts of the rows under `labels` (all zero with labels = -1 at the start of a
 * run) and on return those of the new labels (only rows whose label changed are moved). When a
 * cluster is empty the centroids are NOT updated (out[2] = -1): relocate on a copy of sums /
 * counts, then update (sklearn relocates before the M-step). */
int ottohip_kmeans_lloyd_iter(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* centroids, int k,
                              int32_t* labels, int64_t* sums, int64_t* counts, double* out, void* stream);
/* Half-precision rows of a KMeans matrix (C2's E-step reads 208 B per row instead of 400 at dim 100): f16
 * copies of X's rows and their exact f32 squared norms are kept in the context, and lloyd_steps on this same X
 * (pointer, n, dim) scores with them; rows whose two best clusters are too close for the f16 scores go to the
 * exact f32 kernel, so labels are those of the f32 E-step. X must not change until detach_half (or ctx_trim).
 * Replaces nothing in the reference (sklearn's float64 Lloyd, model/kmeans_sessions.py:152-159): a device
 * data-layout step of the same labels. OTTOHIP_KM_H16=0 ignores the attached rows. */
int ottohip_kmeans_attach_half(ottohip_ctx* ctx, const float* X, int64_t n, int dim, void* stream);
int ottohip_kmeans_detach_half(ottohip_ctx* ctx);
/* Up to max_steps lloyd_iter steps with a single device->host copy: after each step the device
 * applies sklearn's stop checks (no label changed; shift^2 <= tol; an empty cluster, which leaves
 * the centroids untouched for the host's relocation) and the later steps do nothing. out (HOST
 * double[6]) = out[0..3] of the last step run, steps run, stop reason (0 none, 1 no label changed,
 * 2 shift^2 <= tol, 3 empty cluster). Shapes the MFMA E-step does not take run one step. */
int ottohip_kmeans_lloyd_steps(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* centroids, int k,
                               int32_t* labels, int64_t* sums, int64_t* counts, int max_steps, double tol,
                               double* out, void* stream);
/* lloyd_steps for TWO independent runs (two n_init runs of :152-159) in lockstep: one read of X per step
 * scores both (the step is bound by the X stream). centroids / labels / sums / counts are HOST arrays
 * of the two runs' device pointers, max_steps (HOST int[2]) the step budget of each run (0: the run sits
 * out); out (HOST double[12]) = the 6 values of lloyd_steps per run. Each
 * run's labels, centres, stop step and reason equal lloyd_steps on that run alone (no distance bounds
 * here). OTTOHIP_ELIMIT for shapes outside the pair kernel (32 < k <= 64, dim <= 112): run them one
 * at a time. */
int ottohip_kmeans_lloyd_steps_pair(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* const* centroids,
                                    int k, int32_t* const* labels, int64_t* const* sums, int64_t* const* counts,
                                    const int* max_steps, double tol, double* out, void* stream);
/* lloyd_steps for n_runs (1..4) independent runs in lockstep (the n_init runs of :152-159, 4 at a time):
 * one read of X per step scores all of them; a decided row whose label changes is applied to its run's
 * fixed-point sums by a move list. Arrays as in lloyd_steps_pair with n_runs entries; out (HOST
 * double[6 * n_runs]). Each run's labels, centres, stop step and reason equal lloyd_steps on that run
 * alone (no distance bounds in lockstep). OTTOHIP_ELIMIT outside 32 < k <= 64, dim <= 112. */
int ottohip_kmeans_lloyd_steps_multi(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* const* centroids,
                                     int k, int32_t* const* labels, int64_t* const* sums, int64_t* const* counts,
                                     const int* max_steps, int n_runs, double tol, double* out, void* stream);
/* The E-step of lloyd_steps is a split-precision pass (x = hi + lo and c = hi + lo in bf16, three bf16
 * MFMA products, a rigorous error bound) that decides every row whose two best scores are separated
 * beyond the bound, plus the exact f32 kernel on the remaining near ties: labels, sums and stop
 * checks are bit-identical to the exact kernel on every row (out[0] then covers the near ties only).
 * (OTTOHIP_KM_SPLIT=0: the exact kernel on every row).
 * Rows are skipped by distance bounds carried across steps and calls (Hamerly's upper bound to the
 * own centre and one lower bound to all others, moved by each centre's shift since the bounds were
 * set): a row whose bounds separate beyond the exact kernel's error keeps its label unscored, the
 * same label the exact kernel gives it. The bounds belong to (X, labels, n, dim, k) of the previous
 * lloyd_steps call on the context; a row with label -1 (a new run) is always scored, and every other
 * kmeans entry point that writes labels discards them. Between calls, change labels only through the
 * library or by resetting them to -1. (OTTOHIP_KM_BOUNDS=0: every row scored each step.) */
int ottohip_kmeans_farthest(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids,
                            const int32_t* labels, int m, int64_t* rows, float* d2, void* stream);
int ottohip_kmeans_relocate(ottohip_ctx* ctx, int64_t* sums, int64_t* counts, int k, int dim, const float* vecs,
                            const int32_t* old_new, int m, void* stream);
int ottohip_kmeans_inertia(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids,
                           const int32_t* labels, double* inertia, void* stream);
/* sklearn KMeans(init='random') initial centres: numpy RandomState(seed) (legacy MT19937)
 * replica. ottohip_rs_permutation_head(rs, n, k, out) == rs.permutation(n)[:k] (out HOST int64[k])
 * and advances the stream exactly as numpy does, so successive calls give the n_init runs'
 * seeds (model/kmeans_sessions.py:152-159 -> sklearn 1.2 _init_centroids). Host-only, thread-safe
 * per handle; n < 2^32. */
typedef struct ottohip_rs ottohip_rs;
int ottohip_rs_create(uint32_t seed, ottohip_rs** out);
int ottohip_rs_permutation_head(ottohip_rs* rs, int64_t n, int k, int64_t* out);
void ottohip_rs_destroy(ottohip_rs* rs);
/* column statistics and centering for KMeans.fit (sklearn subtracts the column mean before the
 * runs and scales tol by the mean column variance): sum_x[d] = sum x, sum_sq[d] = sum (x - center[d])^2
 * (center NULL = 0), both device int64 in 2^-24 fixed point (exact: shards all-reduce them); dim <= 128 */
int ottohip_col_sums(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* center, int64_t* sum_x,
                     int64_t* sum_sq, void* stream);
int ottohip_center_rows(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* mean, float* out,
                        void* stream);
/* C3 count_popularity (model/count_popularity.py:53-85) for one clustering: per (cluster, aid)
 * n_{clicks,carts,orders} and *_7d (ts > ts_7d), ordinal rank desc within the cluster (ties: aid
 * asc) clipped to 999, rows with min rank <= keep_top_k. session_cl: dense cluster per session. */
typedef struct ottohip_pop ottohip_pop;
int ottohip_popularity_ranks(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions,
                             const int32_t* aid, const int32_t* ts, const int8_t* type, const int32_t* session_cl,
                             int32_t n_items, int32_t n_clusters, int32_t ts_7d, int keep_top_k,
                             ottohip_pop** out, int64_t* n_out, void* stream);
/* C3 in two parts, for sessions sharded over ranks: pop_counts ADDS this rank's
 * per (cluster, aid) counters into counts (device u32 [6][n_clusters * n_items]: clicks, carts, orders,
 * then the *_7d ones); the host all-reduces them; popularity_from_counts ranks them exactly as
 * ottohip_popularity_ranks does (which is pop_counts on zeroed counters + popularity_from_counts). */
int ottohip_pop_counts(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions, const int32_t* aid,
                       const int32_t* ts, const int8_t* type, const int32_t* session_cl, int32_t n_items,
                       int32_t n_clusters, int32_t ts_7d, uint32_t* counts, void* stream);
int ottohip_popularity_from_counts(ottohip_ctx* ctx, const uint32_t* counts, int32_t n_items, int32_t n_clusters,
                                   int keep_top_k, ottohip_pop** out, int64_t* n_out, void* stream);
/* rows sorted by (cluster, aid); ranks6 [n x 6]: clicks, carts, orders, clicks_7d, carts_7d, orders_7d */
int ottohip_pop_copy(const ottohip_pop* p, int32_t* aid, int32_t* cluster, int16_t* ranks6, void* stream);
void ottohip_pop_free(ottohip_pop* p);
/* R7 (model/retrieve.py:604-625): cos and Euclidean distance between the session embedding and
 * each candidate's item embedding; a session without an embedding (sess_has[s] == 0) or an item
 * without one gives cos 0, eucl -1 (the inner joins + fill_null of :621-625). */
int ottohip_session_item_similarity(ottohip_ctx* ctx, const int64_t* cand_off, int64_t n_sessions,
                                    const int32_t* aid_next, const float* sess_emb, const uint8_t* sess_has,
                                    const int32_t* row_of_aid, int32_t n_aid_map, const float* emb, int dim,
                                    float* cos_out, float* eucl_out, void* stream);

/* ---- Multi-GPU exchange -------------------------------------------------
 * The reference is single-process; these calls replace the cross-file groupby of
 * concat_files_w_stats (model/count_co_events.py:168) when files are dealt over G ranks.
 * Each rank counts its own whole files (ottohip_covis_count), packs its rows by owner and
 * exchanges them (all-to-all-v issued by the host layer over RCCL); the owner rebuilds a
 * table that equals the single-GPU table restricted to {aid : owner(aid) == rank}.
 * Record = 4 x u32 {rule << 29 | aid, aid_next, count, count_ge2} (requires aid < 2^29). */
int ottohip_owner_of(int32_t aid, int n_parts); /* owner rank of an aid: multiplicative hash, range-reduced */
/* out_records: device, >= n_rows records; part_counts: HOST [n_parts] rows per owner, records
 * of owner p follow those of owners < p. */
int ottohip_table_pack_by_owner(ottohip_ctx* ctx, const ottohip_table* t, int n_parts, void* out_records,
                                int64_t* part_counts, void* stream);
/* merge-sum received records (duplicates of a (rule, aid, aid_next) key are summed) into a new
 * table; file_stats (HOST, n_rules entries, may be NULL) supplies the GLOBAL file_rows /
 * file_rows_ge2 (all-reduced by the caller) that ottohip_table_finalize needs. */
/* install GLOBAL per-file row statistics on a shard (all-reduced by the caller): the N that
 * concat_files_w_stats tests against 1e8 / 3e8 (:131, :135) is a whole-dataset quantity */
int ottohip_table_set_file_stats(ottohip_table* t, int rule, int64_t file_rows, int64_t file_rows_ge2);
int ottohip_table_from_records(ottohip_ctx* ctx, const void* records, int64_t n, int n_rules, int32_t n_items,
                               const ottohip_rule_stats* file_stats, ottohip_table** out, void* stream);

/* Pair-level exchange (the scalable path, used by otto-recommender_amd/dist.py): each rank
 * emits the pair words of its own whole files with rows laid out owner-major, so the words
 * for owner p are one contiguous segment; the owner receives every rank's segment plus a
 * piece list (row_key << 32 | n_words per (source, row)), assembles one word range per row
 * and runs the same reduce as ottohip_covis_count. Words carry GLOBAL file ids (file_ids),
 * so the per-file count>=2 rule (count_co_events.py:131-132) is exact across ranks.
 * ottohip_covis_emit runs S1-S3 (prep, count, row layout) and reports per-owner sizes;
 * ottohip_emit_write then writes the words and pieces into caller device buffers (the
 * all-to-all send buffers). No other count call may run on ctx in between. */
typedef struct ottohip_emit ottohip_emit;
int ottohip_covis_emit(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules, int n_rules,
                       const ottohip_covis_params* params, const int32_t* file_ids /* host [n_files], NULL = 0.. */,
                       int32_t n_files_total, int n_parts, ottohip_emit** out,
                       int64_t* words_per_part /* host [n_parts] */, int64_t* rows_per_part /* host [n_parts] */,
                       void* stream);
int ottohip_emit_write(ottohip_emit* em, uint32_t* words, uint64_t* pieces, void* stream);
void ottohip_emit_free(ottohip_emit* em);
/* words / pieces: every source's segment for this rank, concatenated in the same source order */
int ottohip_covis_reduce_received(ottohip_ctx* ctx, const ottohip_rule* rules, int n_rules,
                                  const ottohip_covis_params* params, int32_t n_files_total, const uint32_t* words,
                                  int64_t n_words, const uint64_t* pieces, int64_t n_pieces, ottohip_table** out,
                                  void* stream);
/* the same with per-file options (global file ids; the owner's histograms cover its own rows, the
 * host all-reduces them) */
int ottohip_covis_reduce_received_opts(ottohip_ctx* ctx, const ottohip_rule* rules, int n_rules,
                                       const ottohip_covis_params* params, int32_t n_files_total, const uint32_t* words,
                                       int64_t n_words, const uint64_t* pieces, int64_t n_pieces,
                                       const ottohip_file_opts* opts, ottohip_table** out, void* stream);

/* ---- Word2Vec top-K similarity (model/w2vec_aids.py:98-173) ------------------------------
 * Replaces load_index_faiss_ivff (:98-110) + get_top_k_similar_faiss (:125-173): exact L2
 * search (the reference's IVFFlat nlist 100 / nprobe 3 is approximate). The index packs the
 * caller's fp32 embeddings [n_items x dim] (device, kept referenced) into a bf16 MFMA operand;
 * ottohip_knn_topk returns, per query row, the k nearest rows in ascending squared L2
 * distance (ties by row index), distances exact in fp32 (candidates from bf16 MFMA scores,
 * reranked: 24 per query, 4 of margin). dim <= 126, k <= 20. query_rows (device, n_q) index the embedding rows
 * (get_top_k_similar_faiss queries words_q, a subset of words); NULL = rows 0..n_q-1. */
typedef struct ottohip_knn_index ottohip_knn_index;
int ottohip_knn_index_create(ottohip_ctx* ctx, const float* emb, int64_t n_items, int dim,
                             ottohip_knn_index** out, void* stream);
int ottohip_knn_topk(ottohip_ctx* ctx, const ottohip_knn_index* index, const int32_t* query_rows,
                     int64_t n_q, int k, int32_t* out_idx, float* out_d2, void* stream);
void ottohip_knn_index_free(ottohip_knn_index* index);

/* Test hooks for the device primitives the engine is built from (parity tests only). */
int ottohip_test_exclusive_scan_u32(ottohip_ctx* ctx, const uint32_t* in, uint64_t* out, int64_t n,
                                    uint64_t* total_host, void* stream);
int ottohip_test_radix_sort_pairs(ottohip_ctx* ctx, uint32_t* keys, uint32_t* vals, int64_t n,
                                  int bits, void* stream);
/* cross-lane moves of one wave on in[64] (device): out[k*64 + l] for k = 0..5 the value of lane
 * l ^ (1 << k); k = 6, 7: inclusive sum / max scan; k = 8, 9: lanes l-1 / l+1 (0 off the ends) */
int ottohip_test_lanes(const uint32_t* in, uint32_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif

// Count-table and context objects shared by the C-ABI translation units (abi.hip, shard.hip).
#pragma once
#include <algorithm>
#include "common.h"

using namespace ottohip;

// device buffers of one count table (reused across calls through the context's spare slot)
struct TableBufs {
  uint64_t cap = 0;
  uint8_t* rule = nullptr;
  int32_t* aid = nullptr;
  int32_t* aid_next = nullptr;
  uint32_t* count = nullptr;
  uint32_t* count_ge2 = nullptr;
  void release() {
    dev_free(rule);
    dev_free(aid);
    dev_free(aid_next);
    dev_free(count);
    dev_free(count_ge2);
    *this = TableBufs();
  }
  int alloc(uint64_t n) {
    if (dev_alloc(reinterpret_cast<void**>(&rule), n, "tab_rule") ||
        dev_alloc(reinterpret_cast<void**>(&aid), n * 4, "tab_aid") ||
        dev_alloc(reinterpret_cast<void**>(&aid_next), n * 4, "tab_aid_next") ||
        dev_alloc(reinterpret_cast<void**>(&count), n * 4, "tab_count") ||
        dev_alloc(reinterpret_cast<void**>(&count_ge2), n * 4, "tab_count_ge2")) {
      release();
      set_error("table allocation for %llu rows failed", (unsigned long long)n);
      return OTTOHIP_ENOMEM;
    }
    cap = n;
    return 0;
  }
};

struct ottohip_ctx : public Ctx {
  TableBufs spare;  // buffers of the last freed table, reused by the next count
  uint64_t gen = 0;  // count calls so far (emit handles refer to the workspace of one call)
};

constexpr int TABLE_MAX_IDS = 256;  // rule ids of a table's rows (part ids: ottohip_covis_count_parts)
struct KeptEmission;  // a count's emitted words and rows, kept for ottohip_table_count_parts (abi.hip)
void kept_free(KeptEmission* k);
struct ottohip_table {
  int device = 0;
  int n_rules = 0;
  int32_t n_items = 0;  // aid range [0, n_items) of the rows
  int64_t n_rows = 0;   // valid rows (sum over rules)
  int64_t n_slots = 0;  // entries of the row arrays; holes carry rule = 0xFF
  TableBufs b;
  uint32_t sym_mask = 0;  // rules stored once per unordered pair (aid <= aid_next): readers add the mirrors
  int sym(int rule) const { return (int)((sym_mask >> rule) & 1u); }
  ottohip_rule_stats stats[TABLE_MAX_IDS];  // per rule (or per part of a ottohip_covis_count_parts table)
  ottohip_ctx* ctx = nullptr;
  KeptEmission* kept = nullptr;  // ottohip_file_opts.keep_words: the count's words, for ottohip_table_count_parts
  bool aid_ordered = true;       // a rule's (part's) slots are in aid order (false: explicit mirror rows)
  // rows are type-major in a count's table: the first slot of each row type (types 0..2) and the end, written on the
  // device by the count (type_slots_dev, read back on first use); a rule's rows lie in its type's slot range
  uint64_t* type_slots_dev = nullptr;
  int64_t type_slots[4] = {0, 0, 0, 0};
  bool type_slots_known = false;
  int8_t rule_type[TABLE_MAX_IDS] = {};  // -1: unknown (scan every slot)
  int part_stats_pending = 0;    // part-mode tables: the per-part rows / pairs are counted when first read
  hipEvent_t produced = nullptr; // part-mode tables: recorded on the producer's stream after the reduce; the
                                 // deferred statistics wait on it (the producer may be a non-blocking stream)
};
// a part-mode table's per-part statistics (rows, pairs per rule byte), counted on first use (abi.hip)
namespace ottohip {
int ensure_part_stats(const ottohip_table* t);
}

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

template <class T>
static int d2h(T* host, const T* dev, size_t n, hipStream_t s) {
  OH_HIP(hipMemcpyAsync(host, dev, n * sizeof(T), hipMemcpyDeviceToHost, s));
  OH_HIP(hipStreamSynchronize(s));
  return 0;
}

static inline unsigned grid_for(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, ceil_div(n, t)); }

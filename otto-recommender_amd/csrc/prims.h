#pragma once
#include "common.h"

namespace ottohip {
// out[i] = sum(in[0..i)), 64-bit; optional device total
int exclusive_scan_u32(Ctx* ctx, const uint32_t* in, uint64_t* out, int64_t n, uint64_t* total,
                       hipStream_t s);
int exclusive_scan_u64(Ctx* ctx, const uint64_t* in, uint64_t* out, int64_t n, uint64_t* total,
                       hipStream_t s);
// stable LSD sort of (key, val) by key bits [0, bits); ping-pongs with the *_alt buffers and
// returns the buffers holding the result in keys/vals
// iota_vals: the input values are their own indices (0..n-1); the first pass generates them
// instead of reading vals (vals still provides the buffer)
// skip (with iota_vals): the first pass drops keys with (key & mask) == inv and the later passes sort the
// *n_out kept pairs (the first pass' total, read back on the host)
struct SortSkip {
  uint32_t mask, inv;
  int64_t* n_out;
};
int radix_sort_pairs(Ctx* ctx, uint32_t*& keys, uint32_t*& vals, uint32_t* keys_alt, uint32_t* vals_alt,
                     int64_t n, int bits, hipStream_t s, bool iota_vals = false, const SortSkip* skip = nullptr);
// one stable 8-bit pass on digit (key >> shift) & 255
int radix_pass(Ctx* ctx, const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout, int64_t n,
               int shift, hipStream_t s, const uint64_t** digit_start = nullptr, int* n_tiles = nullptr);
}  // namespace ottohip

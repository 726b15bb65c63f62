// 32-byte key order (lexicographic over the key bytes; keys are 4 little-endian u64
// words): comparisons and binary search shared by the fast-sync request match
// (nodedata.h) and the resident forest (forest.h).
#pragma once
#include "trie_ops.h"
namespace khst {

// lexicographic compare of two 32-byte keys held as 4 little-endian words
KH_HD int key_cmp(const uint64_t* a, const uint64_t* b) {
  for (int j = 0; j < 4; ++j) {
    uint64_t x = bswap64(a[j]), y = bswap64(b[j]);
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

// first index in sorted keys[0, n) not less than k
KH_HD uint64_t key_lower_bound(const uint64_t* keys, uint64_t n, const uint64_t* k) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (key_cmp(keys + 4 * mid, k) < 0)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

}  // namespace khst

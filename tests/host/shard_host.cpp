// Host build of at2-node_amd/csrc/at2v_shard.h (the index-range sharding the library's multi-GPU entry points use),
// exported for tests/test_shard_host.py, which checks it against at2v/dist.py.
#include <cstddef>
#include <cstdint>

#include "at2v_shard.h"

extern "C" {
size_t sh_per_rank(size_t n, int world) { return at2v::shard_per_rank(n, world); }
size_t sh_words_per_rank(size_t n, int world) { return at2v::shard_words_per_rank(n, world); }
void sh_rank_range(size_t n, int world, int rank, size_t* lo, size_t* hi) {
  const at2v::Range r = at2v::rank_range(n, world, rank);
  *lo = r.lo;
  *hi = r.hi;
}
void sh_rank_words(size_t n, int world, int rank, size_t* dst, size_t* src, size_t* words) {
  const at2v::WordCopy w = at2v::rank_words(n, world, rank);
  *dst = w.dst_word;
  *src = w.src_word;
  *words = w.words;
}
void sh_device_range(size_t n, size_t G, size_t g, size_t* lo, size_t* hi) {
  const at2v::Range r = at2v::device_range(n, G, g);
  *lo = r.lo;
  *hi = r.hi;
}
int sh_offsets_valid(const uint32_t* off, size_t n) { return at2v::offsets_valid(off, n) ? 1 : 0; }
void sh_rebase(const uint32_t* off, size_t a, size_t m, uint32_t* out) { at2v::rebase_offsets(off, a, m, out); }
}

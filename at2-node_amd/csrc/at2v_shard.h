// at2v_shard.h — index-range sharding of a verify batch over GPUs, host side.
//
// Header-only and free of HIP/RCCL so the CPU suite runs the same code (tests/host/shard_host.cpp, checked against
// at2v/dist.py's shard_bounds / padded_words_per_rank). Used by at2v_api.hip for:
//   * one process per GPU (at2v_verify_batch_sharded, at2v_verify_shard_gather_device): rank r owns records
//     [r*per, min(n, (r+1)*per)) with per = ceil(ceil(n/world)/64)*64, and contributes per/32 verdict words to an
//     in-place all-gather, so the node bitmap holds world*per/32 words, rank r's at word r*per/32;
//   * one process, several devices (at2v_verify_batch with at2v_opts.num_gpus > 1): shard g owns the 64-record
//     chunks [chunks*g/G, chunks*(g+1)/G), so its verdict words start at a word-aligned place of the caller's array.
// The consumer of the bitmap is the deliver/apply loop of /root/reference/src/bin/server/rpc.rs:156-173.
#pragma once
#include <cstddef>
#include <cstdint>

namespace at2v {

constexpr size_t kShardAlign = 64;  // records per wave chunk = two verdict words

struct Range {
  size_t lo, hi;  // [lo, hi) record indices
  size_t size() const { return hi > lo ? hi - lo : 0; }
};

// Multi-process: records per rank, padded to whole chunks (every rank contributes the same word count).
inline size_t shard_per_rank(size_t n, int world) {
  const size_t w = world > 0 ? (size_t)world : 1;
  const size_t per = (n + w - 1) / w;
  return (per + kShardAlign - 1) / kShardAlign * kShardAlign;
}

// Verdict words every rank contributes to the all-gather (at least 2 even for n = 0: RCCL needs a count > 0).
inline size_t shard_words_per_rank(size_t n, int world) { return shard_per_rank(n ? n : 1, world) / 32; }

inline Range rank_range(size_t n, int world, int rank) {
  const size_t per = shard_per_rank(n ? n : 1, world);
  const size_t lo = (size_t)rank * per < n ? (size_t)rank * per : n;
  const size_t hi = lo + per < n ? lo + per : n;
  return {lo, hi};
}

// Where rank r's gathered words go in the caller's ceil(n/32)-word verdict array: dst_word = lo/32 (lo is a multiple
// of 64), from word r*words_per_rank of the padded node bitmap, ceil((hi-lo)/32) words (0 for an empty rank).
struct WordCopy {
  size_t dst_word, src_word, words;
};
inline WordCopy rank_words(size_t n, int world, int rank) {
  const Range r = rank_range(n, world, rank);
  return {r.lo / 32, (size_t)rank * shard_words_per_rank(n, world), (r.size() + 31) / 32};
}

// Single process, G devices: balanced whole chunks per device.
inline Range device_range(size_t n, size_t G, size_t g) {
  const size_t chunks = (n + kShardAlign - 1) / kShardAlign;
  auto at = [&](size_t k) {
    const size_t v = chunks * k / (G ? G : 1) * kShardAlign;
    return v < n ? v : n;
  };
  return {at(g), at(g + 1)};
}

// msg_off[0..n] non-decreasing. Evaluated on the WHOLE batch before any per-rank or per-device work, so every rank of a
// collective call reaches the same verdict from the same input and either all of them join the all-gather or none.
inline bool offsets_valid(const uint32_t* off, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return false;
  return true;
}

// Offsets of records [a, a+m) relative to the first of them (the message slice that is uploaded); m+1 values.
// Requires offsets_valid over [a, a+m].
inline void rebase_offsets(const uint32_t* off, size_t a, size_t m, uint32_t* out) {
  const uint32_t base = off[a];
  for (size_t i = 0; i <= m; ++i) out[i] = off[a + i] - base;
}

}  // namespace at2v

// cgx_hash.h -- 64-bit content hash of host memory, shared by the op-level
// matrix residency check (cgx_mvops.cpp) and the reader's binary cache key
// (cgx_io.cpp).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <thread>
#include <vector>

namespace cgx {

// 64-bit content hash of a byte range (xxHash64's construction, written
// here): each 8-byte word goes through a multiply-rotate-multiply round of
// one of 4 lanes, so a bit flip in any word diffuses over the lane and two
// flips cannot cancel the way they did in the round-2 multiply-xor lanes
// (negating a symmetric pair a_ij / a_ji left the hash
// unchanged).  Chunks on host threads (the count depends on the size only),
// chunk hashes folded in order, final avalanche.
constexpr unsigned long long kP1 = 0x9E3779B185EBCA87ULL, kP2 = 0xC2B2AE3D27D4EB4FULL,
                             kP3 = 0x165667B19E3779F9ULL, kP4 = 0x85EBCA77C2B2AE63ULL,
                             kP5 = 0x27D4EB2F165667C5ULL;
inline unsigned long long rotl64(unsigned long long x, int r) { return (x << r) | (x >> (64 - r)); }
inline unsigned long long hround(unsigned long long acc, unsigned long long w) {
  return rotl64(acc + w * kP2, 31) * kP1;
}
inline unsigned long long hmerge(unsigned long long h, unsigned long long v) {
  return (h ^ hround(0, v)) * kP1 + kP4;
}
inline unsigned long long avalanche(unsigned long long h) {
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  return h ^ (h >> 32);
}

inline unsigned long long hash_bytes(const void *p, size_t bytes) {
  const unsigned char *b = (const unsigned char *)p;
  const size_t words = bytes / 8;
  const int nt = (int)std::max<size_t>(1, std::min<size_t>(16, words >> 20));
  std::vector<unsigned long long> part((size_t)nt);
  auto work = [&](int t) {
    const size_t lo = words * t / nt, hi = words * (t + 1) / nt;
    unsigned long long v[4] = {kP1 + kP2, kP2, 0, 0ULL - kP1};
    size_t i = lo;
    for (; i + 4 <= hi; i += 4)
      for (int l = 0; l < 4; ++l) {
        unsigned long long w;
        memcpy(&w, b + 8 * (i + l), 8);
        v[l] = hround(v[l], w);
      }
    unsigned long long h = rotl64(v[0], 1) + rotl64(v[1], 7) + rotl64(v[2], 12) + rotl64(v[3], 18);
    for (int l = 0; l < 4; ++l) h = hmerge(h, v[l]);
    h += (unsigned long long)(hi - lo) * 8;
    for (; i < hi; ++i) {
      unsigned long long w;
      memcpy(&w, b + 8 * i, 8);
      h = rotl64(h ^ hround(0, w), 27) * kP1 + kP4;
    }
    part[(size_t)t] = avalanche(h);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
  unsigned long long h = kP5 + bytes;
  for (unsigned long long x : part) h = hmerge(h, x);
  for (size_t i = words * 8; i < bytes; ++i) h = rotl64(h ^ (b[i] * kP5), 11) * kP1;
  return avalanche(h);
}

}  // namespace cgx

// srd_xxh3.h -- XXH3-64 (seed 0, default secret) for device code.
//
// The reference hashes with xxhash-rust 0.8.15 `xxh3_64`
// (src/storage_engine/digest/compute_hash.rs:25-27, :64-77) and uses the same
// function as the HashMap/HashSet hasher of the key index
// (src/storage_engine/digest/xxh3_build_hasher.rs:11-13): a u64 key_hash is
// hashed as its 8 little-endian bytes (the len 4..8 path below).
// Restated from the published XXH3 algorithm; pinned against
// tests/hash_stability_tests.rs goldens in tests/test_gpu_parity.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srd {

__device__ __constant__ static const uint8_t kXxhSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

__device__ __forceinline__ uint64_t x_rd64(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}
__device__ __forceinline__ uint32_t x_rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint64_t x_sec64(int o) { return x_rd64(kXxhSecret + o); }
__device__ __forceinline__ uint64_t x_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t x_fold(uint64_t a, uint64_t b) {
  return (a * b) ^ __umul64hi(a, b);
}
__device__ __forceinline__ uint64_t x_av3(uint64_t h) {
  h ^= h >> 37; h *= 0x165667919E3779F9ull; return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t x_av64(uint64_t h) {
  h ^= h >> 33; h *= 0xC2B2AE3D27D4EB4Full; h ^= h >> 29; h *= 0x165667B19E3779F9ull; return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t x_rrmxmx(uint64_t h, uint64_t len) {
  h ^= x_rotl(h, 49) ^ x_rotl(h, 24);
  h *= 0x9FB21C651E98DF25ull;
  h ^= (h >> 35) + len;
  h *= 0x9FB21C651E98DF25ull;
  return h ^ (h >> 28);
}

// xxh3_64 of the 8 little-endian bytes of v (the Xxh3BuildHasher input).
__device__ __forceinline__ uint64_t xxh3_64_u64(uint64_t v) {
  const uint64_t bf = 0x1cad21f72c81017cull ^ 0xdb979083e96dd4deull;  // sec[8..16) ^ sec[16..24)
  uint64_t i1 = (uint32_t)v, i2 = v >> 32;
  return x_rrmxmx((i2 + (i1 << 32)) ^ bf, 8);
}

__device__ __forceinline__ uint64_t x_mix16(const uint8_t* in, int so) {
  return x_fold(x_rd64(in) ^ x_sec64(so), x_rd64(in + 8) ^ x_sec64(so + 8));
}

// General xxh3_64 (one thread per input).
__device__ inline uint64_t xxh3_64(const uint8_t* in, uint64_t len) {
  if (len <= 16) {
    if (len > 8) {
      uint64_t lo = x_rd64(in) ^ (x_sec64(24) ^ x_sec64(32));
      uint64_t hi = x_rd64(in + len - 8) ^ (x_sec64(40) ^ x_sec64(48));
      uint64_t acc = len + __builtin_bswap64(lo) + hi + x_fold(lo, hi);
      return x_av3(acc);
    }
    if (len >= 4) {
      uint64_t i1 = x_rd32(in), i2 = x_rd32(in + len - 4);
      return x_rrmxmx((i2 + (i1 << 32)) ^ (x_sec64(8) ^ x_sec64(16)), len);
    }
    if (len > 0) {
      uint32_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
      uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
      uint64_t bf = (uint64_t)(x_rd32(kXxhSecret) ^ x_rd32(kXxhSecret + 4));
      return x_av64((uint64_t)comb ^ bf);
    }
    return x_av64(x_sec64(56) ^ x_sec64(64));
  }
  if (len <= 128) {
    uint64_t acc = len * 0x9E3779B185EBCA87ull;
    if (len > 32) {
      if (len > 64) {
        if (len > 96) {
          acc += x_mix16(in + 48, 96);
          acc += x_mix16(in + len - 64, 112);
        }
        acc += x_mix16(in + 32, 64);
        acc += x_mix16(in + len - 48, 80);
      }
      acc += x_mix16(in + 16, 32);
      acc += x_mix16(in + len - 32, 48);
    }
    acc += x_mix16(in, 0);
    acc += x_mix16(in + len - 16, 16);
    return x_av3(acc);
  }
  if (len <= 240) {
    uint64_t acc = len * 0x9E3779B185EBCA87ull, acc_end;
    unsigned nb = (unsigned)len / 16;
    for (unsigned i = 0; i < 8; i++) acc += x_mix16(in + 16 * i, 16 * i);
    acc_end = x_mix16(in + len - 16, 136 - 17);
    acc = x_av3(acc);
    for (unsigned i = 8; i < nb; i++) acc_end += x_mix16(in + 16 * i, 16 * (i - 8) + 3);
    return x_av3(acc + acc_end);
  }
  uint64_t acc[8] = {0xC2B2AE3Dull, 0x9E3779B185EBCA87ull, 0xC2B2AE3D27D4EB4Full,
                     0x165667B19E3779F9ull, 0x85EBCA77C2B2AE63ull, 0x85EBCA77ull,
                     0x27D4EB2F165667C5ull, 0x9E3779B1ull};
  const uint64_t nb_blocks = (len - 1) / 1024;
  auto acc512 = [&](const uint8_t* p, int so) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t dv = x_rd64(p + 8 * i);
      uint64_t dk = dv ^ x_sec64(so + 8 * i);
      acc[i ^ 1] += dv;
      acc[i] += (uint64_t)(uint32_t)dk * (dk >> 32);
    }
  };
  for (uint64_t b = 0; b < nb_blocks; b++) {
    for (int n = 0; n < 16; n++) acc512(in + b * 1024 + n * 64, n * 8);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t a = acc[i];
      a ^= a >> 47;
      a ^= x_sec64(128 + 8 * i);
      a *= 0x9E3779B1ull;
      acc[i] = a;
    }
  }
  uint64_t nbs = ((len - 1) - 1024 * nb_blocks) / 64;
  for (uint64_t n = 0; n < nbs; n++) acc512(in + nb_blocks * 1024 + n * 64, (int)n * 8);
  acc512(in + len - 64, 192 - 64 - 7);
  uint64_t r = len * 0x9E3779B185EBCA87ull;
#pragma unroll
  for (int i = 0; i < 4; i++)
    r += x_fold(acc[2 * i] ^ x_sec64(11 + 16 * i), acc[2 * i + 1] ^ x_sec64(11 + 16 * i + 8));
  return x_av3(r);
}

}  // namespace srd

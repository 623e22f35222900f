// srd_crc.h -- IEEE CRC-32 algebra shared by host and device code.
//
// The reference computes CRC-32/ISO-HDLC with crc32fast 1.5.0
// (src/storage_engine/digest/compute_checksum.rs:15-20): reflected polynomial
// 0xEDB88320, init and xorout 0xFFFFFFFF, little-endian storage.
//
// Notation: crc_raw(D) = the CRC register after feeding D into a zeroed
// register (no init, no xorout).  In the reflected representation (bit 31 =
// x^0, bit 30 = x^1, ...) the register is a polynomial modulo P, and
//   crc_raw(A || B) = mulp(x^(8|B|), crc_raw(A)) ^ crc_raw(B)
//   CRC32(D)        = crc_raw(D) ^ CRC32(0^|D|)
//   CRC32(D)        = ~crc_raw(D with 0xFFFFFFFF xored into bytes 0..3) (|D|>=4)
// which is what lets 64-lane waves compute per-line CRCs independently and
// combine them (lane weights, per-tile suffix values) -- see DESIGN.md §3.
#pragma once
#include <stdint.h>

#ifndef SRD_HD
#if defined(__HIPCC__)
#define SRD_HD __host__ __device__
#else
#define SRD_HD
#endif
#endif

namespace srd {

static constexpr uint32_t kPoly = 0xEDB88320u;
static constexpr uint32_t kX0 = 0x80000000u;  // x^0 in reflected form

// a(x) * b(x) mod P, reflected.  Branch-free (32 fixed steps).
SRD_HD inline uint32_t mulp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int i = 31; i >= 0; --i) {
    p ^= ((a >> i) & 1u) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
  }
  return p;
}

// Host-side tables: 4 slice tables, lane weights, init/zero corrections and
// the inverse powers used by the per-entry combine.
struct CrcTables {
  uint32_t tab[4][256];     // slice-by-4 (tab[0] = byte table)
  uint32_t lw[64];          // x^(512*(63-l))   lane weight of line l in a tile
  uint32_t winit[64];       // x^(512*(63-j)) * crc_raw(FFFFFFFF || 0^60)
  uint32_t zero_crc[64];    // CRC32(0^n), n < 64
  uint32_t x32768;          // x^(8*4096)       one tile
  uint32_t pow8[64];        // x^(8*2^k)
  uint32_t invpow[4097];    // x^(-8d), d = 0..4096
};

inline uint32_t host_crc_raw_bytes(const CrcTables& t, uint32_t s, const uint8_t* p, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) s = t.tab[0][(s ^ p[i]) & 0xff] ^ (s >> 8);
  return s;
}

// x^(8n) via the pow8 table
inline uint32_t host_xpow8(const CrcTables& t, uint64_t n) {
  uint32_t r = kX0;
  for (int k = 0; n; k++, n >>= 1)
    if (n & 1) r = mulp(t.pow8[k], r);
  return r;
}

inline void build_crc_tables(CrcTables& t) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kPoly : (c >> 1);
    t.tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; i++)
    for (int k = 1; k < 4; k++)
      t.tab[k][i] = (t.tab[k - 1][i] >> 8) ^ t.tab[0][t.tab[k - 1][i] & 0xff];
  // pow8[k] = x^(8*2^k)
  uint32_t x8 = kX0;
  for (int i = 0; i < 8; i++) x8 = (x8 >> 1);  // x^8: bit 31-8
  t.pow8[0] = x8;
  for (int k = 1; k < 64; k++) t.pow8[k] = mulp(t.pow8[k - 1], t.pow8[k - 1]);
  for (int l = 0; l < 64; l++) t.lw[l] = host_xpow8(t, 64ull * (63 - l));
  t.x32768 = host_xpow8(t, 4096);
  uint8_t ff[64] = {0xff, 0xff, 0xff, 0xff};
  uint32_t delta = host_crc_raw_bytes(t, 0, ff, 64);
  for (int j = 0; j < 64; j++) t.winit[j] = mulp(t.lw[j], delta);
  uint8_t z[64] = {0};
  for (int n = 0; n < 64; n++) t.zero_crc[n] = ~host_crc_raw_bytes(t, 0xffffffffu, z, n);
  // x^-1: normal form (P(x)+1)/x = 0x82608EDB; reflect to our representation
  uint32_t nrm = 0x82608EDBu, xinv = 0;
  for (int i = 0; i < 32; i++)
    if (nrm & (1u << i)) xinv |= 1u << (31 - i);
  uint32_t xinv8 = kX0;
  for (int i = 0; i < 8; i++) xinv8 = mulp(xinv, xinv8);
  t.invpow[0] = kX0;
  for (int d = 1; d <= 4096; d++) t.invpow[d] = mulp(xinv8, t.invpow[d - 1]);
}

}  // namespace srd

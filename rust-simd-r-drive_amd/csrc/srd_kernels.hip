// srd_kernels.hip -- MI355X (gfx950) kernels of the validate+index hot path.
//
// Reference path being replaced (jzombie/rust-simd-r-drive v0.16.3-alpha):
//   DataStore::open           src/storage_engine/data_store.rs:84-117
//   recover_valid_chain       src/storage_engine/data_store.rs:383-482
//   KeyIndexer::build         src/storage_engine/key_indexer.rs:98-124
//   is_valid_checksum         simd-r-drive-entry-handle/src/entry_handle.rs:260-275
//
// Pipeline:
//   1. scan_kernel   one streaming pass over the file.  Each wave owns spans of
//                    16 tiles (4 KiB tile = 64 lines x 64 B, one line per
//                    lane).  Per tile it (a) finds chain-node candidates with
//                    a zero-triple filter + wave-cooperative exact check,
//                    (b) computes every line's raw CRC with LDS slice-by-4
//                    tables, (c) weights lines by x^(512(63-l)) and runs a
//                    64-lane suffix-XOR scan, so any 64-aligned range's CRC
//                    can later be assembled from O(1) per-tile values.
//   2. link_kernel   parent lookup per candidate (binary search in the span
//                    of the target) -> node / root / miss.
//   3. walk + mark   the chain from final_len, run-compressed (consecutive
//                    candidates that link to their predecessor form a run).
//   4. finalize      per chain entry: CRC from per-tile values (a few GF(2)
//                    multiplies), slow path recomputes a tile when a piece is
//                    missing.
//   5. index         XXH3-hashed open-addressing table, latest wins.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srd_crc.h"
#include "srd_xxh3.h"

namespace srd {


typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

constexpr int TILE = 4096;
constexpr int SPAN_TILES = 4;
constexpr uint64_t SPAN_BYTES = (uint64_t)TILE * SPAN_TILES;
constexpr int64_t PAR_ROOT = -1;
constexpr int64_t PAR_MISS = -2;

// flags of a candidate record
constexpr uint32_t F_TOMB = 1u, F_TAIL = 2u, F_SXM = 4u;
constexpr int F_SUF_SHIFT = 3;        // 2 bits: 0 value, 1 next-tile T, 2 next-tile SX1, 3 missing
// the recorded sxm / suf value is a lower-half partial (line < 32): true value =
// mul16k(v) ^ SX_32 of the tile holding m (sxm) or the entry start (suf kind 0) -- see lo_fix()
constexpr uint32_t F_SXM_LO = 32u, F_SUF_LO = 64u;
// single-candidate record of the optimistic scan: link_record applies the
// node test (F_NT); F_ZB = the byte at m - 1 is 0 (the tombstone rule's byte
// when p == m - 1)
constexpr uint32_t F_NT = 256u, F_ZB = 512u;

struct DevTables {
  uint32_t tab[4][256];
  uint32_t lw[64];
  uint32_t winit[64];
  uint32_t zero_crc[64];
  uint32_t x32768;
  uint32_t pow8[64];
  uint32_t invpow[4097];
  alignas(16) uint32_t nib[8 * 16 * 32];  // half-tile lane-weight nibble tables
  uint32_t m16k[4][256];           // v -> v * x^16384 byte tables
  alignas(16) uint32_t last[3][4][256];   // chain q's last slice-by-4 step, shifted: v -> v * x^(32 + 128 (3 - q))
  uint32_t xtile[65];              // X^e, X = x^32768 (one tile), e = 0..64
  uint32_t xt64[65];               // X^(64 q), q = 0..64 (with xtile: X^n for n < 4160 in one multiply)
  uint32_t mx64[4][256];           // v -> v * X^64 byte tables (the long-entry Horner step)
  // the writer's coalesced lane layout (lane l holds the 16-byte pieces at
  // 1024 j + 16 l of a 4 KiB block): the same slice-by-4 chains and lane-
  // weight nibbles with the pieces' own distances
  alignas(16) uint32_t last_c[3][4][256];  // v -> v * x^(32 + 8192 (3 - q))
  alignas(16) uint32_t nib_c[8 * 16 * 32];  // c -> c * x^(128 (31 - l % 32))
  uint32_t m4096[4][256];                   // v -> v * x^4096 (512 bytes: the half-lanes' distance)
  uint32_t m32k[4][256];                    // v -> v * x^32768 (one tile step in one multiply)
  uint32_t mtk[3][4][256];                  // v -> v * x^(32768 (j + 2)): 2-4 tile steps in one multiply
};
__device__ DevTables g_tabs;
#ifdef SRD_WAVE_STAMPS
__device__ uint64_t g_wave_stamp[8192 + 1024];  // [w]: wave w's end; [8192 + b]: block b's start;
#ifdef SRD_WAVE_STAMPS
__device__ uint64_t g_wave_clk[4096 + 256];  // s_memtime (shader clock) at wave w's end / block b's start: the scan's clock
#endif
                                                // [8192 + 256 + b]: its tables loaded; [8192 + 512 + b]: its
                                                // XCC_ID; [8192 + 1023]: the epilogue's end
#endif

// The scan's wave partition (both passes; link_record inverts it).  Block b of g
// takes the resident spans [st(b), st(b+1)), st(b) = b*ns/g; inside a block
// wave v takes the share [cw(v), cw(v+1)) (units of 1/65536) of the block's
// spans.  Waves of one SIMD do not progress equally: the SIMD issues for
// its oldest waves first, so with an even split waves 0-3 (the oldest on
// each SIMD) finished ~15% before waves 12-15 (tools/wave_stamps.py); the
// per-slot shares wq[v] (scan_weights: fitted to the wave stamps) even out
// the finish times.  The optimistic pass replaces st(b) by a device table
// (XPart, XCD-aware block shares) once a context has scanned a store of the
// same span count and grid.
struct ScanPart {
  uint64_t s_lo;   // first resident span
  uint64_t ns;     // resident spans
  uint32_t g;      // scan blocks
  uint32_t nw;     // waves per scan block (<= 16; the launch's variant sets it, scan_geom)
  uint32_t wq[16];  // share of wave slot v of each block; wq[0] + .. + wq[nw-1] == 65536
  uint32_t cw[17];  // cumulative: cw[v] = wq[0] + .. + wq[v-1] (part_fill_cw)
  const uint64_t* bs;  // device: st(0..g) (XPart::bs of this call), nullptr: st(b) = b*ns/g
};

// XCD-aware block shares (the optimistic scan).  The dispatcher hands block b
// to XCD (b + r) mod 8, r fixed per HW queue, and the XCDs do not stream at
// one speed: on a box the odd XCDs ran their blocks 4-5 % slower than the even
// ones, the pattern the same for consecutive calls (tools/xcc_stamps.py,
// profiles/r06/xcc_stamps_r6e.txt) -- with equal blocks the slow XCDs set the
// scan's end.  Every scan block records the XCD it ran on (HW_REG_XCC_ID) and
// its duration; link2_kernel's block 0 turns them into each XCD's speed (a
// moving average over the calls) and the next call's block
// starts, each block sized by its XCD's speed (clamped to +-XP_CLAMP), into
// the other half of a double-buffered table: call k reads bs[k & 1], writes
// bs[(k + 1) & 1] (the host flips the parity; it uses the table only for the
// span count and grid it was made for).
constexpr uint32_t XP_MAX_BLOCKS = 1024;
constexpr float XP_CLAMP = 0.10f;
struct XPart {
  uint64_t bs[2][XP_MAX_BLOCKS + 1];  // block starts (resident-relative spans) per parity
  uint32_t xcc[XP_MAX_BLOCKS];        // the XCD each block of the last scan ran on
  uint32_t dur[XP_MAX_BLOCKS];        // its duration (s_memrealtime ticks, 10 ns)
  uint64_t t0[XP_MAX_BLOCKS];         // its start (ticks)
  float w[8];                         // each XCD's relative speed (0: none measured yet)
  uint64_t scan_ticks;                // the last scan: first block start -> last block end (idx_emit publishes it)
};
__host__ __device__ __forceinline__ void part_fill_cw(ScanPart& p) {
  p.cw[0] = 0;
  for (uint32_t v = 0; v < 16; v++) p.cw[v + 1] = p.cw[v] + (v < p.nw ? p.wq[v] : 0u);
}
// cumulative share of the waves below v (v <= 16)
__host__ __device__ __forceinline__ uint64_t part_cw(const ScanPart& p, uint32_t v) { return p.cw[v]; }
__host__ __device__ __forceinline__ uint64_t part_block_start(const ScanPart& p, uint64_t b) {
  if (p.bs) return p.bs[b];  // (device pointer: host code sizes with the even split, bs unset)
  return b * p.ns / p.g;
}
// wave v of block b: resident-relative spans [*r0, *r1)
__host__ __device__ __forceinline__ void part_wave_range(const ScanPart& p, uint64_t b, uint32_t v,
                                                         uint64_t* r0, uint64_t* r1) {
  const uint64_t bs = part_block_start(p, b), nb = part_block_start(p, b + 1) - bs;
  *r0 = bs + ((nb * part_cw(p, v)) >> 16);
  *r1 = bs + ((nb * part_cw(p, v + 1)) >> 16);
}
// the scan wave (b * nw + v) holding resident-relative span rel < ns
__device__ __forceinline__ uint64_t part_span_wave(const ScanPart& p, uint64_t rel) {
  uint64_t b;
  if (p.bs) {  // the last block whose start is <= rel (empty blocks are skipped over)
    uint64_t lo = 0, hi = p.g - 1;
    while (lo < hi) {
      const uint64_t mid = (lo + hi + 1) >> 1;
      if (p.bs[mid] <= rel) lo = mid; else hi = mid - 1;
    }
    b = lo;
  } else {
    b = rel * p.g / p.ns;
    while (b + 1 < p.g && part_block_start(p, b + 1) <= rel) b++;
  }
  const uint64_t bs = part_block_start(p, b), nb = part_block_start(p, b + 1) - bs, o = rel - bs;
  uint32_t v = 0;
#pragma unroll
  for (uint32_t j = 1; j < 16; j++) v += j < p.nw && o >= ((nb * part_cw(p, j)) >> 16) ? 1u : 0u;
  return b * p.nw + v;
}

struct ScanArgs {
  ScanPart part;
  const uint8_t* file;
  uint64_t flen;
  uint64_t n_tiles, n_spans;
  uint32_t cap;
  uint32_t* tile;                  // [4*n_tiles]: half-tile partials h_0, h_1, SX_32 (tile_sx())
  uint32_t* span_count;
  uint64_t* c_m;                   // [n_spans*cap] candidate metadata offsets
  // the records in two 16-byte halves (structure of arrays): c_rec[g] = {p,
  // flags, crc_stored} -- all link2 reads --, c_rec1[g] = {key_hash, sxm, suf}
  u32x4* c_rec;                    // [slots] {p_lo, p_hi, flags, crc}
  u32x4* c_rec1;                   // [slots] {kh_lo, kh_hi, sxm, suf}
  unsigned long long* counters;    // [0] max root tail, [1] find_top's tail (optimistic pass), [2] overflow
  uint32_t filt_hb;               // (file_len-1) >> 32: bound of a node's p-byte 4 (p < file_len < 2^40)
  // span mode (entry-range shard): tiles [k_lo, n_tiles) are resident, k_lo a
  // multiple of SPAN_TILES; only nodes with m > m_lo are recorded (m_lo = the
  // shard's lower tail; 0 = whole file, where m >= 1)
  uint64_t k_lo;
  uint64_t m_lo;
  // zeroed by block 0 before its scan (folds two memset launches into the
  // scan): the glue's plan words and the span-count scan's sentinel
  uint32_t* zero_words;
  uint32_t n_zero_words;
  uint32_t* sentinel;
  // per-wave results, reduced by the last block to finish (no atomics on the
  // counters, no memset, no span-base scan launch): wave w's record count
  // (bit 63: a span overflowed its slots), its largest root tail; the last
  // block writes k_total[0] = the record total, k_total[1] = 1 + the last
  // record's slot, counters[0] (max root tail), [1] (find_top's tail), [2]
  // (overflow); `done` counts the finished blocks (the last block resets it
  // to 0).  The glue works in slot space (w * wcap + r): no wave bases.
  uint64_t* wave_total;
  uint64_t* wave_root;
  uint64_t* k_total;
  uint32_t* done;
  // optimistic pass: the records of scan wave w are DENSE in file order at
  // [w*wcap, (w+1)*wcap) (consecutive span flushes fill whole cache lines;
  // per-span slots left most lines partial: +0.11 ms of HBM writes at C2);
  // span_first[s] = index of span s's first record inside its wave's region
  // (the full pass keeps span*cap + slot)
  uint32_t* span_first;
  uint64_t wcap;
  // the link step (link2_kernel, over the same arguments) works in slot
  // space: record r of wave w is slot w*wcap + r.  k_total[1] = 1 + the slot
  // of the last record (0: none)
  int32_t* d_par;                  // [slots] the parent's slot, PAR_ROOT or PAR_MISS
  unsigned long long* childof;     // [slots] claims on parents (claim_word)
  uint32_t gen;                    // this call's claim generation
  uint64_t span_lo;                // span mode: the shard's lower tail (0 = whole file)
  uint32_t* zero2;                 // zeroed by block 0 as well: the index's bucket fills
  uint32_t n_zero2;
  // host-side only: the scan variant to launch (0 = the build's default;
  // SRD_DEBUG_API builds A/B the others inside one context)
  uint32_t variant;
  // XCD-aware block shares (optimistic pass; nullptr: off): the scan records
  // each block's XCD and duration, link2's block 0 writes the next call's
  // block starts into xp->bs[xp_next]
  XPart* xp;
  uint32_t xp_next;
};

__device__ __forceinline__ uint32_t ld_dw_guarded(const uint8_t* f, uint64_t n, uint64_t o) {
  if (o + 4 <= n) return *(const uint32_t*)(f + o);
  uint32_t v = 0;
  for (int k = 0; k < 4; k++)
    if (o + k < n) v |= (uint32_t)f[o + k] << (8 * k);
  return v;
}
__device__ __forceinline__ uint64_t ld_u64_unaligned(const uint8_t* f, uint64_t o) {
  uint64_t v = 0;
  for (int k = 0; k < 8; k++) v |= (uint64_t)f[o + k] << (8 * k);
  return v;
}
__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t* f, uint64_t o) {
  uint32_t v = 0;
  for (int k = 0; k < 4; k++) v |= (uint32_t)f[o + k] << (8 * k);
  return v;
}
__device__ __forceinline__ uint64_t prepad64(uint64_t o) { return (64 - (o & 63)) & 63; }

// Stores of results another kernel reads (the glue's outputs, the scan's
// records and tile values): relaxed system-scope stores (sc0 sc1), written
// through the XCD's L2 instead of sitting there dirty.  Dirty lines were
// written back while the scan streamed (and at every kernel's end, before the
// next one started); in the same process, scan + glue write-through vs the
// round-5 policies (plain scan stores, nontemporal glue stores): call -2.3 /
// -4.5 % on two boxes, and the contexts' spread shrank (profiles/r06/
// lib_ab_store_policy_*.txt).  SRD_GLUE_STORE: 0 nontemporal (round 5), 1
// system scope (default), 2 agent scope (a timing A/B knob).
#ifndef SRD_GLUE_STORE
#define SRD_GLUE_STORE 1
#endif
template <class T, class V>
__device__ __forceinline__ void srd_gst(T* p, V v) {
  if constexpr (SRD_GLUE_STORE == 1) __hip_atomic_store(p, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else if constexpr (SRD_GLUE_STORE == 2) __hip_atomic_store(p, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __builtin_nontemporal_store((T)v, p);
}

// A claim on a parent: the generation in the high word (stale words of
// earlier calls lose any atomicMax), ~g in the low word, so the claimer with
// the SMALLEST slot (file order) holds the parent.  The real child of p is
// the first node after p in file order; a false candidate that resolves to p
// lies later (C3: a candidate 8 bytes past some metadata reads that entry's
// CRC as its prev field, and one in ~7000 such CRCs equals a real tail below
// 4 GiB) -- with the largest claimer winning it took the parent from the real
// child, and every C3 call went through the retry rounds.
__device__ __forceinline__ unsigned long long claim_word(uint32_t gen, uint64_t g) {
  return ((unsigned long long)gen << 32) | (0xffffffffull - (g & 0xffffffffull));
}
// the 20-byte metadata record at m (entry_metadata.rs:75-112), any alignment;
// reads the dwords covering [m, m + 20) (the buffer is padded past file_len)
__device__ __forceinline__ void ld_meta(const uint8_t* f, uint64_t m, uint64_t* kh, uint64_t* p, uint32_t* crc) {
  const uint32_t* q = (const uint32_t*)(f + (m & ~3ull));
  const uint32_t sh = (uint32_t)(m & 3) * 8;
  uint32_t w[6], v[5];
#pragma unroll
  for (int i = 0; i < 6; i++) w[i] = q[i];
#pragma unroll
  for (int i = 0; i < 5; i++) v[i] = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
  *kh = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
  *p = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
  *crc = v[4];
}
// zero the bytes of dword v (file offset o) at or past n
__device__ __forceinline__ uint32_t mask_past_end(uint32_t v, uint64_t o, uint64_t n) {
  if (o + 4 <= n) return v;
  if (o >= n) return 0u;
  return v & ((1u << (8 * (uint32_t)(n - o))) - 1u);
}
__device__ __forceinline__ uint32_t mask_past_end32(uint32_t v, uint32_t o, uint32_t n) {
  if (o + 4 <= n) return v;
  if (o >= n) return 0u;
  return v & ((1u << (8 * (n - o))) - 1u);
}

// raw buffer resource over [base, base + bytes) for stores whose unused lanes
// pass OOB_OFF (out of range: the hardware drops them)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t OOB_OFF = 0xFFFFFFFFu;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);  // gfx9 raw dword format
}

__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbit(hi, lo, sh);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}

// --------------------------------------------------------------------------
// 1. the fused streaming scan
// --------------------------------------------------------------------------
// LDS: slice-by-4 CRC tables replicated 32 times (lane l reads copy l%32,
// so the 32 lanes of a ds_read_b32 group hit at most 2 distinct addresses per
// bank), the lane-weight nibble tables (entry (pos,nib) of lane l at word
// ((pos*16+nib)*64 + l): every lane its own bank, conflict-free) and one
// 24-dword window per wave for the cooperative candidate check.
constexpr int SCAN_WAVES_V2 = 16;
struct alignas(2048) ScanLds {
  // the last slice-by-4 step of 16-byte chain q (q < 3) with the chain's
  // join shift folded in: byte i of s -> (b << 8i) * x^(32 + 128 (3 - q)),
  // so the line CRC is the XOR of the four chains' last steps (crc_line4)
  uint32_t last[3 * 4 * 256];      // 12 KiB, not replicated; first, so its
                                   // lookups carry the table base in the ds_read offset field (no base VGPRs)
  uint32_t tab[4 * 256 * 32];      // 128 KiB slice-by-4 tables, conflict-free (layout: tab_lookup)
  uint32_t nib[8 * 16 * 32];       // 16 KiB: c -> c * x^(512*(31 - l%32)), bank = l%32
  uint32_t win[SCAN_WAVES_V2][24];
  // the epilogue's block reduction
  uint64_t s_root[SCAN_WAVES_V2], s_ovf[SCAN_WAVES_V2];
  uint32_t s_last;
};
static_assert(offsetof(ScanLds, nib) % 2048 == 0, "lane_weight_or ORs nibble bits 7-10 into the table base");

// Slice-by-4 with v_perm addressing.  LDS layout of the 4 tables: word
// b*64 + (t&1)*32 + c (+ 16384*(t>>1)), c = lane%32 -> byte address
// [t>>1 : b : (t&1)*128 + 4c], so the lookup address of byte j of s is ONE
// v_perm_b32(s, R_t) and every 32-lane group hits 32 distinct banks.
__device__ __forceinline__ uint32_t tab_lookup(const ScanLds& L, uint32_t s, uint32_t R, uint32_t sel) {
  const uint32_t addr = __builtin_amdgcn_perm(s, R, sel);
  return *(const uint32_t*)((const char*)L.tab + addr);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // one v_bitop3_b32
}
__device__ __forceinline__ uint32_t mulfix(uint32_t v, const uint32_t* __restrict__ m) {
  return m[v & 0xff] ^ m[256 + ((v >> 8) & 0xff)] ^ m[512 + ((v >> 16) & 0xff)] ^ m[768 + (v >> 24)];
}
// The raw CRC-32 of a lane's 64-byte line by slice-by-4 as 4 independent
// 16-byte chains (4 dependent LDS round trips instead of 16): raw(line) = a x^384 ^ b x^256 ^ c x^128 ^ d for
// the chains' raw CRCs a..d, and chain q's last step looks its bytes up in
// tables that already carry the x^(128 (3 - q)) shift (ScanLds::last), so the
// joins cost no lookups of their own.
__device__ __forceinline__ uint32_t crc_line4(const uint32_t (&d)[16], const ScanLds& L, const uint32_t (&R)[4]) {
  constexpr uint32_t SEL0 = 0x0c020400u, SEL1 = 0x0c020500u, SEL2 = 0x0c020600u, SEL3 = 0x0c020700u;
  uint32_t s[4] = {d[0], d[4], d[8], d[12]};
#pragma unroll
  for (int j = 0; j < 3; j++) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t t3 = tab_lookup(L, s[q], R[3], SEL0), t2 = tab_lookup(L, s[q], R[2], SEL1);
      const uint32_t t1 = tab_lookup(L, s[q], R[1], SEL2), t0 = tab_lookup(L, s[q], R[0], SEL3);
      s[q] = xor3(xor3(t3, t2, d[4 * q + j + 1]), t1, t0);
    }
  }
  uint32_t v[4];
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const uint32_t* m = L.last + 1024 * q;
    v[q] = xor3(m[s[q] & 0xff], m[256 + ((s[q] >> 8) & 0xff)], m[512 + ((s[q] >> 16) & 0xff)]) ^ m[768 + (s[q] >> 24)];
  }
  v[3] = xor3(tab_lookup(L, s[3], R[3], SEL0), tab_lookup(L, s[3], R[2], SEL1), tab_lookup(L, s[3], R[1], SEL2)) ^
         tab_lookup(L, s[3], R[0], SEL3);
  return xor3(v[0], v[1], v[2]) ^ v[3];
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
constexpr int DPP_WAVE_SHL1 = 0x130;  // lane i <- lane i+1 (0 past the end)
constexpr int DPP_WAVE_SHR1 = 0x138;  // lane i <- lane i-1
constexpr int DPP_ROW_SHL = 0x100;    // + n: lane i <- lane i+n inside a row of 16

// c * x^(512*(31 - lane%32)) via 8 nibble lookups: the lane weight relative
// to the end of the lane's HALF of the tile (lanes >= 32: relative to the
// tile end, i.e. final; lanes < 32: relative to line 31, corrected on use).
__device__ __forceinline__ uint32_t lane_weight(uint32_t c, const uint32_t* __restrict__ nib, int lane) {
  uint32_t v[8];
  const char* base = (const char*)(nib + (lane & 31));
#pragma unroll
  for (int pos = 0; pos < 8; pos++) {
    const uint32_t nb = __builtin_amdgcn_ubfe(c, 4 * pos, 4);
    v[pos] = *(const uint32_t*)(base + pos * 2048 + (nb << 7));  // nib[((pos*16 + nb) << 5) + lane%32]
  }
  return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6] ^ v[7]);
}
// v_writelane_b32 (the LLVM intrinsic; this clang has no builtin for it):
// lane `lane` (uniform) of `old` takes `val`
__device__ int srd_llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t writelane_u32(uint32_t val, int lane, uint32_t old) {
  return (uint32_t)srd_llvm_writelane((int)val, lane, (int)old);
}
// LDS byte offsets (address space 3) for explicit address arithmetic
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ uint32_t lds_ld(uint32_t off) {
  return *(const __attribute__((address_space(3))) uint32_t*)(uintptr_t)off;
}
// crc_line4 with each level's 16 lookups issued together: the scheduler
// otherwise issues two chains' 8 lookups and drains them before the other
// two chains' (8 dependent LDS round trips per line instead of 4).  Groups:
// per level the 16 address VALU, the 16 LDS reads, then the XORs.
__device__ __forceinline__ uint32_t crc_line4_wide(const uint32_t (&d)[16], const ScanLds& L, const uint32_t (&R)[4]) {
  constexpr uint32_t SEL0 = 0x0c020400u, SEL1 = 0x0c020500u, SEL2 = 0x0c020600u, SEL3 = 0x0c020700u;
  uint32_t s[4] = {d[0], d[4], d[8], d[12]};
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 3; j++) {
    uint32_t t[4][4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      t[q][3] = tab_lookup(L, s[q], R[3], SEL0);
      t[q][2] = tab_lookup(L, s[q], R[2], SEL1);
      t[q][1] = tab_lookup(L, s[q], R[1], SEL2);
      t[q][0] = tab_lookup(L, s[q], R[0], SEL3);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) s[q] = xor3(xor3(t[q][3], t[q][2], d[4 * q + j + 1]), t[q][1], t[q][0]);
    __builtin_amdgcn_sched_group_barrier(0x0002, 16, 0);  // the 16 lookup addresses
    __builtin_amdgcn_sched_group_barrier(0x0100, 16, 0);  // the 16 LDS reads
    __builtin_amdgcn_sched_group_barrier(0x0002, 8, 0);   // the XORs
  }
  // the last level: chains 0-2 through the shifted tables (ScanLds::last,
  // byte i of s at word 1024 q + 256 i + byte), chain 3 through tab
  const uint32_t lb = lds_off(L.last);
  uint32_t t[4][4];
#pragma unroll
  for (int q = 0; q < 3; q++)
#pragma unroll
    for (int i = 0; i < 4; i++) t[q][i] = lds_ld(lb + 4096u * q + 1024u * i + 4u * ((s[q] >> (8 * i)) & 0xffu));
  t[3][3] = tab_lookup(L, s[3], R[3], SEL0);
  t[3][2] = tab_lookup(L, s[3], R[2], SEL1);
  t[3][1] = tab_lookup(L, s[3], R[1], SEL2);
  t[3][0] = tab_lookup(L, s[3], R[0], SEL3);
  uint32_t v[4];
#pragma unroll
  for (int q = 0; q < 4; q++) v[q] = xor3(t[q][0], t[q][1], t[q][2]) ^ t[q][3];
  __builtin_amdgcn_sched_group_barrier(0x0002, 16, 0);
  __builtin_amdgcn_sched_group_barrier(0x0100, 16, 0);
  const uint32_t r = xor3(v[0], v[1], v[2]) ^ v[3];
  __builtin_amdgcn_sched_barrier(0);
  return r;
}
// lane_weight for the scan, whose nib table sits at a 2 KiB-aligned LDS
// offset: the nibble's address bits (7-10) are OR-ed into the lane's base
// (one v_and_or_b32 after the shift instead of and + add)
__device__ __forceinline__ uint32_t lane_weight_or(uint32_t c, uint32_t lbase) {
  uint32_t v[8];
#pragma unroll
  for (int pos = 0; pos < 8; pos++) {
    const int sh = 4 * pos - 7;  // nibble pos -> address bits 7-10
    const uint32_t x = sh < 0 ? c << (-sh) : c >> sh;
    v[pos] = lds_ld(((x & 0x780u) | lbase) + pos * 2048);
  }
  return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6] ^ v[7]);
}
__device__ __forceinline__ uint32_t mul16k(uint32_t v, const uint32_t* __restrict__ m) {
  return m[v & 0xff] ^ m[256 + ((v >> 8) & 0xff)] ^ m[512 + ((v >> 16) & 0xff)] ^ m[768 + (v >> 24)];
}
// Half-tile suffix XOR: lanes >= 32 get XOR_{i>=l} u_i (the true SX_l);
// lanes < 32 get XOR_{l<=i<32} u_i (true SX_l = mul16k(.) ^ SX_32).
__device__ __forceinline__ uint32_t half_suffix_xor(uint32_t v, int lane) {
  v ^= dpp<DPP_ROW_SHL + 1>(v);
  v ^= dpp<DPP_ROW_SHL + 2>(v);
  v ^= dpp<DPP_ROW_SHL + 4>(v);
  v ^= dpp<DPP_ROW_SHL + 8>(v);
  // rows 0 and 2 add the totals of rows 1 and 3 (held by lanes 16, 48):
  // row_newbcast:0 on rows 1 and 3 only ({0, T1, 0, T3}), then
  // v_permlane16_swap against zero moves rows 1 / 3 down to rows 0 / 2
  const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150, 0xA, 0xF, false);
  const auto sw = __builtin_amdgcn_permlane16_swap(t, 0u, false, false);
  (void)lane;
  return v ^ sw[1];
}

// the LDS tables of the line-CRC machinery (crc_line*, lane_weight); ends
// with a block barrier.  One 1024-thread block: every thread issues its three
// global loads (one table word, 16 B of the nibble tables, 16 B of the last-
// step tables) before any LDS store, then writes its word's 32 replicas with
// 16-byte stores (a load -> store loop per word took ~10 us of the scan)
// COAL: the writer's coalesced lane layout (DevTables::last_c / nib_c)
template <bool COAL = false>
__device__ __forceinline__ void load_crc_lds(ScanLds& lds) {
  static_assert(SCAN_WAVES_V2 * 64 == 1024 && sizeof(lds.nib) == 1024 * 16 && sizeof(lds.last) <= 1024 * 16,
                "one 16-byte piece of nib / last per thread");
  const uint32_t u = threadIdx.x;  // tab word u: hi = u >> 9, b = (u >> 1) & 255, t = 2 hi + (u & 1)
  const uint32_t tv = g_tabs.tab[2 * (u >> 9) + (u & 1)][(u >> 1) & 255];
  const u32x4 nv = ((const u32x4*)(COAL ? g_tabs.nib_c : g_tabs.nib))[u];
  constexpr uint32_t NLAST = sizeof(lds.last) / 16;
  const u32x4 lv = ((const u32x4*)(COAL ? &g_tabs.last_c[0][0][0] : &g_tabs.last[0][0][0]))[u < NLAST ? u : 0];
  u32x4* const tr = (u32x4*)(lds.tab + 32 * u);  // tab_lookup's layout: word (hi, b, t & 1, copy)
#pragma unroll
  for (int j = 0; j < 8; j++) tr[j] = u32x4{tv, tv, tv, tv};
  ((u32x4*)lds.nib)[u] = nv;
  if (u < NLAST) ((u32x4*)lds.last)[u] = lv;
  __syncthreads();
}
// lane l's slice-by-4 lookup bases (tab_lookup)
__device__ __forceinline__ void crc_lane_bases(uint32_t (&R)[4], int lane) {
#pragma unroll
  for (int t = 0; t < 4; t++) R[t] = ((uint32_t)(t >> 1) << 16) | ((uint32_t)(t & 1) * 128u + 4u * (lane & 31));
}

// recover_valid_chain's outer loop (data_store.rs:388-479) walks the cursor t
// down from file_len and skips every t whose metadata fails its first test,
// entry_start < metadata_offset (:390-420; entry_start = prev + prepad(prev),
// or prev for a tombstone, u64 wrapping).  The optimistic pass starts at the
// largest t that passes it -- file_len itself for an intact store, file_len -
// 7 after b"CORRUPT" was appended (persistence_tests.rs:126-173) -- searched
// within TOP_WINDOW bytes below file_len (whole file; a shard's tail is
// given: only t = file_len).  Returns t when its entry is a strong node (p >=
// 20, p < m, a nonzero checksum field, the prepad / tombstone rule) or a root
// (p == 0: one entry spans [0, t)); 0 otherwise, and the full pass decides.
// Every candidate the scan records lies at or below t - 20: a strong node
// above it would pass the same test.
constexpr uint32_t TOP_WINDOW = 256;
__device__ __forceinline__ uint64_t find_top(const uint8_t* file, uint64_t flen, bool search) {
  const int lane = threadIdx.x & 63;
  const uint32_t steps = search ? TOP_WINDOW / 64 : 1;
  for (uint32_t s = 0; s < steps; s++) {
    const uint64_t d = (uint64_t)s * 64 + (uint64_t)lane;  // t = flen - d
    const bool has = (search || lane == 0) && flen >= 21 + d;
    const uint64_t m = (has ? flen - d : flen) - 20;      // flen >= 21 (the caller's guard)
    uint64_t kh, p;
    uint32_t crc;
    ld_meta(file, m, &kh, &p, &crc);
    const uint32_t bw = *(const uint32_t*)(file + ((m - 1) & ~3ull));
    const bool zb = ((bw >> (8 * ((m - 1) & 3))) & 0xffu) == 0;  // byte m - 1: the tombstone byte when p == m - 1
    const bool tomb = m > p && m - p == 1 && zb;
    const uint64_t es = tomb ? p : p + prepad64(p);
    const uint64_t pass = __ballot(has && es < m);
    if (!pass) continue;
    const int l = __builtin_ctzll(pass);  // the largest passing t of the step
    // (readlane returns int: widen through uint32_t, or bit 31 sign-extends)
    const uint64_t pl = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(p >> 32), l) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)p, l);
    const uint32_t cl = (uint32_t)__builtin_amdgcn_readlane(crc, l);
    const bool zl = __builtin_amdgcn_readlane((uint32_t)zb, l) != 0;
    const uint64_t t = flen - ((uint64_t)s * 64 + (uint64_t)l), ml = t - 20, dp = ml - pl;
    const bool strong = pl >= 20 && pl < ml && cl != 0 && (dp > prepad64(pl) || (dp == 1 && zl));
    return (pl == 0 || strong) ? t : 0;
  }
  return 0;
}

// Link record r of scan wave w (slot w*wcap + r; the optimistic pass, after
// the scan): the deferred node test of a single-candidate record
// (data_store.rs:404-470), its parent -- the previous record in file order
// when that record's metadata sits at p - 20, else a binary search in the
// parent's span -- and the claim on it (the earliest claimer wins).
__device__ void link_record(const ScanArgs& a, uint64_t w, uint64_t r) {
  const uint64_t gi = w * a.wcap + r;
  uint64_t gprev = 0;
  bool hp = true;
  if (r > 0) {
    gprev = gi - 1;
  } else if (w == 0) {
    hp = false;  // the first resident record: nothing before it is resident
  } else {
    const uint64_t wt = a.wave_total[w - 1] & ~(1ull << 63);
    hp = wt > 0 && wt <= a.wcap;  // an overflowed wave fails the pass anyway (ST_OVERFLOW)
    gprev = (w - 1) * a.wcap + (hp ? wt - 1 : 0);
  }
  // the record two back too (the same cache line, beside the others): C2's
  // false candidates sit one byte past a real record's metadata (a CRC whose
  // low byte is 0), so the real child of that record finds its parent there
  // instead of by a dependent search (~1/256 of the records; each one was
  // a whole block's critical path)
  const bool hp2 = r >= 2;
  const uint64_t m = a.c_m[gi], mprev = hp ? a.c_m[gprev] : 0, mprev2 = hp2 ? a.c_m[gi - 2] : 0;
  const u32x4 r0 = a.c_rec[gi];  // {p, flags, crc}: the record's half link2 needs
  const uint64_t p = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);
  bool node = true, tomb = false;
  if (r0[2] & F_NT) {
    // single-candidate record, deferred node test; F_ZB is the byte at m - 1,
    // the tombstone byte when p == m - 1
    const uint64_t dp = m - p;
    tomb = dp == 1 && (r0[2] & F_ZB);
    node = p >= 20 && p < m && (tomb || dp > prepad64(p));
  }
  const uint64_t mp = p - 20;  // p >= 20 for nodes
  const uint64_t sp2 = (mp + 14) / SPAN_BYTES;  // span s holds m in [16 KiB s - 14, +16 KiB)
  // in a store without garbage the parent is the previous record: one load
  int64_t par = hp && mprev == mp ? (int64_t)gprev : hp2 && mprev2 == mp ? (int64_t)(gi - 2) : PAR_MISS;
  // Otherwise a record at mp needs mp's prev field pp = u64 at p - 12 with
  // 20 <= pp < mp (every record is a strong node, data_store.rs:404-470).
  // One 8-byte file read settles most misses here: a false candidate's p is
  // whatever its checksum bytes held (C3: ~940 K of them per call, p
  // anywhere in the first 4 GiB), whose "parent" bytes are payload: no
  // binary search in a random span for it.  pp == 0 is the root rule below.
  // (Resident bytes only: in span mode p - 20 may lie below the span.)
  uint64_t pp = 1;
  const bool res = mp >= a.k_lo * (uint64_t)TILE;
  if (node && par == PAR_MISS && res) pp = ld_u64_unaligned(a.file, p - 12);
  const bool maybe_rec = !res || (pp >= 20 && pp < mp);
  if (node && par == PAR_MISS && maybe_rec && sp2 >= a.part.s_lo && sp2 < a.n_spans) {
    const uint64_t w2 = part_span_wave(a.part, sp2 - a.part.s_lo);
    const uint32_t f2 = a.span_first[sp2];
    const uint32_t n2 = (uint32_t)min<uint64_t>(a.span_count[sp2], a.wcap - min<uint64_t>(f2, a.wcap));
    uint32_t lo = 0, hi = n2;
    const uint64_t* cm = a.c_m + w2 * a.wcap + f2;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (cm[mid] < mp) lo = mid + 1; else hi = mid;
    }
    if (lo < n2 && cm[lo] == mp) par = (int64_t)(w2 * a.wcap + f2 + lo);
  }
  if (!node) {
    par = PAR_MISS;  // no parent, no root
  } else if (par == PAR_MISS) {
    if (a.span_lo) {
      if (p == a.span_lo) par = PAR_ROOT;  // the shard's first entry (its parent is the previous shard's last)
    } else if (p >= 21 && pp == 0) {
      par = PAR_ROOT;  // the parent is the root entry (prev 0), data_store.rs:404-416
    }
  }
  // (plain stores: written through like the scan's records, link2's own
  // words made the glue 3-5 us slower, profiles/r06/lib_ab_store_policy_r6u.txt)
  if (tomb) a.c_rec[gi] = u32x4{r0[0], r0[1], r0[2] | F_TOMB, r0[3]};
  a.d_par[gi] = (int32_t)par;
  if (par >= 0) atomicMax(&a.childof[par], claim_word(a.gen, gi));
}

// The link step (optimistic pass), one block per scan wave right after the
// scan: every record of the wave's region through link_record.  (Round 4
// tried it inside the scan's epilogue -- each block linking its own records
// once its tiles were done, the last block the records that needed another
// block's: the early blocks' work hid, but the last block's ~4 K (C2) to
// ~40 K (C3) records in one block sat on the scan's critical path, and the
// scan ran 6 % (C2) to 11 % (C3) longer for a 22 us kernel saved.)
// LINK_WPB scan waves per block (256 threads each; 2: 20.7 -> 24.0 us at C2,
// profiles/r05/kernel_stats_r5k.csv)
constexpr uint32_t LINK_WPB = 1;
// The next call's block starts (XPart, block 0 of link2_kernel, 256 threads,
// after its own records: off the critical path of the call): each XCD's speed
// = spans / ticks summed over its blocks of this scan, relative to the mean
// over the XCDs, then w = 0.25 w + 0.75 that (the pattern changes over tens
// of calls: profiles/r06/xcc_blocks_r6{e,g}.json), clamped to 1 +- XP_CLAMP; block b gets a
// share of the spans proportional to the speed of the XCD it ran on (the
// block -> XCD map is fixed per HW queue).  st(0) = 0, st(g) = ns, and no
// block exceeds (1 + XP_CLAMP) / (1 - XP_CLAMP) of the even share + 1 span
// (the host's slot-space bound, optimistic_pass).
__device__ void xpart_update(const ScanArgs& a) {
  __shared__ unsigned long long s_sp[8], s_du[8], s_t0, s_t1;
  __shared__ float s_w[8];
  __shared__ double s_pre[256 / 64 + 1];
  XPart* xp = a.xp;
  const ScanPart& p = a.part;
  const uint32_t g = p.g, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t < 8) { s_sp[t] = 0; s_du[t] = 0; }
  if (t == 0) { s_t0 = ~0ull; s_t1 = 0; }
  __syncthreads();
  for (uint32_t b = t; b < g; b += 256) {
    const uint32_t x = xp->xcc[b] & 7u;
    const uint64_t t0 = xp->t0[b], du = xp->dur[b];
    atomicAdd(&s_sp[x], (unsigned long long)(part_block_start(p, b + 1) - part_block_start(p, b)));
    atomicAdd(&s_du[x], (unsigned long long)du);
    atomicMin(&s_t0, (unsigned long long)t0);
    atomicMax(&s_t1, (unsigned long long)(t0 + du));
  }
  __syncthreads();
  if (t == 0) {
    xp->scan_ticks = s_t1 > s_t0 ? s_t1 - s_t0 : 0;  // (the host's load-pattern choice, via idx_emit)
    float sp[8], mean = 0;
    int nx = 0;
    for (int x = 0; x < 8; x++) {
      sp[x] = s_du[x] && s_sp[x] ? (float)s_sp[x] / (float)s_du[x] : 0.f;
      if (sp[x] > 0) { mean += sp[x]; nx++; }
    }
    mean = nx ? mean / nx : 1.f;
    for (int x = 0; x < 8; x++) {
      const float m = sp[x] > 0 ? sp[x] / mean : 1.f, old = xp->w[x];
      float v = old > 0 ? 0.25f * old + 0.75f * m : m;
      v = fminf(fmaxf(v, 1.f - XP_CLAMP), 1.f + XP_CLAMP);
      xp->w[x] = v;
      s_w[x] = v;
    }
  }
  __syncthreads();
  // st(b) = round(ns * (q_0 + .. + q_(b-1)) / sum q), q_b = the speed of b's XCD
  auto q_of = [&](uint32_t b) -> double { return b < g ? (double)s_w[xp->xcc[b] & 7u] : 0.0; };
  double part = 0;
  for (uint32_t b = t; b < g; b += 256) part += q_of(b);
#pragma unroll
  for (int o = 32; o; o >>= 1) part += __shfl_xor(part, o);
  if (lane == 0) s_pre[wv] = part;
  __syncthreads();
  const double tot = s_pre[0] + s_pre[1] + s_pre[2] + s_pre[3];
  __syncthreads();
  uint64_t* nb = xp->bs[a.xp_next];
  double acc = 0;  // the prefix of the chunks before this one
  for (uint32_t b0 = 0; b0 < g; b0 += 256) {
    const uint32_t b = b0 + t;
    const double q = q_of(b);
    double x = q;  // inclusive wave prefix
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(x, o);
      if ((int)lane >= o) x += y;
    }
    if (lane == 63) s_pre[wv] = x;
    __syncthreads();
    double wpre = 0, ctot = 0;
    for (uint32_t i = 0; i < 4; i++) {
      wpre += i < wv ? s_pre[i] : 0.0;
      ctot += s_pre[i];
    }
    __syncthreads();
    if (b < g) nb[b] = b == 0 ? 0 : (uint64_t)((double)p.ns * ((acc + wpre + x - q) / tot) + 0.5);
    acc += ctot;
  }
  if (t == 0) nb[g] = p.ns;
}
// The optimistic scan's per-wave results reduced (the scan kernel has no
// last-block epilogue in this pass): k_total[0] = the records, k_total[1] =
// 1 + the last record's slot, counters[0] = the largest root tail,
// counters[2] = a region overflowed.  Blocks [0, ceil(n_waves / 256)) of
// link2_kernel, one scan wave per thread, after their own records, combine
// their slices with four global atomics (the scan's block 0 zeroed the
// words); link_record reads wave_total directly, the glue kernels after
// link2 read these.
__device__ void scan_reduce(const ScanArgs& a, uint32_t n_waves) {
  __shared__ unsigned long long s_sum, s_smax, s_rmax, s_ovf;
  if (threadIdx.x == 0) { s_sum = 0; s_smax = 0; s_rmax = 0; s_ovf = 0; }
  __syncthreads();
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint64_t sum = 0, smax = 0, rmax = 0, o = 0;
  if (i < n_waves) {
    const uint64_t v = a.wave_total[i], cnt = v & ~(1ull << 63);
    sum = cnt;
    o = v >> 63;
    rmax = a.wave_root[i];
    if (cnt) smax = (uint64_t)i * a.wcap + min(cnt, a.wcap);
  }
  rmax = wave_max_u64(rmax);
  smax = wave_max_u64(smax);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    o |= __shfl_xor(o, d);
    sum += __shfl_xor(sum, d);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&s_sum, (unsigned long long)sum);
    atomicMax(&s_smax, (unsigned long long)smax);
    atomicMax(&s_rmax, (unsigned long long)rmax);
    atomicOr(&s_ovf, (unsigned long long)o);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd((unsigned long long*)&a.k_total[0], s_sum);
    atomicMax((unsigned long long*)&a.k_total[1], s_smax);
    atomicMax((unsigned long long*)&a.counters[0], s_rmax);
    atomicOr((unsigned long long*)&a.counters[2], s_ovf);
  }
}
__global__ __launch_bounds__(256 * LINK_WPB) void link2_kernel(ScanArgs a, uint32_t n_waves) {
  const uint64_t w = (uint64_t)blockIdx.x * LINK_WPB + threadIdx.x / 256;
  if (w < n_waves) {
    const uint64_t nrec = min(a.wave_total[w] & ~(1ull << 63), a.wcap);  // records past wcap: ST_OVERFLOW
    for (uint64_t r = threadIdx.x % 256; r < nrec; r += 256) link_record(a, w, r);
  }
  if ((uint64_t)blockIdx.x * 256 < n_waves) scan_reduce(a, n_waves);
  // the next call's block starts in a block of the first dispatch round that
  // reduces no slice (C2: 4096 waves -> blocks 0-15 reduce, 16 does this)
  if (a.xp && blockIdx.x == min((n_waves + 255) / 256, gridDim.x - 1)) xpart_update(a);
}

// ---- coalesced nontemporal tile loads (the product scan's, round 5) ----
// The scan's line-per-lane loads (lane l: 16 B at 64 l + 16 j) stream at
// ~6.0-6.1 TB/s; loads whose every instruction reads 1 KiB contiguous, with
// the nontemporal bit, at ~6.75 TB/s (tools/stream_map_probe.hip,
// profiles/r05/stream_cpol_probe.txt; nt on the line-per-lane pattern: 3.6).
// The load puts lane l = 16 B + 4 A + C on 16 B at 1024 j + 256 A + 64 C + 16 B
// (quarter B of line 16 j + 4 A + C; every instruction reads its 1 KiB whole,
// each 16-lane row 16 B of 16 lines), so the quarter index sits in lane bits
// 4-5 and two register <-> lane field swaps by v_permlane16/32_swap move line L
// to lane L, quarter q to dwords 4q..4q+3: 16 VALU per tile.  (Rounds 5-6a
// put the quarter in lane bits 2-3 -- 256 contiguous bytes per row -- and
// needed 32 DPP bank swaps + 16 copies more for the same loads: the
// quarter-in-row layout streams alike and the scan runs 1-2 % faster at C2,
// 4-5 % at C3, profiles/r06/variant_ab_rowq_c{2,3}.txt)
__device__ __forceinline__ uint32_t coal_lane_off(int lane, int j) {
  return 1024u * (uint32_t)j + 256u * (((uint32_t)lane >> 2) & 3u) + 64u * ((uint32_t)lane & 3u) +
         16u * ((uint32_t)lane >> 4);
}
template <int RB, bool P32>
__device__ __forceinline__ void coal_pswap(uint32_t (&d)[16]) {  // register bit RB <-> lane bit 4 (P32: 5)
#pragma unroll
  for (int r0 = 0; r0 < 4; r0++) {
    if (r0 & RB) continue;
    const int r1 = r0 | RB;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const auto w = P32 ? __builtin_amdgcn_permlane32_swap(d[4 * r0 + i], d[4 * r1 + i], false, false)
                         : __builtin_amdgcn_permlane16_swap(d[4 * r0 + i], d[4 * r1 + i], false, false);
      d[4 * r0 + i] = w[0];
      d[4 * r1 + i] = w[1];
    }
  }
}
__device__ __forceinline__ void coal_to_lines(uint32_t (&d)[16]) {
  coal_pswap<1, false>(d);
  coal_pswap<2, true>(d);
}

// line-per-lane tile loads (round 4's product): the scan of large stores
// (scan_variant_for); one 16-wave block per CU for every variant
constexpr int SCAN_LINES = 34;
constexpr int scan_nw(int) { return SCAN_WAVES_V2; }

// WIDE: stores above 2^40 bytes (prev offsets up to 48 bits, key_indexer.rs:12-15):
// the level-1 filter looks for the two zero bytes m+14, m+15 at any alignment
template <bool FULL, bool WIDE, int V = 0>
__global__ __launch_bounds__(SCAN_WAVES_V2 * 64) __attribute__((amdgpu_waves_per_eu(4, 4)))
void scan_kernel(ScanArgs a) {
  constexpr int NW = SCAN_WAVES_V2;
  // The product loads each tile coalesced + nontemporal and transposes it in
  // registers (coal_to_lines); SCAN_LINES = round 4's line-per-lane loads
  // (the pass measures both per store: srd_api.hip scan_variant_tune).  Timing-only
  // ablations of SRD_DEBUG_API builds (results wrong; tools/variant_ab.py):
  // 7 = the ring's coalesced loads alone (each tile XOR-folded), 8 = the whole
  // coalesced tile body on two L2-resident tiles per block (no HBM stream).
  // Round 1-5's rejected variants (rotated tables, 2-deep ring, straight-line
  // first flagged line, ...) are in git history.
  static_assert(V == 0 || V == SCAN_LINES || V == 7 || V == 8, "scan variants: 0, SCAN_LINES, 7, 8");
  constexpr bool COALT = V != SCAN_LINES;
  constexpr bool MEMONLY = V == 7, NOHBM = V == 8;
  uint32_t memonly_acc = 0;
  using Lds = ScanLds;
  __shared__ Lds lds;
  constexpr uint64_t RQ_LANES = 64;  // lanes of the record queue rq
  if (blockIdx.x == 0) {
    for (uint32_t i = threadIdx.x; i < a.n_zero_words; i += blockDim.x) a.zero_words[i] = 0;
    for (uint32_t i = threadIdx.x; i < a.n_zero2; i += blockDim.x) a.zero2[i] = 0;
    if (threadIdx.x == 0 && a.sentinel) *a.sentinel = 0;
    if (!FULL && threadIdx.x == 0) {  // link2's scan_reduce combines into these
      a.k_total[0] = 0;
      a.k_total[1] = 0;
      a.counters[0] = 0;
      a.counters[2] = 0;
    }
  }
  uint64_t xp_t0 = 0;  // (thread 0) the block's start, XCD-aware shares
  if (a.xp && threadIdx.x == 0) xp_t0 = __builtin_amdgcn_s_memrealtime();
#ifdef SRD_WAVE_STAMPS
  if (threadIdx.x == 0) {
    g_wave_stamp[8192 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x < 256) g_wave_clk[4096 + blockIdx.x] = __builtin_amdgcn_s_memtime();
    uint32_t xcc, hwid;  // the physical XCD and CU the block runs on (tools/xcc_stamps.py)
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    if (blockIdx.x < 256) g_wave_stamp[8192 + 512 + blockIdx.x] = ((uint64_t)hwid << 32) | xcc;
  }
#endif
  load_crc_lds(lds);
#ifdef SRD_WAVE_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 256) g_wave_stamp[8192 + 256 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif

  const int lane = threadIdx.x & 63;
  // wave id via readfirstlane: provably uniform, so all tile bookkeeping
  // below (k, B, span, bounds) stays in SGPRs / scalar branches
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t R[4];
  crc_lane_bases(R, lane);
  const uint8_t* __restrict__ file = a.file;
  const uint64_t flen = a.flen;
  uint32_t* win = lds.win[wv];
  const uint32_t nib_lane = lds_off(lds.nib) + 4u * (lane & 31);  // 2 KiB-aligned table base + the lane's bank
  auto line_crc = [&](const uint32_t (&x)[16]) -> uint32_t { return crc_line4(x, lds, R); };
  auto lane_wt = [&](uint32_t c) -> uint32_t { return lane_weight_or(c, nib_lane); };

  // contiguous tile range per wave (whole spans, ScanPart)
  const uint64_t total_waves = (uint64_t)gridDim.x * NW;
  const uint64_t w = (uint64_t)blockIdx.x * NW + wv;
  uint64_t r0, r1;
  part_wave_range(a.part, blockIdx.x, (uint32_t)wv, &r0, &r1);
  uint64_t k0 = (a.part.s_lo + r0) * SPAN_TILES;
  uint64_t k1 = min((a.part.s_lo + r1) * SPAN_TILES, a.n_tiles);
  if (k0 >= k1) k0 = k1 = a.k_lo;  // no tiles (the loops below do nothing): the wave joins the epilogue

  // the optimistic pass's start (find_top); none: the waves skip their tiles,
  // record nothing (zero span counts) and the glue reports ST_NOSTART, so the
  // full pass starts ~0.9 ms earlier
  const uint64_t top = FULL ? 0 : find_top(file, flen, a.m_lo == 0);
  if (!FULL && top == 0) {
    const uint64_t sa = k0 / SPAN_TILES, sb = (k1 + SPAN_TILES - 1) / SPAN_TILES;
    for (uint64_t sp = sa + lane; sp < sb; sp += 64) {
      a.span_count[sp] = 0;
      a.span_first[sp] = 0;
    }
    k0 = k1 = a.k_lo;
  }

  uint32_t count = 0;
  uint64_t wtotal = 0;  // wave-uniform: records of the wave's spans
  bool ovf = false;     // wave-uniform: a span had more candidates than slots
  // store batching (registers, flushed with few wide stores): per-tile values
  // of 16 tiles, span counts of 64 spans, and up to 64 records of the span
  // per-tile values, lanes 4 (k % 16) + j of the 16-tile group's register
  // (two: a group can complete in the middle of a ring round, whose later
  // tiles already fill the next group), and span counts / first records in
  // lane span % 64 of scnt / sfirst; stored by the next store point once a
  // group completes (16 tiles, 64 spans) or the wave ends -- few, whole-line
  // stores (one real store per tile and per span was 15 % of the scan)
  uint32_t tacc0 = 0, tacc1 = 0, scnt = 0, sfirst = 0;
  bool tg_pend = false, sg_pend = false;  // uniform: a group to store
  uint64_t tg_base = 0, sg_base = 0;
  uint32_t tg_par = 0, tg_lo = 0, tg_hi = 0, sg_lo = 0, sg_hi = 0;
  uint32_t rq[10];
#pragma unroll
  for (int i = 0; i < 10; i++) rq[i] = 0;
  // records buffered in rq: the wave's records [flushed, wtotal + count) sit
  // in lanes [0, wtotal + count - flushed) (< 64); they are written out with
  // whole-line stores once >= FLUSH_AT are pending (and at the wave's end):
  // a real store holds the prefetch ring's vmcnt waits until it completes,
  // so few large flushes beat one per span
  uint64_t flushed = 0;  // wave-uniform
  uint64_t rvalid = 0;   // wave-uniform: bit j = record flushed + j is in lane j (multi-candidate lines store directly)

  // Unconditional loads: the buffer is readable to srd_padded_size(flen)
  // (no loads under divergent/uniform branches, so the compiler's vmcnt
  // waits never have to drain the prefetch ring).  The tile's code (CRC,
  // lane weights, suffix XOR, filter) is one basic block.
  const uint64_t nohbm_k = (a.part.s_lo + part_block_start(a.part, blockIdx.x)) * SPAN_TILES;
  auto load_tile = [&](uint64_t k, uint32_t (&o)[16]) {
    if constexpr (COALT) {
      const uint8_t* tb = file + (NOHBM ? nohbm_k + (k & 1) : k) * (uint64_t)TILE;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)(tb + coal_lane_off(lane, j)));
        o[4 * j] = v[0]; o[4 * j + 1] = v[1]; o[4 * j + 2] = v[2]; o[4 * j + 3] = v[3];
      }
      return;
    }
    const u32x4* q = (const u32x4*)(file + k * (uint64_t)TILE + 64ull * lane);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      // plain loads: this 64 B-per-lane pattern runs at ~3.8 TB/s with nt, ~6.1 without
      const u32x4 v = q[j];
      o[4 * j] = v[0]; o[4 * j + 1] = v[1]; o[4 * j + 2] = v[2]; o[4 * j + 3] = v[3];
    }
  };

  // Candidate coverage: lane l of tile k tests the positions
  // m in [L-14, L+49] (L = B + 64 l): a node's zero bytes m+13..m+15 hold an
  // aligned zero halfword inside the lane's OWN line, so no lookahead is
  // needed.  Tile k covers [B-14, B+4082), span s covers
  // [16 KiB s - 14, 16 KiB (s+1) - 14) -- link_record looks parents up in
  // span (m + 14) / 16 KiB.  The slow path stages the 22-dword window
  // [L-16, L+72) in LDS: win[0..3] the previous line's tail, win[4..19] the
  // line, win[20..21] the next line's head; win[22] holds the previous
  // tile's SX partial of line 63 (= its true SX_63).
  const uint32_t hb = a.filt_hb;
  uint64_t rootmax = 0;
  {
    // the line just before this wave's first tile: its tail bytes and its raw
    // CRC (= SX_63 of tile k0-1) seed the window; all lanes load it
    uint32_t pl[16];
    const bool has_prev = k0 > a.k_lo;  // the line before the resident range reads as zeros
    const u32x4* q = (const u32x4*)(file + (has_prev ? k0 * (uint64_t)TILE - 64 : k0 * (uint64_t)TILE));
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const u32x4 v = q[j];
      pl[4 * j] = v[0]; pl[4 * j + 1] = v[1]; pl[4 * j + 2] = v[2]; pl[4 * j + 3] = v[3];
    }
    const uint32_t cp = line_crc(pl);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 4; j++) win[j] = has_prev ? pl[12 + j] : 0u;
      win[22] = has_prev ? cp : 0u;
    }
  }

  // first 8 bytes of tile k+1 (line 63's window) by a SCALAR load: the slow
  // loop must not touch a register of the vector prefetch ring, or the
  // compiler drains the whole ring (vmcnt(0)) in front of it
  auto next_head = [&](uint64_t k, uint32_t* n0, uint32_t* n1) {
    const __attribute__((address_space(4))) uint32_t* q =
        (const __attribute__((address_space(4))) uint32_t*)(file + (k + 1) * (uint64_t)TILE);
    *n0 = q[0];
    *n1 = q[1];
  };

  // TAIL (compile-time): tile k lies within TILE + 64 bytes of file_len, so
  // bytes >= flen must read as 0.  Only the last <= 2 tiles of the file are
  // tail tiles; they run after the ring loop, because masking ring registers
  // under a branch inside the loop makes the compiler drain the whole
  // prefetch ring (vmcnt(0)) at the loop header.
  auto process = [&](uint64_t k, uint32_t (&d)[16], auto tail_c) {
    if constexpr (MEMONLY) {
#pragma unroll
      for (int j = 0; j < 16; j++) memonly_acc ^= d[j];
      __builtin_amdgcn_s_setprio(0);
      return;
    }
    constexpr bool tail_tile = decltype(tail_c)::value;
    if constexpr (COALT) coal_to_lines(d);  // lane l <- line l
    const uint64_t B = k * (uint64_t)TILE;
    const uint64_t span = k / SPAN_TILES;
    // bytes left in the file from B (uniform, 32-bit: every in-tile test below
    // is relative to B, so the uniform bookkeeping stays on the scalar unit)
    const uint64_t rem64 = flen - B;
    const uint32_t remu = (rem64 >> 32) ? 0xFFFFFFFFu : (uint32_t)rem64;
    if (tail_tile) {
#pragma unroll
      for (int j = 0; j < 16; j++) d[j] = mask_past_end32(d[j], 64u * lane + 4 * j, remu);
    }

    // the filter first: its VALU fills the CRC's LDS waits and the suffix
    // XOR's DPP hazard slots (same basic block)
    // ---- filter, level 1: any aligned zero halfword in the lane's line
    //      (packed 16-bit min over the 16 dwords: 1 VALU per dword); level 2
    //      (exact, per position) in the slow path.  WIDE: any two adjacent
    //      zero bytes, the last one possibly the next line's first ----
    uint64_t slow;
    if (!WIDE) {
      // a tree, not a chain: back-to-back dependent v_pk_min_u16 need an
      // s_nop between them on gfx950 (15 per tile as a chain)
      u16x2 zm[8];
#pragma unroll
      for (int i = 0; i < 8; i++)
        zm[i] = __builtin_elementwise_min(__builtin_bit_cast(u16x2, d[i]), __builtin_bit_cast(u16x2, d[i + 8]));
#pragma unroll
      for (int w = 4; w > 0; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; i++) zm[i] = __builtin_elementwise_min(zm[i], zm[i + w]);
      const uint32_t z = __builtin_bit_cast(uint32_t, zm[0]);
      slow = __ballot(((z - 0x00010001u) & ~z & 0x80008000u) != 0);  // a zero halfword (exact)
    } else {
      uint32_t nx = __shfl_down(d[0], 1);
      if (lane == 63) {
        uint32_t n0, n1;
        next_head(k, &n0, &n1);
        nx = tail_tile ? mask_past_end32(n0, TILE, remu) : n0;
      }
      uint32_t hz = 0;
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint32_t y = d[i] | alignb(i < 15 ? d[i < 15 ? i + 1 : 15] : nx, d[i], 8);
        hz |= (y - 0x01010101u) & ~y & 0x80808080u;  // a zero byte of y = two zero bytes in a row
      }
      slow = __ballot(hz != 0);
    }
    // ---- per-line raw CRC, lane weight, 64-lane suffix XOR ----
    // Wave priority over the LDS-latency chains (the CRC's lookups here, the
    // flagged-line window below): a wave in them wins the issue arbitration,
    // so its next round of lookups goes out as soon as the last returns,
    // while the other waves fill the gaps (same-box A/B: -4 %)
    __builtin_amdgcn_s_setprio(3);
    const uint32_t c = line_crc(d);
    __builtin_amdgcn_s_setprio(0);
    const uint32_t hx = half_suffix_xor(lane_wt(c), lane);
    // per-tile values: lanes 0, 1 their half partials, lane 32 the true SX_32.
    // Buffered in lanes 4(k%16) + {0,1,2} of tacc; one 256-B store per 16
    // tiles.  Every store of this loop is an UNCONDITIONAL buffer store whose
    // unused lanes carry an out-of-range offset (dropped by the hardware): a
    // store under a branch makes the count of memory ops between a prefetch
    // load and its wait path-dependent, and the compiler then waits for the
    // store's completion too (measured: ~10 % of the kernel).
    {
      const int t = (int)(k & 15);
      const uint32_t v0 = __builtin_amdgcn_readlane(hx, 0), v1 = __builtin_amdgcn_readlane(hx, 1),
                     v2 = __builtin_amdgcn_readlane(hx, 32);
      // (branch-free: a uniform branch here split the tile's basic block)
      const bool odd = (k >> 4) & 1;
      uint32_t tv = odd ? tacc1 : tacc0;
      tv = writelane_u32(v0, 4 * t, tv);
      tv = writelane_u32(v1, 4 * t + 1, tv);
      tv = writelane_u32(v2, 4 * t + 2, tv);
      tacc0 = odd ? tacc0 : tv;
      tacc1 = odd ? tv : tacc1;
      if (t == 15 || k + 1 == k1) {  // uniform: the group is complete
        const uint64_t g = k & ~15ull;
        tg_pend = true;
        tg_base = g;
        tg_par = odd ? 1u : 0u;
        tg_lo = (uint32_t)(max(g, k0) - g) * 4;
        tg_hi = 4u * t + 4u;
      }
    }

    // Re-define d by an empty asm once its loads have been consumed: a loop
    // that stores and uses a register last written by a pending VMEM load
    // makes the compiler flush vmcnt to 0 in the loop preheader, draining the
    // prefetch ring on every flagged tile.
    // (one statement: an asm per register put an s_nop hazard guard after each)
    asm volatile("" : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]),
                 "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13]), "+v"(d[14]), "+v"(d[15]));

    // (the flagged-line chain one level below the CRC's: -1.3 % vs equal)
    if (slow) __builtin_amdgcn_s_setprio(2);
    while (slow) {
      const int f = __builtin_ctzll(slow);
      slow &= slow - 1;
      // stage [L-16, L+72) from lane f alone: its line, the previous line's
      // tail and the next line's head moved into every lane by DPP (one exec
      // group, 16-byte LDS stores); f == 0: the previous tile's tail is
      // already in win[0..3]; f == 63: the next tile's head by a scalar load
      const uint32_t p12 = dpp<DPP_WAVE_SHR1>(d[12]), p13 = dpp<DPP_WAVE_SHR1>(d[13]),
                     p14 = dpp<DPP_WAVE_SHR1>(d[14]), p15 = dpp<DPP_WAVE_SHR1>(d[15]);
      uint32_t n0 = dpp<DPP_WAVE_SHL1>(d[0]), n1 = dpp<DPP_WAVE_SHL1>(d[1]);
      if (f == 63) {
        next_head(k, &n0, &n1);
        if (tail_tile) {
          n0 = mask_past_end32(n0, TILE, remu);
          n1 = mask_past_end32(n1, TILE + 4, remu);
        }
      }
      if (lane == f) {
        if (f > 0) *(u32x4*)&win[0] = u32x4{p12, p13, p14, p15};
#pragma unroll
        for (int j = 0; j < 4; j++) *(u32x4*)&win[4 + 4 * j] = u32x4{d[4 * j], d[4 * j + 1], d[4 * j + 2], d[4 * j + 3]};
        *(u32x2*)&win[20] = u32x2{n0, n1};
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint32_t b = lane;
      const int r = 64 * f + (int)b - 14;  // m - B, in [-14, 4081]
      const uint32_t o = b + 2;            // m's byte offset in the window
      const int base = (int)(o >> 2);
      const uint32_t sh = (o & 3) * 8;
      uint32_t W[6];
#pragma unroll
      for (int i = 0; i < 6; i++) W[i] = win[base + i];
      const uint32_t tdw = win[(o - 1) >> 2];
      const uint32_t hxp = win[22];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // level 2, exact: p >> 32 <= (file_len-1) >> 32 (roots: p == 0 pass too)
      const uint32_t f3 = alignb(W[4], W[3], sh);
      const uint32_t f2 = alignb(W[3], W[2], sh);
      const uint32_t f4 = alignb(W[5], W[4], sh);
      const uint32_t u = (uint32_t)(r + 20);  // t - B >= 6
      const bool inrange = (u <= remu) && ((int64_t)B + r > (int64_t)a.m_lo);
      if (!FULL) {
        // optimistic pass: only strong nodes (p >= 20 so p != 0, crc field
        // != 0) are recorded; a chain through any other node fails the shape
        // check and goes to the full pass, so nothing else is needed here
        const uint64_t pm = __ballot(inrange && f3 <= hb && (f2 | f3) != 0 && f4 != 0);
        if (!pm) continue;
        if ((pm & (pm - 1)) == 0) {
          // one possible node (the common case: one metadata record per
          // line): the record -- m, p, key_hash, crc, the two suffix values
          // only the scan has, and the position flags -- goes to lane `count`
          // of the record registers; link_record applies the node test
          // (data_store.rs:404-470) beside its parent lookup (F_NT).
          const int bl = __builtin_ctzll(pm);
          const int rs = 64 * f + bl - 14;
          const uint64_t m = B + (int64_t)rs;
          const uint32_t s2 = __builtin_amdgcn_readlane(f2, bl), s3 = __builtin_amdgcn_readlane(f3, bl);  // p
          const uint32_t os = (uint32_t)bl + 2;
          const uint32_t stb = (__builtin_amdgcn_readlane(tdw, bl) >> (((os - 1) & 3) * 8)) & 0xffu;
          const uint32_t s0 = __builtin_amdgcn_readlane(alignb(W[1], W[0], sh), bl);
          const uint32_t s1 = __builtin_amdgcn_readlane(alignb(W[2], W[1], sh), bl);
          const uint32_t s4 = __builtin_amdgcn_readlane(f4, bl);
          const uint32_t REC_KIND = F_NT | (stb == 0 ? F_ZB : 0u);
          const uint32_t us = (uint32_t)(rs + 20);
          const uint32_t js = (us + ((0u - us) & 63u)) >> 6;
          const uint32_t hs = __builtin_amdgcn_readlane(hx, (int)(js & 63));
          const int lm = rs >> 6;
          const uint32_t hm = lm < 0 ? (uint32_t)__builtin_amdgcn_readfirstlane(hxp)
                                     : (uint32_t)__builtin_amdgcn_readlane(hx, lm & 63);
          const uint64_t r = wtotal + count;  // the record's index in the wave's region
          if (r < a.wcap) {
            const uint32_t kind = js < 64 ? 0u : (js == 64 ? 1u : 2u);
            const uint32_t fl = REC_KIND | ((rs & 63) == 0 ? F_TAIL : 0u) | F_SXM |
                                (kind << F_SUF_SHIFT) | (lm >= 0 && lm < 32 ? F_SXM_LO : 0u) |
                                ((js & 63) < 32 ? F_SUF_LO : 0u);
            if (r - flushed < RQ_LANES) {
              // record r -> lane r - flushed of the record registers
              const int li = (int)(r - flushed);
              rq[0] = writelane_u32((uint32_t)m, li, rq[0]);
              rq[1] = writelane_u32((uint32_t)(m >> 32), li, rq[1]);
              rq[2] = writelane_u32(hm, li, rq[2]);
              rq[3] = writelane_u32(hs, li, rq[3]);
              rq[4] = writelane_u32(fl, li, rq[4]);
              rq[5] = writelane_u32(s2, li, rq[5]);
              rq[6] = writelane_u32(s3, li, rq[6]);
              rq[7] = writelane_u32(s0, li, rq[7]);
              rq[8] = writelane_u32(s1, li, rq[8]);
              rq[9] = writelane_u32(s4, li, rq[9]);
              rvalid |= 1ull << (r - flushed);
            } else if (lane == 0) {
              const uint64_t gi = w * a.wcap + r;
              a.c_m[gi] = m;
              a.c_rec[gi] = u32x4{s2, s3, fl, s4};
              a.c_rec1[gi] = u32x4{s0, s1, hm, hs};
            }
          } else {
            ovf = true;
          }
          count++;
          continue;
        }
      } else if (!__ballot(f3 <= hb)) {
        continue;
      }
      const uint32_t tbyte = (tdw >> (((o - 1) & 3) * 8)) & 0xffu;
      const uint32_t f0 = alignb(W[1], W[0], sh), f1 = alignb(W[2], W[1], sh);
      // recover_valid_chain's node test (data_store.rs:404-470) at m = B + r
      const uint64_t roots = FULL ? __ballot(inrange && (f2 | f3) == 0) : 0ull;
      if (roots) rootmax = B + (uint64_t)(64 * f - 14 + 20) + (63 - __builtin_clzll(roots));  // increasing in (k, f)
      const uint64_t m = B + (int64_t)r;
      const uint64_t p = (uint64_t)f2 | ((uint64_t)f3 << 32);
      const uint64_t dp = m - p;
      const bool tomb = dp == 1 && tbyte == 0;
      const uint32_t pp = (0u - f2) & 63u;  // prepad(p)
      const bool isnode = inrange && p >= 20 && p < m && (tomb || dp > pp);
      const bool strong = isnode && (FULL || f4 != 0);
      const uint64_t cm = __ballot(strong);
      if (!cm) continue;
      const uint32_t js = (u + ((0u - u) & 63u)) >> 6;  // line of the next entry's start
      const uint32_t hs = __shfl(hx, (int)(js & 63));
      const int lm = r >> 6;                             // m's line (-1: previous tile's line 63)
      const uint32_t hm0 = __shfl(hx, lm & 63);
      const uint32_t hm = lm < 0 ? hxp : hm0;
      if (FULL ? count + __popcll(cm) > a.cap : wtotal + count + __popcll(cm) > a.wcap) ovf = true;
      if (strong) {
        const uint32_t idx = count + __popcll(cm & ((1ull << lane) - 1));
        if (FULL ? idx < a.cap : wtotal + idx < a.wcap) {
          const uint64_t gi = FULL ? span * a.cap + idx : w * a.wcap + wtotal + idx;
          const uint32_t kind = js < 64 ? 0u : (js == 64 ? 1u : 2u);
          const uint32_t fl = (tomb ? F_TOMB : 0u) | ((r & 63) == 0 ? F_TAIL : 0u) | F_SXM | (kind << F_SUF_SHIFT) |
                              (lm >= 0 && lm < 32 ? F_SXM_LO : 0u) | ((js & 63) < 32 ? F_SUF_LO : 0u);
          a.c_m[gi] = m;
          a.c_rec[gi] = u32x4{f2, f3, fl, f4};
          a.c_rec1[gi] = u32x4{f0, f1, hm, hs};
        }
      }
      count += __popcll(cm);
    }
    __builtin_amdgcn_s_setprio(0);
    // carry the last line's tail and SX_63 into the next tile's window
    if (lane == 63) {
#pragma unroll
      for (int j = 0; j < 4; j++) win[j] = d[12 + j];
      win[22] = hx;
    }
    // span end: its record count and first record into lane span % 64
    if ((k + 1) % SPAN_TILES == 0 || k + 1 == k1) {  // uniform
      const uint32_t sp = (uint32_t)(span & 63);
      scnt = (uint32_t)lane == sp ? count : scnt;
      sfirst = (uint32_t)lane == sp ? (uint32_t)wtotal : sfirst;
      if (sp == 63 || k + 1 == k1) {  // the 64-span group is complete
        const uint64_t sg = span & ~63ull;
        sg_pend = true;
        sg_base = sg;
        sg_lo = (uint32_t)(max(sg, k0 / SPAN_TILES) - sg);
        sg_hi = sp;
      }
      wtotal += count;
      count = 0;
    }
  };

  // A store point after the tiles [kf, kf + nt): a completed 16-tile group
  // of per-tile values, the buffered records once >= FLUSH_AT are pending
  // (and at the wave's end), a completed 64-span group of span counts / first
  // records.  Six UNCONDITIONAL buffer stores whose unused lanes carry an
  // out-of-range offset (dropped by the hardware): a store under a branch
  // makes the count of memory ops between a prefetch load and its wait
  // path-dependent, and the compiler then waits for the store's completion
  // too (~10 % of the kernel).  Their issue slots are not free either (all
  // six per tile cost 7-8 %, profiles/r04/variant_ab_no_stores.txt), so the
  // ring loop runs one store point per round of 3 tiles, not one per tile (a
  // round completes at most one group of either kind).
  // the store points' cache policy (buffer-store aux bits): sc0 sc1, written
  // through the XCD's L2 (srd_gst above; 0 = plain write-back: the round-5
  // stores, 2 = nt, 16 = sc1 -- timing A/B builds)
#ifndef SRD_SCAN_STORE_AUX
#define SRD_SCAN_STORE_AUX 17
#endif
  constexpr int SCAN_STORE_AUX = SRD_SCAN_STORE_AUX;
  auto store_point = [&](uint64_t kf, uint32_t nt) {
    if constexpr (MEMONLY) return;
    const bool last = kf + nt == k1;  // uniform
    {
      const uint32_t off = tg_pend && (uint32_t)lane - tg_lo < tg_hi - tg_lo ? 4u * lane : OOB_OFF;
      __builtin_amdgcn_raw_buffer_store_b32(tg_par ? tacc1 : tacc0, out_rsrc(a.tile + 4 * tg_base, 256), off, 0, SCAN_STORE_AUX);
      tg_pend = false;
    }
    {
      // (optimistic pass only; the full pass stores its records directly)
      constexpr uint64_t FLUSH_AT = 40;  // (60: +-0, profiles/r05/variant_ab_store_ablations_coal.txt)
      const uint64_t pend = wtotal + count - flushed;  // records pending (lanes [0, min(pend, 64)))
      const bool fl = pend >= FLUSH_AT || last;  // uniform
      const bool wr = fl && ((rvalid >> lane) & 1);
      const uint64_t rb = w * a.wcap + flushed;  // lane 0's record
      const uint32_t rn = (uint32_t)min<uint64_t>(a.wcap - min(flushed, a.wcap), 64);  // slots left (OOB past)
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{rq[0], rq[1]}, out_rsrc(a.c_m + rb, rn * 8),
                                            wr ? 8u * lane : OOB_OFF, 0, SCAN_STORE_AUX);
      // the record's halves: {p, flags, crc}, {key_hash, sxm, suf}
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{rq[5], rq[6], rq[4], rq[9]}, out_rsrc(a.c_rec + rb, rn * 16),
                                             wr ? 16u * lane : OOB_OFF, 0, SCAN_STORE_AUX);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{rq[7], rq[8], rq[2], rq[3]}, out_rsrc(a.c_rec1 + rb, rn * 16),
                                             wr ? 16u * lane : OOB_OFF, 0, SCAN_STORE_AUX);
      if (fl) {
        flushed = wtotal + count;
        rvalid = 0;
      }
    }
    {
      const uint32_t soff = sg_pend && (uint32_t)lane >= sg_lo && (uint32_t)lane <= sg_hi ? 4u * lane : OOB_OFF;
      __builtin_amdgcn_raw_buffer_store_b32(scnt, out_rsrc(a.span_count + sg_base, 256), soff, 0, SCAN_STORE_AUX);
      __builtin_amdgcn_raw_buffer_store_b32(sfirst, out_rsrc(a.span_first + sg_base, 256), soff, 0, SCAN_STORE_AUX);
      sg_pend = false;
    }
  };

  // register ring (3 buffers: 2 tiles in flight while one is processed;
  // measured best with the 4-chain line CRC, whose registers a 4th buffer
  // would spill).
  // Loads are clamped, never skipped (tiles up to n_tiles+1 are readable).
  // kt = the first tail tile (flen - kt*TILE < TILE + 64)
  const uint64_t kt = flen >= (uint64_t)TILE + 64 ? (flen - TILE - 64) / TILE + 1 : 0;
  const uint64_t km = min(k1, max(k0, kt));  // ring part: [k0, km)
  const uint32_t nk = (uint32_t)(km - k0);
  const std::false_type body{};
  uint32_t A[16], Bv[16], Cv[16];
  // vmcnt counts loads and stores in issue order, and the compiler's wait
  // counts at the loop header are the minimum over its entries.  In the
  // steady state every tile's loads are followed by process()'s 6
  // unconditional stores (tile values, span records, span count / first); without
  // them on the entry path the first iteration's shorter queue sets every
  // wait of the loop, which then waits for part of the next tile early.
  // Dummy stores (out-of-range offsets: dropped by the hardware; distinct,
  // or the compiler merges them as dead stores) give the entry the same queue.
  auto pad_stores = [&](uint32_t g) {
    constexpr uint32_t NST = MEMONLY ? 0u : 6u;  // a store point's unconditional stores
#pragma unroll
    for (uint32_t i = 0; i < NST; i++)
      __builtin_amdgcn_raw_buffer_store_b32(0u, out_rsrc(a.tile, 256), OOB_OFF - 64u * (NST * g + i), 0, 0);
  };
  // Whole rounds of 3 tiles only: a break between the tiles of a round
  // reaches the loop latch, and that (never taken) latch -> header path
  // would shorten the compiler's wait counts as well.  The <= 2 remaining
  // ring tiles run in the unpipelined loop below with the file's tail tiles.
  constexpr uint32_t RD = 3;  // ring depth
  const uint32_t nfull = nk / RD;
  // (the entry's queue = the loop latch's: with a store point per tile the
  // stores of one tile follow every load; with one per round, only tile
  // B's loads have a store point behind them before the loop comes round)
  load_tile(k0, A);
  // A's loads strictly before B's: the scheduler interleaved the two tiles'
  // coalesced loads here, and the loop's first wait (the minimum over its
  // entries) then waited for 3 of the next tile's loads too (vmcnt 11
  // instead of 14): -0.2 to -1 % scan (profiles/r05/variant_ab_prologue_order*.txt)
  if constexpr (COALT) __builtin_amdgcn_sched_barrier(0);
  load_tile(k0 + 1, Bv);
  pad_stores(1);
  for (uint32_t i = 0; i < nfull; i++) {
    const uint32_t j = RD * i;
    // priority from the tile's prefetch loads through its CRC (process()
    // drops it after the lookups): -1.6 % same-box A/B over priority on the
    // CRC alone
    __builtin_amdgcn_s_setprio(3);
    load_tile(k0 + min(j + 2, nk), Cv);
    process(k0 + j, A, body);
    __builtin_amdgcn_s_setprio(3);
    load_tile(k0 + min(j + 3, nk), A);
    process(k0 + j + 1, Bv, body);
    __builtin_amdgcn_s_setprio(3);
    load_tile(k0 + min(j + 4, nk), Bv);
    process(k0 + j + 2, Cv, body);
    store_point(k0 + j, 3);
  }
  const uint64_t kr = k0 + (uint64_t)RD * nfull;
  // the ring's remainder and the file's last <= 2 tiles (masked: a tail
  // tile's bytes past file_len read as 0; a no-op on the others)
  for (uint64_t k = kr; k < k1; k++) {
    load_tile(k, A);
    process(k, A, std::true_type{});
    store_point(k, 1);
  }

  if constexpr (MEMONLY) {
    if (memonly_acc == 0x12345678u) a.counters[3] = memonly_acc;  // (keeps the loads)
  }
  // ---- epilogue: per-wave results ----
  if (lane == 0) {
    a.wave_total[w] = wtotal | (ovf ? (1ull << 63) : 0ull);
    a.wave_root[w] = rootmax;  // wave-uniform already
#ifdef SRD_WAVE_STAMPS  // timing-only build (tools/wave_stamps.py): each wave's end, 100 MHz clock
    if (w < 8192) g_wave_stamp[w] = __builtin_amdgcn_s_memrealtime();
    if (w < 4096) g_wave_clk[w] = __builtin_amdgcn_s_memtime();
#endif
  }
  if (a.xp) {  // (uniform) every wave of the block is done: its XCD and duration
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < XP_MAX_BLOCKS) {
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      a.xp->xcc[blockIdx.x] = xcc & 7u;
      a.xp->dur[blockIdx.x] = (uint32_t)min<uint64_t>(__builtin_amdgcn_s_memrealtime() - xp_t0, 0xFFFFFFFFull);
      a.xp->t0[blockIdx.x] = xp_t0;
    }
  }
  if constexpr (!FULL) {
    // The optimistic pass: no last-block reduction here.  Its agent-scope
    // release (an L2 write-back of every block's XCD, ~4 MB of dirty record
    // lines) and the reduction sat on the critical path of every call: the
    // last block ended 7-8 us before the kernel did (tools/wave_stamps.py,
    // profiles/r06/wave_stamps_r6m.txt).  link2_kernel's block 0 reduces the
    // wave totals instead (scan_reduce), after the kernel boundary;
    // find_top's tail (the same value in every wave) goes out from block 0.
    if (blockIdx.x == 0 && threadIdx.x == 0) a.counters[1] = top;
    return;
  }
  // (the full pass: the last block to finish reduces them -- cdna guide: plain
  // stores, vmcnt(0), barrier, lane-0 agent release, add; the last block
  // acquires before reading)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t& s_last = lds.s_last;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = atomicAdd(a.done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // totals of the wave counts: thread t owns waves [t*q, (t+1)*q).  q <= 4
  // (up to 256 blocks): the thread's waves are loaded together into
  // registers (one round trip instead of 2q dependent ones: the last block's
  // epilogue is on the critical path of every call)
  constexpr int QR = 4;
  uint64_t* s_wsum = (uint64_t*)lds.tab;  // the CRC tables are dead now
  uint64_t* s_smax = s_wsum + NW;
  uint64_t* s_root = lds.s_root;
  uint64_t* s_ovf = s_smax + NW;
  const uint32_t T = blockDim.x, t = threadIdx.x;
  const uint64_t q = (total_waves + T - 1) / T;
  uint64_t sum = 0, rmax = 0, o = 0, smax = 0;
  auto take = [&](uint64_t i, uint64_t v, uint64_t rt) {
    const uint64_t cnt = v & ~(1ull << 63);
    sum += cnt;
    o |= v >> 63;
    rmax = max(rmax, rt);
    if (cnt) smax = max(smax, i * a.wcap + min(cnt, a.wcap));  // 1 + the wave's last slot
  };
  if (q <= QR) {
    uint64_t vt[QR], vr[QR];
#pragma unroll
    for (int j = 0; j < QR; j++) {
      const uint64_t i = min(t * q + j, total_waves - 1);
      vt[j] = a.wave_total[i];
      vr[j] = a.wave_root[i];
    }
#pragma unroll
    for (int j = 0; j < QR; j++)
      if ((uint64_t)j < q && t * q + j < total_waves) take(t * q + j, vt[j], vr[j]);
  } else {
    for (uint64_t i = t * q; i < min((t + 1) * q, total_waves); i++) take(i, a.wave_total[i], a.wave_root[i]);
  }
  rmax = wave_max_u64(rmax);
  smax = wave_max_u64(smax);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    o |= __shfl_xor(o, d);
    sum += __shfl_xor(sum, d);
  }
  if (lane == 0) { s_wsum[wv] = sum; s_root[wv] = rmax; s_ovf[wv] = o; s_smax[wv] = smax; }
  __syncthreads();
  if (t == 0) {
    uint64_t mr = 0, oo = 0, tot = 0, sm = 0;
    for (int i = 0; i < NW; i++) {
      mr = max(mr, s_root[i]);
      oo |= s_ovf[i];
      tot += s_wsum[i];
      sm = max(sm, s_smax[i]);
    }
    a.k_total[0] = tot;
    a.k_total[1] = sm;
    a.counters[0] = mr;
    a.counters[1] = top;  // the optimistic pass's start tail (find_top; 0: none)
    a.counters[2] = oo;
    *a.done = 0;  // for the next launch on this context
#ifdef SRD_WAVE_STAMPS
    g_wave_stamp[8192 + 1023] = __builtin_amdgcn_s_memrealtime();
#endif
  }
}

// --------------------------------------------------------------------------
// 2. parent lookup
// --------------------------------------------------------------------------
struct LinkArgs {
  const uint8_t* file;
  uint64_t flen, n_spans;
  uint32_t cap;
  const uint32_t* span_count;
  const uint64_t* span_base;  // exclusive prefix of min(count, cap)
  const uint64_t* c_m;
  const u32x4* c_rec;
  uint64_t* d_m;
  int64_t* d_par;
  uint64_t* d_slot;
};

// LINK_LANES lanes per span, 256 / LINK_LANES spans per block: the full
// pass records ~11 candidates per C2 span (the real node and the weak ones
// its checksum bytes make), each a chain of dependent loads with a random
// file read, so one record per lane (4 lanes and a loop: ~3 records each)
constexpr uint32_t LINK_LANES = 16;
__global__ __launch_bounds__(256) void link_kernel(LinkArgs a) {
  const uint64_t sp = (uint64_t)blockIdx.x * (256 / LINK_LANES) + (threadIdx.x / LINK_LANES);
  if (sp >= a.n_spans) return;
  const uint32_t n = min(a.span_count[sp], a.cap);
  const uint64_t gb = a.span_base[sp];
  for (uint32_t i = threadIdx.x % LINK_LANES; i < n; i += LINK_LANES) {
    const uint64_t gi = sp * a.cap + i;
    const u32x4 r0 = a.c_rec[gi];
    const uint64_t m = a.c_m[gi], p = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);
    const uint64_t mp = p - 20;  // p >= 20 by construction
    const uint64_t sp2 = (mp + 14) / SPAN_BYTES;  // span s holds m in [16 KiB s - 14, 16 KiB (s+1) - 14)
    // the parent is usually the previous record of the span: one load instead
    // of a binary search
    int64_t par = (i > 0 && a.c_m[gi - 1] == mp) ? (int64_t)(gb + i - 1) : PAR_MISS;
    if (par == PAR_MISS) {
      // The metadata the parent would have at p - 20, read from the file:
      // its prev == 0 makes it the root entry (data_store.rs:404-416);
      // otherwise only bytes that pass the node test can be a recorded
      // candidate, so the binary search runs for those alone (the weak
      // nodes a record's checksum and zero prepad leave have random "prev"
      // values: their parents mostly fail here, one line read instead of
      // three to four dependent ones)
      uint64_t pkh, pp;
      uint32_t pcrc;
      ld_meta(a.file, mp, &pkh, &pp, &pcrc);
      const uint64_t dp = mp - pp;
      if (pp == 0) {
        if (p >= 21) par = PAR_ROOT;
      } else if (pp >= 20 && pp < mp && (dp > prepad64(pp) || dp == 1) && sp2 < a.n_spans) {
        uint32_t lo = 0, hi = min(a.span_count[sp2], a.cap);
        const uint64_t* cm = a.c_m + sp2 * a.cap;
        while (lo < hi) {
          uint32_t mid = (lo + hi) >> 1;
          if (cm[mid] < mp) lo = mid + 1; else hi = mid;
        }
        if (lo < min(a.span_count[sp2], a.cap) && cm[lo] == mp) par = (int64_t)(a.span_base[sp2] + lo);
      }
    }
    const uint64_t g = gb + i;
    a.d_m[g] = m;
    a.d_par[g] = par;
    a.d_slot[g] = gi;
  }
}

// --------------------------------------------------------------------------
// 3. chain walk over runs (single thread) + marking
// --------------------------------------------------------------------------
struct WalkState {
  int64_t status;      // 1 ok, -1 miss (cannot conclude), -2 no start
  uint64_t n_int;      // intervals [h, x] in an index space
  uint64_t chain_len;  // entries incl. root
  uint64_t root_t;     // tail of the chain's root entry
  uint64_t final_len;
  uint64_t start;      // start index in the walk space
  int64_t pad[2];
};

// idx space: 0..n-1 ; par_of(i) gives par in the same space ; runhead[i]
__global__ void walk_kernel(const int64_t* par, const uint32_t* runhead, const uint64_t* slot,
                            const u32x4* c_rec, uint64_t* ints, WalkState* ws, uint64_t max_ints) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t x = ws->start, n = 0, len = 1;
  int64_t status = 1;
  while (true) {
    uint64_t h = runhead[x] - 1;  // runhead holds (run head index + 1)
    if (n < max_ints) { ints[2 * n] = h; ints[2 * n + 1] = x; }
    n++;
    len += x - h + 1;
    int64_t q = par[h];
    if (q == PAR_ROOT) {
      const u32x4 r0 = c_rec[slot[h]];
      ws->root_t = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);
      break;
    }
    if (q < 0) { status = -1; break; }
    x = (uint64_t)q;
  }
  ws->status = status;
  ws->n_int = n;
  ws->chain_len = len;
}

// Leaf pruning: a chain node other than the start always has a child (the
// next chain entry links to it), so nodes nobody links to (false candidates)
// are dropped before run compression.  core[g] = has a child || g == start.
__global__ void child_kernel(const int64_t* par, uint64_t n, uint8_t* core) {
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  int64_t p = par[g];
  if (p >= 0) core[p] = 1;
}
// run keys and heads are g + 1 in 32 bits (the host bounds the node count
// below 2^32 - 1: half the bytes of the max-scans)
__global__ void core_key_kernel(uint8_t* core, const WalkState* ws, uint64_t n, uint32_t* key) {
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  if (g == ws->start) core[g] = 1;
  key[g] = core[g] ? (uint32_t)(g + 1) : 0u;
}
// runs over core nodes: head if its parent is not the previous core node
__global__ void head_key_kernel(const uint8_t* core, const int64_t* par, const uint32_t* cmax, uint64_t n,
                                uint32_t* key) {
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  uint32_t k = 0;
  if (core[g]) {
    const uint64_t prev1 = g ? cmax[g - 1] : 0;  // previous core index + 1
    const bool cont = prev1 && par[g] == (int64_t)(prev1 - 1);
    k = cont ? 0u : (uint32_t)(g + 1);
  }
  key[g] = k;
}

// onpath[i] = 1 if i is a core node inside one of the (descending) intervals
__global__ void mark_kernel(const uint64_t* ints, const WalkState* ws, uint64_t n, const uint8_t* core,
                            uint32_t* onpath) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (!core[i]) { onpath[i] = 0; return; }
  uint64_t ni = ws->n_int;
  // intervals sorted by descending h (and x); find first with h <= i
  uint64_t lo = 0, hi = ni;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (ints[2 * mid] > i) lo = mid + 1; else hi = mid;
  }
  onpath[i] = (lo < ni && ints[2 * lo + 1] >= i) ? 1u : 0u;
}

// chain index c (1..) -> walk-space index
__global__ void scatter_chain_kernel(const uint32_t* onpath, const uint32_t* cpos, uint64_t n,
                                     const uint64_t* map, uint64_t* chain_g) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !onpath[i]) return;
  chain_g[1 + cpos[i]] = map ? map[i] : i;
}

// --------------------------------------------------------------------------
// full mode: statuses by pointer jumping
// --------------------------------------------------------------------------
// Statuses (1: reaches a root, 2: reaches a miss) by pointer jumping over
// runs of CORE nodes (something links to them).  The full pass records every
// node, also the weak ones a metadata record's checksum and zero prepad leave
// (~2 per entry at C2: leaves whose random "prev" mostly misses), so chain
// nodes are rarely adjacent; among core nodes they are: a core node whose
// parent is the previous core node continues that one's run.  Runs share
// their head's status and only heads jump (to the head of their parent's
// run); a leaf then takes its parent's status.  A torn C2 store: one run.
__global__ void status_init_kernel(const int64_t* par, const uint8_t* core, const uint32_t* chead, uint64_t n,
                                   uint8_t* st, int64_t* jmp) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n || !core[g] || chead[g] != g + 1) return;  // core run heads only
  const int64_t p = par[g];
  st[g] = p == PAR_ROOT ? 1 : (p == PAR_MISS ? 2 : 0);
  jmp[g] = p >= 0 ? (int64_t)chead[p] - 1 : p;  // a parent has a child: it is core
}
// prev (nullable): the previous round's change flag -- a round after one in
// which no head jumped has nothing left to do (every head resolved)
__global__ void status_round_kernel(uint64_t n, const uint8_t* core, const uint32_t* chead, uint8_t* st,
                                    int64_t* jmp, unsigned int* changed, const unsigned int* prev) {
  if (prev && *prev == 0) return;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x) {
    if (!core[g] || chead[g] != g + 1 || st[g]) continue;
    const int64_t j = jmp[g];
    const uint8_t s = st[j];
    if (s) st[g] = s;
    else { jmp[g] = jmp[j]; *changed = 1; }
  }
}
__global__ void status_spread_core_kernel(uint64_t n, const uint8_t* core, const uint32_t* chead, uint8_t* st) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n && core[g] && chead[g] != g + 1) st[g] = st[chead[g] - 1];
}
__global__ void status_spread_leaf_kernel(uint64_t n, const int64_t* par, const uint8_t* core, uint8_t* st) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n || core[g]) return;
  const int64_t p = par[g];
  st[g] = p == PAR_ROOT ? 1 : (p == PAR_MISS ? 2 : st[p]);
}
__global__ void core_flag_key_kernel(const uint8_t* core, uint64_t n, uint32_t* key) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) key[g] = core[g] ? (uint32_t)(g + 1) : 0u;
}

// the largest valid node: a block maximum per block (same-address atomics
// serialise: even one per wave, ~16K of them, took 0.83 ms at C2), then one
// block reduces them
__global__ __launch_bounds__(256) void valid_max_kernel(const uint8_t* st, uint64_t n, uint64_t* bmax,
                                                        uint32_t* vflag) {
  __shared__ uint64_t wm[4];
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool v = g < n && st[g] == 1;
  if (g < n) vflag[g] = v;
  const uint64_t b = __ballot(v);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = b ? (g & ~63ull) + 64 - __builtin_clzll(b) : 0;  // max g + 1
  __syncthreads();
  if (threadIdx.x == 0) bmax[blockIdx.x] = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
}
// *out = max of the per-block maxima (best_g1 = 1 + the valid node with the
// largest tail, 0 if none); *meta = d_m[best_g1 - 1], that node's metadata
// offset (one host wait reads both)
__global__ __launch_bounds__(1024) void max_reduce_kernel(const uint64_t* v, uint64_t n, unsigned long long* out,
                                                          const uint64_t* d_m, unsigned long long* meta) {
  __shared__ uint64_t wm[16];
  uint64_t m = 0;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) m = max(m, v[i]);
  m = wave_max_u64(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; w++) m = max(m, wm[w]);
    *out = m;
    *meta = m ? d_m[m - 1] : 0ull;
  }
}
// remap parents into the compacted valid space
__global__ void remap_kernel(const uint64_t* vlist, const uint64_t* nv, const int64_t* par,
                             const uint64_t* vpos, int64_t* vpar, uint64_t* vslot,
                             const uint64_t* slot) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *nv) return;
  uint64_t g = vlist[i];
  int64_t p = par[g];
  int64_t vp = p >= 0 ? (int64_t)vpos[p] : p;
  vpar[i] = vp;
  vslot[i] = slot[g];
}

// --------------------------------------------------------------------------
// 4. finalize: per chain entry outputs + CRC from the per-tile values
// --------------------------------------------------------------------------
struct FinArgs {
  const uint8_t* file;
  uint64_t flen;
  uint64_t n_chain;
  const uint64_t* chain_g;   // [n_chain], entry 0 = root (unused)
  const uint64_t* slot;      // dense g -> record slot
  const int64_t* par;        // dense g -> dense parent
  const WalkState* ws;
  const uint64_t* c_m;
  const u32x4* c_rec;        // {p, flags, crc} (ScanArgs::c_rec)
  const u32x4* c_rec1;       // {key_hash, sxm, suf}
  const uint32_t* tile;      // [4k..4k+2] per-tile values (tile_T / tile_SX1)
  int no_crc;
  // device-side plan (sync-free path): when set, n_chain / root_t come from
  // device memory and a nonzero *status disables the kernel
  // and chain_g holds record slots (the parent of chain entry c >= 2 is entry c-1)
  const uint64_t* d_n_chain;
  const uint64_t* d_root_t;
  const uint32_t* d_status;
  // chain entries before the first candidate: 1 (entry 0 is the root entry
  // with prev 0, not a candidate) or 0 (span mode: the shard's first entry,
  // prev == the shard's lower tail, is a candidate record)
  uint32_t coff;
  // outputs
  uint64_t *o_mo, *o_kh, *o_prev, *o_start, *o_len;
  uint64_t* o_packed;  // nullable: pack(tag16, meta_off48) per chain entry (the optimistic pass's index alias)
  uint32_t *o_crc_st, *o_crc, *o_pieces;  // o_pieces: bit0 suf ok, bit1 sxm ok (slow path input)
  uint32_t *o_suf, *o_sxm, *o_tail;
  uint8_t* o_ok;
  uint64_t* slow_list;
  unsigned long long* n_slow;
  unsigned long long* n_bad;
};

// crc_raw of bytes [floor64(m), m) (<= 63 bytes) in one round trip: the
// 64-byte line at floor64(m) by four independent 16-byte loads (the store is
// readable to srd_padded_size, so the whole line is), then <= 15 slice-by-4
// word steps and <= 3 byte steps from registers.  (A word load per step made
// every step wait for its own HBM round trip: up to 18 dependent loads per
// entry, which set C3's finalize pass time.)  tab(t, b) = slice table t, byte b.
template <class Tab>
__device__ __forceinline__ uint32_t tail_crc_line(const uint8_t* file, uint64_t m, Tab tab) {
  const uint64_t L = m & ~63ull;
  const uint32_t r = (uint32_t)(m - L);
  if (r == 0) return 0;
  const u32x4* lp = (const u32x4*)(file + L);
  const u32x4 q0 = lp[0], q1 = lp[1], q2 = lp[2], q3 = lp[3];
  const uint32_t w[16] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3],
                          q2[0], q2[1], q2[2], q2[3], q3[0], q3[1], q3[2], q3[3]};
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 15; i++) {
    if (4u * i + 4u <= r) {
      s ^= w[i];
      s = tab(3, s & 0xff) ^ tab(2, (s >> 8) & 0xff) ^ tab(1, (s >> 16) & 0xff) ^ tab(0, s >> 24);
    }
  }
  uint32_t pw = 0;  // the partial word w[r / 4] (selects: no indexed register access)
#pragma unroll
  for (int i = 0; i < 16; i++) pw = (uint32_t)i == (r >> 2) ? w[i] : pw;
  for (uint32_t b = 0; b < (r & 3u); b++) s = tab(0, (s ^ (pw >> (8 * b))) & 0xff) ^ (s >> 8);
  return s;
}
__device__ __forceinline__ uint32_t tail_crc(const uint8_t* file, uint64_t m) {
  return tail_crc_line(file, m, [](int t, uint32_t b) { return g_tabs.tab[t][b]; });
}

// per-tile values: tile[4k] / tile[4k+1] = half-tile partials of lines 0 / 1,
// tile[4k+2] = SX_32.  A lower-half partial v becomes the true suffix value
// SX_j = v * x^16384 ^ SX_32.
__device__ __forceinline__ uint32_t mul16k_g(uint32_t v) {
  return g_tabs.m16k[0][v & 0xff] ^ g_tabs.m16k[1][(v >> 8) & 0xff] ^ g_tabs.m16k[2][(v >> 16) & 0xff] ^
         g_tabs.m16k[3][v >> 24];
}
__device__ __forceinline__ uint32_t lo_fix(const uint32_t* tile, uint64_t k, uint32_t v) {
  return mul16k_g(v) ^ tile[4 * k + 2];
}
__device__ __forceinline__ uint32_t tile_T(const uint32_t* tile, uint64_t k) { return lo_fix(tile, k, tile[4 * k]); }
__device__ __forceinline__ uint32_t tile_SX1(const uint32_t* tile, uint64_t k) {
  return lo_fix(tile, k, tile[4 * k + 1]);
}

__device__ __forceinline__ uint32_t crc_from_pieces(uint64_t s, uint64_t m, uint32_t suf, uint32_t sxm,
                                                    uint32_t tail, const uint32_t* tile) {
  const uint64_t len = m - s;
  if (len < 64) return tail ^ g_tabs.zero_crc[len];
  const uint64_t k0 = s / TILE, k1 = m / TILE;
  const uint32_t j0 = (uint32_t)((s % TILE) / 64);
  uint32_t acc = suf ^ g_tabs.winit[j0];
  uint32_t y;
  if (k0 == k1) {
    y = acc ^ sxm;
  } else {
    for (uint64_t k = k0 + 1; k < k1; k++) acc = mulp(g_tabs.x32768, acc) ^ tile_T(tile, k);
    y = mulp(g_tabs.x32768, acc) ^ tile_T(tile, k1) ^ sxm;
  }
  const uint64_t dd = (k1 + 1) * TILE - m;
  return ~(mulp(g_tabs.invpow[dd], y) ^ tail);
}

// whole tiles a finalize thread combines serially (longer entries go to the
// slow list, a wave each).  C3 glue (tools/lib_ab.py, contexts interleaved):
// 4 -> 1.66 ms, 8 -> 1.61, 16 -> 1.57, 32 -> 1.57; C2 (entries of 2 tiles)
// unchanged
#ifndef SRD_LONG_TILES
#define SRD_LONG_TILES 16
#endif
constexpr uint64_t LONG_TILES = SRD_LONG_TILES;
constexpr uint64_t NO_REC = ~0ull;
__device__ void finalize_one(const FinArgs& a, uint64_t c, uint64_t root_t);
__device__ bool finalize_core(const FinArgs& a, uint64_t c, uint64_t gi, int64_t pgi, uint64_t root_t, uint64_t* kh_out);
__global__ void finalize_kernel(FinArgs a) {
  uint64_t n = a.n_chain, root_t = 0;
  if (a.d_status) {
    if (*a.d_status) return;
    n = *a.d_n_chain;
    root_t = *a.d_root_t;
  } else if (a.ws) {
    root_t = a.ws->root_t;
  }
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (uint64_t)gridDim.x * blockDim.x)
    finalize_one(a, c, root_t);
}
__device__ void finalize_one(const FinArgs& a, uint64_t c, uint64_t root_t) {
  uint64_t gi = NO_REC;
  int64_t pgi = -1;
  if (c >= a.coff) {
    const uint64_t g = a.chain_g[c];
    gi = a.d_status ? g : a.slot[g];
    // plan mode: chain_g holds record slots and the parent of entry c > coff
    // is entry c - 1; otherwise the dense parent of g
    const int64_t pg = a.d_status ? (c >= a.coff + 1 ? 0 : PAR_ROOT) : a.par[g];
    if (pg >= 0) pgi = (int64_t)(a.d_status ? a.chain_g[c - 1] : a.slot[pg]);
  }
  uint64_t kh;
  if (finalize_core(a, c, gi, pgi, root_t, &kh)) {
    const unsigned long long w = atomicAdd(a.n_slow, 1ull);
    a.slow_list[w] = c;
  }
}

// Chain entry c: its candidate record gi (NO_REC: the root entry, from
// root_t) and its parent's record pgi (< 0: the parent is the root entry or
// lies outside the span).  Writes every output; returns true when the CRC
// needs slow_one (o_pieces / o_suf / o_sxm / o_tail hold its inputs then).
__device__ bool finalize_core(const FinArgs& a, uint64_t c, uint64_t gi, int64_t pgi, uint64_t root_t,
                              uint64_t* kh_out) {
  uint64_t mo, kh, p, start, len;
  uint32_t crc_st, suf = 0, sxm = 0, tail = 0, pieces = 0;
  bool tomb;
  if (gi == NO_REC) {
    const uint64_t t = root_t;
    mo = t - 20;
    kh = ld_u64_unaligned(a.file, mo);
    crc_st = ld_u32_unaligned(a.file, mo + 16);
    p = 0;
    tomb = false;  // start is 0 either way
    start = 0;
    suf = tile_T(a.tile, 0);
    pieces = 1;
  } else {
    mo = a.c_m[gi];
    const u32x4 r0 = a.c_rec[gi], r1 = a.c_rec1[gi];
    p = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);
    kh = (uint64_t)r1[0] | ((uint64_t)r1[1] << 32);
    crc_st = r0[3];
    const uint32_t fl = r0[2];
    tomb = fl & F_TOMB;
    start = tomb ? p : p + prepad64(p);
    if (fl & F_SXM) {
      sxm = (fl & F_SXM_LO) ? lo_fix(a.tile, mo / TILE, r1[2]) : r1[2];
      pieces |= 2;
    }
    if (fl & F_TAIL) { tail = 0; pieces |= 4; }
    if (pgi >= 0) {
      const uint32_t pfl = a.c_rec[pgi][2], psuf = a.c_rec1[pgi][3];
      const uint32_t kind = (pfl >> F_SUF_SHIFT) & 3;
      const uint64_t k0 = start / TILE;  // kind 0: the parent's tile; 1, 2: the next one
      if (kind == 0) { suf = (pfl & F_SUF_LO) ? lo_fix(a.tile, k0, psuf) : psuf; pieces |= 1; }
      else if (kind == 1) { suf = tile_T(a.tile, k0); pieces |= 1; }
      else if (kind == 2) { suf = tile_SX1(a.tile, k0); pieces |= 1; }
    } else if (start == 0) {
      suf = tile_T(a.tile, 0);
      pieces |= 1;
    }
  }
  *kh_out = kh;
  // A piece no record holds (the root entry's metadata-line suffix, its
  // child's start-line suffix: the root has no candidate record) comes from
  // the per-tile values when its line is 0, 1 or 32 of the tile (C1/C2/C5:
  // root metadata at 4096, the child's start at 4160); else slow_kernel
  // recomputes it
  if (!(pieces & 1)) {
    const uint64_t k = start / TILE;
    const uint32_t j = (uint32_t)((start % TILE) / 64);
    if (j == 0) { suf = tile_T(a.tile, k); pieces |= 1; }
    else if (j == 1) { suf = tile_SX1(a.tile, k); pieces |= 1; }
    else if (j == 32) { suf = a.tile[4 * k + 2]; pieces |= 1; }
  }
  if (!(pieces & 2)) {
    const uint64_t k = mo / TILE;
    const uint32_t j = (uint32_t)((mo % TILE) / 64);
    if (j == 0) { sxm = tile_T(a.tile, k); pieces |= 2; }
    else if (j == 1) { sxm = tile_SX1(a.tile, k); pieces |= 2; }
    else if (j == 32) { sxm = a.tile[4 * k + 2]; pieces |= 2; }
  }
  len = mo - start;
  a.o_mo[c] = mo;
  a.o_kh[c] = kh;
  if (a.o_packed) a.o_packed[c] = ((kh >> 48) << 48) | (mo & 0xFFFFFFFFFFFFull);  // key_indexer.rs:79-85
  a.o_prev[c] = p;
  a.o_start[c] = start;
  a.o_len[c] = len;
  a.o_crc_st[c] = crc_st;
  if (a.no_crc) { a.o_crc[c] = 0; a.o_ok[c] = 0; return false; }
  if (tomb) {
    const uint32_t crc = 0xD202EF8Du;  // CRC32(b"\0"): the tombstone byte is 0 by the rule
    a.o_crc[c] = crc;
    a.o_ok[c] = crc == crc_st;
    if (crc != crc_st) atomicAdd(a.n_bad, 1ull);
    return false;
  }
  if (!(pieces & 4)) tail = tail_crc(a.file, mo);  // re-read the partial last line
  const bool need_long = len >= 64;
  // entries spanning many whole tiles combine them with one wave (slow_kernel)
  const bool many_tiles = need_long && mo / TILE > start / TILE + 1 + LONG_TILES;
  if (!need_long || ((pieces & 1) && (pieces & 2) && !many_tiles)) {
    const uint32_t crc = crc_from_pieces(start, mo, suf, sxm, tail, a.tile);
    a.o_crc[c] = crc;
    a.o_ok[c] = crc == crc_st;
    if (crc != crc_st) atomicAdd(a.n_bad, 1ull);
    return false;
  }
  a.o_pieces[c] = pieces;
  a.o_suf[c] = suf;
  a.o_sxm[c] = sxm;
  a.o_tail[c] = tail;
  return true;
}



// Recompute, with one wave, SX at line j of tile k (bytes past flen read as 0;
// the buffer is readable to srd_padded_size).  tab = the 4x256 CRC table in LDS.
__device__ uint32_t tile_probe_sx(const uint8_t* file, uint64_t flen, uint64_t k, uint32_t j, const uint32_t* tab) {
  const int lane = threadIdx.x & 63;
  const uint64_t L = k * TILE + 64ull * lane;
  const u32x4* p = (const u32x4*)(file + L);
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const u32x4 v = p[q];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const uint64_t o = L + 16 * q + 4 * e;
      uint32_t w = v[e];
      if (o + 4 > flen) w = o >= flen ? 0u : (w & (0xffffffffu >> (8 * (4 - (uint32_t)(flen - o)))));
      s ^= w;
      s = tab[768 + (s & 0xff)] ^ tab[512 + ((s >> 8) & 0xff)] ^ tab[256 + ((s >> 16) & 0xff)] ^ tab[s >> 24];
    }
  }
  uint32_t sx = mulp(g_tabs.lw[lane], s);
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t v = __shfl_down(sx, o);
    if (lane + o < 64) sx ^= v;
  }
  return __shfl(sx, (int)j);
}

// x^(8n) for any n (binary exponentiation over pow8[k] = x^(8*2^k))
__device__ __forceinline__ uint32_t xpow8_dev(uint64_t n) {
  uint32_t r = kX0;
  for (int k = 0; n; k++, n >>= 1)
    if (n & 1) r = mulp(g_tabs.pow8[k], r);
  return r;
}
__device__ __forceinline__ uint32_t xpow8_any(uint64_t n) { return xpow8_dev(n); }

// crc_from_pieces with the whole tiles between the start tile k0 and the
// metadata tile k1 combined by the 64 lanes of the calling wave: lane l
// Horner-combines tiles k0+1+l, +65+l, ... with X^64 steps, weights its sum by
// X^(distance of its last tile to tile k1-1), and the wave XOR-reduces.
// mulp(a, b) for wave-uniform a, b, by the whole wave (every lane gets the
// product): mulp adds b * x^(31 - i) for every set bit i of a; lane i < 32
// builds its term from b with (31 - i) / 8 byte steps through the CRC table
// R (crc8: v * x^8 = (v >> 8) ^ R[v & 0xff], LDS) and the remaining bit
// steps, then the 32 terms are XOR-reduced -- ~45 instructions instead of
// mulp's 32 dependent 7-instruction steps (the slow path runs four per entry)
__device__ __forceinline__ uint32_t mulp_wave(uint32_t a, uint32_t b, const uint32_t* R) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 31;
  const uint32_t e = 31u - (uint32_t)i;
  uint32_t t = b;
  for (uint32_t k = 0; k < (e >> 3); k++) t = (t >> 8) ^ R[t & 0xffu];
  for (uint32_t r = 0; r < (e & 7u); r++) t = (t >> 1) ^ ((t & 1u) ? kPoly : 0u);
  uint32_t v = ((a >> i) & 1u) ? t : 0u;
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o);
  return v;  // lanes 32-63 reduce the same 32 terms
}

// the tables of the slow path in LDS: every input of an entry's combine is a
// table word, and from global memory each was a dependent round trip
// (latency, not arithmetic, set the slow path's time: ~10 us per entry)
struct SlowLds {
  uint32_t tab[1024];  // slice-by-4 CRC tables (tab[0..255]: the byte step R)
  uint32_t mx[1024];   // v -> v * X^64 byte tables
  uint32_t m16k[1024];  // v -> v * x^16384 byte tables (tile_T's lower-half fix)
  uint32_t invpow[4097];
  uint32_t xtile[65], xt64[65], winit[64], zero_crc[64];
  uint32_t x32768;
};
__device__ __forceinline__ void load_slow_lds(SlowLds& L) {
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
    L.tab[i] = g_tabs.tab[i >> 8][i & 255];
    L.mx[i] = (&g_tabs.mx64[0][0])[i];
    L.m16k[i] = (&g_tabs.m16k[0][0])[i];
  }
  for (int i = threadIdx.x; i < 4097; i += blockDim.x) L.invpow[i] = g_tabs.invpow[i];
  for (int i = threadIdx.x; i < 65; i += blockDim.x) {
    L.xtile[i] = g_tabs.xtile[i];
    L.xt64[i] = g_tabs.xt64[i];
    if (i < 64) {
      L.winit[i] = g_tabs.winit[i];
      L.zero_crc[i] = g_tabs.zero_crc[i];
    }
  }
  if (threadIdx.x == 0) L.x32768 = g_tabs.x32768;
}

__device__ uint32_t crc_from_pieces_wave(uint64_t s, uint64_t m, uint32_t suf, uint32_t sxm, uint32_t tail,
                                         const uint32_t* tile, const SlowLds& L) {
  const uint32_t* mx64 = L.mx;
  const uint32_t* R = L.tab;
  const int lane = threadIdx.x & 63;
  const uint64_t len = m - s;
  if (len < 64) return tail ^ L.zero_crc[len];
  const uint64_t k0 = s / TILE, k1 = m / TILE;
  const uint32_t j0 = (uint32_t)((s % TILE) / 64);
  uint32_t acc = suf ^ L.winit[j0];
  uint32_t y;
  if (k0 == k1) {
    y = acc ^ sxm;
  } else {
    const uint64_t n = k1 - k0 - 1;  // whole tiles between
    // the last tile's values first (needed at the end), then the lane's
    // tiles 4 at a time: their loads issued together, then the Horner steps
    // (a dependent load chain per tile took ~10 us per C3 entry)
    const uint32_t e0 = tile[4 * k1], e2 = tile[4 * k1 + 2];
    uint32_t h = 0;
    uint64_t jl = 0;
    bool any = false;
    for (uint64_t jb = lane; jb < n; jb += 256) {
      uint32_t t0[4], t2[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint64_t j = jb + 64 * q, k = k0 + 1 + (j < n ? j : 0);
        t0[q] = tile[4 * k];
        t2[q] = tile[4 * k + 2];
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint64_t j = jb + 64 * q;
        if (j < n) {
          h = mulfix(h, mx64) ^ mulfix(t0[q], L.m16k) ^ t2[q];  // h * X^64 ^ tile_T(k0 + 1 + j)
          jl = j;
          any = true;
        }
      }
    }
    uint32_t v = any ? mulp(L.xtile[n - 1 - jl], h) : 0u;  // n-1-jl < 64
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
    // acc * X^n ^ mid, then one more tile step into k1
    const uint32_t xn = n < 64 * 65 ? mulp_wave(L.xt64[n >> 6], L.xtile[n & 63], R) : xpow8_any(n * (uint64_t)TILE);
    acc = mulp_wave(xn, acc, R) ^ v;
    y = mulp_wave(L.x32768, acc, R) ^ (mulfix(e0, L.m16k) ^ e2) ^ sxm;
  }
  const uint64_t dd = (k1 + 1) * TILE - m;
  return ~(mulp_wave(L.invpow[dd], y, R) ^ tail);
}

// one wave per slow entry (a piece of the combine was not recorded, or the
// entry spans more than LONG_TILES whole tiles)
// (SLOW_WAVES waves per block share the LDS tables; few blocks keep the
// launch cheap when the list is empty, the common case)
constexpr int SLOW_WAVES = 4;
// one wave: chain entry c's CRC from its recorded inputs (o_start / o_mo /
// o_pieces / o_suf / o_sxm / o_tail), recomputing missing pieces from the
// file.  tab, mx: the CRC and X^64 byte tables in LDS.
__device__ void slow_one(const FinArgs& a, uint64_t c, const SlowLds& L) {
  const uint32_t* tab = L.tab;
  const uint64_t s = a.o_start[c], m = a.o_mo[c];
  const uint32_t pieces = a.o_pieces[c], tail = a.o_tail[c];
  uint32_t suf = a.o_suf[c], sxm = a.o_sxm[c];
  if (!(pieces & 1)) suf = tile_probe_sx(a.file, a.flen, s / TILE, (uint32_t)((s % TILE) / 64), tab);
  if (!(pieces & 2)) sxm = tile_probe_sx(a.file, a.flen, m / TILE, (uint32_t)((m % TILE) / 64), tab);
  const uint32_t crc = crc_from_pieces_wave(s, m, suf, sxm, tail, a.tile, L);
  if ((threadIdx.x & 63) == 0) {
    a.o_crc[c] = crc;
    a.o_ok[c] = crc == a.o_crc_st[c];
    if (crc != a.o_crc_st[c]) atomicAdd(a.n_bad, 1ull);
  }
}
__global__ __launch_bounds__(SLOW_WAVES * 64) void slow_kernel(FinArgs a) {
  __shared__ SlowLds L;
  const unsigned long long ns = *a.n_slow;
  if ((uint64_t)blockIdx.x * SLOW_WAVES >= ns) return;
  load_slow_lds(L);
  __syncthreads();
  for (uint64_t w = (uint64_t)blockIdx.x * SLOW_WAVES + (threadIdx.x >> 6); w < ns;
       w += (uint64_t)gridDim.x * SLOW_WAVES)
    slow_one(a, a.slow_list[w], L);
}

// --------------------------------------------------------------------------
// 5. KeyIndexer::build -- latest wins, tombstones included
// --------------------------------------------------------------------------
constexpr uint64_t EMPTY_KEY = ~0ull;

__global__ void index_insert_kernel(const uint64_t* kh, const uint64_t* mo, uint64_t n, uint64_t* keys,
                                    unsigned long long* vals, uint64_t mask, unsigned long long* special) {
  uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const uint64_t k = kh[c];
  const unsigned long long v = mo[c] + 1;
  if (k == EMPTY_KEY) { atomicMax(special, v); return; }
  uint64_t i = xxh3_64_u64(k) & mask;
  while (true) {
    unsigned long long old = atomicCAS((unsigned long long*)&keys[i], (unsigned long long)EMPTY_KEY,
                                       (unsigned long long)k);
    if (old == EMPTY_KEY || old == k) { atomicMax(&vals[i], v); return; }
    i = (i + 1) & mask;
  }
}
__global__ void index_latest_kernel(const uint64_t* kh, const uint64_t* mo, uint64_t n, const uint64_t* keys,
                                    const unsigned long long* vals, uint64_t mask,
                                    const unsigned long long* special, uint32_t* latest) {
  uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const uint64_t k = kh[c];
  const unsigned long long v = mo[c] + 1;
  unsigned long long best;
  if (k == EMPTY_KEY) best = *special;
  else {
    uint64_t i = xxh3_64_u64(k) & mask;
    while (keys[i] != k) i = (i + 1) & mask;
    best = vals[i];
  }
  latest[c] = best == v;
}
// Xxh3BuildHasher over a key_hash (xxh3_build_hasher.rs:11-13): xxh3_64(le8(k))
__global__ void index_hash_kernel(const uint64_t* keys, uint64_t n, uint64_t* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = xxh3_64_u64(keys[i]);
}
__global__ void index_emit_kernel(const uint64_t* kh, const uint64_t* mo, const uint32_t* latest,
                                  const uint32_t* pos, uint64_t n, uint64_t* okey, uint64_t* opacked) {
  uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n || !latest[c]) return;
  const uint64_t k = kh[c];
  okey[pos[c]] = k;
  opacked[pos[c]] = ((k >> 48) << 48) | (mo[c] & 0xFFFFFFFFFFFFull);  // key_indexer.rs:79-85
}

// --------------------------------------------------------------------------
// batch digests (compute_checksum / compute_hash_batch)
// --------------------------------------------------------------------------

// one wave per range; range bytes may have any alignment
__global__ __launch_bounds__(64) void crc_batch_kernel(const uint8_t* buf, const uint64_t* offs,
                                                       const uint64_t* lens, uint64_t n, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint8_t* p = buf + offs[i];
    const uint64_t len = lens[i];
    uint32_t acc = 0;
    uint64_t o = 0;
    for (; o + TILE <= len; o += TILE) {  // full 4 KiB blocks
      uint32_t s = 0;
      const uint8_t* q = p + o + 64 * lane;
      for (int b = 0; b < 64; b++) s = g_tabs.tab[0][(s ^ q[b]) & 0xff] ^ (s >> 8);
      uint32_t u = mulp(g_tabs.lw[lane], s);
      for (int w = 32; w > 0; w >>= 1) u ^= __shfl_xor(u, w);
      acc = mulp(g_tabs.x32768, acc) ^ u;
    }
    const uint64_t rem = len - o;
    // remainder: line i covers [64i, min(64i+64, rem))
    uint32_t u = 0;
    const uint64_t ls = 64ull * lane;
    if (ls < rem) {
      const uint64_t le = ls + 64 < rem ? ls + 64 : rem;
      uint32_t s = 0;
      for (uint64_t b = ls; b < le; b++) s = g_tabs.tab[0][(s ^ p[o + b]) & 0xff] ^ (s >> 8);
      u = mulp(xpow8_dev(rem - le), s);
    }
    for (int w = 32; w > 0; w >>= 1) u ^= __shfl_xor(u, w);
    if (lane == 0) {
      const uint32_t raw = mulp(xpow8_dev(rem), acc) ^ u;
      out[i] = raw ^ ~mulp(xpow8_dev(len), 0xFFFFFFFFu);
    }
  }
}

__global__ void xxh3_batch_kernel(const uint8_t* keys, const uint64_t* offs, const uint64_t* lens, uint64_t n,
                                  uint64_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = xxh3_64(keys + offs[i], lens[i]);
}

// --------------------------------------------------------------------------
// synthetic store writer (checksum-on-append, data_store.rs:847-939)
// --------------------------------------------------------------------------
__device__ __forceinline__ uint64_t synth_word(uint64_t seed, uint64_t entry, uint64_t word) {
  uint64_t z = seed + ((entry << 32) + word + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// one wave per entry; entry_off[i] = prev tail (where the prepad starts)
// `out` is indexed by absolute file offset; bytes below clip_lo (a multiple
// of 64) are not written (span mode: they precede the shard's resident range).
// Entry i of this launch is global entry id0 + i (its key and payload seed).
__global__ __launch_bounds__(64) void synth_kernel(uint8_t* out, const uint64_t* entry_off,
                                                   const uint64_t* lens, uint64_t fixed_len, uint64_t n,
                                                   uint64_t seed, uint64_t id0, uint64_t clip_lo) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint64_t tail = entry_off[i];
    const uint64_t len = lens ? lens[i] : fixed_len;
    const uint64_t pad = prepad64(tail);
    const uint64_t st = tail + pad;  // 64-aligned
    const uint64_t id = id0 + i;
    if (lane < (int)pad && tail + lane >= clip_lo) out[tail + lane] = 0;
    // payload: 8-byte words
    uint32_t acc = 0;
    for (uint64_t blk = 0; blk < len; blk += TILE) {
      const uint64_t ls = blk + 64ull * lane;
      uint32_t s = 0;
      uint64_t le = ls + 64 < len ? ls + 64 : len;
      if (ls < len) {
        for (uint64_t w = ls / 8; w * 8 < le; w++) {
          const uint64_t v = synth_word(seed, id, w);
          const uint64_t nb = le - w * 8 < 8 ? le - w * 8 : 8;
          if (st + w * 8 >= clip_lo) {
            if (nb == 8) *(uint64_t*)(out + st + w * 8) = v;  // st is 64-aligned
            else for (uint64_t b = 0; b < nb; b++) out[st + w * 8 + b] = (uint8_t)(v >> (8 * b));
          }
          for (uint64_t b = 0; b < nb; b++) s = g_tabs.tab[0][(s ^ (uint32_t)(v >> (8 * b))) & 0xff] ^ (s >> 8);
        }
      }
      const uint64_t bl = len - blk < TILE ? len - blk : TILE;
      uint32_t u = ls < len ? mulp(xpow8_dev(bl - (le - blk)), s) : 0u;
      for (int w = 32; w > 0; w >>= 1) u ^= __shfl_xor(u, w);
      acc = mulp(xpow8_dev(bl), acc) ^ u;
    }
    if (lane == 0) {
      const uint32_t crc = acc ^ ~mulp(xpow8_dev(len), 0xFFFFFFFFu);
      // key "bench-key-{i}"
      uint8_t key[32] = {'b', 'e', 'n', 'c', 'h', '-', 'k', 'e', 'y', '-'};
      uint8_t dig[24];
      int nd = 0;
      uint64_t v = id;
      do { dig[nd++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
      for (int q = 0; q < nd; q++) key[10 + q] = dig[nd - 1 - q];
      const uint64_t kh = xxh3_64(key, 10 + nd);
      uint8_t mbuf[20];
      for (int b = 0; b < 8; b++) mbuf[b] = (uint8_t)(kh >> (8 * b));
      for (int b = 0; b < 8; b++) mbuf[8 + b] = (uint8_t)(tail >> (8 * b));
      for (int b = 0; b < 4; b++) mbuf[16 + b] = (uint8_t)(crc >> (8 * b));
      for (int b = 0; b < 20; b++)
        if (st + len + b >= clip_lo) out[st + len + b] = mbuf[b];
    }
  }
}

}  // namespace srd

// srd_writer.hip -- checksum-on-append batch writer (BASELINE config C5).
//
// Reference being replaced (jzombie/rust-simd-r-drive v0.16.3-alpha):
//   DataStoreWriter::batch_write           src/storage_engine/data_store.rs:838-843
//   batch_write_with_key_hashes            src/storage_engine/data_store.rs:847-939
//   compute_hash_batch (XXH3-64 of keys)   src/storage_engine/digest/compute_hash.rs:64-77
//   compute_checksum (CRC-32 of payloads)  src/storage_engine/digest/compute_checksum.rs:15-20
//   EntryMetadata::serialize               simd-r-drive-entry-handle/src/entry_metadata.rs:75-93
//
// One wave per entry (persistent grid of 16-wave blocks): the wave hashes the
// key, zero-fills the prepad, streams the payload into its 64-byte-aligned
// place in the output (4 KiB per step; lane l moves the 16-byte pieces at
// 1024 j + 16 l, so every load and store instruction covers one contiguous
// KiB) while computing its CRC with the scan's LDS slice-by-4 machinery
// (four chains per lane, lane weights, a half-wave XOR per 4 KiB, with the
// pieces' own distances in the tables), and writes the 20-byte metadata
// (key_hash, prev_offset = the previous tail, crc) after it.
// The layout (every entry's previous tail) comes from srd_batch_layout on the
// host: prepad_len makes each start depend on all earlier lengths.

namespace srd {

struct WriteArgs {
  const uint8_t* pay;           // payload bytes (srd_write_entry.src is relative to it)
  const uint8_t* keys;          // key bytes (key_src relative to it)
  const srd_write_entry* ent;   // n entries
  uint64_t n;
  uint8_t* out;                 // out[j] = file byte (base + j)
  uint64_t base;                // 64-aligned file offset of out[0]
  uint64_t* kh_out;             // [n] key hashes
  uint64_t* mo_out;             // [n] metadata offsets (the index's offsets)
  unsigned int* null_only;      // nullable: write_stream's check (data_store.rs:783-797), set when a payload is all NULL bytes
};

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
  return v;
}
// v * x^16384 for a wave-uniform v by SCALAR loads of the byte tables (the
// table words are uniform too: no LDS, no vector memory)
__device__ __forceinline__ uint32_t mul16k_u(uint32_t v) {
  const __attribute__((address_space(4))) uint32_t* m =
      (const __attribute__((address_space(4))) uint32_t*)&g_tabs.m16k[0][0];
  return m[v & 0xff] ^ m[256 + ((v >> 8) & 0xff)] ^ m[512 + ((v >> 16) & 0xff)] ^ m[768 + (v >> 24)];
}
// v * x^4096 (512 bytes) for a wave-uniform v by scalar loads
__device__ __forceinline__ uint32_t mul4096_u(uint32_t v) {
  const __attribute__((address_space(4))) uint32_t* m =
      (const __attribute__((address_space(4))) uint32_t*)&g_tabs.m4096[0][0];
  return m[v & 0xff] ^ m[256 + ((v >> 8) & 0xff)] ^ m[512 + ((v >> 16) & 0xff)] ^ m[768 + (v >> 24)];
}
// v * x^32768 (one 4 KiB block) = two x^16384 steps
__device__ __forceinline__ uint32_t mul_tile_u(uint32_t v) { return mul16k_u(mul16k_u(v)); }
// a table word at a wave-uniform index, by a scalar load
__device__ __forceinline__ uint32_t tab_u(const uint32_t* p) {
  return *(const __attribute__((address_space(4))) uint32_t*)p;
}
// x^(8 n) mod P for a wave-uniform n (xpow8_dev with scalar table loads)
__device__ __forceinline__ uint32_t xpow8_u(uint64_t n) {
  uint32_t r = kX0;
  for (int k = 0; n; k++, n >>= 1)
    if (n & 1) r = mulp(tab_u(&g_tabs.pow8[k]), r);
  return r;
}

// 64 readable bytes for the lanes whose line is no whole in-bounds payload
// line (their bytes are read one by one instead): the payload ring's loads
// stay unconditional
__device__ u32x4 g_wdummy[4];

// One wave per entry, entries w, w + W, ... of the batch (W waves in the
// grid).  The 4 KiB blocks of the wave's entries form one sequence; a 2-deep
// register ring keeps the next block's loads in flight while the current
// one is stored and checksummed.  Per block: lane l moves its four 16-byte
// pieces (1024 j + 16 l, j < 4) and computes their raw CRCs from the same
// registers (crc_line4_wide: one slice-by-4 chain per piece, the last step of
// pieces 0-2 shifted by their distance to piece 3 -- last_c), weighted by
// lane (lane_weight_or with nib_c: x^(128 (31 - l % 32))) and XOR-reduced per
// half-wave (half_suffix_xor): raw CRC of the block = (lo * x^4096) ^ hi.  The
// key hashes (XXH3-64, compute_hash.rs:25-27) are computed 64 at a time, one
// entry per lane, not by one lane per entry.
// V: variants of the SRD_DEBUG_API build (tools/writer_ab.py): 1 = the copy
// alone (no CRC, wrong outputs), 2 = the CRC alone (no payload stores, wrong
// outputs), 9 = round 3's lane = 64-byte line layout.  Measured (one process,
// two contexts, profiles/r04/writer_ab_*.txt): with lane = line the copy alone
// took as long as the whole kernel (2.13 vs 2.14 ms) while the runtime's
// device-to-device copy of the same bytes took 1.56-1.86 ms -- the strided
// 16-byte stores (each instruction touching every line of the block) were the
// bound; coalesced stores alone cut the copy to 1.89 ms.  The coalesced lanes
// with the CRC: 2.02 -> 1.97 ms.  Rejected: nontemporal payload stores (2x
// slower), a 3-deep register ring (+0.6 %, and +0.5 % with coalesced lanes).
template <int V = 0>
__global__ __launch_bounds__(SCAN_WAVES_V2 * 64, 1) void write_kernel(WriteArgs a) {
  // CO (the product layout): coalesced lanes -- lane l moves the 16-byte
  // pieces at 1024 j + 16 l of each 4 KiB block (one contiguous KiB per load /
  // store instruction) and checksums them with the same four slice-by-4
  // chains, the chains' and lanes' distances in their own tables
  // (DevTables::last_c, nib_c, m4096)
  constexpr bool CO = V != 9;
  __shared__ ScanLds lds;
  load_crc_lds<CO>(lds);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t R[4];
  crc_lane_bases(R, lane);
  const uint32_t nib_lane = lds_off(lds.nib) + 4u * (lane & 31);
  const uint64_t W = (uint64_t)gridDim.x * SCAN_WAVES_V2;
  const uint64_t w = (uint64_t)blockIdx.x * SCAN_WAVES_V2 + wv;
  if (w >= a.n) return;
  const bool pay_al = ((uintptr_t)a.pay & 15) == 0;
  uint64_t last_len = ~0ull;  // cache of ~(x^(8 len) * 0xFFFFFFFF) for runs of equal lengths
  uint32_t last_fix = 0;

  auto vec_line = [&](const srd_write_entry& e, uint64_t b) -> bool {
    return !(e.flags & SRD_ENTRY_TOMB) && pay_al && (e.src & 15) == 0 && b * TILE + 64ull * lane + 64 <= e.len;
  };
  // CO: piece j of the lane is a whole in-bounds 16-byte vector
  auto vec_piece = [&](const srd_write_entry& e, uint64_t b, int j) -> bool {
    return !(e.flags & SRD_ENTRY_TOMB) && pay_al && (e.src & 15) == 0 &&
           b * TILE + 1024ull * j + 16ull * lane + 16 <= e.len;
  };
  auto load_blk = [&](const srd_write_entry& e, uint64_t b, uint32_t (&o)[16]) {
    if constexpr (CO) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const u32x4* q =
            vec_piece(e, b, j) ? (const u32x4*)(a.pay + e.src + b * TILE + 1024ull * j + 16ull * lane) : &g_wdummy[j];
        const u32x4 v = *q;
        o[4 * j] = v[0]; o[4 * j + 1] = v[1]; o[4 * j + 2] = v[2]; o[4 * j + 3] = v[3];
      }
      return;
    }
    const u32x4* q = vec_line(e, b) ? (const u32x4*)(a.pay + e.src + b * TILE + 64ull * lane) : g_wdummy;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const u32x4 v = q[j];
      o[4 * j] = v[0]; o[4 * j + 1] = v[1]; o[4 * j + 2] = v[2]; o[4 * j + 3] = v[3];
    }
  };

  uint64_t i = 0, b = 0, khl = 0, gend = 0;
  srd_write_entry e;
  // the wave's entry descriptors by SCALAR loads (constant address space: the
  // table is read-only here): as vector loads they joined the ring's vmcnt
  // queue and their wait drained it -- the previous unit's stores included
  auto ent_s = [&](uint64_t k) {
    const __attribute__((address_space(4))) uint64_t* q =
        (const __attribute__((address_space(4))) uint64_t*)(a.ent + k);
    srd_write_entry x;
    x.src = q[0];
    x.len = q[1];
    x.key_src = q[2];
    x.tail = q[3];
    const uint64_t kf = q[4];
    x.key_len = (uint32_t)kf;
    x.flags = (uint32_t)(kf >> 32);
    return x;
  };
  // entry p's metadata ends at t (p's layout: data_store.rs:863-931), so the
  // wave of p writes the prepad that follows it (the metadata store below)
  auto meets = [&](const srd_write_entry& p, uint64_t t) -> bool {
    const uint64_t pmo = (p.flags & SRD_ENTRY_TOMB) ? p.tail + 1 : p.tail + prepad64(p.tail) + p.len;
    return pmo + 20 == t;
  };
  uint32_t acc = 0, any = 0;
  // one unit of the sequence: block b of entry i (a tombstone is one unit
  // without a block); returns whether a next unit exists in the group (its
  // loads went to nx)
  // the unit after (i0, b0) of entry e0
  struct Unit {
    uint64_t i, b;
    srd_write_entry e;
  };
  auto advance = [&](uint64_t i0, uint64_t b0, const srd_write_entry& e0) -> Unit {
    const uint64_t nb = (e0.flags & SRD_ENTRY_TOMB) ? 1 : (e0.len + TILE - 1) / TILE;
    Unit u{i0, b0 + 1, e0};
    if (u.b >= nb) {
      u.i = i0 + W;
      u.b = 0;
      if (u.i < gend) u.e = ent_s(u.i);
    }
    return u;
  };
  auto step = [&](uint32_t (&d)[16], uint32_t (&nx)[16]) -> bool {
    const bool tomb = e.flags & SRD_ENTRY_TOMB;
    const uint64_t nb = tomb ? 1 : (e.len + TILE - 1) / TILE;
    const Unit u2 = advance(i, b, e);
    const uint64_t i2 = u2.i, b2 = u2.b;
    const srd_write_entry e2 = u2.e;
    load_blk(e2, b2, nx);  // (past the group: a block of this entry again, or the dummy -- harmless)
    const int jl = (int)(((i - w) / W) % 64);  // the entry's lane in khl
    const uint64_t kh = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(khl >> 32), jl) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)khl, jl);
    // Every store of a unit is an UNCONDITIONAL buffer store whose unused
    // lanes fall outside the descriptor's range (dropped by the hardware):
    // stores under a branch made the count of memory ops between a block's
    // loads and their wait path-dependent, and the ring's wait then also
    // waited for the previous unit's stores to complete (the scan's rule)
    const uint64_t pad = tomb ? 0 : prepad64(e.tail), st = e.tail + pad;  // data_store.rs:907-914
    // the zero bytes before the payload: the prepad on an entry's first
    // block, the single NULL byte of a tombstone (data_store.rs:864-897)
    // (an entry's prepad is written by the wave of the batch's previous entry,
    // with that entry's metadata -- one whole line instead of two partial
    // ones from two waves -- when that entry's metadata ends at this entry's
    // tail; the batch's first entry, and one whose table predecessor ends
    // elsewhere (a caller-built, gapped or reordered srd_batch_write_device
    // table), writes its own)
    bool own_pad = i == 0;
    if (!tomb && b == 0 && i > 0) own_pad = !meets(ent_s(i - 1), e.tail);  // uniform
    const uint32_t nz = tomb ? 1u : (b == 0 && own_pad ? (uint32_t)pad : 0u);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, out_rsrc(a.out + (e.tail - a.base), nz), (uint32_t)lane, 0, 0);
    bool done = tomb;
    uint32_t crc = 0xD202EF8Du;  // CRC32(b"\0")
    uint64_t mo = e.tail + 1;
    if (!tomb) {
      uint8_t* dst = a.out + (st - a.base);  // 64-aligned when out is
      if (b == 0) {
        acc = 0;
        any = 0;
      }
      const uint64_t o = b * TILE + 64ull * lane;
      const bool vec = CO ? true : vec_line(e, b);
      bool vp[4];
#pragma unroll
      for (int j = 0; j < 4; j++) vp[j] = CO ? vec_piece(e, b, j) : vec;
      if constexpr (CO) {
        // a partial (or unaligned) piece: byte by byte, zero past the payload
        const uint8_t* src = a.pay + e.src;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (!vp[j]) {
            const uint64_t oj = b * TILE + 1024ull * j + 16ull * lane;
            const uint32_t nl = oj < e.len ? (uint32_t)min<uint64_t>(16, e.len - oj) : 0u;
#pragma unroll
            for (int k = 0; k < 4; k++) {
              uint32_t wd = 0;
#pragma unroll
              for (int kb = 0; kb < 4; kb++) {
                const uint32_t q = 4u * k + kb;
                if (q < nl) {
                  const uint8_t v = src[oj + q];
                  dst[oj + q] = v;
                  wd |= (uint32_t)v << (8 * kb);
                }
              }
              d[4 * j + k] = wd;
            }
          }
        }
      } else if (!vec) {
        // a partial (or unaligned) line: byte by byte, zero past the payload
        // (extra memory ops on this path only: the ring's waits stay right)
        const uint32_t nl = o < e.len ? (uint32_t)min<uint64_t>(64, e.len - o) : 0u;
        const uint8_t* src = a.pay + e.src;
        // (static register indices only: a dynamic d[q >> 2] put a ring
        // array in scratch)
#pragma unroll
        for (int j = 0; j < 16; j++) {
          uint32_t wd = 0;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const uint32_t q = 4u * j + k;
            if (q < nl) {
              const uint8_t v = src[o + q];
              dst[o + q] = v;
              wd |= (uint32_t)v << (8 * k);
            }
          }
          d[j] = wd;
        }
      }
      {
        const __amdgpu_buffer_rsrc_t rb = out_rsrc(dst + b * TILE, TILE);
#pragma unroll
        for (int j = 0; j < 4; j++)
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{d[4 * j], d[4 * j + 1], d[4 * j + 2], d[4 * j + 3]}, rb,
                                                 vp[j] && V != 2 ? (CO ? 16u * lane + 1024u * j : 64u * lane + 16u * j)
                                                                 : OOB_OFF,
                                                 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 16; j++) any |= d[j];
      // raw CRC of this 4 KiB block (zero-padded past the payload)
      const uint32_t hx = V == 1 ? d[0] ^ d[15] : half_suffix_xor(lane_weight_or(crc_line4_wide(d, lds, R), nib_lane), lane);
      const uint32_t lo = __builtin_amdgcn_readlane(hx, 0), hi = __builtin_amdgcn_readlane(hx, 32);
      const uint32_t raw = (CO ? mul4096_u(lo) : mul16k_u(lo)) ^ hi;
      acc = b ? mul_tile_u(acc) ^ raw : raw;
      if (b + 1 == nb) {
        if (a.null_only && !__ballot(any != 0) && lane == 0) atomicOr(a.null_only, 1u);
        const uint64_t z = nb * TILE - e.len;  // trailing zero padding of the last block, < 4096
        // (uniform values: scalar table loads, which leave the ring's vmcnt queue alone)
        if (z) acc = mulp(tab_u(&g_tabs.invpow[z]), acc);
        if (e.len != last_len) {
          last_len = e.len;
          last_fix = ~mulp(xpow8_u(e.len), 0xFFFFFFFFu);
        }
        crc = acc ^ last_fix;  // crc32fast: init and xorout 0xFFFFFFFF
        mo = st + e.len;
        done = true;
      }
    }
    // EntryMetadata::serialize: key_hash LE, prev_offset LE, checksum LE
    // (bytes 0-19, one per lane), then the zero prepad of the batch's next
    // entry up to its payload start (data_store.rs:907-914; a tombstone has
    // none), so the line holding both is written whole by this wave; the
    // (key_hash, metadata offset) pair
    {
      // the next entry's prepad only when it follows this entry (meets(); a
      // table out of order or with gaps: 20 bytes, the next entry's wave writes
      // its own prepad)
      uint64_t next_start = mo + 20;
      if (i + 1 < a.n) {
        const srd_write_entry en = ent_s(i + 1);
        if (en.tail == mo + 20) next_start = (en.flags & SRD_ENTRY_TOMB) ? en.tail : en.tail + prepad64(en.tail);
      }
      const uint32_t nb_meta = done ? (uint32_t)(next_start - mo) : 0u;  // 20 .. 83
      const uint64_t v = lane < 8 ? kh : lane < 16 ? e.tail : (uint64_t)crc;
      const __amdgpu_buffer_rsrc_t rm = out_rsrc(a.out + (mo - a.base), nb_meta);
      __builtin_amdgcn_raw_buffer_store_b8(lane < 20 ? (uint8_t)(v >> (8 * (lane & 7))) : (uint8_t)0, rm, (uint32_t)lane, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, rm, 64u + (uint32_t)lane, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)kh, (uint32_t)(kh >> 32)}, out_rsrc(a.kh_out + i, done ? 8u : 0u),
                                            8u * lane, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)mo, (uint32_t)(mo >> 32)}, out_rsrc(a.mo_out + i, done ? 8u : 0u),
                                            8u * lane, 0, 0);
    }
    i = i2;
    b = b2;
    e = e2;
    return i < gend;
  };
  uint32_t cur[16], nxt[16];
  // groups of 64 entries of the wave: their key hashes first (one per lane,
  // outside the ring), then the ring over the group's blocks
  for (uint64_t g0 = w; g0 < a.n; g0 += 64 * W) {
    {
      const uint64_t ij = g0 + (uint64_t)lane * W;
      khl = 0;
      if (ij < a.n) {
        const srd_write_entry ej = a.ent[ij];
        khl = (ej.flags & SRD_ENTRY_HASHED) ? ej.key_src : xxh3_64(a.keys + ej.key_src, ej.key_len);
      }
    }
    gend = min(a.n, g0 + 64 * W);
    i = g0;
    b = 0;
    e = ent_s(i);
    load_blk(e, 0, cur);
    // the ring: two register blocks, the roles swapped every unit
    while (step(cur, nxt) && step(nxt, cur)) {
    }
  }
}

}  // namespace srd

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
// place in the output (4 KiB per step, one 64-byte line per lane) while
// computing its CRC with the scan's LDS line-CRC machinery (crc_line1 +
// lane weights + a wave XOR-reduce per 4 KiB), and writes the 20-byte
// metadata (key_hash, prev_offset = the previous tail, crc) after it.
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
// v * x^32768 (one 4 KiB block) = two x^16384 byte-table steps
__device__ __forceinline__ uint32_t mul_tile(uint32_t v) { return mul16k(mul16k(v, &g_tabs.m16k[0][0]), &g_tabs.m16k[0][0]); }

__global__ __launch_bounds__(SCAN_WAVES_V2 * 64, 1) void write_kernel(WriteArgs a) {
  __shared__ ScanLds lds;
  load_crc_lds(lds);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t R[4];
  crc_lane_bases(R, lane);
  uint64_t last_len = ~0ull;   // cache of ~(x^(8 len) * 0xFFFFFFFF) for runs of equal lengths
  uint32_t last_fix = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * SCAN_WAVES_V2 + wv; i < a.n; i += (uint64_t)gridDim.x * SCAN_WAVES_V2) {
    const srd_write_entry e = a.ent[i];
    // key hash (lane 0; compute_hash.rs:25-27 = xxh3_64 with seed 0)
    uint64_t kh = e.key_src;  // SRD_ENTRY_HASHED: batch_write_with_key_hashes / write_stream_with_key_hash
    if (!(e.flags & SRD_ENTRY_HASHED) && lane == 0) kh = xxh3_64(a.keys + e.key_src, e.key_len);
    kh = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(kh >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)kh);
    uint32_t crc;
    uint64_t mo;
    if (e.flags & SRD_ENTRY_TOMB) {
      // tombstone: the single NULL byte, no prepad (data_store.rs:864-897)
      if (lane == 0) a.out[e.tail - a.base] = 0;
      crc = 0xD202EF8Du;  // CRC32(b"\0")
      mo = e.tail + 1;
    } else {
      const uint64_t pad = prepad64(e.tail), st = e.tail + pad;  // data_store.rs:907-914
      if ((uint64_t)lane < pad) a.out[e.tail - a.base + lane] = 0;
      const uint8_t* src = a.pay + e.src;
      uint8_t* dst = a.out + (st - a.base);  // 64-aligned when out is
      const bool fast_src = ((uintptr_t)src & 15) == 0;
      uint32_t acc = 0, any = 0;
      const uint64_t nb = (e.len + TILE - 1) / TILE;
      for (uint64_t b = 0; b < nb; b++) {
        const uint64_t o = b * TILE + 64ull * lane;
        const uint32_t nl = o < e.len ? (uint32_t)min<uint64_t>(64, e.len - o) : 0u;
        uint32_t d[16];
        if (nl == 64 && fast_src) {
          const u32x4* q = (const u32x4*)(src + o);
          u32x4* w = (u32x4*)(dst + o);
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const u32x4 v = q[j];
            w[j] = v;
            d[4 * j] = v[0]; d[4 * j + 1] = v[1]; d[4 * j + 2] = v[2]; d[4 * j + 3] = v[3];
          }
        } else {
#pragma unroll
          for (int j = 0; j < 16; j++) d[j] = 0;
          for (uint32_t q = 0; q < nl; q++) {
            const uint8_t v = src[o + q];
            dst[o + q] = v;
            d[q >> 2] |= (uint32_t)v << (8 * (q & 3));
          }
        }
#pragma unroll
        for (int j = 0; j < 16; j++) any |= d[j];
        // raw CRC of this 4 KiB block (zero-padded past the payload)
        const uint32_t u = lane_weight(crc_line1(d, lds, R), lds.nib, lane);
        const uint32_t lo = wave_xor(lane < 32 ? u : 0u), hi = wave_xor(lane < 32 ? 0u : u);
        const uint32_t raw = mul16k(lo, &g_tabs.m16k[0][0]) ^ hi;
        acc = mul_tile(acc) ^ raw;
      }
      if (a.null_only && !__ballot(any != 0) && lane == 0) atomicOr(a.null_only, 1u);
      const uint64_t z = nb * TILE - e.len;  // trailing zero padding of the last block, < 4096
      if (z) acc = mulp(g_tabs.invpow[z], acc);
      if (e.len != last_len) {
        last_len = e.len;
        last_fix = ~mulp(xpow8_dev(e.len), 0xFFFFFFFFu);
      }
      crc = acc ^ last_fix;  // crc32fast: init and xorout 0xFFFFFFFF
      mo = st + e.len;
    }
    // EntryMetadata::serialize: key_hash LE, prev_offset LE, checksum LE
    if (lane < 20) {
      const uint64_t v = lane < 8 ? kh : lane < 16 ? e.tail : (uint64_t)crc;
      a.out[mo - a.base + lane] = (uint8_t)(v >> (8 * (lane & 7)));
    }
    if (lane == 0) {
      a.kh_out[i] = kh;
      a.mo_out[i] = mo;
    }
  }
}

}  // namespace srd

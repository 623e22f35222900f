// srd_index.hip -- the device KeyIndexer and batched keyed reads
// (adopt the index the validate pass built on the GPU
// instead of re-inserting it into a host HashMap, and serve batched lookups).
//
// Reference being replaced (jzombie/rust-simd-r-drive v0.16.3-alpha):
//   KeyIndexer (HashMap<u64, u64>)      src/storage_engine/key_indexer.rs:98-124, get_packed :164-167
//   batch_read / batch_read_hashed_keys src/storage_engine/data_store.rs:1111-1158
//   read_entry_with_context             src/storage_engine/data_store.rs:502-565
//
// Table: open addressing over 2^k slots (load <= 1/2), keys[] then packed[]
// (two u64 arrays); an empty slot holds packed == ~0 (a packed value is
// tag16 << 48 | offset48 with offset < file_len, never all ones).  Keys are
// unique (an index), so an insert only claims a slot: CAS on packed.

namespace srd {

constexpr uint64_t TBL_EMPTY = ~0ull;

__device__ __forceinline__ uint64_t idx_slot(uint64_t k, uint32_t log2cap) {
  k ^= k >> 29;  // key hashes are XXH3 outputs already; one mix keeps clustered inputs spread
  return (k * 0x9E3779B97F4A7C15ull) >> (64 - log2cap);
}

__global__ void idx_table_insert_kernel(const uint64_t* keys, const uint64_t* packed, uint64_t n, uint64_t* tkeys,
                                        unsigned long long* tpacked, uint32_t log2cap) {
  const uint64_t mask = (1ull << log2cap) - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i], p = packed[i];
    uint64_t s = idx_slot(k, log2cap);
    for (;;) {  // terminates: at most cap/2 keys
      if (atomicCAS(tpacked + s, (unsigned long long)TBL_EMPTY, (unsigned long long)p) == TBL_EMPTY) {
        tkeys[s] = k;
        break;
      }
      s = (s + 1) & mask;
    }
  }
}

__device__ __forceinline__ uint64_t idx_get_packed(const uint64_t* tkeys, const uint64_t* tpacked, uint32_t log2cap,
                                                   uint64_t k) {
  const uint64_t mask = (1ull << log2cap) - 1;
  uint64_t s = idx_slot(k, log2cap);
  for (;;) {
    const uint64_t p = tpacked[s];
    if (p == TBL_EMPTY) return TBL_EMPTY;
    if (tkeys[s] == k) return p;
    s = (s + 1) & mask;
  }
}

__global__ void idx_get_packed_kernel(const uint64_t* tkeys, const uint64_t* tpacked, uint32_t log2cap,
                                      const uint64_t* q, uint64_t n, uint64_t* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = idx_get_packed(tkeys, tpacked, log2cap, q[i]);
}

// read_entry_with_context (data_store.rs:502-565) per query: [start, end) of
// the entry's payload, or (0, 0) for None (absent, tag mismatch against the
// verification hash, out of range, or a tombstone)
__global__ void batch_read_kernel(const uint64_t* tkeys, const uint64_t* tpacked, uint32_t log2cap,
                                  const uint8_t* file, uint64_t flen, const uint64_t* q, const uint64_t* verify,
                                  uint64_t n, uint64_t* out_start, uint64_t* out_end) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t start = 0, end = 0;
    const uint64_t p = idx_get_packed(tkeys, tpacked, log2cap, q[i]);
    const uint64_t off = p & 0xFFFFFFFFFFFFull;
    bool ok = p != TBL_EMPTY;
    if (ok && verify) ok = (p >> 48) == (verify[i] >> 48);  // tag_from_key(non_hashed_key), :513-521
    ok = ok && off + 20 <= flen;                               // :524-526
    if (ok) {
      const uint64_t prev = ld_u64_unaligned(file, off + 8);  // EntryMetadata.prev_offset
      uint64_t s = prev + prepad64(prev);                     // :533-535
      if (off > prev && off - prev == 1 && file[prev] == 0) s = prev;  // tombstone: no prepad, :539-544
      if (s < off) {                                         // :546-548 (off <= flen already)
        if (!(off - s == 1 && file[s] == 0)) {               // tombstone -> None, :551-553
          start = s;
          end = off;
        }
      }
    }
    out_start[i] = start;
    out_end[i] = end;
  }
}

}  // namespace srd

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

// The payload range of the entry whose metadata is at `off`, with the
// reference's bounds, prepad and tombstone rules (read_entry_with_context
// :524-553, par_iter_entries :322-353, EntryIterator::next
// entry_iterator.rs:85-118); false for None (out of range / tombstone).
__device__ __forceinline__ bool entry_range(const uint8_t* file, uint64_t flen, uint64_t off, uint64_t* start,
                                            uint64_t* end) {
  if (off + 20 > flen) return false;
  const uint64_t prev = ld_u64_unaligned(file, off + 8);  // EntryMetadata.prev_offset
  uint64_t s = prev + prepad64(prev);
  if (off > prev && off - prev == 1 && file[prev] == 0) s = prev;  // tombstone: no prepad
  if (s >= off) return false;
  if (off - s == 1 && file[s] == 0) return false;  // tombstone -> None
  *start = s;
  *end = off;
  return true;
}

// par_iter_entries over the index: flags, ranges and the kept bytes
// (range + metadata, EntryHandle::file_size) for estimate_compaction_savings
__global__ __launch_bounds__(256) void iter_flag_kernel(const uint8_t* file, uint64_t flen, const uint64_t* packed,
                                                        uint64_t n, uint32_t* flag, uint64_t* st, uint64_t* en,
                                                        unsigned long long* kept) {
  __shared__ unsigned long long part[4];
  unsigned long long mine = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t s = 0, e = 0;
    const bool ok = entry_range(file, flen, packed[i] & 0xFFFFFFFFFFFFull, &s, &e);
    flag[i] = ok;
    st[i] = s;
    en[i] = e;
    if (ok) mine += e - s + 20;
  }
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mine;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(kept, part[0] + part[1] + part[2] + part[3]);
}

// EntryIterator order (newest first = the index's file order reversed)
__global__ void iter_emit_kernel(const uint8_t* file, const uint64_t* packed, const uint32_t* flag, const uint32_t* pos,
                                 uint64_t n, uint64_t n_valid, const uint64_t* st, const uint64_t* en,
                                 uint64_t* out_start, uint64_t* out_end, uint64_t* out_meta, uint64_t* out_kh) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (!flag[i]) continue;
    const uint64_t j = n_valid - 1 - pos[i];
    const uint64_t off = packed[i] & 0xFFFFFFFFFFFFull;
    out_start[j] = st[i];
    out_end[j] = en[i];
    if (out_meta) out_meta[j] = off;
    if (out_kh) out_kh[j] = ld_u64_unaligned(file, off);
  }
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
    if (ok && !entry_range(file, flen, off, &start, &end)) start = end = 0;
    out_start[i] = start;
    out_end[i] = end;
  }
}

// compact's layout (data_store.rs:706-719 -> write_stream_with_key_hash per
// entry, :758-825, tail from 0): entry j's payload starts at
// P_j = roundup64(tail_j) and tail_{j+1} = P_j + len_j + 20, so
// P_{j+1} = P_j + roundup64(len_j + 20) -- an exclusive prefix sum of
// roundup64(len + 20), no sequential walk.
__global__ void compact_sizes_kernel(const uint64_t* st, const uint64_t* en, uint64_t n, uint64_t* rlen) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    rlen[i] = (en[i] - st[i] + 20 + 63) & ~63ull;
}

__global__ void compact_entries_kernel(const uint64_t* st, const uint64_t* en, const uint64_t* kh,
                                       const uint64_t* pstart, uint64_t n, srd_write_entry* ent, uint64_t* new_len) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t tail = j ? pstart[j - 1] + (en[j - 1] - st[j - 1]) + 20 : 0;
    ent[j] = srd_write_entry{st[j], en[j] - st[j], kh[j], tail, 0u, SRD_ENTRY_HASHED};
    if (j == n - 1) *new_len = pstart[j] + (en[j] - st[j]) + 20;
  }
}

}  // namespace srd

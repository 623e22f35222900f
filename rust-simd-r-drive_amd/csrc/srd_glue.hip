// srd_glue.hip -- sync-free glue of the optimistic pass (included by srd_api.hip
// after srd_kernels.hip).
//
// Everything between the streaming scan and the final result runs with the
// counts kept in device memory (struct Plan); the host enqueues the pass and
// waits once, on the outcome idx_emit publishes to pinned host memory:
//
//   scan            (srd_kernels.hip) strong candidates only, each wave's
//                   records dense in its region (ScanPart); block 0 zeroes
//                   the plan and the index bucket fills
//   link2           (srd_kernels.hip) one block per scan wave: every
//                   record's node test, parent (the previous record, else a
//                   binary search in the parent's span, skipped when the
//                   would-be parent's prev field rules a record out) and the
//                   claim on it, the earliest claimer winning (claim_word).
//                   Slot space throughout: record r of wave w is slot
//                   w*wcap + r
//   check           shape test from the claims alone: the core nodes (claimed
//                   by someone, or the start node at file_len - 20) must form
//                   ONE chain from the start down to a root -- each core node's
//                   parent claimed by it, exactly one core node linking to a
//                   root.  Leaves (false candidates nobody links to) are
//                   ignored, the pruning recover_valid_chain's walk gets from
//                   only following back-pointers from file_len
//                   (data_store.rs:404-470).  Per-block core counts.  A failed
//                   test retries with more prune rounds (marks_from_claims),
//                   then sends the call to the full pass; it never changes a
//                   result.
//   chain_finalize  plan (every block derives it, block 0 publishes), the chain
//                   rank of each core node, the per-entry outputs and CRC from
//                   the scan's pieces (entries that need a wave go to the
//                   call's slow list), and KeyIndexer::build's bucket claims +
//                   scatter
//   idx_dedup       the slow list (one wave per entry), then one block per
//                   XXH3 bucket: marks the non-latest entries
//                   (generation bytes); none marked -> the index aliases
//                   (o_kh, o_packed)
//   idx_emit        compacts the latest entries in chain order (or nothing,
//                   aliased) and publishes the outcome (PUB_WORDS) to the host
//
// Generation tags (claim_word: gen and ~g in one u64; lgen bytes for the non-latest marks)
// make the per-node marks self-invalidating between calls, so no per-call
// memsets are needed.
#pragma once

namespace srd {

// The glue's per-entry outputs (~100 MB per C2 call) are not left as dirty
// lines in L2: round 3 made them nontemporal (written back while the NEXT
// call's scan streamed the store: scan -1 %, call -1 %, profiles/r03/
// scan_record_regions_ab.txt), round 6 writes them through (srd_gst,
// srd_kernels.hip)
#define GST(ptr, val) srd_gst(&(ptr), (val))  // (srd_kernels.hip: written through the XCD's L2)

struct Plan {
  uint64_t K;          // dense candidates
  uint64_t n_chain;    // chain entries incl. the root entry
  uint64_t root_t;     // tail of the root entry
  uint64_t start;      // dense index of the node at file_len - 20, or ~0
  uint64_t n_index;
  uint64_t n_bad;      // chain entries whose CRC mismatches
  uint64_t n_slow;     // finalize entries handed to slow_kernel
  uint64_t chain_core; // core nodes (n_chain - 1 on success)
  uint64_t max_root, top_gap, overflow;  // the scan counters; top_gap = file_len - the start tail (find_top)
  uint32_t status;     // ST_* bits; 0 = the optimistic result is final
  uint32_t nroot;      // core nodes linking to a root
  uint32_t troot;      // file_len itself is a root tail
  uint32_t idx_overflow;
  uint32_t idx_alias;  // every chain entry is its key's latest: the index IS (o_kh, o_packed) (idx_emit)
};
constexpr uint32_t ST_NOSTART = 1, ST_SHAPE = 2, ST_ROOTS = 4, ST_OVERFLOW = 16;
constexpr uint64_t NO_NODE = ~0ull;

constexpr int GLUE_BLOCKS = 1024;  // chunked grid of the count/scatter kernels
constexpr int GLUE_THREADS = 256;

// rank of `f` among the 256 flags of this block iteration (exclusive) and the
// iteration's total; wsum is LDS[4]
__device__ __forceinline__ uint32_t block_rank256(bool f, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t bal = __ballot(f);
  const uint32_t pre = (uint32_t)__popcll(bal & ((1ull << lane) - 1));
  if (lane == 0) wsum[w] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t v = wsum[i];
    off += i < w ? v : 0u;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return off + pre;
}

// the same for NW-wave blocks (wsum: LDS[NW])
template <int NW>
__device__ __forceinline__ uint32_t block_rank_n(bool f, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t bal = __ballot(f);
  const uint32_t pre = (uint32_t)__popcll(bal & ((1ull << lane) - 1));
  if (lane == 0) wsum[w] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    const uint32_t v = wsum[i];
    off += i < w ? v : 0u;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return off + pre;
}
template <int NW>
__device__ __forceinline__ uint32_t block_sum_n(uint32_t v, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) wsum[w] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) t += wsum[i];
  __syncthreads();
  return t;
}
// chunked grid of the shape check and the fused chain finalize (which also
// builds the index histogram and scatter of its chain positions)
constexpr int CHAIN_BLOCKS = 256;
constexpr int CHAIN_THREADS = 1024;
constexpr int CHAIN_WAVES = CHAIN_THREADS / 64;

__device__ __forceinline__ uint32_t block_sum256(uint32_t v, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) wsum[w] = v;
  __syncthreads();
  const uint32_t t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return t;
}

__device__ __forceinline__ void chunk_of(uint64_t n, uint64_t* lo, uint64_t* hi) {
  const uint64_t ch = (n + gridDim.x - 1) / gridDim.x;
  *lo = min(n, (uint64_t)blockIdx.x * ch);
  *hi = min(n, *lo + ch);
}

// sum of part[0 .. blockIdx.x) (exclusive prefix of this block) and of all
// np partials, by every block itself (np <= 1024; replaces a one-block scan launch)
__device__ __forceinline__ void block_prefix(const uint32_t* part, uint32_t np, uint32_t* wsum, uint64_t* before,
                                             uint64_t* total) {
  uint32_t b = 0, t = 0;
  for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
    const uint32_t v = part[i];
    t += v;
    b += i < blockIdx.x ? v : 0u;
  }
  *before = block_sum256(b, wsum);
  *total = block_sum256(t, wsum);
}



// exclusive scan of up to 1024 partials with one 1024-thread block
__device__ uint64_t block_scan_partials(const uint32_t* part, uint32_t np, uint32_t* part_ex) {
  __shared__ uint64_t s[1024];
  const uint32_t t = threadIdx.x;
  uint64_t v = t < np ? part[t] : 0;
  s[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint64_t a = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += a;
    __syncthreads();
  }
  if (t < np) part_ex[t] = (uint32_t)(s[t] - v);
  const uint64_t total = s[1023];
  __syncthreads();
  return total;
}

struct ShapeArgs {
  const uint8_t* file;
  uint64_t flen;
  uint32_t gen;
  // slot space (scan_kernel's link phase): record r of scan wave w is slot
  // w*wcap + r, r < min(wave_total[w], wcap); the chain blocks take the scan
  // waves in order, wpb each (block_waves)
  const uint64_t* Kp;  // [0] records, [1] 1 + the slot of the last record (0: none)
  const uint64_t* wave_total;
  uint64_t wcap;
  uint32_t n_waves, wpb;
  uint64_t n_slots;     // n_waves * wcap
  const uint64_t* c_m;  // the records' metadata offsets
  const int32_t* d_par;  // the parent's slot / PAR_ROOT / PAR_MISS
  const u32x4* c_rec;
  const uint32_t* has_child;  // retry rounds: the prune marks
  uint64_t* childof;
  uint8_t* flag;
  uint32_t* part;       // [CHAIN_BLOCKS] core records per chain block (check_kernel)
  uint32_t* wpart;      // [CHAIN_BLOCKS * CHAIN_WAVES] core records per wave chunk (check_kernel)
  const unsigned long long* counters;
  Plan* plan;
  uint32_t coff;     // chain entries before the first candidate (1 whole file, 0 span mode)
  uint32_t* zero;    // child2_kernel zeroes [zero, zero + n_zero): the index's bucket fills and chunk counts
  uint32_t n_zero;
  // FUSED chain_finalize: the chain block whose look-back is treated as timed
  // out (SRD_LB_FAIL_BLOCK at context creation, a test knob); ~0u = none
  uint32_t lb_fail;
};

// the slot of the node at the start tail find_top chose (the scan's
// counters[1]; no candidate lies above it): the last record
__device__ __forceinline__ uint64_t start_node(const ShapeArgs& a) {
  const uint64_t t = a.counters[1], s1 = a.Kp[1];
  return (s1 && t >= 21 && a.c_m[s1 - 1] == t - 20) ? s1 - 1 : NO_NODE;
}
// a record region overflowed (ST_OVERFLOW: the records past it were not
// stored or linked) -- the shape kernels must not read the slot arrays;
// chain_finalize reports the status and the host retries larger
__device__ __forceinline__ bool dense_incomplete(const ShapeArgs& a) { return a.counters[2] != 0; }

// Chain block b's records: scan waves [b*wpb, (b+1)*wpb) in file order,
// flattened (s_pre: LDS[wpb + 1], the exclusive prefix of their record
// counts); returns the block's record count.  slot_of maps a block index to
// its slot.
constexpr uint32_t BW_MAX = 64;  // wpb bound (the host checks)
__device__ __forceinline__ uint32_t block_waves(const ShapeArgs& a, uint32_t* s_pre) {
  const uint64_t w0 = (uint64_t)blockIdx.x * a.wpb;
  const uint32_t t = threadIdx.x, lane = t & 63;
  if (t < 64) {
    const uint64_t w = w0 + lane;
    const uint32_t c = lane < a.wpb && w < a.n_waves ? (uint32_t)min(a.wave_total[w] & ~(1ull << 63), a.wcap) : 0u;
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= (uint32_t)d) x += y;
    }
    s_pre[lane + 1] = x;
    if (lane == 0) s_pre[0] = 0;
  }
  __syncthreads();
  return s_pre[a.wpb];
}
__device__ __forceinline__ uint64_t slot_of(const ShapeArgs& a, const uint32_t* s_pre, uint32_t i) {
  uint32_t v = 0;  // the largest v < wpb with s_pre[v] <= i
  for (uint32_t st = BW_MAX / 2; st; st >>= 1)
    if (v + st < a.wpb && s_pre[v + st] <= i) v += st;
  return ((uint64_t)blockIdx.x * a.wpb + v) * a.wcap + (i - s_pre[v]);
}

// Core nodes of the current round: the start node, or a node some node of
// the previous round links to (has_child[g] == gen), whose own parent was
// found (a record or the root rule).  Round 1's marks come from the link
// phase's claims (every node with a found parent); each prune round keeps
// only the parents of the previous round's core nodes, so a false chain of L
// candidates (a false node whose "prev" happens to be another false node's
// tail) drops out after L rounds, while an intact chain from the start node
// stays core throughout.  The retry kernels run over every slot: a slot
// without a record is never core (no claim or mark of this generation
// reaches it -- parents are records), so its stale words are never used.
__device__ __forceinline__ bool is_core(const ShapeArgs& a, uint64_t g, uint64_t start) {
  if (g == start) return true;
  const int64_t p = a.d_par[g];
  return a.has_child[g] == a.gen && (p >= 0 || p == PAR_ROOT);
}

// the retry's round-0 marks: the nodes the link phase's claims were made on
__global__ __launch_bounds__(256) void marks_from_claims_kernel(ShapeArgs a, uint32_t* marks_out) {
  if (dense_incomplete(a)) return;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < a.n_slots; g += (uint64_t)gridDim.x * blockDim.x)
    if ((a.childof[g] >> 32) == a.gen) marks_out[g] = a.gen;
}

__global__ __launch_bounds__(256) void prune_kernel(ShapeArgs a, uint32_t* marks_out, uint32_t gen_out) {
  if (dense_incomplete(a)) return;
  const uint64_t start = start_node(a);
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < a.n_slots; g += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t p = a.d_par[g];
    if (p >= 0 && is_core(a, g, start)) marks_out[p] = gen_out;
  }
}

__global__ __launch_bounds__(256) void child2_kernel(ShapeArgs a) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n_zero; i += gridDim.x * blockDim.x) a.zero[i] = 0;
  if (dense_incomplete(a)) return;
  const uint64_t start = start_node(a);
  const uint64_t K = a.n_slots;
  // CR nodes per thread per pass: loads first (no store in between)
  constexpr int CR = 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g0 < K; g0 += CR * stride) {
    int64_t par[CR];
    uint32_t hc[CR];
#pragma unroll
    for (int r = 0; r < CR; r++) {
      const uint64_t g = g0 + r * stride, gg = g < K ? g : g0;
      par[r] = a.d_par[gg];
      hc[r] = a.has_child[gg];
    }
#pragma unroll
    for (int r = 0; r < CR; r++) {
      const uint64_t g = g0 + r * stride;
      if (g >= K) break;
      const int64_t p = par[r];
      if (p >= 0 && (g == start || hc[r] == a.gen)) a.childof[p] = claim_word(a.gen, g);  // is_core(g)
    }
  }
}

// The core nodes (the start node, and every node something links to whose own
// parent was found) must form ONE chain from the start down to one root:
//   (1) a core node's parent is a core node (else: dangling),
//   (2) it holds the claim on its parent (else: another node claims it -- a
//       branch, or a leaf that won the claim: the retry rounds decide),
//   (3) exactly one core node links to a root (nroot, chain_finalize).
// Then following parents from any core node ends at that root, and no node
// has two core children: the core set is a single path, and its top is the
// start node (no node lies above file_len - 20), so every core node but the
// start has a core child without a test of its own.  Leaves (false
// candidates nobody links to) are ignored -- recover_valid_chain's walk only
// follows back-pointers from file_len (data_store.rs:404-470).  Round 0
// reads the link phase's claims (core: (childof[g] >> 32) == gen); the retry
// rounds, the prune marks and child2's core-only claims.
__global__ __launch_bounds__(CHAIN_THREADS) void check_kernel(ShapeArgs a) {
  __shared__ uint32_t wsum[CHAIN_WAVES];
  __shared__ uint32_t s_pre[BW_MAX + 1];
  if (dense_incomplete(a)) return;
  const uint64_t start = start_node(a);
  const uint64_t tag = (uint64_t)a.gen << 32;
  const bool marks = a.has_child != nullptr;  // retry rounds
  const uint32_t n = block_waves(a, s_pre);
  uint32_t cnt = 0;
  bool fail = false;
  // wave chunks: wave wi takes the block's records [c0, c1) (chain_finalize
  // ranks them with the same chunks and the per-chunk counts, no barriers);
  // CR records per lane per pass, their loads issued level by level: the
  // node's own words (parent, claim), then its parent's
  const uint32_t wi = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t chunk = (n + CHAIN_WAVES - 1) / CHAIN_WAVES;
  const uint32_t c0 = min(n, wi * chunk), c1 = min(n, c0 + chunk);
  constexpr int CR = 4;
  for (uint32_t base = c0; base < c1; base += CR * 64) {
    uint64_t g[CR], cg[CR], cp[CR];
    int64_t par[CR], pp[CR];
    uint32_t hc[CR], hp[CR];
    bool in[CR];
#pragma unroll
    for (int r = 0; r < CR; r++) {
      const uint32_t i = base + (uint32_t)r * 64 + lane;
      in[r] = i < c1;
      g[r] = slot_of(a, s_pre, in[r] ? i : c0);
      par[r] = a.d_par[g[r]];
      cg[r] = a.childof[g[r]];
      hc[r] = marks ? a.has_child[g[r]] : 0u;
    }
#pragma unroll
    for (int r = 0; r < CR; r++) {
      const uint64_t q = par[r] >= 0 ? (uint64_t)par[r] : g[r];
      pp[r] = a.d_par[q];
      cp[r] = a.childof[q];
      hp[r] = marks ? a.has_child[q] : 0u;
    }
#pragma unroll
    for (int r = 0; r < CR; r++) {
      if (!in[r]) break;
      const int64_t p = par[r];
      const bool linked = marks ? hc[r] == a.gen : (cg[r] & ~0xffffffffull) == tag;
      const bool core = g[r] == start || (linked && (p >= 0 || p == PAR_ROOT));  // is_core(g)
      GST(a.flag[g[r]], (uint8_t)core);
      if (!core) continue;
      cnt++;
      const bool plinked = marks ? hp[r] == a.gen : (cp[r] & ~0xffffffffull) == tag;
      if (p == PAR_ROOT) {
        atomicAdd(&a.plan->nroot, 1u);
        const u32x4 r0 = a.c_rec[g[r]];
        a.plan->root_t = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);
      } else if (p < 0 || !((uint64_t)p == start || (plinked && (pp[r] >= 0 || pp[r] == PAR_ROOT)))) {
        fail = true;  // dangling: the chain through g is broken (only the start node can get here)
      } else if (cp[r] != claim_word(a.gen, g[r])) {
        fail = true;  // branch: another node holds the claim on the same parent
      }
    }
  }
  {
    uint32_t wc = cnt;
#pragma unroll
    for (int o = 32; o; o >>= 1) wc += __shfl_xor(wc, o);
    if (lane == 0) a.wpart[blockIdx.x * CHAIN_WAVES + wi] = wc;
  }
  const uint32_t tot = block_sum_n<CHAIN_WAVES>(cnt, wsum);
  if (__syncthreads_or(fail) && threadIdx.x == 0) atomicOr(&a.plan->status, ST_SHAPE);
  if (threadIdx.x == 0) a.part[blockIdx.x] = tot;
}

// KeyIndexer::build's bucket layout (shared with chain_finalize_kernel, which
// builds the histogram, claims the bucket ranges and scatters its chain
// positions itself)
constexpr int IDX_HBLOCKS = 256;  // histogram / scatter blocks of the stand-alone build
constexpr int IDX_TCAP = 2048;       // max entries per bucket (load <= 1/2)
// the host picks the fewest buckets with <= IDX_BUCKET_AVG expected entries
// each (fewer buckets, fewer range claims; a bucket of Poisson(1280) stays far
// below IDX_TCAP, and an overflowing one sends the build to the global table)
constexpr int IDX_BUCKET_AVG = 1280;
constexpr uint64_t IDX_EMPTY = ~0ull;
constexpr int PUB_WORDS = 7;  // flags, n_chain, n_index, n_bad, K, top_gap, the scan's ticks (XPart; 0: none)

struct IdxArgs {
  const uint64_t* kh;    // chain key hashes (o_kh)
  const uint64_t* mo;    // chain meta offsets (o_mo)
  const uint64_t* n_dev; // &plan->n_chain
  const uint32_t* status;
  uint32_t log2_nbk;
  // Buckets of fixed capacity IDX_TCAP: bucket k owns srec[k*IDX_TCAP, ...).
  // Each block claims a range per bucket with one atomicAdd on bfill[k] (no
  // histogram scan).  bfill (nbk) is zero before the claims.
  uint32_t* bfill;
  uint64_t* srec;        // idx_rec(key, chain index) per entry, in its bucket's range
  uint8_t* latest;       // [n] == lgen: NOT the latest entry of its key (idx_dedup writes only those)
  uint8_t lgen;          // this build's generation (1..255; the host clears the array on wrap)
  uint32_t alias;        // fused pass: with no non-latest entry idx_emit writes nothing (Plan::idx_alias)
  // fused pass: idx_emit's block 0 publishes the call's outcome straight to
  // pinned host memory (PUB_WORDS words, each (seq << 32) | value) as soon
  // as it starts -- the host reads it there instead of waiting for the plan
  // copy and the stream's completion signal
  uint64_t* pub;
  uint32_t pub_seq;
  uint32_t* ccount;      // [GLUE_BLOCKS] NON-latest entries per chain chunk (idx_dedup -> idx_emit; zero before)
  const uint64_t* scan_ticks;  // nullable: XPart::scan_ticks of this call's scan (published)
  uint64_t* okey;
  uint64_t* opacked;
  Plan* plan;
};

__device__ __forceinline__ uint64_t idx_n(const IdxArgs& a) { return *a.status ? 0 : *a.n_dev; }

// ---------------------------------------------------------------------------
// The plan (every block decides it from the same inputs; block 0 publishes
// it) fused with the whole per-entry stage: chain rank of every core node
// (block prefix of check_kernel's per-chunk core counts + a block rank), the
// outputs and the CRC of each chain entry (finalize_core), the entries whose
// CRC needs a wave (long entries, missing pieces: slow_one, run by this
// block's 16 waves after each round), and the index histogram and scatter
// of the bucketed KeyIndexer::build over this block's chain positions.
// Replaces the plan/scatter, finalize, slow, histogram and scatter launches.
template <int NW>
__device__ __forceinline__ void block_prefix_n(const uint32_t* part, uint32_t np, uint32_t* wsum, uint64_t* before,
                                               uint64_t* total) {
  uint32_t b = 0, t = 0;
  for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
    const uint32_t v = part[i];
    t += v;
    b += i < blockIdx.x ? v : 0u;
  }
  *before = block_sum_n<NW>(b, wsum);
  *total = block_sum_n<NW>(t, wsum);
}

__device__ __forceinline__ uint32_t idx_bucket(uint64_t key, uint32_t log2_nbk) {
  return (uint32_t)(xxh3_64_u64(key) >> (64 - log2_nbk));
}
// A bucket record in 8 bytes: the chain index in the high word, the low word
// of the key's Xxh3BuildHasher hash (xxh3_64_u64, key_indexer.rs:98-124 hashes
// with it; its top bits are the bucket) in the low word.  idx_dedup
// deduplicates by that 32-bit partial key and checks every entry that loses to
// another one against the full key_hash (the chain's key array): a partial
// match of two different keys is detected there and the bucket is redone with
// the full keys.  16-byte (key, index) records wrote and read 8 bytes more per
// entry.
__device__ __forceinline__ uint64_t idx_rec(uint64_t hh, uint64_t c) { return (c << 32) | (uint32_t)hh; }

// block ranks of R rounds of flags at once (one LDS exchange): round r's
// flags rank after every flag of rounds < r; wsum is LDS[R * NW]
template <int NW, int R>
__device__ __forceinline__ uint32_t block_rank_rounds(const bool* f, uint32_t* wsum, uint32_t* rank) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t pre[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint64_t bal = __ballot(f[r]);
    pre[r] = (uint32_t)__popcll(bal & lt);
    if (lane == 0) wsum[r * NW + w] = (uint32_t)__popcll(bal);
  }
  __syncthreads();
  uint32_t acc = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    uint32_t off = 0, t = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      const uint32_t v = wsum[r * NW + i];
      off += i < w ? v : 0u;
      t += v;
    }
    rank[r] = acc + off + pre[r];
    acc += t;
  }
  __syncthreads();
  return acc;
}

// chain entries per thread per pass of chain_finalize_kernel: the per-entry
// work is a chain of four dependent loads (flag -> parent/slot -> records ->
// parent record, tile values, table words); the R entries' loads of each level
// are issued together
#ifndef SRD_FIN_R
#define SRD_FIN_R 2
#endif
constexpr int FIN_R = SRD_FIN_R;
constexpr uint32_t WSLOW = 256;  // per-wave slow-entry queue (LDS) of chain_finalize_kernel

// one chain entry's inputs (finalize_core's, loaded level by level)
struct FinIn {
  uint64_t mo, p;
  uint32_t crc_st, fl, sxv;   // record: r1[0], r1[3], r1[1]
  uint32_t pfl, psuf;         // parent record: r1[3], r1[2] (pfl = 3 << F_SUF_SHIFT: no parent record)
  u32x4 t0, t1;               // per-tile values of the start tile k0 and the metadata tile k1
};
// the tables finalize_in reads, in LDS
struct FinLds {
  uint32_t tab[1024];         // CRC slice-by-4
  uint32_t m16k[1024];        // v -> v * x^16384
  uint32_t m32k[1024];        // v -> v * x^32768 (a tile step)
  uint32_t mtk[3 * 1024];     // v -> v * x^(32768 (j + 2)), j = 0..2 (2-4 tile steps)
  uint32_t winit[64], zero_crc[64];
  uint32_t invpow[4097];
};

__device__ __forceinline__ uint32_t mul16k_lds(const uint32_t* m16k, uint32_t v) {
  return m16k[v & 0xff] ^ m16k[256 + ((v >> 8) & 0xff)] ^ m16k[512 + ((v >> 16) & 0xff)] ^ m16k[768 + (v >> 24)];
}

// crc_raw of bytes [floor64(m), m) (tail_crc_line) with the CRC table in LDS
__device__ __forceinline__ uint32_t tail_crc_lds(const uint8_t* file, uint64_t m, const uint32_t* tab) {
  return tail_crc_line(file, m, [tab](int t, uint32_t b) { return tab[256 * t + b]; });
}

// finalize_core (srd_kernels.hip) for a candidate chain entry from its
// preloaded inputs: the same outputs, bit for bit; true = slow_one needed
__device__ __forceinline__ bool finalize_in(const FinArgs& a, uint64_t c, const FinIn& e, const FinLds& t) {
  const uint32_t* m16k = t.m16k;
  const uint64_t mo = e.mo, p = e.p;
  const uint32_t fl = e.fl;
  const bool tomb = fl & F_TOMB;
  const uint64_t start = tomb ? p : p + prepad64(p);
  const uint64_t k0 = start / TILE, k1 = mo / TILE;
  uint32_t suf = 0, sxm = 0, tail = 0, pieces = 0;
  if (fl & F_SXM) {
    sxm = (fl & F_SXM_LO) ? mul16k_lds(m16k, e.sxv) ^ e.t1[2] : e.sxv;
    pieces |= 2;
  }
  if (fl & F_TAIL) pieces |= 4;
  const uint32_t kind = (e.pfl >> F_SUF_SHIFT) & 3;
  if (kind == 0) { suf = (e.pfl & F_SUF_LO) ? mul16k_lds(m16k, e.psuf) ^ e.t0[2] : e.psuf; pieces |= 1; }
  else if (kind == 1) { suf = mul16k_lds(m16k, e.t0[0]) ^ e.t0[2]; pieces |= 1; }
  else if (kind == 2) { suf = mul16k_lds(m16k, e.t0[1]) ^ e.t0[2]; pieces |= 1; }
  if (!(pieces & 1)) {  // the start line's suffix from the per-tile values (line 0, 1 or 32)
    const uint32_t j = (uint32_t)((start % TILE) / 64);
    if (j == 0) { suf = mul16k_lds(m16k, e.t0[0]) ^ e.t0[2]; pieces |= 1; }
    else if (j == 1) { suf = mul16k_lds(m16k, e.t0[1]) ^ e.t0[2]; pieces |= 1; }
    else if (j == 32) { suf = e.t0[2]; pieces |= 1; }
  }
  if (!(pieces & 2)) {
    const uint32_t j = (uint32_t)((mo % TILE) / 64);
    if (j == 0) { sxm = mul16k_lds(m16k, e.t1[0]) ^ e.t1[2]; pieces |= 2; }
    else if (j == 1) { sxm = mul16k_lds(m16k, e.t1[1]) ^ e.t1[2]; pieces |= 2; }
    else if (j == 32) { sxm = e.t1[2]; pieces |= 2; }
  }
  const uint64_t len = mo - start;
  GST(a.o_start[c], start);  // o_mo / o_kh / o_prev / o_crc_st: stored by the caller
  GST(a.o_len[c], len);
  if (a.no_crc) { a.o_crc[c] = 0; a.o_ok[c] = 0; return false; }
  uint32_t crc;
  if (tomb) {
    crc = 0xD202EF8Du;  // CRC32(b"\0"): the tombstone byte is 0 by the rule
  } else {
    if (!(pieces & 4)) tail = tail_crc_lds(a.file, mo, t.tab);
    const bool need_long = len >= 64;
    const bool many_tiles = need_long && k1 > k0 + 1 + LONG_TILES;
    if (need_long && !((pieces & 1) && (pieces & 2) && !many_tiles)) {
      a.o_pieces[c] = pieces;
      a.o_suf[c] = suf;
      a.o_sxm[c] = sxm;
      a.o_tail[c] = tail;
      return true;
    }
    if (!need_long) {
      crc = tail ^ t.zero_crc[len];
    } else {  // crc_from_pieces
      uint32_t acc = suf ^ t.winit[(start % TILE) / 64], y;
      if (k0 == k1) {
        y = acc ^ sxm;
      } else {
        // the whole tiles 4 at a time (their values loaded together): acc =
        // acc * X^r ^ T_0 X^(r-1) ^ ... ^ T_(r-1) for the group's r <= 4
        // tiles (X = x^32768, tile_T(k) = mul16k(T_lo) ^ SX_32), so the
        // dependent chain is one table multiply per 4 tiles, not per tile
        // (the same 32 lookups per 4 tiles; C3's 2-16-tile entries)
        const u32x4* t4 = (const u32x4*)a.tile;
        for (uint64_t kb = k0 + 1; kb < k1; kb += 4) {
          u32x4 tv[4];
#pragma unroll
          for (int q = 0; q < 4; q++) tv[q] = t4[kb + q < k1 ? kb + q : k1];
          const uint32_t r = (uint32_t)min<uint64_t>(k1 - kb, 4);
          uint32_t T[4];
#pragma unroll
          for (int q = 0; q < 4; q++) T[q] = mul16k_lds(m16k, tv[q][0]) ^ tv[q][2];
          // X^j tables: j = 1 m32k, j = 2..4 mtk[j - 2]
          auto xt = [&](uint32_t j) -> const uint32_t* { return j == 1 ? t.m32k : t.mtk + 1024 * (j - 2); };
          uint32_t v = mul16k_lds(xt(r), acc) ^ T[r - 1];
          if (r >= 2) v ^= mul16k_lds(t.m32k, T[r - 2]);
          if (r >= 3) v ^= mul16k_lds(t.mtk, T[r - 3]);
          if (r >= 4) v ^= mul16k_lds(t.mtk + 1024, T[0]);
          acc = v;
        }
        y = mul16k_lds(t.m32k, acc) ^ (mul16k_lds(m16k, e.t1[0]) ^ e.t1[2]) ^ sxm;
      }
      crc = ~(mulp(t.invpow[(k1 + 1) * TILE - mo], y) ^ tail);
    }
  }
  GST(a.o_crc[c], crc);
  GST(a.o_ok[c], (uint8_t)(crc == e.crc_st));
  if (crc != e.crc_st) atomicAdd(a.n_bad, 1ull);
  return false;
}

// ---- the fused shape check (FUSED chain_finalize_kernel, round 0) ----
// Each chain block checks its own records (check_kernel's test), then learns
// the core records of the blocks before it by a decoupled look-back over one
// 8-byte granule per block: {tag = 24 bits of the call generation (never 0),
// state (1 = the block's own aggregate, 2 = its inclusive prefix), the shape
// failure bit, the root-linked core nodes (saturating at 3), the core count}.
// The data is the flag (the cdna guide's Guideline 16, form R2): relaxed
// agent-scope atomic stores and loads, no fence, no per-call memset (a stale
// granule carries another call's tag).  A block only waits for LOWER blocks,
// dispatched before it, so the grid cannot deadlock; a bounded spin that runs
// out publishes state 3 (a POISONED inclusive prefix): every later block's
// look-back stops there and fails too, so the plan (the last block) carries
// ST_LOOKBACK and the host takes the full pass -- a timed-out block never
// passes a partial prefix on as if it were complete (ShapeArgs::lb_fail forces
// the timeout in one block: tests/test_gpu_parity.py::test_lookback_fallback).
constexpr uint32_t ST_LOOKBACK = 32;
#ifdef SRD_GLUE_STAMPS  // timing-only build (tools/glue_stamps.py): per-block phase ends of chain_finalize<true>
__device__ uint64_t g_glue_stamp[CHAIN_BLOCKS * 8];
#define GLUE_STAMP(i) \
  do { if (FUSED && threadIdx.x == 0) g_glue_stamp[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define GLUE_STAMP(i) do {} while (0)
#endif
constexpr uint64_t LB_CNT = (1ull << 35) - 1;
__device__ __forceinline__ uint64_t lb_pack(uint32_t tag, uint32_t st, bool fail, uint32_t nr, uint64_t cnt) {
  return ((uint64_t)tag << 40) | ((uint64_t)st << 38) | ((uint64_t)fail << 37) | ((uint64_t)min(nr, 3u) << 35) |
         (cnt & LB_CNT);
}
__device__ __forceinline__ uint32_t lb_tag(uint32_t gen) { return gen % 0xFFFFFFu + 1u; }
// wave 0 of block b: the exclusive prefix of blocks [0, b) -- core count,
// failure, root-linked nodes; false when the spin bound ran out or the
// inclusive prefix it stops at is poisoned (state 3: a lower block timed out)
__device__ bool lb_lookback(unsigned long long* desc, uint32_t b, uint32_t tag, uint64_t* cnt, bool* fail,
                            uint32_t* nr) {
  typedef __attribute__((address_space(1))) unsigned long long gu64;
  const uint32_t lane = threadIdx.x & 63;
  uint64_t sum = 0;
  bool f = false;
  uint32_t n = 0;
  uint32_t spins = 0;
  for (int64_t j = (int64_t)b - 1; j >= 0; j -= 64) {
    const int64_t idx = j - (int64_t)lane;
    uint64_t v;
    for (;;) {  // until every lane's granule carries this call's tag (lanes past block 0: a zero prefix)
      v = idx >= 0 ? __hip_atomic_load((gu64*)(desc + idx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : lb_pack(tag, 2, false, 0, 0);
      const bool ok = (v >> 40) == tag && ((v >> 38) & 3) != 0;
      if (__all(ok)) break;
      if (++spins > (1u << 22)) return false;  // uniform
      __builtin_amdgcn_s_sleep(2);
    }
    const uint32_t stv = (uint32_t)(v >> 38) & 3u;
    const uint64_t inc = __ballot(stv >= 2);
    const uint32_t first = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
    const bool take = lane <= first;
    if (__ballot(take && stv == 3)) return false;  // (uniform) a poisoned prefix
    uint64_t c = take ? (v & LB_CNT) : 0;
    uint32_t r = take ? (uint32_t)((v >> 35) & 3) : 0u;
    uint32_t fl = take ? (uint32_t)((v >> 37) & 1) : 0u;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
      c += __shfl_xor(c, o);
      r += __shfl_xor(r, o);
      fl |= __shfl_xor(fl, o);
    }
    sum += c;
    n += r;
    f = f || fl;
    if (inc) break;
  }
  *cnt = sum;
  *fail = f;
  *nr = n;
  return true;
}

// the previous lane's value (DPP wave_shr:1), lane 0 taking `lane0` (the
// previous pass's lane 63): record i's neighbour i - 1 in a pass of 64
__device__ __forceinline__ uint32_t prev_lane(uint32_t v, uint32_t lane0) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, DPP_WAVE_SHR1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t prev_lane64(uint64_t v, uint64_t lane0) {
  return (uint64_t)prev_lane((uint32_t)v, (uint32_t)lane0) | ((uint64_t)prev_lane((uint32_t)(v >> 32), (uint32_t)(lane0 >> 32)) << 32);
}
__device__ __forceinline__ uint64_t lane63_64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, 63) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), 63) << 32);
}

// FUSED (round 0 of the optimistic pass): check_kernel's shape test of the
// block's own records first, the chain ranks from the look-back instead of
// check_kernel's per-block totals, the plan written by the LAST block once
// its prefix holds every block -- one launch and one pass over the slot
// words fewer.  The retry rounds (prune marks) keep check_kernel + !FUSED.
template <bool FUSED>
__global__ __launch_bounds__(CHAIN_THREADS) void chain_finalize_kernel(ShapeArgs a, FinArgs f, IdxArgs ia,
                                                                      uint32_t log2_nbk,
                                                                      unsigned long long* lb_desc) {
  __shared__ uint32_t wsum[CHAIN_WAVES * FIN_R];
  __shared__ uint32_t s_pre[BW_MAX + 1];
  __shared__ uint32_t wslow[CHAIN_WAVES][WSLOW];
  __shared__ FinLds lt;
  uint32_t* const tab = lt.tab;
  extern __shared__ uint32_t hist[];
  // the LDS tables' words first, into registers: their loads overlap the
  // plan's dependent ones below (one round trip instead of a load -> store
  // loop after the plan)
  static_assert(CHAIN_THREADS == 1024, "one word of each 1024-word table per thread");
  GLUE_STAMP(0);
  const uint32_t ti = threadIdx.x;
  const uint32_t r_tab = g_tabs.tab[ti >> 8][ti & 255],
                 r_m16k = (&g_tabs.m16k[0][0])[ti], r_m32k = (&g_tabs.m32k[0][0])[ti];
  uint32_t r_mtk[3];
#pragma unroll
  for (int j = 0; j < 3; j++) r_mtk[j] = (&g_tabs.mtk[j][0][0])[ti];
  uint32_t r_inv[4];
#pragma unroll
  for (int j = 0; j < 4; j++) r_inv[j] = g_tabs.invpow[ti + 1024 * j];
  const uint32_t r_inv_last = g_tabs.invpow[4096];
  const uint32_t r_winit = g_tabs.winit[ti & 63], r_zc = g_tabs.zero_crc[ti & 63];
  const uint64_t K = a.Kp[0];
  const bool incomplete = dense_incomplete(a);
  uint64_t before = 0, total = 0;
  if constexpr (!FUSED)
    block_prefix_n<CHAIN_WAVES>(a.part, incomplete ? 0u : (uint32_t)CHAIN_BLOCKS, wsum, &before, &total);
  Plan* pl = a.plan;
  uint32_t st = FUSED ? 0u : pl->status;  // check_kernel's shape bits (FUSED: this kernel's own, below)
  // whole file only: the start tail is itself a root tail (prev 0): one
  // entry spans [0, t) (recover_valid_chain's walk ends at once)
  const uint64_t top = a.counters[1];
  // (the prev field at top - 12 by two aligned dword pairs: the buffer is
  // padded past file_len)
  auto ld_prev_at = [&](uint64_t o) -> uint64_t {
    const uint32_t* q = (const uint32_t*)(a.file + (o & ~3ull));
    const uint32_t sh = (uint32_t)(o & 3) * 8, w0 = q[0], w1 = q[1], w2 = q[2];
    return (uint64_t)alignb(w1, w0, sh) | ((uint64_t)alignb(w2, w1, sh) << 32);
  };
  const bool troot = a.coff && top >= 21 && ld_prev_at(top - 12) == 0;
  uint64_t root_t = troot ? top : FUSED ? 0 : pl->root_t;
  if (a.counters[2]) st |= ST_OVERFLOW;
  // the start node: !FUSED now; FUSED lazily -- it can only be the last
  // record (slot s1 - 1), so the shape check tests g == s1 - 1 and reads
  // that record's c_m only there, and the last block settles ST_NOSTART /
  // ST_OVERFLOW with the plan (the other blocks' work is discarded then)
  const uint64_t s1 = a.Kp[1];
  const uint64_t start = FUSED ? NO_NODE : incomplete ? NO_NODE : start_node(a);
  if (!FUSED && start == NO_NODE) st |= ST_NOSTART;
  if (!FUSED && pl->nroot != 1) st |= ST_ROOTS;
  if (FUSED) st = 0;  // (settled by the last block)
  if (!FUSED) __syncthreads();  // this block has read pl->status / nroot / root_t before block 0 rewrites them
  const uint32_t nbk = 1u << log2_nbk;
  // the plan: !FUSED block 0 now; FUSED the last block, once the look-back
  // has every block's count (or now, when the counters alone decide)
  auto write_plan = [&](uint32_t s2, uint64_t tot) {
    pl->K = K;
    pl->max_root = a.counters[0];
    pl->top_gap = top ? a.flen - top : 0;
    pl->overflow = a.counters[2];
    pl->troot = troot;
    if (troot) {  // the start tail is itself a root tail: chain = that one entry
      pl->status = 0;
      pl->n_chain = 1;
      pl->root_t = top;
      pl->chain_core = 0;
    } else {
      if (!FUSED) pl->start = start;
      pl->status = s2;
      pl->chain_core = tot;
      pl->n_chain = s2 ? 0 : a.coff + tot;
    }
  };
  const bool plan_block = FUSED ? blockIdx.x + 1 == gridDim.x : blockIdx.x == 0;
  if (!FUSED && plan_block && threadIdx.x == 0) write_plan(st, total);
  if (FUSED && troot && plan_block && threadIdx.x == 0) write_plan(0, 0);
  if (st && !troot) return;
  // FUSED: the shape check of this block's records (check_kernel, round 0),
  // then the look-back; per-wave core counts in LDS
  __shared__ uint32_t s_vcnt[BW_MAX];  // FUSED: core records per scan wave of the block
  __shared__ uint64_t s_lb[2];
  __shared__ uint32_t s_fail, s_nroot, s_lbok;
  __shared__ unsigned long long s_root_t;
  if constexpr (FUSED) {
    if (!troot) {
      if (threadIdx.x == 0) { s_fail = 0; s_nroot = 0; s_root_t = 0; }
      __syncthreads();
      const uint64_t tag = (uint64_t)a.gen << 32;
      const uint32_t wi = threadIdx.x >> 6, lane = threadIdx.x & 63;
      // chain wave wi takes the block's scan waves wi, wi + 16, ... whole:
      // record r of scan wave w is slot w * wcap + r, so no slot map (the
      // waves' record counts differ by the scan's wave shares, ~ +-15 %).
      // The parent of a record is almost always the previous record (slot g
      // - 1): its words come from the neighbour lane (prev_lane), not a load
      uint32_t nr = 0;
      bool fail = false;
      constexpr int CR = 4;
      for (uint32_t v = wi; v < a.wpb; v += CHAIN_WAVES) {
        const uint64_t w = (uint64_t)blockIdx.x * a.wpb + v;
        const uint32_t n = w < a.n_waves ? (uint32_t)min(a.wave_total[w] & ~(1ull << 63), a.wcap) : 0u;
        const uint64_t gb = w * a.wcap;
        int64_t c_par = PAR_MISS;  // the previous pass's lane-63 words
        uint64_t c_cg = 0;
        uint32_t cnt = 0;
        for (uint32_t base = 0; base < n; base += CR * 64) {
          uint64_t g[CR], cg[CR], cp[CR];
          int64_t par[CR], pp[CR];
          bool in[CR], need[CR];
#pragma unroll
          for (int r = 0; r < CR; r++) {
            const uint32_t i = base + (uint32_t)r * 64 + lane;
            in[r] = i < n;
            g[r] = gb + (in[r] ? i : 0u);
            par[r] = a.d_par[g[r]];
            cg[r] = a.childof[g[r]];
          }
          bool any = false;
#pragma unroll
          for (int r = 0; r < CR; r++) {
            const uint32_t i = base + (uint32_t)r * 64 + lane;
            const int64_t l0p = r ? (int64_t)(int32_t)__builtin_amdgcn_readlane((uint32_t)par[r - 1], 63) : c_par;
            const uint64_t l0c = r ? lane63_64(cg[r - 1]) : c_cg;
            pp[r] = (int64_t)(int32_t)prev_lane((uint32_t)par[r], (uint32_t)l0p);
            cp[r] = prev_lane64(cg[r], l0c);
            need[r] = in[r] && par[r] >= 0 && !(i > 0 && (uint64_t)par[r] == g[r] - 1);
            any = any || need[r];
          }
          if (__ballot(any)) {  // (uniform) a parent elsewhere: its words by a load
#pragma unroll
            for (int r = 0; r < CR; r++)
              if (need[r]) {
                pp[r] = a.d_par[par[r]];
                cp[r] = a.childof[par[r]];
              }
          }
          c_par = (int64_t)(int32_t)__builtin_amdgcn_readlane((uint32_t)par[CR - 1], 63);
          c_cg = lane63_64(cg[CR - 1]);
#pragma unroll
          for (int r = 0; r < CR; r++) {
            if (!in[r]) break;
            const int64_t p = par[r];
            const bool linked = (cg[r] & ~0xffffffffull) == tag;
            // g == the start node: the last record, at the start tail's metadata
            const bool is_st = s1 && g[r] == s1 - 1 && top >= 21 && a.c_m[g[r]] == top - 20;
            const bool core = is_st || (linked && (p >= 0 || p == PAR_ROOT));  // is_core(g)
            GST(a.flag[g[r]], (uint8_t)core);
            if (!core) continue;
            cnt++;
            const bool plinked = (cp[r] & ~0xffffffffull) == tag;
            if (p == PAR_ROOT) {
              nr++;
              const u32x4 r0 = a.c_rec[g[r]];
              s_root_t = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);  // (any one: nroot != 1 fails the call)
            } else if (p < 0 || !(((uint64_t)p == s1 - 1 && a.c_m[p] == top - 20) ||
                                  (plinked && (pp[r] >= 0 || pp[r] == PAR_ROOT)))) {
              fail = true;  // dangling (a parent that is the start node is core: never here in practice)
            } else if (cp[r] != claim_word(a.gen, g[r])) {
              fail = true;  // branch
            }
          }
        }
#pragma unroll
        for (int o = 32; o; o >>= 1) cnt += __shfl_xor(cnt, o);
        if (lane == 0) s_vcnt[v] = cnt;
      }
#pragma unroll
      for (int o = 32; o; o >>= 1) nr += __shfl_xor(nr, o);
      if (lane == 0 && nr) atomicAdd(&s_nroot, nr);
      if (__ballot(fail) && lane == 0) s_fail = 1;
      __syncthreads();
      GLUE_STAMP(1);
      // the LDS tables and the bucket counts now: wave 0's look-back below
      // overlaps the other waves' stores (one barrier for both)
      for (uint32_t k = threadIdx.x; k < nbk; k += blockDim.x) hist[k] = 0;
      tab[ti] = r_tab;
      lt.m16k[ti] = r_m16k;
      lt.m32k[ti] = r_m32k;
#pragma unroll
      for (int j = 0; j < 3; j++) lt.mtk[1024 * j + ti] = r_mtk[j];
#pragma unroll
      for (int j = 0; j < 4; j++) lt.invpow[ti + 1024 * j] = r_inv[j];
      if (ti == 0) lt.invpow[4096] = r_inv_last;
      if (ti < 64) {
        lt.winit[ti] = r_winit;
        lt.zero_crc[ti] = r_zc;
      }
      uint32_t btot = 0;
      for (uint32_t v = 0; v < a.wpb; v++) btot += s_vcnt[v];
      const uint32_t ltag = lb_tag(a.gen);
      typedef __attribute__((address_space(1))) unsigned long long gu64;
      if (threadIdx.x == 0 && blockIdx.x > 0)
        __hip_atomic_store((gu64*)(lb_desc + blockIdx.x), lb_pack(ltag, 1, s_fail, s_nroot, btot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (wi == 0) {
        uint64_t pc = 0;
        bool pf = false;
        uint32_t pn = 0;
        const bool ok = blockIdx.x != a.lb_fail && lb_lookback(lb_desc, blockIdx.x, ltag, &pc, &pf, &pn);
        if (lane == 0) {
          const bool f2 = pf || s_fail;
          const uint32_t n2 = pn + s_nroot;
          __hip_atomic_store((gu64*)(lb_desc + blockIdx.x),
                             ok ? lb_pack(ltag, 2, f2, n2, pc + btot) : lb_pack(ltag, 3, true, 0, 0), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          s_lb[0] = pc;
          s_lb[1] = pc + btot;
          s_lbok = ok;
          if (plan_block) {  // every block's count, failure and root links are in the prefix
            const uint64_t stn = incomplete ? NO_NODE : start_node(a);
            pl->start = stn;
            write_plan((ok ? 0u : ST_LOOKBACK) | (f2 ? ST_SHAPE : 0u) | (n2 != 1 ? ST_ROOTS : 0u) |
                           (a.counters[2] ? ST_OVERFLOW : 0u) | (stn == NO_NODE ? ST_NOSTART : 0u),
                       pc + btot);
          }
        }
      }
      __syncthreads();
      GLUE_STAMP(2);
      before = s_lb[0];
      total = s_lb[1];  // (this block's inclusive prefix; the last block's is the total)
      if (!s_lbok) return;
      root_t = s_root_t;
    }
  }
  if (!FUSED || troot) {  // (FUSED: stored beside the look-back above)
    for (uint32_t k = threadIdx.x; k < nbk; k += blockDim.x) hist[k] = 0;
    tab[ti] = r_tab;
    lt.m16k[ti] = r_m16k;
    lt.m32k[ti] = r_m32k;
#pragma unroll
    for (int j = 0; j < 3; j++) lt.mtk[1024 * j + ti] = r_mtk[j];
#pragma unroll
    for (int j = 0; j < 4; j++) lt.invpow[ti + 1024 * j] = r_inv[j];
    if (ti == 0) lt.invpow[4096] = r_inv_last;
    if (ti < 64) {
      lt.winit[ti] = r_winit;
      lt.zero_crc[ti] = r_zc;
    }
    __syncthreads();
  }
  GLUE_STAMP(3);
  // the root entry (whole file: chain entry 0, no candidate record); its
  // CRC's slow path, if any, runs after the candidates
  bool root_slow = false;
  // (FUSED: the block holding the root-linked core node -- it alone knows
  // root_t -- or block 0 for a start tail that is itself a root)
  const bool root_block = FUSED && !troot ? root_t != 0 : blockIdx.x == 0;
  if (root_block && a.coff && threadIdx.x == 0) {
    uint64_t kh;
    root_slow = finalize_core(f, 0, NO_REC, -1, root_t, &kh);
    atomicAdd(&hist[idx_bucket(kh, log2_nbk)], 1u);
  }
  uint64_t bend = a.coff + before;  // the end of this block's chain positions
  if (FUSED && !troot) {
    // the same scan waves per chain wave as the check above; a scan wave's
    // chain positions start at this block's prefix + the core records of the
    // block's earlier scan waves
    const uint32_t wi = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t lt_mask = (1ull << lane) - 1;
    uint32_t btot = 0;
    for (uint32_t v = 0; v < a.wpb; v++) btot += s_vcnt[v];
    bend += btot;
    auto wave_sync = [&]() {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    const u32x4* t4 = (const u32x4*)f.tile;
    for (uint32_t v = wi; v < a.wpb; v += CHAIN_WAVES) {
      const uint64_t w = (uint64_t)blockIdx.x * a.wpb + v;
      const uint32_t n = w < a.n_waves ? (uint32_t)min(a.wave_total[w] & ~(1ull << 63), a.wcap) : 0u;
      const uint64_t gb = w * a.wcap;
      uint32_t voff = 0;
      for (uint32_t u = 0; u < v; u++) voff += s_vcnt[u];
      uint64_t run = a.coff + before + voff;  // this scan wave's next chain position
      const uint64_t run0 = run;
      uint32_t nsq = 0;  // wave-uniform: entries in the wave's slow queue
      auto flush_slow = [&]() {
        if (!nsq) return;
        wave_sync();
        unsigned long long sbase = 0;
        if (lane == 0) sbase = atomicAdd(f.n_slow, (unsigned long long)nsq);
        sbase = __shfl(sbase, 0);
        for (uint32_t q = lane; q < nsq; q += 64) f.slow_list[sbase + q] = run0 + wslow[wi][q];
        wave_sync();
      };
      uint32_t c_fl = 3u << F_SUF_SHIFT, c_suf = 0;  // the previous pass's lane-63 record words
      for (uint32_t base = 0; base < n; base += 64 * FIN_R) {
        bool fl[FIN_R];
        uint64_t gi[FIN_R], kh[FIN_R];
        int64_t par[FIN_R];
        uint32_t psuf[FIN_R];
        FinIn e[FIN_R];
        // level 1: core flag, parent and the record itself, all at the slot
#pragma unroll
        for (int r = 0; r < FIN_R; r++) {
          const uint32_t i = base + (uint32_t)r * 64 + lane;
          gi[r] = gb + (i < n ? i : 0u);
          fl[r] = i < n && a.flag[gi[r]];
          par[r] = a.d_par[gi[r]];
          e[r].mo = f.c_m[gi[r]];
          const u32x4 r0 = f.c_rec[gi[r]], r1 = f.c_rec1[gi[r]];
          e[r].p = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);
          kh[r] = (uint64_t)r1[0] | ((uint64_t)r1[1] << 32);
          e[r].crc_st = r0[3];
          e[r].sxv = r1[2];
          e[r].fl = r0[2];
          psuf[r] = r1[3];
        }
        uint32_t rank[FIN_R], tot = 0;
#pragma unroll
        for (int r = 0; r < FIN_R; r++) {
          const uint64_t b = __ballot(fl[r]);
          rank[r] = tot + (uint32_t)__popcll(b & lt_mask);
          tot += (uint32_t)__popcll(b);
        }
        // level 2: the parent's record words -- the previous record's (the
        // neighbour lane) when it is the parent, else a load -- and the tile
        // values.  A root-linked candidate has no parent record (start 0)
        bool any = false, need[FIN_R];
#pragma unroll
        for (int r = 0; r < FIN_R; r++) {
          const uint32_t i = base + (uint32_t)r * 64 + lane;
          const uint32_t l0f = r ? (uint32_t)__builtin_amdgcn_readlane(e[r - 1].fl, 63) : c_fl;
          const uint32_t l0s = r ? (uint32_t)__builtin_amdgcn_readlane(psuf[r - 1], 63) : c_suf;
          const uint32_t nf = prev_lane(e[r].fl, l0f), ns = prev_lane(psuf[r], l0s);
          need[r] = fl[r] && par[r] >= 0 && !(i > 0 && (uint64_t)par[r] == gi[r] - 1);
          any = any || need[r];
          e[r].pfl = par[r] >= 0 ? nf : (3u << F_SUF_SHIFT);
          e[r].psuf = ns;
          // idle lanes read the last tile's values (resident in span mode too)
          const uint64_t mo = fl[r] ? e[r].mo : f.flen - 1;
          const uint64_t st0 = !fl[r] ? mo : (e[r].fl & F_TOMB) ? e[r].p : e[r].p + prepad64(e[r].p);
          e[r].t0 = t4[st0 / TILE];
          e[r].t1 = t4[mo / TILE];
        }
        if (__ballot(any)) {  // (uniform)
#pragma unroll
          for (int r = 0; r < FIN_R; r++)
            if (need[r]) {
              e[r].pfl = f.c_rec[par[r]][2];
              e[r].psuf = f.c_rec1[par[r]][3];
            }
        }
        c_fl = (uint32_t)__builtin_amdgcn_readlane(e[FIN_R - 1].fl, 63);
        c_suf = (uint32_t)__builtin_amdgcn_readlane(psuf[FIN_R - 1], 63);
        // the record's own outputs and the index histogram while those loads fly
#pragma unroll
        for (int r = 0; r < FIN_R; r++) {
          if (!fl[r]) continue;
          const uint64_t c = run + rank[r];
          GST(f.o_mo[c], e[r].mo);
          GST(f.o_kh[c], kh[r]);
          GST(f.o_packed[c], ((kh[r] >> 48) << 48) | (e[r].mo & 0xFFFFFFFFFFFFull));  // key_indexer.rs:79-85
          GST(f.o_prev[c], e[r].p);
          GST(f.o_crc_st[c], e[r].crc_st);
          atomicAdd(&hist[idx_bucket(kh[r], log2_nbk)], 1u);
        }
#pragma unroll
        for (int r = 0; r < FIN_R; r++) {
          const uint64_t c = run + rank[r];
          const bool slow = fl[r] && finalize_in(f, c, e[r], lt);
          const uint64_t sb = __ballot(slow);
          const uint32_t k = (uint32_t)__popcll(sb);
          if (k) {
            if (nsq + k > WSLOW) {
              flush_slow();
              nsq = 0;
            }
            if (slow) wslow[wi][nsq + __popcll(sb & lt_mask)] = (uint32_t)(c - run0);
            nsq += k;
          }
        }
        run += tot;
      }
      flush_slow();
    }
  } else if (!troot) {
    const uint32_t n = block_waves(a, s_pre);
    // wave chunks as in check_kernel: wave wi ranks its records from its
    // chunk's offset (the per-chunk core counts) with ballots -- the waves
    // never wait for each other inside the loop
    const uint32_t wi = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t lt_mask = (1ull << lane) - 1;
    uint32_t woff, btot;
    {
      const uint32_t v = lane < CHAIN_WAVES ? a.wpart[blockIdx.x * CHAIN_WAVES + lane] : 0u;
      uint32_t x = lane < wi ? v : 0u, y = v;
#pragma unroll
      for (int o = 32; o; o >>= 1) {
        x += __shfl_xor(x, o);
        y += __shfl_xor(y, o);
      }
      woff = x;
      btot = y;
    }
    bend += btot;
    uint64_t run = a.coff + before + woff;  // this wave's next chain position
    const uint64_t run0 = run;
    uint32_t nsq = 0;  // wave-uniform: entries in the wave's slow queue
    // (the queue passes values between lanes through LDS: wavefront fences
    // and a wave barrier order the writers' stores before the reads here and
    // the reads before the slots' reuse, as scan_kernel's window does)
    auto wave_sync = [&]() {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto flush_slow = [&]() {
      if (!nsq) return;
      wave_sync();
      unsigned long long sbase = 0;
      if (lane == 0) sbase = atomicAdd(f.n_slow, (unsigned long long)nsq);
      sbase = __shfl(sbase, 0);
      for (uint32_t q = lane; q < nsq; q += 64) f.slow_list[sbase + q] = run0 + wslow[wi][q];
      wave_sync();
    };
    const uint32_t chunk = (n + CHAIN_WAVES - 1) / CHAIN_WAVES;
    const uint32_t c0 = min(n, wi * chunk), c1 = min(n, c0 + chunk);
    const u32x4* t4 = (const u32x4*)f.tile;
    for (uint32_t base = c0; base < c1; base += 64 * FIN_R) {
      bool fl[FIN_R];
      uint64_t gi[FIN_R], kh[FIN_R];
      int64_t par[FIN_R];
      FinIn e[FIN_R];
      // level 1: core flag, parent and the record itself, all at the record's
      // slot (idle lanes: the chunk's first record)
#pragma unroll
      for (int r = 0; r < FIN_R; r++) {
        const uint32_t i = base + (uint32_t)r * 64 + lane;
        gi[r] = slot_of(a, s_pre, i < c1 ? i : c0);
        fl[r] = i < c1 && a.flag[gi[r]];
        par[r] = a.d_par[gi[r]];
        e[r].mo = f.c_m[gi[r]];
        const u32x4 r0 = f.c_rec[gi[r]], r1 = f.c_rec1[gi[r]];
        e[r].p = (uint64_t)r0[0] | ((uint64_t)r0[1] << 32);
        kh[r] = (uint64_t)r1[0] | ((uint64_t)r1[1] << 32);
        e[r].crc_st = r0[3];
        e[r].sxv = r1[2];
        e[r].fl = r0[2];
      }
      uint32_t rank[FIN_R], tot = 0;
#pragma unroll
      for (int r = 0; r < FIN_R; r++) {
        const uint64_t b = __ballot(fl[r]);
        rank[r] = tot + (uint32_t)__popcll(b & lt_mask);
        tot += (uint32_t)__popcll(b);
      }
      // level 2: the parent's record, the tile values and table words.  k0
      // (the entry's start tile) is resident: start >= p >= the span's lower
      // tail in span mode.  A root-linked candidate (par == PAR_ROOT) has no
      // parent record: its suffix comes from the per-tile values (start 0)
#pragma unroll
      for (int r = 0; r < FIN_R; r++) {
        const uint64_t pg = fl[r] && par[r] >= 0 ? (uint64_t)par[r] : gi[r];
        e[r].pfl = par[r] >= 0 ? f.c_rec[pg][2] : (3u << F_SUF_SHIFT);
        e[r].psuf = f.c_rec1[pg][3];
        // idle lanes read the last tile's values (resident in span mode too)
        const uint64_t mo = fl[r] ? e[r].mo : f.flen - 1;
        const uint64_t st0 = !fl[r] ? mo : (e[r].fl & F_TOMB) ? e[r].p : e[r].p + prepad64(e[r].p);
        e[r].t0 = t4[st0 / TILE];
        e[r].t1 = t4[mo / TILE];
      }
      // the record's own outputs and the index histogram while those loads fly
#pragma unroll
      for (int r = 0; r < FIN_R; r++) {
        if (!fl[r]) continue;
        const uint64_t c = run + rank[r];
        GST(f.o_mo[c], e[r].mo);
        GST(f.o_kh[c], kh[r]);
        GST(f.o_packed[c], ((kh[r] >> 48) << 48) | (e[r].mo & 0xFFFFFFFFFFFFull));  // key_indexer.rs:79-85
        GST(f.o_prev[c], e[r].p);
        GST(f.o_crc_st[c], e[r].crc_st);
        atomicAdd(&hist[idx_bucket(kh[r], log2_nbk)], 1u);
      }
      // entries whose CRC needs a wave go to the call's slow list (idx_dedup's
      // blocks run them, one wave each), gathered in the wave's LDS queue:
      // one list claim per wave and WSLOW entries
#pragma unroll
      for (int r = 0; r < FIN_R; r++) {
        const uint64_t c = run + rank[r];
        const bool slow = fl[r] && finalize_in(f, c, e[r], lt);
        const uint64_t sb = __ballot(slow);
        const uint32_t k = (uint32_t)__popcll(sb);
        if (k) {
          if (nsq + k > WSLOW) {
            flush_slow();
            nsq = 0;
          }
          if (slow) wslow[wi][nsq + __popcll(sb & lt_mask)] = (uint32_t)(c - run0);
          nsq += k;
        }
      }
      run += tot;
    }
    flush_slow();
  }
  if (root_slow) f.slow_list[atomicAdd(f.n_slow, 1ull)] = 0;  // (block 0, thread 0 only)
  __syncthreads();
  GLUE_STAMP(4);
  // KeyIndexer::build's scatter for this block's chain positions [clo, run)
  // (block 0 from 0: the root entry): claim the block's range of every
  // bucket, then one (key, position) record per entry into it; the keys are
  // re-read from o_kh (written above by this block: L2-hot)
  for (uint32_t k = threadIdx.x; k < nbk; k += blockDim.x) {
    const uint32_t n = hist[k];
    hist[k] = n ? atomicAdd(&ia.bfill[k], n) : 0u;
  }
  __syncthreads();
  GLUE_STAMP(5);
  // this block's chain positions [clo, chi) (block 0 from 0: the root entry;
  // FUSED: the root block scatters position 0 on its own below)
  uint64_t clo, chi;
  if constexpr (FUSED) {
    clo = troot ? 0 : a.coff + before;
    chi = troot ? (blockIdx.x == 0 ? 1 : 0) : bend;
    if (!troot && root_block && a.coff && threadIdx.x == 0) {
      const uint64_t h0 = xxh3_64_u64(f.o_kh[0]);
      const uint32_t bk = (uint32_t)(h0 >> (64 - log2_nbk));
      const uint32_t pos = atomicAdd(&hist[bk], 1u);
      if (pos < IDX_TCAP) ia.srec[(uint64_t)bk * IDX_TCAP + pos] = idx_rec(h0, 0);
    }
  } else {
    const uint64_t n_chain = troot ? 1 : a.coff + total;
    clo = min(n_chain, blockIdx.x ? a.coff + before : 0);
    chi = min(n_chain, bend);
  }
  constexpr int SR = 4;  // keys loaded together per pass
  for (uint64_t base = clo; base < chi; base += SR * CHAIN_THREADS) {
    uint64_t k[SR];
#pragma unroll
    for (int r = 0; r < SR; r++) {
      const uint64_t c = base + (uint64_t)r * CHAIN_THREADS + threadIdx.x;
      k[r] = f.o_kh[c < chi ? c : clo];
    }
#pragma unroll
    for (int r = 0; r < SR; r++) {
      const uint64_t c = base + (uint64_t)r * CHAIN_THREADS + threadIdx.x;
      if (c >= chi) break;
      const uint64_t hh = xxh3_64_u64(k[r]);
      const uint32_t bk = (uint32_t)(hh >> (64 - log2_nbk));
      const uint32_t pos = atomicAdd(&hist[bk], 1u);
      if (pos < IDX_TCAP) ia.srec[(uint64_t)bk * IDX_TCAP + pos] = idx_rec(hh, c);  // else: idx_dedup flags the bucket
    }
  }
  GLUE_STAMP(6);
}

// --------------------------------------------------------------------------
// KeyIndexer::build, bucketed
// --------------------------------------------------------------------------
// KeyIndexer::build's bucketing in one launch: each block histograms its chunk in LDS, claims its
// ranges of the buckets (one atomicAdd per bucket) and scatters the chunk --
// no per-(block, bucket) base table in HBM and the keys read once more from
// L2 instead of from a second launch (dedup takes the latest position, so the
// order inside a bucket does not matter)
__global__ __launch_bounds__(256) void idx_hist_scatter_kernel(IdxArgs a) {
  extern __shared__ uint32_t lds_u32[];
  const uint32_t nbk = 1u << a.log2_nbk;
  for (uint32_t k = threadIdx.x; k < nbk; k += blockDim.x) lds_u32[k] = 0;
  __syncthreads();
  uint64_t lo, hi;
  chunk_of(idx_n(a), &lo, &hi);
  for (uint64_t c = lo + threadIdx.x; c < hi; c += blockDim.x)
    atomicAdd(&lds_u32[xxh3_64_u64(a.kh[c]) >> (64 - a.log2_nbk)], 1u);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nbk; k += blockDim.x) {
    const uint32_t n = lds_u32[k];
    lds_u32[k] = n ? atomicAdd(&a.bfill[k], n) : 0u;
  }
  __syncthreads();
  for (uint64_t c = lo + threadIdx.x; c < hi; c += blockDim.x) {
    const uint64_t hh = xxh3_64_u64(a.kh[c]);
    const uint32_t bk = (uint32_t)(hh >> (64 - a.log2_nbk));
    const uint32_t pos = atomicAdd(&lds_u32[bk], 1u);
    if (pos < IDX_TCAP) a.srec[(uint64_t)bk * IDX_TCAP + pos] = idx_rec(hh, c);  // else: idx_dedup flags the bucket
  }
}

// one block per bucket: latest-wins dedup in LDS.  First, the chain entries
// chain_finalize listed for a wave each (long entries, missing CRC pieces;
// f.n_slow == nullptr: none) are spread over all the dedup blocks' waves --
// balanced over the whole grid instead of queued behind their own
// finalize block (C3: ~340K entries of 5-256 tiles)
// The outcome words (PUB_WORDS, each (seq << 32) | value) to pinned host
// memory with system-scope stores; the host accepts them once all carry this
// call's seq
__device__ __forceinline__ void publish_outcome(const IdxArgs& a, const Plan* pl, uint64_t n, uint64_t nl_total) {
  const uint64_t tag = (uint64_t)a.pub_seq << 32;
  const uint32_t fl = (pl->status & 0xffu) | (a.alias && nl_total == 0 ? 0x100u : 0u) | (pl->idx_overflow ? 0x200u : 0u);
  const uint64_t w[PUB_WORDS] = {tag | fl, tag | (uint32_t)pl->n_chain, tag | (uint32_t)(n - nl_total),
                                 tag | (uint32_t)pl->n_bad, tag | (uint32_t)pl->K, tag | (uint32_t)pl->top_gap,
                                 tag | (a.scan_ticks ? (uint32_t)min<uint64_t>(*a.scan_ticks, 0xFFFFFFFFull) : 0u)};
#pragma unroll
  for (int i = 0; i < PUB_WORDS; i++) __hip_atomic_store(a.pub + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The table is sized for 4 blocks per CU (36 KiB of LDS; 512 threads each):
// C2's 1024 buckets then run in one round instead of two.  DD_SLOTS = 1.5 x
// IDX_TCAP, so any bucket that fits its capacity fits the table (load <= 2/3;
// with the bucket count's average fill of 640-1280 entries, <= ~0.45)
constexpr int DD_SLOTS = 3 * IDX_TCAP / 2;
constexpr uint32_t DD_EMPTY32 = 0xFFFFFFFFu;  // an empty partial-key slot (a partial key equal to it is stored as - 1)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) void idx_dedup_kernel(IdxArgs a, FinArgs f) {
  __shared__ unsigned long long dd_lds[DD_SLOTS + DD_SLOTS / 2];
  unsigned long long* const keys = dd_lds;
  uint32_t* const vals = (uint32_t*)(dd_lds + DD_SLOTS);
  __shared__ uint32_t special, collide;
  if (f.n_slow) {
    const unsigned long long ns = *f.n_slow;
    constexpr uint32_t NW = 512 / 64;
    if ((uint64_t)blockIdx.x * NW < ns) {
      static_assert(sizeof(SlowLds) <= sizeof(dd_lds), "the slow path's tables in the hash table's LDS");
      SlowLds& L = *reinterpret_cast<SlowLds*>(dd_lds);  // before the table's own use
      load_slow_lds(L);
      __syncthreads();
      for (uint64_t q = (uint64_t)blockIdx.x * NW + (threadIdx.x >> 6); q < ns; q += (uint64_t)gridDim.x * NW)
        slow_one(f, f.slow_list[q], L);
      __syncthreads();
    }
  }
  if (*a.status) return;
  const uint32_t k = blockIdx.x;
  const uint32_t fill = a.bfill[k];
  if (fill == 0) return;
  if (fill > IDX_TCAP) {  // skewed bucket (entries beyond the capacity were dropped): the host
    if (threadIdx.x == 0) a.plan->idx_overflow = 1;  // reruns the global-table build
    return;
  }
  const uint64_t lo = (uint64_t)k * IDX_TCAP, hi = lo + fill;
  // each thread's <= IDX_TCAP / 512 records (loaded before the table is
  // cleared) and their slots stay in registers between the insert and the
  // lookup pass
  constexpr int DR = IDX_TCAP / 512;
  uint64_t rec[DR];
  uint32_t slot[DR];
  bool in[DR], mark[DR];
#pragma unroll
  for (int r = 0; r < DR; r++) {
    const uint64_t i = lo + (uint64_t)r * 512 + threadIdx.x;
    in[r] = i < hi;
    rec[r] = a.srec[in[r] ? i : lo];
    mark[r] = false;
  }
  uint32_t slots = 64;
  while (slots < 2 * (hi - lo) && slots < 2048) slots <<= 1;  // load <= 1/2 up to 1024 entries
  const bool pw2 = slots >= 2 * (hi - lo);  // else DD_SLOTS, the slot by a multiply-high
  if (!pw2) slots = DD_SLOTS;
  const uint32_t M = slots - 1;
  auto slot_of = [&](uint32_t h) { return pw2 ? h & M : (uint32_t)(((uint64_t)h * DD_SLOTS) >> 32); };
  // pass 1: latest-wins by the 32-bit partial key (the records' low words)
  uint32_t* const hkeys = (uint32_t*)dd_lds;  // (the exact pass's 64-bit key words reused)
  for (uint32_t i = threadIdx.x; i < slots; i += blockDim.x) { hkeys[i] = DD_EMPTY32; vals[i] = 0; }
  if (threadIdx.x == 0) { special = 0; collide = 0; }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < DR; r++) {
    if (!in[r]) break;
    const uint32_t h = (uint32_t)rec[r], hk = h == DD_EMPTY32 ? DD_EMPTY32 - 1 : h;
    const uint32_t v = (uint32_t)(rec[r] >> 32) + 1;
    uint32_t s = slot_of(h);
    while (true) {
      const uint32_t old = atomicCAS(&hkeys[s], DD_EMPTY32, hk);
      if (old == DD_EMPTY32 || old == hk) { atomicMax(&vals[s], v); break; }
      s = s == M ? 0u : s + 1;
    }
    slot[r] = s;
  }
  __syncthreads();
  // an entry that lost to a later one is NOT its key's latest only if the
  // winner carries the same full key (the chain's key array); otherwise two
  // keys share the partial key: the bucket is redone with the full keys
#pragma unroll
  for (int r = 0; r < DR; r++) {
    if (!in[r]) break;
    const uint32_t c = (uint32_t)(rec[r] >> 32), best = vals[slot[r]];
    if (best != c + 1) {
      if (a.kh[c] == a.kh[best - 1]) mark[r] = true;
      else collide = 1;
    }
  }
  __syncthreads();
  if (collide) {  // (uniform) pass 2: the full keys, gathered
    uint64_t key[DR];
#pragma unroll
    for (int r = 0; r < DR; r++) key[r] = in[r] ? a.kh[(uint32_t)(rec[r] >> 32)] : 0;
    for (uint32_t i = threadIdx.x; i < slots; i += blockDim.x) { keys[i] = IDX_EMPTY; vals[i] = 0; }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < DR; r++) {
      if (!in[r]) break;
      const uint32_t v = (uint32_t)(rec[r] >> 32) + 1;
      if (key[r] == IDX_EMPTY) { atomicMax(&special, v); continue; }
      uint32_t s = slot_of((uint32_t)xxh3_64_u64(key[r]));
      while (true) {
        const unsigned long long old = atomicCAS(&keys[s], (unsigned long long)IDX_EMPTY, (unsigned long long)key[r]);
        if (old == IDX_EMPTY || old == key[r]) { atomicMax(&vals[s], v); break; }
        s = s == M ? 0u : s + 1;
      }
      slot[r] = s;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < DR; r++) {
      if (!in[r]) break;
      const uint32_t c = (uint32_t)(rec[r] >> 32);
      mark[r] = (key[r] == IDX_EMPTY ? special : vals[slot[r]]) != c + 1;
    }
  }
  // the per-chunk count of the entries that are NOT the latest of their key
  // (idx_emit's prefix: position = c - non-latest before c; a store without
  // overwrites makes no atomics here).  Only the (rare) non-latest entries are
  // marked: a byte store per entry, scattered over the chain, costs
  // partial-line writes for every key
  const uint64_t n = idx_n(a);
  const uint64_t ch = n ? (n + GLUE_BLOCKS - 1) / GLUE_BLOCKS : 1;  // chunk_of's chunk at GLUE_BLOCKS blocks
#pragma unroll
  for (int r = 0; r < DR; r++) {
    if (!mark[r]) continue;
    const uint32_t c = (uint32_t)(rec[r] >> 32);
    a.latest[c] = a.lgen;
    atomicAdd(&a.ccount[c / ch], 1u);
  }
}

// the index in chain order of each key's latest entry: entry c goes to
// c - (entries before c that are not the latest of their key); launched on
// GLUE_BLOCKS blocks (idx_dedup's chunks)
__global__ __launch_bounds__(256) void idx_emit_kernel(IdxArgs a) {
  __shared__ uint32_t wsum[4];
  const uint64_t n = idx_n(a);
  uint64_t nl_before = 0, nl_total = 0;
  block_prefix(a.ccount, GLUE_BLOCKS, wsum, &nl_before, &nl_total);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.plan->n_index = n - nl_total;
    a.plan->idx_alias = a.alias && nl_total == 0;
    // (every value < 2^31: the dense capacity bounds K and the chain)
    if (a.pub) publish_outcome(a, a.plan, n, nl_total);
  }
  // every entry the latest of its key (a store without overwrites): the
  // index is the chain's (key_hash, packed) arrays chain_finalize wrote
  if (a.alias && nl_total == 0) return;
  uint64_t lo, hi;
  chunk_of(n, &lo, &hi);
  uint64_t run = lo - nl_before;
  // ER rounds of 256 positions per pass: their flags and keys are loaded
  // together and ranked with one LDS exchange
  constexpr int ER = 4;
  __shared__ uint32_t wsum_r[4 * ER];
  for (uint64_t base = lo; base < hi; base += ER * 256) {
    bool f[ER];
    uint64_t key[ER], mo[ER];
#pragma unroll
    for (int r = 0; r < ER; r++) {
      const uint64_t c = base + (uint64_t)r * 256 + threadIdx.x, cc = c < hi ? c : lo;
      f[r] = c < hi && a.latest[cc] != a.lgen;
      key[r] = a.kh[cc];
      mo[r] = a.mo[cc];
    }
    uint32_t rank[ER];
    const uint32_t tot = block_rank_rounds<4, ER>(f, wsum_r, rank);
#pragma unroll
    for (int r = 0; r < ER; r++) {
      if (!f[r]) continue;
      a.okey[run + rank[r]] = key[r];
      a.opacked[run + rank[r]] = ((key[r] >> 48) << 48) | (mo[r] & 0xFFFFFFFFFFFFull);  // key_indexer.rs:79-85
    }
    run += tot;
  }
}

// --------------------------------------------------------------------------
// Index exchange between entry-range shards: partition (key_hash, value)
// pairs by owner rank, stable (chain order kept inside every owner's run),
// so that after an all-to-all each owner's received runs are in shard order
// = file order and the bucketed build's latest-wins-by-position is exact.
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t owner_of(uint64_t key, uint32_t world) {
  return (uint32_t)(((key >> 32) * (uint64_t)world) >> 32);  // key hashes are XXH3 outputs: uniform
}
constexpr uint32_t PART_MAX_WORLD = 64;
struct PartArgs {
  const uint64_t* keys;
  const uint64_t* vals;
  uint64_t n;
  uint32_t world;
  uint32_t* cnt;  // [world * GLUE_BLOCKS + 1], owner-major
  uint32_t* off;  // exclusive scan of cnt
  uint64_t* out;  // [2n] interleaved (key, value), grouped by owner; or [n] keys when out_v is set
  uint64_t* out_v;   // nullable: [n] values (separate arrays: an owner pulls its run with two plain copies)
  uint64_t* counts;  // [world]
};
__global__ __launch_bounds__(256) void part_count_kernel(PartArgs a) {
  __shared__ uint32_t h[PART_MAX_WORLD];
  for (uint32_t o = threadIdx.x; o < a.world; o += blockDim.x) h[o] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.cnt[(uint64_t)a.world * GLUE_BLOCKS] = 0;
  __syncthreads();
  uint64_t lo, hi;
  chunk_of(a.n, &lo, &hi);
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&h[owner_of(a.keys[i], a.world)], 1u);
  __syncthreads();
  for (uint32_t o = threadIdx.x; o < a.world; o += blockDim.x) a.cnt[(uint64_t)o * GLUE_BLOCKS + blockIdx.x] = h[o];
}
// Stable scatter by owner: PR rounds of 256 pairs per pass, each wave ranks
// its lanes per owner with one ballot per owner, and the block orders the
// (round, wave) groups with one LDS exchange -- three barriers per 1024
// pairs (it was two per owner per 256).
__global__ __launch_bounds__(256) void part_scatter_kernel(PartArgs a) {
  constexpr int PR = 4;
  __shared__ uint32_t wcnt[PR][4][PART_MAX_WORLD];
  __shared__ uint32_t run[PART_MAX_WORLD];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1;
  for (uint32_t o = threadIdx.x; o < a.world; o += blockDim.x) run[o] = a.off[(uint64_t)o * GLUE_BLOCKS + blockIdx.x];
  __syncthreads();
  uint64_t lo, hi;
  chunk_of(a.n, &lo, &hi);
  for (uint64_t base = lo; base < hi; base += PR * 256) {
    uint64_t k[PR], v[PR];
    uint32_t own[PR], rk[PR];
#pragma unroll
    for (int r = 0; r < PR; r++) {
      const uint64_t i = base + (uint64_t)r * 256 + threadIdx.x;
      const bool in = i < hi;
      k[r] = in ? a.keys[i] : 0;
      v[r] = in ? a.vals[i] : 0;
      own[r] = in ? owner_of(k[r], a.world) : ~0u;
    }
#pragma unroll
    for (int r = 0; r < PR; r++) {
      uint32_t wc = 0;
      rk[r] = 0;
      for (uint32_t o = 0; o < a.world; o++) {
        const uint64_t b = __ballot(own[r] == o);
        if (own[r] == o) rk[r] = (uint32_t)__popcll(b & lt);
        if (lane == o) wc = (uint32_t)__popcll(b);
      }
      if (lane < a.world) wcnt[r][w][lane] = wc;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PR; r++) {
      if (own[r] == ~0u) continue;
      const uint32_t o = own[r];
      uint32_t before = run[o];
      for (int rr = 0; rr < PR; rr++)
        for (uint32_t ww = 0; ww < 4; ww++)
          before += (rr < r || (rr == r && ww < w)) ? wcnt[rr][ww][o] : 0u;
      const uint64_t pos = (uint64_t)before + rk[r];
      if (a.out_v) {
        a.out[pos] = k[r];
        a.out_v[pos] = v[r];
      } else {
        a.out[2 * pos] = k[r];
        a.out[2 * pos + 1] = v[r];
      }
    }
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < a.world; o += blockDim.x) {
      uint32_t t = 0;
      for (int rr = 0; rr < PR; rr++)
        for (uint32_t ww = 0; ww < 4; ww++) t += wcnt[rr][ww][o];
      run[o] += t;
    }
    __syncthreads();
  }
}
__global__ void part_counts_kernel(PartArgs a) {
  const uint32_t o = threadIdx.x;
  if (o < a.world) a.counts[o] = a.off[(uint64_t)(o + 1) * GLUE_BLOCKS] - a.off[(uint64_t)o * GLUE_BLOCKS];
}
// An owner's runs pulled from every shard in ONE launch (blockIdx.y = the
// source shard; its run read over xGMI straight from the source GPU's HBM,
// peer access enabled) instead of two hipMemcpyPeerAsync per source: each
// small copy cost a blit launch of ~5 us on the owner's stream
// With src_cnt set, the run lengths come from the sources' partition counts
// in their own HBM (part_counts_kernel's words, read over xGMI) instead of a
// host round trip per source: source s's run for this owner starts at
// sum(cnt_s[q], q < owner) in its partitioned arrays and lands at
// sum(cnt_s'[owner], s' < s) here; *d_total = the owner's pair count (the
// index build's n, on the device).
struct GatherArgs {
  const uint64_t* src_k[PART_MAX_WORLD];
  const uint64_t* src_v[PART_MAX_WORLD];
  const uint64_t* src_cnt[PART_MAX_WORLD];  // nullable: dst_off / src_k / src_v are final (host counts)
  uint64_t dst_off[PART_MAX_WORLD + 1];
  uint64_t* dst_k;
  uint64_t* dst_v;
  uint64_t* d_total;
  uint32_t owner, nsrc;
};
__global__ __launch_bounds__(256) void gather_runs_kernel(GatherArgs a) {
  const uint32_t s = blockIdx.y;
  __shared__ uint64_t s_run[3];  // source offset, length, destination offset
  if (a.src_cnt[0]) {
    if (threadIdx.x == 0) {
      uint64_t off = 0, dst = 0;
      for (uint32_t q = 0; q < a.owner; q++) off += a.src_cnt[s][q];
      for (uint32_t t = 0; t < s; t++) dst += a.src_cnt[t][a.owner];
      const uint64_t len = a.src_cnt[s][a.owner];
      s_run[0] = off;
      s_run[1] = len;
      s_run[2] = dst;
      if (blockIdx.x == 0 && s + 1 == a.nsrc) *a.d_total = dst + len;
    }
    __syncthreads();
  }
  const bool dev = a.src_cnt[0] != nullptr;
  const uint64_t o = dev ? s_run[2] : a.dst_off[s], n = dev ? s_run[1] : a.dst_off[s + 1] - o;
  const uint64_t* __restrict__ sk = a.src_k[s] + (dev ? s_run[0] : 0);
  const uint64_t* __restrict__ sv = a.src_v[s] + (dev ? s_run[0] : 0);
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    a.dst_k[o + j] = sk[j];
    a.dst_v[o + j] = sv[j];
  }
}

// interleaved pairs -> key / value arrays (the bucketed build's input)
__global__ void deinterleave_kernel(const uint64_t* pairs, uint64_t n, uint64_t* k, uint64_t* v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    k[i] = pairs[2 * i];
    v[i] = pairs[2 * i + 1];
  }
}

}  // namespace srd

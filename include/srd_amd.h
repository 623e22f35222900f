/*
 * srd_amd.h -- C ABI of the MI355X-native open-time hot path of SIMD R Drive
 * (jzombie/rust-simd-r-drive v0.16.3-alpha): validation-chain recovery,
 * per-payload IEEE CRC-32 check, and the latest-wins key-index rebuild,
 * plus the batch digest entry points.
 *
 * Plain pointers and sizes only (no torch / HIP types).  `stream` arguments
 * are `hipStream_t` passed as `void*` (NULL = the context's own stream).
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to the reference repo root):
 *
 *   srd_recover_valid_chain   <- DataStore::recover_valid_chain
 *                                src/storage_engine/data_store.rs:383-482
 *   srd_key_indexer_build     <- KeyIndexer::build
 *                                src/storage_engine/key_indexer.rs:98-124
 *   srd_validate_index(_device) <- the two calls inside DataStore::open
 *                                (data_store.rs:89 and :108) fused with
 *                                EntryHandle::is_valid_checksum
 *                                (simd-r-drive-entry-handle/src/entry_handle.rs:260-275)
 *                                over every chain entry
 *   srd_crc32_batch(_device)  <- compute_checksum
 *                                src/storage_engine/digest/compute_checksum.rs:15-20
 *   srd_xxh3_64_batch(_device) <- compute_hash_batch
 *                                src/storage_engine/digest/compute_hash.rs:64-77
 *   srd_xxh3_64               <- compute_hash  (compute_hash.rs:25-27)
 *
 * Semantics (bit-exact with the reference):
 *   - final_len = largest tail t <= file_len whose backward chain is
 *     structurally valid down to offset 0 (0 if none), exactly as the
 *     reference's byte-wise outer loop finds it.
 *   - chain = entries of the chain ending at final_len, in file order.
 *   - crc_computed = IEEE CRC-32 (crc32fast) of each chain payload;
 *     crc_ok = (crc_computed == stored little-endian checksum).
 *   - index = key_hash -> pack(tag16 = key_hash >> 48, meta_off48), latest
 *     entry per key_hash wins, tombstones INCLUDED (as KeyIndexer::build).
 * Errors: 0 = ok; negative = HIP / allocation / argument error
 * (srd_last_error() has the message).  Invalid chains and bad CRCs are
 * data, never errors.  Arithmetic on offsets wraps like release-mode Rust.
 */
#ifndef SRD_AMD_H
#define SRD_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRD_OK 0
#define SRD_ERR_HIP (-1)
#define SRD_ERR_ALLOC (-2)
#define SRD_ERR_ARG (-3)
#define SRD_ERR_INTERNAL (-4)

/* srd_device_result.mode */
#define SRD_MODE_OPTIMISTIC 0      /* the chain was proven through recorded nodes from the largest tail
                                      within 256 B of file_len that passes recover_valid_chain's first
                                      test (file_len for an intact store, below it for a short torn tail) */
#define SRD_MODE_FULL 1            /* full pass (torn tail / corrupt store / unusual structure) */
#define SRD_MODE_SPAN_UNPROVEN 3   /* span mode: the shard's chain was not proven; use the whole-file path */

/* srd_device_result.full_reason: why the optimistic pass left the call to
 * the full pass (mode SRD_MODE_FULL) or left a span unproven
 * (SRD_MODE_SPAN_UNPROVEN); SRD_FULL_NONE when it decided.  The full pass
 * costs ~1.8x the optimistic one, so a store that always lands here (e.g. one
 * above ~1 TiB: SRD_FULL_SLOT_SPACE) is visible instead of silently slower. */
#define SRD_FULL_NONE 0
#define SRD_FULL_FORCED 1     /* SRD_FLAG_FORCE_FULL */
#define SRD_FULL_SLOT_SPACE 2 /* scan waves x candidate slots per wave >= the glue's 31-bit slot space */
#define SRD_FULL_WAVES 3      /* more scan waves per chain block than the shape check's bound */
#define SRD_FULL_NO_START 4   /* no strong node or root at the start tail (find_top): torn / corrupt end */
#define SRD_FULL_UNPROVEN 5   /* the recorded nodes do not prove one chain (shape / root count) */
#define SRD_FULL_CAP 6        /* the candidate slots per span could not grow further */
#define SRD_FULL_LOOKBACK 7   /* the fused shape check's decoupled look-back timed out (a chain block
                                 waited too long for a lower one): nothing it computed is used */

/* option flags */
#define SRD_FLAG_FORCE_FULL 1u   /* skip the optimistic (strong-candidate) pass */
#define SRD_FLAG_NO_CRC 2u       /* structural recovery + index only */
/* host-input staging (srd_validate_index / _multi).  Default: pinned input is
 * copied directly; any other memory (the mmap) goes through double-buffered
 * pinned bounce buffers that host threads fill (taking the mapping's page
 * faults on several cores) while the previous chunks DMA -- measured at the
 * pinned-buffer rate on MI355X (end to end). */
#define SRD_FLAG_STAGE_PAGEABLE 4u /* one pageable hipMemcpy (measurement baseline) */
#define SRD_FLAG_STAGE_REGISTER 8u /* hipHostRegister the range (read-only) for one DMA copy;
                                      bounce buffers when registration is refused */

typedef struct srd_ctx srd_ctx; /* one device + stream + reusable workspace */

int srd_ctx_create(int device, srd_ctx **out);
void srd_ctx_destroy(srd_ctx *ctx);
/* The HIP stream the context launches on (hipStream_t as void*). */
void *srd_ctx_stream(srd_ctx *ctx);
/* Device bytes the context holds now: its workspace buffers (candidate
 * records, per-slot glue words, result arrays, index buckets, ...) plus its
 * staging copy of a host store, if any.  The optimistic pass sizes its
 * per-slot arrays by slot space (~S / 2048 slots of ~160 B for an S-byte
 * store at the default 8 slots per 16 KiB span: DESIGN.md section 3). */
uint64_t srd_ctx_device_bytes(srd_ctx *ctx);
/* The tile-load pattern of the context's last optimistic scan: 0 coalesced
 * loads + in-register transpose, 1 line per lane (the pass measures both on
 * each new store and keeps the faster: DESIGN.md section 4.1); -1 before any. */
int srd_ctx_scan_loads(srd_ctx *ctx);
/* The load-pattern trial of the current store: ms[0] / ms[1] = the fastest
 * device-timed optimistic scan with coalesced / line-per-lane loads so far (0
 * if not measured); returns the choice (0, 1) or -1 while still measuring
 * (or pinned by SRD_SCAN_LOADS, or with XCD-aware shares off). */
int srd_ctx_scan_trial(srd_ctx *ctx, double *ms);
const char *srd_last_error(void);
/* The sha256 of the sources this library was compiled from (csrc/ +
 * include/srd_amd.h, rust-simd-r-drive_amd/src_hash.py), 64 hex digits;
 * the Python mirror refuses a library whose hash differs from the sources
 * beside it, and bench.py / smoke print it. */
const char *srd_build_info(void);
/* HIP-event timing of the validate calls on ctx: SRD_TIMING_NONE (the
 * default), SRD_TIMING_SCAN (the streaming scan's launches: events stamped by
 * the scan dispatch itself, hipExtLaunchKernel -- bench.py's roofline),
 * SRD_TIMING_CALL (+ marker events around the whole call, ~10 us each).  Not
 * part of the reference interface. */
#define SRD_TIMING_NONE 0
#define SRD_TIMING_SCAN 1
#define SRD_TIMING_CALL 2
int srd_ctx_set_timing(srd_ctx *ctx, int level);
/* With SRD_TIMING_SCAN: stamp only every n-th scan launch (n >= 1; 1 = every
 * launch, the default).  The event-stamped launch costs ~7 us more wall time
 * than a plain one; a systematic sample keeps that off most calls. */
int srd_ctx_set_timing_every(srd_ctx *ctx, int n);

/* HIP-event timings on the context stream: the summed duration (ms) and the
 * count of the streaming scan kernel launches of every validate call since the
 * previous srd_ctx_timings call (the scans' event pairs are read out here, not
 * inside the calls), and the device span of the last call (0 unless the
 * timing level includes them). */
int srd_ctx_timings(srd_ctx *ctx, double *scan_ms, int *scan_launches,
                    double *total_ms);
/* The individual scan durations (ms) summed by the last srd_ctx_timings
 * read, in launch order: copies up to cap of them to out and returns how
 * many there were (< 0: error). */
int srd_ctx_scan_list(srd_ctx *ctx, float *out, int cap);

/* Result of one validate+index pass whose arrays live in DEVICE memory owned
 * by the context (valid until the next call on the same ctx). */
typedef struct {
  uint64_t file_len;
  uint64_t final_len;      /* recover_valid_chain */
  uint64_t n_chain;        /* entries on the chain ending at final_len */
  uint64_t n_index;        /* KeyIndexer entries */
  uint64_t n_crc_bad;      /* chain entries whose CRC does not match */
  uint64_t n_candidates;   /* chain-node candidates recorded by the scan */
  uint64_t full_reason;    /* SRD_FULL_*: why the optimistic pass did not decide (0 when it did) */
  uint32_t mode;           /* 0 = optimistic pass sufficed, 1 = full pass */
  uint32_t reserved;       /* host results: 1 = arrays owned by the context */
  /* chain, file order; device pointers */
  uint64_t *meta_off, *key_hash, *prev_offset, *payload_start, *payload_len;
  uint32_t *crc_stored, *crc_computed;
  uint8_t *crc_ok;
  /* index (chain order of the latest entry per key); device pointers */
  uint64_t *index_key_hash, *index_packed;
} srd_device_result;

/* Bytes the device buffer handed to srd_validate_index_device must be
 * readable for: file_len rounded up to 4 KiB plus 8 KiB of slack (contents
 * past file_len are ignored).  The streaming kernel loads whole 4 KiB tiles
 * unconditionally so its prefetch ring never drains on a bounds branch. */
uint64_t srd_padded_size(uint64_t file_len);

/* Device-resident validate+index over `file_len` bytes at `d_file`
 * (device pointer, 16-byte aligned, readable to srd_padded_size(file_len);
 * the bytes are the mmap'd store). */
int srd_validate_index_device(srd_ctx *ctx, const uint8_t *d_file,
                              uint64_t file_len, uint32_t flags,
                              srd_device_result *out);

/* Entry-range shard of a store (multi-GPU, one process per GPU; no
 * collective inside).  `d_span` holds file bytes [span_off, hi) -- span_off a
 * multiple of 16 KiB and <= lo, readable to srd_padded_size(hi - span_off) --
 * where lo and hi are entry tails: lo = the previous shard's last tail, hi =
 * this shard's last tail (hi = file_len for the last shard).  Proves that the
 * backward chain from hi reaches an entry whose prev_offset == lo and returns
 * that chain segment (file order, absolute offsets), every payload's CRC and
 * the shard-local latest-wins index.  final_len = hi when proven; otherwise
 * mode = SRD_MODE_SPAN_UNPROVEN, final_len = 0 and the caller falls back to
 * the whole-file path (a torn tail, for example, can only be recovered there,
 * recover_valid_chain's byte-wise outer loop is global).  The shards' chains
 * compose to the whole file's chain when shard 0 has lo = 0 (whole-file rule)
 * and each shard's lo equals the previous shard's hi.  lo == 0 with
 * span_off == 0 is exactly srd_validate_index_device (the whole-file rule:
 * final_len may lie below hi in any mode); a shard is proven iff
 * final_len == hi and mode != SRD_MODE_SPAN_UNPROVEN. */
int srd_validate_span_device(srd_ctx *ctx, const uint8_t *d_span,
                             uint64_t span_off, uint64_t lo, uint64_t hi,
                             uint32_t flags, srd_device_result *out);

/* Shard boundaries of an arbitrary store (host pre-pass, no GPU): cuts[0] = 0,
 * cuts[world] = file_len, and cuts[r] (0 < r < world) the highest byte t at
 * or below r * file_len / world (searched down to 64 MiB below it) whose
 * backward walk passes recover_valid_chain's node test (data_store.rs:404-470)
 * for 8 hops without reaching offset 0.  Non-decreasing; a cut with no candidate repeats the previous
 * one (an empty shard).  The cuts are guesses that srd_validate_span_device
 * plus the composition check prove or refute: [cuts[r], cuts[r+1]) are rank
 * r's lo / hi. */
int srd_shard_cuts(const uint8_t *file, uint64_t file_len, uint32_t world,
                   uint64_t *cuts);

/* Index exchange between shards (KeyIndexer semantics, key_indexer.rs:98-124).
 * Partition n (key_hash, value) pairs (device arrays) by owner rank
 * owner = ((key_hash >> 32) * world) >> 32 into d_out_pairs ([2n] u64,
 * interleaved key,value; grouped by owner, input order kept inside a group);
 * counts[world] (host) receives the group sizes.  Synchronises. */
int srd_index_partition_device(srd_ctx *ctx, const uint64_t *d_keys,
                               const uint64_t *d_vals, uint64_t n,
                               uint32_t world, uint64_t *d_out_pairs,
                               uint64_t *counts);

/* KeyIndexer::build over n interleaved (key_hash, meta_off or packed) device
 * pairs in file order (the latest position of a key wins; tombstones are
 * entries like any other).  Writes the index (key_hash, pack(tag16,
 * offset48)) in file order of each key's latest entry to the caller's device
 * arrays (capacity n each); *n_index = its size.  Synchronises. */
int srd_index_build_device(srd_ctx *ctx, const uint64_t *d_pairs, uint64_t n,
                           uint64_t *d_out_keys, uint64_t *d_out_packed,
                           uint64_t *n_index);

/* Same result with host-memory arrays.  `file` is host memory (e.g. the
 * mmap); it is staged to HBM inside.  The arrays live in pinned host memory
 * owned by the context (ctxs[0] for the multi-GPU form), DMA'd there straight
 * from HBM: valid until the next srd_validate_index(_multi) call on that
 * context; srd_result_free releases nothing then, it only clears the struct
 * (reserved == 1 marks such a result). */
typedef srd_device_result srd_result;
int srd_validate_index(srd_ctx *ctx, const uint8_t *file, uint64_t file_len,
                       uint32_t flags, srd_result *out);
void srd_result_free(srd_result *res);

/* DataStore::open of one host store (the mmap) on n GPUs in ONE process,
 * without RCCL (data_store.rs:84-117).  ctxs[i] are distinct
 * contexts (one per GPU; the same device may repeat, the same context may
 * not: SRD_ERR_ARG).  The host pre-pass
 * srd_shard_cuts splits the store into n entry ranges; one host thread per
 * context stages its span [span_off, hi) and runs srd_validate_span_device.
 * The host composes the shards (every shard proven, each lo == the previous
 * hi); then the chain arrays are concatenated and the per-shard indexes are
 * gathered to ctxs[0]'s device (hipMemcpyPeer over xGMI) in shard order and
 * merged latest-wins there (KeyIndexer::build, key_indexer.rs:98-124).  A
 * store that does not compose (a torn tail, corruption, a wrong cut, a shard
 * error) is decided by the whole-file path on ctxs[0].  The result is
 * identical to srd_validate_index's. */
int srd_validate_index_multi(srd_ctx *const *ctxs, uint32_t n_ctx,
                             const uint8_t *file, uint64_t file_len,
                             uint32_t flags, srd_result *out);

/* ---- the same open over a store already resident in the GPUs' HBM ----
 *   srd_validate_index_multi_device <- DataStore::open (data_store.rs:84-117:
 *                                      recover_valid_chain :383-482 +
 *                                      KeyIndexer::build key_indexer.rs:98-124)
 *                                      with the file sharded by entry range over
 *                                      the GPUs of one node, no RCCL
 * Context i holds its shard in its own HBM: d_spans[i] = file bytes
 * [span_offs[i], cuts[i+1]) (span_offs[i] a multiple of 16 KiB, <= cuts[i];
 * span_offs[0] = 0; readable to srd_padded_size(cuts[i+1] - span_offs[i])).
 * cuts[0] = 0 <= cuts[1] <= .. <= cuts[n] = file_len are entry tails (e.g.
 * from the writer's layout or srd_shard_cuts); an empty shard (cuts[i] ==
 * cuts[i+1]) needs no span.  One host thread per context validates its shard;
 * the host composes them.  Index (latest wins over the whole chain):
 *   default: by owner -- shards[i].index_* (device arrays on ctxs[i]'s GPU)
 *            hold the keys with owner ((key_hash >> 32) * n) >> 32 == i, in
 *            file order of each key's latest entry; every owner pulls its runs
 *            from all shards over xGMI (hipMemcpyPeerAsync) in shard order;
 *   SRD_FLAG_MERGE_INDEX: the whole index on ctxs[0]'s GPU
 *            (summary->index_*, the order srd_validate_index_device gives).
 * shards[i] (array of n) = chain segment i (device arrays on ctxs[i]'s GPU,
 * owned by the context until its next call); the segments concatenated in
 * shard order are the chain in file order.  A shard left unproven by its cut
 * (a cut that is no chain tail) is re-validated together with its lower
 * neighbour, the bytes gathered onto that neighbour's GPU over xGMI; a store
 * that still does not compose (a torn tail, corruption, a shard error) is
 * decided by the whole-file path on ctxs[0] (the store gathered there; its
 * whole chain is then shards[0]).  summary (nullable) reports which path
 * decided, the totals and host timings.  Each entry of ctxs must be a
 * distinct context (the same device may repeat).  Synchronises. */
#define SRD_FLAG_MERGE_INDEX 16u
#define SRD_MULTI_COMPOSED 0u   /* every shard proven on its own */
#define SRD_MULTI_NEIGHBOUR 1u  /* a run of unproven shards proven with its lower neighbour */
#define SRD_MULTI_WHOLE_FILE 2u /* the whole-file path decided (torn tail / corruption / shard error) */
typedef struct {
  uint64_t file_len, final_len;  /* final_len: recover_valid_chain's answer */
  uint64_t n_chain, n_index, n_crc_bad, n_candidates;  /* totals */
  uint32_t mode;          /* SRD_MODE_OPTIMISTIC if every shard's pass was optimistic */
  uint32_t path;          /* SRD_MULTI_* */
  uint32_t n_shards;
  uint32_t merged;        /* 1: the index is summary->index_* on ctxs[0] */
  uint32_t shard_errors;  /* shards whose first validation failed with an error */
  uint32_t peer_errors;   /* cross-device copies between GPUs without peer access
                             (hipDeviceEnablePeerAccess refused: staged by the runtime) */
  double validate_ms;     /* host wall time of the slowest shard's validation(s) */
  double exchange_ms;     /* index exchange + builds */
  double total_ms;        /* the whole call */
  uint64_t *index_key_hash, *index_packed; /* merged: device arrays on ctxs[0] */
} srd_multi_summary;
int srd_validate_index_multi_device(srd_ctx *const *ctxs, uint32_t n_ctx,
                                    const uint8_t *const *d_spans,
                                    const uint64_t *span_offs,
                                    const uint64_t *cuts, uint32_t flags,
                                    srd_device_result *shards,
                                    srd_multi_summary *summary);
/* The summary of the last multi-GPU open (host or device input) that had ctx
 * as ctxs[0]: which path decided it, totals, timings. */
int srd_ctx_multi_summary(srd_ctx *ctx, srd_multi_summary *out);
/* Its per-shard validate times (host wall ms of each shard's own thread,
 * re-validations included): copies up to cap of them to out and returns the
 * shard count (< 0: error). */
int srd_ctx_multi_shard_ms(srd_ctx *ctx, double *out, int cap);
/* Staging of the last host-input call on ctx: *mode = 0 pinned input, 1
 * registered mapping, 2 bounce buffers, 3 pageable copy (-1 none yet);
 * *stage_ms = host wall time from the call's start until the store was in
 * HBM (registration / page faults / copies included).  Nullable outputs. */
int srd_ctx_stage_info(srd_ctx *ctx, int *mode, double *stage_ms);

/* The index bucket hash on the device: out[i] = xxh3_64(le8(keys[i])), the
 * Xxh3BuildHasher's Hasher::write (digest/xxh3_build_hasher.rs:11-13) the
 * KeyIndexer HashMap applies to every key_hash.  Asynchronous on `stream`. */
int srd_index_hash_device(srd_ctx *ctx, const uint64_t *d_keys, uint64_t n,
                          uint64_t *d_out, void *stream);

/* Measurement utility (bench.py's roofline.peak_measured; not part of the
 * reference interface): the streaming-read ceiling of the scan's geometry
 * -- one 16-wave block per CU, a contiguous tile range per wave, 64 B per
 * lane, a 3-deep register ring, no work on the bytes -- over the first
 * floor(bytes / 4096) tiles of d_buf, timed `reps` times (after one warm-up
 * run) with HIP events on the context stream.  *best_ms / *median_ms
 * (nullable) over the reps.  Synchronises. */
int srd_stream_probe_device(srd_ctx *ctx, const uint8_t *d_buf, uint64_t bytes,
                            int reps, double *best_ms, double *median_ms);

/* recover_valid_chain: final_len only (host input). */
int srd_recover_valid_chain(srd_ctx *ctx, const uint8_t *file,
                            uint64_t file_len, uint64_t *final_len);

/* KeyIndexer::build over the chain ending at `tail` (host input).  Writes up
 * to `cap` pairs; *n_out = number of index entries. */
int srd_key_indexer_build(srd_ctx *ctx, const uint8_t *file, uint64_t tail,
                          uint64_t *key_hash_out, uint64_t *packed_out,
                          uint64_t cap, uint64_t *n_out);

/* CRC-32 (crc32fast) of n byte ranges [offs[i], offs[i]+lens[i]) of buf. */
int srd_crc32_batch(srd_ctx *ctx, const uint8_t *buf, uint64_t buf_len,
                    const uint64_t *offs, const uint64_t *lens, uint64_t n,
                    uint32_t *out);
int srd_crc32_batch_device(srd_ctx *ctx, const uint8_t *d_buf,
                           const uint64_t *d_offs, const uint64_t *d_lens,
                           uint64_t n, uint32_t *d_out, void *stream);

/* XXH3-64 (seed 0, default secret) of n keys [offs[i], offs[i]+lens[i]). */
int srd_xxh3_64_batch(srd_ctx *ctx, const uint8_t *keys, uint64_t keys_len,
                      const uint64_t *offs, const uint64_t *lens, uint64_t n,
                      uint64_t *out);
int srd_xxh3_64_batch_device(srd_ctx *ctx, const uint8_t *d_keys,
                             const uint64_t *d_offs, const uint64_t *d_lens,
                             uint64_t n, uint64_t *d_out, void *stream);

/* ---- checksum-on-append batch writer (BASELINE config C5) ----
 *   srd_batch_write           <- DataStoreWriter::batch_write
 *                                src/storage_engine/data_store.rs:838-843
 *                                (compute_hash_batch + batch_write_with_key_hashes
 *                                 data_store.rs:847-939, allow_null_bytes = false)
 *   SRD_WRITE_ALLOW_NULL      <- batch_write_with_key_hashes(.., true), the
 *                                tombstone path used by deletes (:864-897)
 * The serialized bytes are exactly what the reference appends to the file:
 * per entry a zero prepad to the next 64-byte boundary (none for a
 * tombstone), the payload, and EntryMetadata{key_hash, prev_offset = the
 * previous tail, crc32(payload)} (entry_metadata.rs:75-93).  The returned
 * (key_hash, metadata offset) pairs are the reference's key_hash_offsets, in
 * entry order, for the caller's index (reindex, data_store.rs:936). */
#define SRD_WRITE_ALLOW_NULL 1u

typedef struct {
  uint64_t src;      /* payload offset in the payload buffer */
  uint64_t len;      /* payload length (1 for a tombstone) */
  uint64_t key_src;  /* key offset in the key buffer (SRD_ENTRY_HASHED: the key hash) */
  uint64_t tail;     /* file tail before this entry (its prev_offset) */
  uint32_t key_len;
  uint32_t flags;    /* SRD_ENTRY_TOMB | SRD_ENTRY_HASHED */
} srd_write_entry;
#define SRD_ENTRY_TOMB 1u   /* NULL-byte payload written as a tombstone */
#define SRD_ENTRY_HASHED 2u /* key_src holds the key hash (batch_write_with_key_hashes) */

/* Host-side layout of a batch appended at file offset `tail`: fills out[n]
 * and *new_tail.  `payloads` (host) is read only to recognise NULL-byte
 * payloads.  Errors (SRD_ERR_ARG, message as the reference's InvalidInput):
 * "Payload cannot be empty.", "NULL-byte payloads cannot be written
 * directly." (without SRD_WRITE_ALLOW_NULL). */
int srd_batch_layout(uint64_t tail, const uint8_t *payloads,
                     const uint64_t *key_offs, const uint64_t *key_lens,
                     const uint64_t *pay_offs, const uint64_t *pay_lens,
                     uint64_t n, uint32_t flags, srd_write_entry *out,
                     uint64_t *new_tail);

/* batch_write from HOST buffers (pin them for full PCIe rate): payload and
 * key bytes are copied to HBM in chunks on a side stream while the writer
 * kernel serializes the previous chunk on the context stream.  The output
 * goes to d_out (device), d_out[j] = file byte (tail & ~63) + j, capacity
 * out_cap bytes; d_out == NULL only computes *new_tail.  kh_out / mo_out
 * (host, nullable) receive the key hashes and metadata offsets. */
int srd_batch_write(srd_ctx *ctx, uint64_t tail, const uint8_t *keys,
                    const uint64_t *key_offs, const uint64_t *key_lens,
                    const uint8_t *payloads, const uint64_t *pay_offs,
                    const uint64_t *pay_lens, uint64_t n, uint32_t flags,
                    uint8_t *d_out, uint64_t out_cap, uint64_t *new_tail,
                    uint64_t *kh_out, uint64_t *mo_out);

/* The writer kernel alone on device-resident inputs (entries from
 * srd_batch_layout, copied to the device by the caller); out[j] = file byte
 * out_base + j (out_base 64-aligned).  Asynchronous on `stream`. */
int srd_batch_write_device(srd_ctx *ctx, const uint8_t *d_keys,
                           const uint8_t *d_payloads,
                           const srd_write_entry *d_entries, uint64_t n,
                           uint8_t *d_out, uint64_t out_base,
                           uint64_t *d_kh_out, uint64_t *d_mo_out,
                           void *stream);

/* ---- device KeyIndexer + batched keyed reads ----
 *   srd_index_table_build_device <- the KeyIndexer HashMap<u64, u64> that
 *                                   DataStore::open fills (key_indexer.rs:98-124),
 *                                   adopted on the GPU from the validate pass's
 *                                   index arrays instead of re-inserted on the host
 *   srd_index_get_packed_device  <- KeyIndexer::get_packed (key_indexer.rs:164-167)
 *   srd_batch_read_hashed_device <- DataStoreReader::batch_read_hashed_keys
 *                                   (data_store.rs:1117-1158) over
 *                                   read_entry_with_context (:502-565)
 *   srd_batch_read               <- DataStoreReader::batch_read (:1111-1115)
 * The table lives in caller-provided device memory of srd_index_table_bytes(n)
 * bytes (open addressing, load <= 1/2).  A read returns the entry's payload
 * range [start, end) in the file, or start == end == 0 for None: key absent,
 * tag mismatch against the verification hash (the reference's collision
 * check), metadata out of range, or a tombstone. */
#define SRD_INDEX_NONE (~(uint64_t)0) /* get_packed: key absent */

uint64_t srd_index_table_bytes(uint64_t n);
/* n unique (key_hash, packed) device pairs (e.g. srd_device_result's index). */
int srd_index_table_build_device(srd_ctx *ctx, const uint64_t *d_keys,
                                 const uint64_t *d_packed, uint64_t n,
                                 void *d_table, uint64_t table_bytes);
int srd_index_get_packed_device(srd_ctx *ctx, const void *d_table,
                                uint64_t table_bytes, const uint64_t *d_hashes,
                                uint64_t n, uint64_t *d_packed_out, void *stream);
/* d_verify_hashes (nullable): compute_hash of the non-hashed keys; the read is
 * None when its tag (hash >> 48) differs from the indexed entry's tag. */
int srd_batch_read_hashed_device(srd_ctx *ctx, const void *d_table,
                                 uint64_t table_bytes, const uint8_t *d_file,
                                 uint64_t file_len, const uint64_t *d_hashes,
                                 const uint64_t *d_verify_hashes, uint64_t n,
                                 uint64_t *d_start, uint64_t *d_end, void *stream);
/* Host keys in, host ranges out: keys hashed on the device (XXH3-64) and
 * verified by their own tags, as batch_read does.  Synchronises. */
int srd_batch_read(srd_ctx *ctx, const void *d_table, uint64_t table_bytes,
                   const uint8_t *d_file, uint64_t file_len, const uint8_t *keys,
                   const uint64_t *key_offs, const uint64_t *key_lens, uint64_t n,
                   uint64_t *start_out, uint64_t *end_out);

/* ---- iteration and compaction over the device index ----
 *   srd_iter_entries_device   <- EntryIterator (entry_iterator.rs:69-126) /
 *                                par_iter_entries (data_store.rs:297-361):
 *                                the latest non-tombstone entry per key, in
 *                                EntryIterator order (newest first)
 *   srd_estimate_compaction_savings_device
 *                             <- estimate_compaction_savings (:605-616)
 *   srd_compact_device        <- compact (:706-749): the latest entries
 *                                re-serialized by write_stream_with_key_hash
 *                                in iter_entries order from offset 0 (the
 *                                write_kernel with prehashed keys), into d_out
 * d_index_packed = srd_device_result.index_packed (n_index values). */
int srd_iter_entries_device(srd_ctx *ctx, const uint8_t *d_file,
                            uint64_t file_len, const uint64_t *d_index_packed,
                            uint64_t n_index, uint64_t *d_start, uint64_t *d_end,
                            uint64_t *d_meta_off, uint64_t *d_key_hash,
                            uint64_t *n_out);
int srd_estimate_compaction_savings_device(srd_ctx *ctx, const uint8_t *d_file,
                                           uint64_t file_len,
                                           const uint64_t *d_index_packed,
                                           uint64_t n_index, uint64_t *savings);
/* d_out == NULL only computes *new_len.  Fails (SRD_ERR_ARG) like the
 * reference when a kept payload is all NULL bytes ("NULL-byte-only streams
 * cannot be written directly."). */
int srd_compact_device(srd_ctx *ctx, const uint8_t *d_file, uint64_t file_len,
                       const uint64_t *d_index_packed, uint64_t n_index,
                       uint8_t *d_out, uint64_t out_cap, uint64_t *new_len,
                       uint64_t *d_key_hash_out, uint64_t *d_meta_off_out);

/* Synthetic store of the BASELINE configs written on the device (the
 * checksum-on-append writer of data_store.rs:847-939 for keys
 * "bench-key-{i}" and counter-mode splitmix64 payloads).  lens==NULL ->
 * every payload is fixed_len bytes.  Returns the file length in *len_out;
 * d_out==NULL only computes the length. */
int srd_synth_store_device(srd_ctx *ctx, uint8_t *d_out, uint64_t n_entries,
                           uint64_t fixed_len, const uint64_t *lens,
                           uint64_t seed, uint64_t *len_out);

/* The shard [lo, hi) of that synthetic store holding entries
 * [first, first + n) (lens, if given, holds the lengths of entries
 * 0 .. first + n - 1), written into d_span = file bytes [span_off, hi)
 * (span_off a multiple of 16 KiB, <= lo; bytes of earlier entries at or past
 * span_off are written too).  d_span == NULL only computes lo / hi. */
int srd_synth_span_device(srd_ctx *ctx, uint8_t *d_span, uint64_t span_off,
                          uint64_t first, uint64_t n, uint64_t fixed_len,
                          const uint64_t *lens, uint64_t seed,
                          uint64_t *lo_out, uint64_t *hi_out);

/* Library self-test of the CRC algebra tables (host only, no GPU). */
int srd_selftest_host(void);

#ifdef __cplusplus
}
#endif
#endif

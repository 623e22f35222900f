/*
 * srd_oracle.h -- CPU restatement of SIMD R Drive's open-time hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X path and the timed CPU baseline (`bench.py` cpu_baseline leg).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product library (rust-simd-r-drive_amd/) never links it.
 *
 * Every function cites the reference file:line it restates
 * (paths relative to jzombie/rust-simd-r-drive v0.16.3-alpha).
 *
 * Parity pins: XXH3-64 against tests/hash_stability_tests.rs:16-100 (golden
 * values, via tests/golden/reference_goldens.json); CRC-32 against the
 * IEEE check value 0xCBF43926 and zlib-generated fixtures (the reference has
 * no CRC golden vectors); chain recovery / index against
 * fixtures written by tests/golden/make_golden.py (an independent pure-Python
 * restatement that uses zlib + python-xxhash for the arithmetic).
 */
#ifndef SRD_ORACLE_H
#define SRD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_METADATA_SIZE 20u
#define ORC_PAYLOAD_ALIGNMENT 64u

/* ---- digest (src/storage_engine/digest/) ---- */
uint64_t orc_xxh3_64(const void *data, size_t len);
void orc_xxh3_64_batch(const uint8_t *buf, const uint64_t *offs,
                       const uint64_t *lens, uint64_t n, uint64_t *out);
uint32_t orc_crc32(const void *data, size_t len);       /* crc32fast-equivalent */
uint32_t orc_crc32_update(uint32_t crc, const void *data, size_t len);
uint32_t orc_crc32_table(const void *data, size_t len); /* portable slice-by-8 */
/* orc_crc32 of buf[starts[i], starts[i] + lens[i]) for i < n, threaded */
void orc_crc32_ranges(const uint8_t *buf, const uint64_t *starts,
                      const uint64_t *lens, uint64_t n, uint32_t *out,
                      int threads);
int orc_has_pclmul(void);

/* ---- format (simd-r-drive-entry-handle/src/) ---- */
uint64_t orc_prepad_len(uint64_t offset);

/* ---- writer (data_store.rs:847-939) ----
 * Appends n entries to `out` (which already holds `tail` bytes).
 * Returns the new tail, or -1 on an invalid payload, -2 on capacity. */
int64_t orc_write_entries(uint8_t *out, uint64_t cap, uint64_t tail,
                          const uint64_t *key_hashes, const uint8_t *payload_buf,
                          const uint64_t *payload_offs,
                          const uint64_t *payload_lens, uint64_t n,
                          int allow_null_bytes);

/* Synthetic store of BASELINE configs: keys bench-key-{i},
 * payload bytes from counter-mode splitmix64 (see srd_oracle.c).
 * lens==NULL -> every payload is `fixed_len` bytes.  Returns the file length
 * (when out==NULL only the length is computed). */
uint64_t orc_synth_store(uint8_t *out, uint64_t n_entries, uint64_t fixed_len,
                         const uint64_t *lens, uint64_t seed);
uint64_t orc_synth_word(uint64_t seed, uint64_t entry, uint64_t word);

/* ---- engine (data_store.rs:383-482, key_indexer.rs:98-124) ---- */
uint64_t orc_recover_valid_chain(const uint8_t *mmap, uint64_t file_len);

typedef struct {
  uint64_t meta_off;
  uint64_t key_hash;
  uint64_t prev_offset;
  uint64_t payload_start;
  uint64_t payload_len;
  uint32_t crc_stored;
  uint32_t crc_computed;
  uint32_t crc_ok;
  uint32_t is_tombstone;
} orc_entry;

/* Entries of the chain ending at `tail`, in FILE order (ascending meta_off).
 * Returns the count (writes at most cap entries; compute_crc!=0 fills the
 * crc_computed/crc_ok fields as EntryHandle::is_valid_checksum would). */
uint64_t orc_chain(const uint8_t *mmap, uint64_t tail, orc_entry *out,
                   uint64_t cap, int compute_crc);

/* KeyIndexer::build: latest-wins (key_hash -> pack(tag, meta_off)),
 * tombstones included.  Output sorted by key_hash.  Returns count. */
uint64_t orc_key_indexer_build(const uint8_t *mmap, uint64_t tail,
                               uint64_t *keys_out, uint64_t *packed_out,
                               uint64_t cap);

/* The timed CPU baseline: DataStore::open (recover + KeyIndexer::build with
 * an XXH3-hashed table) + is_valid_checksum over every chain entry.
 * threads<=1: faithful single thread; threads>1: the CRC pass is split over
 * threads (the par_iter_entries analogue). */
typedef struct {
  uint64_t final_len;
  uint64_t n_chain;
  uint64_t n_index;
  uint64_t n_crc_bad;
  uint64_t crc_xor;      /* xor of all computed CRCs (cheap fingerprint) */
  uint64_t index_xor;    /* xor of (key_hash ^ packed*31) over the index */
  double t_recover_s, t_index_s, t_crc_s;
} orc_stats;
int orc_validate_index(const uint8_t *mmap, uint64_t file_len, int threads,
                       orc_stats *st);

#ifdef __cplusplus
}
#endif
#endif

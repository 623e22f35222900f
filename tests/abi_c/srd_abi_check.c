/*
 * A compiled C caller of the drop-in boundary (TEST INFRASTRUCTURE): built
 * against include/srd_amd.h and linked to libsrd_amd.so exactly as the Rust
 * binding in INTEGRATION.md would be, so the srd_result layout and the
 * calling convention are checked by a C compiler, not by ctypes mirrors.
 *
 *   srd_abi_check --layout
 *       prints sizeof / offsetof of srd_result and srd_write_entry (no GPU);
 *       the CPU test compares them with the #[repr(C)] layout INTEGRATION.md
 *       shows (and with the ctypes mirror).
 *   srd_abi_check STORE FINAL_LEN N_CHAIN N_INDEX [N_CTX]
 *       DataStore::open's pass over the file through srd_validate_index
 *       (N_CTX > 1: srd_validate_index_multi with N_CTX contexts on device
 *       0) and checks the counts plus the internal consistency of the
 *       arrays (chain in file order, every prev the previous tail, crc_ok ==
 *       (crc_computed == crc_stored), index offsets on the chain, tags
 *       = key_hash >> 48).  Exit 0 = ok.
 */
#include <inttypes.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srd_amd.h"

#define F(T, m) printf("\"%s.%s\": %zu, ", #T, #m, offsetof(T, m))

static int fail(const char *what) {
  fprintf(stderr, "srd_abi_check: %s (%s)\n", what, srd_last_error());
  return 1;
}

int main(int argc, char **argv) {
  if (argc == 2 && !strcmp(argv[1], "--layout")) {
    printf("{");
    F(srd_result, file_len); F(srd_result, final_len); F(srd_result, n_chain); F(srd_result, n_index);
    F(srd_result, n_crc_bad); F(srd_result, n_candidates); F(srd_result, full_reason); F(srd_result, mode);
    F(srd_result, reserved); F(srd_result, meta_off); F(srd_result, key_hash); F(srd_result, prev_offset);
    F(srd_result, payload_start); F(srd_result, payload_len); F(srd_result, crc_stored);
    F(srd_result, crc_computed); F(srd_result, crc_ok); F(srd_result, index_key_hash);
    F(srd_result, index_packed);
    F(srd_write_entry, src); F(srd_write_entry, len); F(srd_write_entry, key_src); F(srd_write_entry, tail);
    F(srd_write_entry, key_len); F(srd_write_entry, flags);
    F(srd_multi_summary, file_len); F(srd_multi_summary, final_len); F(srd_multi_summary, n_chain);
    F(srd_multi_summary, n_index); F(srd_multi_summary, n_crc_bad); F(srd_multi_summary, n_candidates);
    F(srd_multi_summary, mode); F(srd_multi_summary, path); F(srd_multi_summary, n_shards);
    F(srd_multi_summary, merged); F(srd_multi_summary, shard_errors); F(srd_multi_summary, peer_errors);
    F(srd_multi_summary, validate_ms); F(srd_multi_summary, exchange_ms); F(srd_multi_summary, total_ms);
    F(srd_multi_summary, index_key_hash); F(srd_multi_summary, index_packed);
    printf("\"sizeof(srd_result)\": %zu, \"sizeof(srd_write_entry)\": %zu, \"sizeof(srd_multi_summary)\": %zu}\n",
           sizeof(srd_result), sizeof(srd_write_entry), sizeof(srd_multi_summary));
    return 0;
  }
  if (argc < 5) {
    fprintf(stderr, "usage: %s --layout | STORE FINAL_LEN N_CHAIN N_INDEX [N_CTX]\n", argv[0]);
    return 2;
  }
  FILE *fp = fopen(argv[1], "rb");
  if (!fp) return fail("cannot open the store");
  fseek(fp, 0, SEEK_END);
  const long len = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  uint8_t *buf = (uint8_t *)malloc(len ? (size_t)len : 1);
  if (len && fread(buf, 1, (size_t)len, fp) != (size_t)len) return fail("short read");
  fclose(fp);
  const uint64_t want_final = strtoull(argv[2], 0, 10), want_chain = strtoull(argv[3], 0, 10),
                 want_index = strtoull(argv[4], 0, 10);
  const int nctx = argc > 5 ? atoi(argv[5]) : 1;
  if (nctx < 1 || nctx > 8) return fail("N_CTX must be 1..8");
  srd_ctx *ctx[8];
  for (int i = 0; i < nctx; i++)
    if (srd_ctx_create(0, &ctx[i]) != SRD_OK) return fail("srd_ctx_create");
  srd_result r;
  memset(&r, 0, sizeof r);
  const int rc = nctx == 1 ? srd_validate_index(ctx[0], buf, (uint64_t)len, 0, &r)
                           : srd_validate_index_multi(ctx, (uint32_t)nctx, buf, (uint64_t)len, 0, &r);
  if (rc != SRD_OK) return fail("srd_validate_index");
  int bad = 0;
  if (r.file_len != (uint64_t)len || r.final_len != want_final || r.n_chain != want_chain || r.n_index != want_index)
    bad |= 1;
  uint64_t prev_tail = 0, nbad = 0;
  for (uint64_t i = 0; i < r.n_chain; i++) {
    if (r.prev_offset[i] != prev_tail) bad |= 2;
    if (r.payload_start[i] + r.payload_len[i] != r.meta_off[i]) bad |= 4;
    if (r.crc_ok[i] != (r.crc_computed[i] == r.crc_stored[i])) bad |= 8;
    nbad += !r.crc_ok[i];
    prev_tail = r.meta_off[i] + 20;
  }
  if (r.n_chain && prev_tail != r.final_len) bad |= 16;
  if (nbad != r.n_crc_bad) bad |= 32;
  for (uint64_t i = 0; i < r.n_index; i++) {
    const uint64_t off = r.index_packed[i] & ((1ull << 48) - 1);
    if (r.index_packed[i] >> 48 != r.index_key_hash[i] >> 48) bad |= 64;
    if (i && off <= (r.index_packed[i - 1] & ((1ull << 48) - 1))) bad |= 128;  /* chain order */
    if (off >= r.final_len) bad |= 256;
  }
  /* the multi-GPU form: which path decided (composed shards / neighbour retry / whole file) */
  int path = -1;
  if (nctx > 1) {
    srd_multi_summary sm;
    if (srd_ctx_multi_summary(ctx[0], &sm) == SRD_OK) path = (int)sm.path;
  }
  printf("{\"final_len\": %" PRIu64 ", \"n_chain\": %" PRIu64 ", \"n_index\": %" PRIu64 ", \"n_crc_bad\": %" PRIu64
         ", \"mode\": %u, \"path\": %d, \"n_ctx\": %d, \"bad\": %d}\n",
         r.final_len, r.n_chain, r.n_index, r.n_crc_bad, r.mode, path, nctx, bad);
  srd_result_free(&r);
  for (int i = 0; i < nctx; i++) srd_ctx_destroy(ctx[i]);
  free(buf);
  return bad ? 1 : 0;
}

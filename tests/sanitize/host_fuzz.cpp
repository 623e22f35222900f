// ASan/UBSan harness for the host code that parses untrusted store bytes
// (TEST INFRASTRUCTURE).  Built by tests/sanitize/Makefile with
// -fsanitize=address,undefined -fno-sanitize-recover=all from the library's
// own host parser (rust-simd-r-drive_amd/csrc/srd_host.cpp) and the oracle
// (oracle/srd_oracle.c).  Runs over every file named on the command line
// (the golden fixtures, including the garbage one) and over random and
// mutated byte strings:
//   - srd_shard_cuts for world 1..9: returns 0, cuts[0] = 0, cuts[w] =
//     file_len, non-decreasing, every non-empty shard not starting at 0
//     (the whole-file rule) >= 21 bytes, every
//     inner cut passes the node test;
//   - srd_batch_layout over random key / payload tables (NULL-byte and empty
//     payloads included): the layout's tails follow prepad_len;
//   - the oracle's recover_valid_chain / chain / KeyIndexer::build.
// Exit status 0 = no sanitizer report and every invariant held.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "srd_host.h"

extern "C" {
#include "srd_oracle.h"
}

static int g_fail = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (!(c)) {                                                        \
      fprintf(stderr, "%s:%d: invariant failed: %s\n", __FILE__, __LINE__, #c); \
      g_fail = 1;                                                      \
    }                                                                  \
  } while (0)

static void check_store(const uint8_t* f, uint64_t n) {
  // heap copy of exactly n bytes so ASan sees any read past the end
  uint8_t* b = (uint8_t*)malloc(n ? n : 1);
  if (n) memcpy(b, f, n);
  for (uint32_t w = 1; w <= 9; w++) {
    std::vector<uint64_t> cuts(w + 1, 7);
    const char* why = "";
    EXPECT(srd_host::shard_cuts(b, n, w, cuts.data(), &why) == 0);
    EXPECT(cuts[0] == 0 && cuts[w] == n);
    for (uint32_t r = 0; r < w; r++) {
      EXPECT(cuts[r] <= cuts[r + 1]);
      EXPECT(cuts[r] == cuts[r + 1] || cuts[r] == 0 || cuts[r + 1] - cuts[r] >= 21);  // lo == 0: whole-file rule
      uint64_t p;
      if (r > 0 && cuts[r] != 0 && cuts[r] != cuts[r - 1]) EXPECT(srd_host::node_at(b, n, cuts[r], &p));
    }
  }
  const uint64_t t = orc_recover_valid_chain(b, n);
  EXPECT(t <= n);
  const uint64_t nc = orc_chain(b, t, nullptr, 0, 0);
  std::vector<orc_entry> e(nc ? nc : 1);
  EXPECT(orc_chain(b, t, e.data(), nc, 1) == nc);
  std::vector<uint64_t> k(nc ? nc : 1), v(nc ? nc : 1);
  EXPECT(orc_key_indexer_build(b, t, k.data(), v.data(), nc) <= nc);
  free(b);
}

static void check_layout(std::mt19937_64& rng) {
  const uint64_t n = rng() % 40;
  std::vector<uint8_t> pay(4096);
  for (auto& x : pay) x = (uint8_t)(rng() % 3 == 0 ? 0 : rng());
  std::vector<uint64_t> ko(n), kl(n), po(n), pl(n);
  for (uint64_t i = 0; i < n; i++) {
    ko[i] = rng() % 100;
    kl[i] = rng() % 40;
    pl[i] = rng() % 5 == 0 ? rng() % 2 : 1 + rng() % 1000;
    po[i] = rng() % (pay.size() - pl[i] + 1);
  }
  std::vector<srd_write_entry> out(n ? n : 1);
  uint64_t tail = rng() % 100000, nt = 0;
  const char* why = "";
  const uint32_t flags = (rng() & 1) ? SRD_WRITE_ALLOW_NULL : 0u;
  const int r = srd_host::batch_layout(tail, pay.data(), ko.data(), kl.data(), po.data(), pl.data(), n, flags,
                                       out.data(), &nt, &why);
  if (r == 0) {
    uint64_t t = tail;
    for (uint64_t i = 0; i < n; i++) {
      EXPECT(out[i].tail == t);
      t = (out[i].flags & SRD_ENTRY_TOMB) ? t + 21 : t + ((64 - (t & 63)) & 63) + pl[i] + 20;
    }
    EXPECT(t == nt);
  } else {
    EXPECT(r == SRD_ERR_ARG && why && *why);
  }
}

int main(int argc, char** argv) {
  std::mt19937_64 rng(12345);
  for (int i = 1; i < argc; i++) {
    FILE* fp = fopen(argv[i], "rb");
    if (!fp) { perror(argv[i]); return 2; }
    std::vector<uint8_t> d;
    uint8_t buf[65536];
    size_t got;
    while ((got = fread(buf, 1, sizeof buf, fp)) > 0) d.insert(d.end(), buf, buf + got);
    fclose(fp);
    check_store(d.data(), d.size());
    // truncations and byte mutations of the fixture
    for (int j = 0; j < 40 && !d.empty(); j++) {
      std::vector<uint8_t> m(d.begin(), d.begin() + (rng() % (d.size() + 1)));
      for (int q = 0; q < 3 && !m.empty(); q++) m[rng() % m.size()] ^= (uint8_t)(1u << (rng() % 8));
      check_store(m.data(), m.size());
    }
  }
  // random byte strings, zero-rich ones (small p fields everywhere) and
  // strings built from repeated forged metadata records
  for (int j = 0; j < 400; j++) {
    std::vector<uint8_t> m(rng() % 3000);
    const int kind = j % 3;
    for (size_t q = 0; q < m.size(); q++) m[q] = kind == 1 ? (uint8_t)(rng() % 8 == 0 ? rng() : 0) : (uint8_t)rng();
    if (kind == 2)
      for (size_t q = 20; q + 20 <= m.size(); q += 20 + rng() % 50) {
        const uint64_t prev = rng() % (q + 1);
        memcpy(&m[q + 8], &prev, 8);
      }
    check_store(m.data(), m.size());
  }
  for (int j = 0; j < 2000; j++) check_layout(rng);
  if (g_fail) return 1;
  printf("host_fuzz ok\n");
  return 0;
}

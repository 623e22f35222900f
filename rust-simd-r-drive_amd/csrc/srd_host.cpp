// srd_host.cpp -- host-only parsing of untrusted store bytes (srd_host.h).
// No HIP: built into the library and, alone, under ASan/UBSan.
#include "srd_host.h"

#include <string.h>

#include <algorithm>

namespace srd_host {

static inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

bool node_at(const uint8_t* f, uint64_t flen, uint64_t t, uint64_t* prev) {
  if (t < 20 || t > flen) return false;
  const uint64_t mo = t - 20, p = rd64(f + mo + 8);
  if (p >= mo) return false;
  // tombstone rule (data_store.rs:404-416): a 1-byte entry whose byte is 0
  // starts at prev itself; otherwise after prepad_len(prev) (:670-673)
  const uint64_t start = (mo - p == 1 && f[p] == 0) ? p : p + ((64 - (p & 63)) & 63);
  if (start >= mo) return false;
  *prev = p;
  return true;
}

// Shard boundaries: cut r is a guessed entry tail at or
// below r*file_len/world.  A byte t is taken as a tail when the backward walk
// from it passes the node test for kCutHops hops without reaching offset 0
// (zero-filled payloads, and CRC bytes read through a zero prepad, look like
// p = 0 / small-p nodes; an 8-hop walk rejects them).  The guess is checked,
// not trusted: the shards' chains compose only if every cut is the tail the
// real chain passes through, and otherwise the caller runs the whole-file
// path.  A non-empty shard is at least 21 bytes (one metadata record and a
// byte of payload): a cut closer than that to the previous one is no cut.
static constexpr int kCutHops = 8;
static constexpr uint64_t kCutScan = 64ull << 20;  // bytes searched below a cut target

static bool plausible_tail(const uint8_t* f, uint64_t flen, uint64_t t) {
  uint64_t cur = t;
  for (int h = 0; h < kCutHops; h++) {
    uint64_t p;
    if (!node_at(f, flen, cur, &p)) return false;
    if (p == 0) return false;
    cur = p;
  }
  return true;
}

int shard_cuts(const uint8_t* file, uint64_t flen, uint32_t world, uint64_t* cuts, const char** why) {
  if (!cuts || world == 0 || (!file && flen)) {
    *why = "bad argument";
    return SRD_ERR_ARG;
  }
  cuts[0] = 0;
  cuts[world] = flen;
  for (uint32_t r = 1; r < world; r++) {
    const uint64_t target = (uint64_t)(((unsigned __int128)flen * r) / world);
    uint64_t got = cuts[r - 1];  // none found: an empty shard
    const uint64_t lo = cuts[r - 1] + 20;  // t > lo: t >= previous cut + 21
    if (target > lo) {
      const uint64_t floor_ = std::max(lo, target > kCutScan ? target - kCutScan : 0);
      for (uint64_t t = target; t > floor_; t--)
        if (plausible_tail(file, flen, t)) { got = t; break; }
    }
    cuts[r] = got;
  }
  // the last shard [cuts[world-1], flen) must be empty or >= 21 bytes too
  for (uint32_t r = world - 1; r >= 1 && flen - cuts[r] < 21 && cuts[r] != flen; r--) cuts[r] = cuts[r - 1];
  return 0;
}

int batch_layout(uint64_t tail, const uint8_t* payloads, const uint64_t* key_offs, const uint64_t* key_lens,
                 const uint64_t* pay_offs, const uint64_t* pay_lens, uint64_t n, uint32_t flags,
                 srd_write_entry* out, uint64_t* new_tail, const char** why) {
  if (n && (!key_offs || !key_lens || !pay_offs || !pay_lens)) {
    *why = "bad argument";
    return SRD_ERR_ARG;
  }
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t len = pay_lens[i];
    if (key_lens[i] > 0xFFFFFFFFull) {
      *why = "key too long";
      return SRD_ERR_ARG;
    }
    srd_write_entry e{pay_offs[i], len, key_offs[i], tail, (uint32_t)key_lens[i], 0u};
    if (payloads && len == 1 && payloads[pay_offs[i]] == 0) {  // payload == NULL_BYTE (data_store.rs:864)
      if (!(flags & SRD_WRITE_ALLOW_NULL)) {
        *why = "NULL-byte payloads cannot be written directly.";
        return SRD_ERR_ARG;
      }
      e.flags = SRD_ENTRY_TOMB;
      tail += 1 + 20;  // no prepad for a tombstone (:871-895)
    } else {
      if (len == 0) {
        *why = "Payload cannot be empty.";
        return SRD_ERR_ARG;
      }
      tail += ((64 - (tail & 63)) & 63) + len + 20;  // prepad_len (:670-673), payload, metadata
    }
    if (out) out[i] = e;
  }
  if (new_tail) *new_tail = tail;
  return 0;
}

}  // namespace srd_host

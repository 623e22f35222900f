// srd_host.h -- host-only parsing of untrusted store bytes (no HIP).
//
// Compiled into libsrd_amd.so (through srd_api.hip) and, on its own with
// -fsanitize=address,undefined, into the sanitizer harness
// (tests/sanitize/host_fuzz.cpp): everything here reads file bytes the
// caller does not vouch for, so it must stay in bounds for any input.
#pragma once
#include <stdint.h>

#include "srd_amd.h"

namespace srd_host {

// recover_valid_chain's node test at tail t (data_store.rs:404-421,
// 429-470): the metadata [t-20, t) has prev p < t-20 and the entry's start
// (p itself for a tombstone, else p + prepad_len(p)) below t-20.
bool node_at(const uint8_t* f, uint64_t flen, uint64_t t, uint64_t* prev);

// srd_shard_cuts (include/srd_amd.h); *why gets the message of an error.
int shard_cuts(const uint8_t* file, uint64_t flen, uint32_t world, uint64_t* cuts, const char** why);

// srd_batch_layout (include/srd_amd.h)
int batch_layout(uint64_t tail, const uint8_t* payloads, const uint64_t* key_offs, const uint64_t* key_lens,
                 const uint64_t* pay_offs, const uint64_t* pay_lens, uint64_t n, uint32_t flags,
                 srd_write_entry* out, uint64_t* new_tail, const char** why);

}  // namespace srd_host

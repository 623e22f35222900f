/* Host overhead probe (timing tool): srd_validate_index_device in a tight C loop on the C2 store, timing level
 * 0 and 1 alternating inside ONE context (the per-context scan spread cancels); prints wall ms per call and the
 * scan's event ms.  Build: make -C tools c_loop (links the in-tree library and libamdhip64). */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include "srd_amd.h"

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

int main(void) {
  srd_ctx* c = NULL;
  if (srd_ctx_create(0, &c)) { fprintf(stderr, "ctx: %s\n", srd_last_error()); return 1; }
  const uint64_t n = 1u << 20;
  uint64_t len = 0;
  srd_synth_store_device(c, NULL, n, 4096, NULL, 0x5EED0001ull, &len);
  uint8_t* d = NULL;
  if (hipMalloc((void**)&d, srd_padded_size(len)) != hipSuccess) return 1;
  if (srd_synth_store_device(c, d, n, 4096, NULL, 0x5EED0001ull, &len)) { fprintf(stderr, "synth: %s\n", srd_last_error()); return 1; }
  hipDeviceSynchronize();
  srd_device_result r;
  double wall[2] = {0, 0}, scan = 0;
  int cnt[2] = {0, 0}, sl = 0;
  for (int round = 0; round < 12; round++) {
    for (int lvl = 0; lvl < 2; lvl++) {
      srd_ctx_set_timing(c, lvl);
      for (int i = 0; i < 3; i++) srd_validate_index_device(c, d, len, 0, &r);  // settle
      double s, ms; int k;
      srd_ctx_timings(c, &s, &k, &ms);
      const double t0 = now_ms();
      for (int i = 0; i < 20; i++) {
        if (srd_validate_index_device(c, d, len, 0, &r)) { fprintf(stderr, "validate: %s\n", srd_last_error()); return 1; }
      }
      const double dt = now_ms() - t0;
      if (r.final_len != len || r.n_chain != n || r.n_crc_bad) { fprintf(stderr, "bad result\n"); return 1; }
      if (round) {
        wall[lvl] += dt;
        cnt[lvl] += 20;
      }
      if (lvl == 1) {
        srd_ctx_timings(c, &s, &k, &ms);
        if (round) { scan += s; sl += k; }
      }
    }
  }
  printf("{\"c_wall_ms_per_call_level0\": %.4f, \"c_wall_ms_per_call_level1\": %.4f, \"scan_ms_events\": %.4f}\n",
         wall[0] / cnt[0], wall[1] / cnt[1], scan / sl);
  hipFree(d);
  srd_ctx_destroy(c);
  return 0;
}

// Read-bandwidth probe for the scan kernel's load structure (timing tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// A: lane owns a 64 B line, 4 x 16 B loads strided 64 B across lanes (scan v2 pattern)
template <bool NT>
__global__ __launch_bounds__(1024) void pat_line(const uint8_t* f, uint64_t ntiles, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  uint64_t w = blockIdx.x * 16 + (threadIdx.x >> 6), tw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t k = w; k < ntiles; k += tw) {
    const u32x4* q = (const u32x4*)(f + k * 4096 + 64 * lane);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      u32x4 v = NT ? __builtin_nontemporal_load(q + j) : q[j];
      acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}
// B: coalesced: instruction j covers bytes [1024 j, 1024 j + 1024) of the tile
template <bool NT>
__global__ __launch_bounds__(1024) void pat_coal(const uint8_t* f, uint64_t ntiles, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  uint64_t w = blockIdx.x * 16 + (threadIdx.x >> 6), tw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t k = w; k < ntiles; k += tw) {
    const u32x4* q = (const u32x4*)(f + k * 4096 + 16 * lane);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      u32x4 v = NT ? __builtin_nontemporal_load(q + 64 * j) : q[64 * j];
      acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}
// C: like B but each wave walks a contiguous span of 16 tiles (scan v2 span order)
template <bool NT>
__global__ __launch_bounds__(1024) void pat_coal_span(const uint8_t* f, uint64_t ntiles, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  uint64_t w = blockIdx.x * 16 + (threadIdx.x >> 6), tw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t sp = w; sp * 16 < ntiles; sp += tw)
    for (int t = 0; t < 16 && sp * 16 + t < ntiles; t++) {
      const u32x4* q = (const u32x4*)(f + (sp * 16 + t) * 4096 + 16 * lane);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        u32x4 v = NT ? __builtin_nontemporal_load(q + 64 * j) : q[64 * j];
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
      }
    }
  if (acc == 0x12345678) out[0] = acc;
}
// D: line pattern, span order (exactly scan v2's addressing)
template <bool NT>
__global__ __launch_bounds__(1024) void pat_line_span(const uint8_t* f, uint64_t ntiles, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  uint64_t w = blockIdx.x * 16 + (threadIdx.x >> 6), tw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t sp = w; sp * 16 < ntiles; sp += tw)
    for (int t = 0; t < 16 && sp * 16 + t < ntiles; t++) {
      const u32x4* q = (const u32x4*)(f + (sp * 16 + t) * 4096 + 64 * lane);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        u32x4 v = NT ? __builtin_nontemporal_load(q + j) : q[j];
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
      }
    }
  if (acc == 0x12345678) out[0] = acc;
}

#define CHK(x) do { hipError_t e = (x); if (e) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
  const uint64_t bytes = 4362076116ull & ~4095ull;
  const uint64_t ntiles = bytes / 4096;
  uint8_t* f; uint32_t* o;
  CHK(hipMalloc(&f, bytes)); CHK(hipMalloc(&o, 64));
  CHK(hipMemset(f, 1, bytes));
  hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  auto run = [&](const char* name, auto kern, int grid) {
    float best = 1e9;
    for (int r = 0; r < 6; r++) {
      hipEventRecord(a);
      kern<<<grid, 1024>>>(f, ntiles, o);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-22s grid %5d  %.3f ms  %.2f TB/s\n", name, grid, best, bytes / (best * 1e-3) / 1e12);
  };
  for (int g : {256, 512, 1024, 4096}) {
    run("line nt", pat_line<true>, g); run("line", pat_line<false>, g);
    run("coal nt", pat_coal<true>, g); run("coal", pat_coal<false>, g);
    run("coal_span nt", pat_coal_span<true>, g); run("coal_span", pat_coal_span<false>, g);
    run("line_span nt", pat_line_span<true>, g); run("line_span", pat_line_span<false>, g);
  }
  return 0;
}

// Read-bandwidth probe (timing tool): does the tile -> wave mapping matter
// when each tile also costs compute?  Line-per-lane loads (the scan's
// pattern), a 2-deep register ring, and D dependent VALU ops per tile.
//   grid-stride : wave w reads tiles w, w + W, w + 2W, ...
//   contiguous  : wave w reads one contiguous range (the scan's mapping)
//   chunk16     : wave w reads 16-tile chunks w, w + W, ...
#include <hip/hip_runtime.h>
#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void ld(const uint8_t* f, uint64_t k, int lane, u32x4 (&o)[4]) {
  const u32x4* q = (const u32x4*)(f + k * 4096 + 64 * lane);
#pragma unroll
  for (int j = 0; j < 4; j++) o[j] = q[j];
}
__device__ __forceinline__ uint32_t work(const u32x4 (&v)[4], uint32_t acc, int D) {
  uint32_t s = acc;
#pragma unroll
  for (int j = 0; j < 4; j++) s ^= v[j][0] ^ v[j][1] ^ v[j][2] ^ v[j][3];
  for (int i = 0; i < D; i++) s = __builtin_amdgcn_alignbit(s, s ^ i, 7) + 0x9E3779B9u;
  return s;
}
// MODE 0 grid-stride, 1 contiguous, 2 chunks of 16
template <int MODE>
__global__ __launch_bounds__(1024) void probe(const uint8_t* f, uint64_t ntiles, int D, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint64_t W = (uint64_t)gridDim.x * 16, w = blockIdx.x * 16 + (threadIdx.x >> 6);
  uint32_t acc = 0;
  auto tile_of = [&](uint64_t i) -> uint64_t {  // i-th tile of this wave
    if (MODE == 0) return w + i * W;
    if (MODE == 1) return w * ((ntiles + W - 1) / W) + i;
    return ((i / 16) * W + w) * 16 + (i % 16);
  };
  uint64_t n = MODE == 1 ? (ntiles + W - 1) / W : (MODE == 0 ? (ntiles - w + W - 1) / W : ntiles / (16 * W) * 16);
  if (MODE == 1) { uint64_t lo = w * n; n = lo >= ntiles ? 0 : (lo + n > ntiles ? ntiles - lo : n); }
  if (!n) return;
  u32x4 a[4], b[4];
  ld(f, tile_of(0), lane, a);
  for (uint64_t i = 0; i < n; i += 2) {
    ld(f, tile_of(i + 1 < n ? i + 1 : i), lane, b);
    acc = work(a, acc, D);
    if (i + 1 >= n) break;
    ld(f, tile_of(i + 2 < n ? i + 2 : i), lane, a);
    acc = work(b, acc, D);
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
  auto run = [&](const char* name, auto kern, int D) {
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(a);
      kern<<<256, 1024>>>(f, ntiles, D, o);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-12s D=%4d  %.3f ms  %.2f TB/s\n", name, D, best, bytes / (best * 1e-3) / 1e12);
  };
  for (int D : {0, 100, 200, 300, 400, 600}) {
    run("grid", probe<0>, D); run("contig", probe<1>, D); run("chunk16", probe<2>, D);
  }
  return 0;
}

// srd_probe.hip -- the streaming-read ceiling of scan_kernel's geometry, measured
// in the same process on the same bytes ("report against both
// the spec peak and a measured stream-read peak"; bench.py's roofline
// peak_measured / frac_measured).  Not part of the reference interface: a
// measurement of what the HBM gives the scan's access pattern when no work is
// done on the bytes.
//
// Geometry = the scan's: one 16-wave block per CU, every wave a contiguous,
// balanced range of 4 KiB tiles, the scan's loads (four 16-byte nontemporal
// loads per lane, every instruction 1 KiB contiguous: coal_lane_off), a
// 3-deep register ring (two tiles in flight while one is folded).  Each tile
// is XOR-folded into one register so the loads stay live (the fold is
// order-free: no transpose); one word per wave is stored only if the fold
// equals a magic value (never, in effect).
#pragma once

namespace srd {

__global__ __launch_bounds__(1024, 1) void stream_probe_kernel(const uint8_t* __restrict__ f, uint64_t ntiles,
                                                               uint32_t* out) {
  constexpr int D = 3;  // ring depth: D - 1 tiles in flight while one is folded
  const int lane = threadIdx.x & 63;
  const uint64_t tw = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t k0 = w * ntiles / tw, k1 = (w + 1) * ntiles / tw;
  if (k0 >= k1) return;
  auto ld = [&](uint64_t k, u32x4 (&o)[4]) {  // the product scan's loads (scan_kernel's load_tile)
    const uint8_t* tb = f + k * (uint64_t)TILE;
#pragma unroll
    for (int j = 0; j < 4; j++) o[j] = __builtin_nontemporal_load((const u32x4*)(tb + coal_lane_off(lane, j)));
  };
  u32x4 ring[D][4];
#pragma unroll
  for (int d = 0; d < D - 1; d++) ld(k0 + d < k1 ? k0 + d : k1 - 1, ring[d]);
  uint32_t acc = lane;
  for (uint64_t k = k0; k < k1; k += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
      const uint64_t kn = k + d + D - 1;
      ld(kn < k1 ? kn : k1 - 1, ring[(d + D - 1) % D]);  // (clamped past the range: re-reads the last tile)
      uint32_t x = acc;
#pragma unroll
      for (int j = 0; j < 4; j++) x ^= ring[d][j][0] ^ ring[d][j][1] ^ ring[d][j][2] ^ ring[d][j][3];
      acc = x;
    }
  }
  if (acc == 0x9E3779B9u) out[w] = acc;
}

}  // namespace srd

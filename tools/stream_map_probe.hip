// Streaming-read probe of the scan's geometry under three tile -> wave maps
// and a per-tile VALU "compute" load (timing tool, not product code).
//   contig : every wave a contiguous range of tiles (the scan's map today)
//   blockil: every block a contiguous range, its 16 waves taking the tiles
//            round-robin (the block streams one front)
//   global : wave w takes tiles w, w + W, w + 2W ... (one front for the chip)
// Per tile: lane l loads line l as four 16-byte loads, a 3-deep register ring
// (the scan's), an XOR fold, then N dependent VALU ops (the compute stand-in).
// Question: does spreading each wave's loads in time (N > 0) cost bandwidth
// by itself, and does the map change that?
// build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_map_probe tools/stream_map_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t TILE = 4096;

// Coalesced pieces -> line per lane.  Lane l = 16A + 4B + C holds, in piece
// j (register field R), quarter C of line 16j + 4A + B (the load at 1024 j +
// 16 l).  Three 2x2-field swaps rotate (R, A, B, C) -> (C, R, A, B): lane L
// then holds line L, quarter q in piece q.
template <int CTRL>
__device__ __forceinline__ uint32_t dppv(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
template <int S, int RB>
__device__ __forceinline__ void tswap(u32x4 (&o)[4], int lane) {  // register bit RB <-> lane bit S (S = 1, 2, 4, 8)
  constexpr int CD = S == 1 ? 0xA0 : S == 2 ? 0x44 : S == 4 ? 0x114 : 0x118;  // lane l <- l - S
  constexpr int CU = S == 1 ? 0xF5 : S == 2 ? 0xEE : S == 4 ? 0x104 : 0x108;  // lane l <- l + S
  const bool hi = (lane & S) != 0, lo = !hi;
  // (the DPP value as the select's FALSE operand: v_cndmask_b32_dpp)
#pragma unroll
  for (int r0 = 0; r0 < 4; r0++) {
    if (r0 & RB) continue;
    const int r1 = r0 | RB;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t a = o[r0][i], b = o[r1][i];
      o[r0][i] = lo ? a : dppv<CD>(b);
      o[r1][i] = hi ? b : dppv<CU>(a);
    }
  }
}
template <int RB, bool P32>
__device__ __forceinline__ void pswap(u32x4 (&o)[4]) {  // register bit RB <-> lane bit 4 (P32: 5)
#pragma unroll
  for (int r0 = 0; r0 < 4; r0++) {
    if (r0 & RB) continue;
    const int r1 = r0 | RB;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const auto w = P32 ? __builtin_amdgcn_permlane32_swap(o[r0][i], o[r1][i], false, false)
                         : __builtin_amdgcn_permlane16_swap(o[r0][i], o[r1][i], false, false);
      o[r0][i] = w[0];
      o[r1][i] = w[1];
    }
  }
}
__device__ __forceinline__ void coal_to_lines(u32x4 (&o)[4], int lane) {
  pswap<1, false>(o);  // R bit 0 <-> lane bit 4
  pswap<2, true>(o);   // R bit 1 <-> lane bit 5
  tswap<4, 1>(o, lane);
  tswap<8, 2>(o, lane);
  tswap<1, 1>(o, lane);
  tswap<2, 2>(o, lane);
}

// The cheaper transpose: the load puts the quarter in lane bits 2-3 (lane l
// = 16A + 4B + C loads 16 B at 1024 j + 256 A + 64 C + 16 B: each 16-lane row
// still reads 256 contiguous bytes), so (R, A, B, C) -> (B, R, A, C) needs
// two field swaps: A by permlane swaps, B by DPP moves under bank masks
// (bank = lane bits 2-3): 16 + 32 VALU, no selects.
template <int S, int RB>
__device__ __forceinline__ void bswap(u32x4 (&o)[4]) {  // register bit RB <-> lane bit S (S = 4, 8)
  constexpr int SHL = 0x100 + S, SHR = 0x110 + S;
  constexpr int HI = S == 4 ? 0xA : 0xC, LO = S == 4 ? 0x5 : 0x3;  // banks with / without lane bit S
#pragma unroll
  for (int r0 = 0; r0 < 4; r0++) {
    if (r0 & RB) continue;
    const int r1 = r0 | RB;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int a = (int)o[r0][i], b = (int)o[r1][i];
      o[r0][i] = (uint32_t)__builtin_amdgcn_update_dpp(a, b, SHR, 0xF, HI, false);  // hi lanes <- b[l - S]
      o[r1][i] = (uint32_t)__builtin_amdgcn_update_dpp(b, a, SHL, 0xF, LO, false);  // lo lanes <- a[l + S]
    }
  }
}
__device__ __forceinline__ uint32_t coal2_off(int lane, int j) {
  return 1024u * j + 256u * ((uint32_t)lane >> 4) + 64u * ((uint32_t)lane & 3) + 16u * (((uint32_t)lane >> 2) & 3);
}
__device__ __forceinline__ void coal2_to_lines(u32x4 (&o)[4]) {
  pswap<1, false>(o);
  pswap<2, true>(o);
  bswap<4, 1>(o);
  bswap<8, 2>(o);
}

// Quarter in lane bits 4-5: lane l = 16A + m loads 16 B at 1024 j + 64 m +
// 16 A (quarter A of line 16 j + m; each instruction still reads 1 KiB
// contiguous, a 16-lane row reads every 4th 16-byte piece of it), so one
// register <-> lane-field swap (v_permlane16/32_swap, 16 instructions)
// puts line L in lane L.
__device__ __forceinline__ uint32_t coal3_off(int lane, int j) {
  return 1024u * j + 64u * ((uint32_t)lane & 15u) + 16u * ((uint32_t)lane >> 4);
}
__device__ __forceinline__ void coal3_to_lines(u32x4 (&o)[4]) {
  pswap<1, false>(o);
  pswap<2, true>(o);
}

// verification: every lane's 16 dwords, loaded line-per-lane and coalesced + transposed
__global__ __launch_bounds__(256) void verify_transpose(const uint8_t* f, uint64_t ntiles, unsigned long long* bad) {
  const int lane = threadIdx.x & 63;
  const uint64_t k = (blockIdx.x * 4ull + (threadIdx.x >> 6)) % ntiles;
  const uint8_t* t = f + k * TILE;
  u32x4 a[4], c[4];
#pragma unroll
  for (int j = 0; j < 4; j++) a[j] = ((const u32x4*)(t + 64ull * lane))[j];
#pragma unroll
  for (int j = 0; j < 4; j++) c[j] = __builtin_nontemporal_load((const u32x4*)(t + 1024ull * j + 16ull * lane));
  if (bad[1] == 2) {
#pragma unroll
    for (int j = 0; j < 4; j++) c[j] = __builtin_nontemporal_load((const u32x4*)(t + coal3_off(lane, j)));
    coal3_to_lines(c);
  } else if (bad[1] == 1) {  // the cheaper pattern
#pragma unroll
    for (int j = 0; j < 4; j++) c[j] = __builtin_nontemporal_load((const u32x4*)(t + coal2_off(lane, j)));
    coal2_to_lines(c);
  } else {
    coal_to_lines(c, lane);
  }
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int i = 0; i < 4; i++) m += a[j][i] != c[j][i];
  if (m) atomicAdd(bad, (unsigned long long)m);
}

template <int MAP, int N, int D, int R = 0, int ST = 0, int LD = 0>
__global__ __launch_bounds__(1024, 1) void probe(const uint8_t* __restrict__ f, uint64_t ntiles, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  __shared__ uint32_t tab[R ? 8192 : 1];  // R > 0: 32 KiB lookup table for the LDS-chain compute
  if (R) {
    for (int i = threadIdx.x; i < (R ? 8192 : 1); i += 1024) tab[i] = (uint32_t)i * 0x9E3779B1u;
    __syncthreads();
  }
  const uint64_t W = (uint64_t)gridDim.x * 16, wl = threadIdx.x >> 6, w = (uint64_t)blockIdx.x * 16 + wl;
  uint64_t k0, k1, step;
  if (MAP == 0) {
    k0 = w * ntiles / W; k1 = (w + 1) * ntiles / W; step = 1;
  } else if (MAP == 1) {
    const uint64_t b0 = blockIdx.x * ntiles / gridDim.x, b1 = (blockIdx.x + 1) * ntiles / gridDim.x;
    k0 = b0 + wl; k1 = b1; step = 16;
  } else if (MAP == 2) {
    k0 = w; k1 = ntiles; step = W;
  } else {  // 3: the contig map's tile count, the loads from two L2-resident tiles per block (compute alone)
    k0 = w * ntiles / W; k1 = (w + 1) * ntiles / W; step = 1;
  }
  if (k0 >= k1) return;
  const uint64_t last = k0 + (k1 - 1 - k0) / step * step;
  auto ld = [&](uint64_t k, u32x4 (&o)[4]) {
    // LD 0: the scan's 64 B per lane; 1: the same, nontemporal; 2: coalesced (1 KiB per
    // instruction, 16 B per lane at 1024 j + 16 l); 3: coalesced, nontemporal
    const uint8_t* t = f + (MAP == 3 ? 2 * blockIdx.x + (k & 1) : k) * TILE;
    if constexpr (LD == 302 || LD == 303) {  // 303: the loads alone (no transpose)
#pragma unroll
      for (int j = 0; j < 4; j++) o[j] = __builtin_nontemporal_load((const u32x4*)(t + coal3_off(lane, j)));
      if (LD == 302) coal3_to_lines(o);
    } else if constexpr (LD == 301) {
#pragma unroll
      for (int j = 0; j < 4; j++) o[j] = __builtin_nontemporal_load((const u32x4*)(t + coal2_off(lane, j)));
      coal2_to_lines(o);
    } else if constexpr (LD == 300) {  // coalesced nontemporal + the register transpose (line per lane)
#pragma unroll
      for (int j = 0; j < 4; j++) o[j] = __builtin_nontemporal_load((const u32x4*)(t + 1024ull * j + 16ull * lane));
      coal_to_lines(o, lane);
    } else if constexpr (LD >= 100) {  // buffer loads, cache policy aux = LD % 100; LD >= 200: coalesced
      constexpr int AUX = LD % 100;
      constexpr bool CO = LD >= 200;
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)t, (short)0, 4096, 0x00020000);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t off = CO ? 1024u * j + 16u * lane : 64u * lane + 16u * j;
        o[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX));
      }
    } else {
    const u32x4* q = (const u32x4*)(t + (LD >= 2 ? 16ull : 64ull) * lane);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const u32x4* pj = q + (LD >= 2 ? 64 * j : j);
      o[j] = (LD & 1) ? __builtin_nontemporal_load(pj) : *pj;
    }
    }
  };
  u32x4 ring[D][4];
#pragma unroll
  for (int d = 0; d < D - 1; d++) {
    const uint64_t kn = k0 + d * step;
    ld(kn <= last ? kn : last, ring[d]);
  }
  uint32_t acc = lane, c = lane;
  for (uint64_t k = k0; k <= last; k += D * step) {
#pragma unroll
    for (int d = 0; d < D; d++) {
      const uint64_t kn = k + (d + D - 1) * step;
      ld(kn <= last ? kn : last, ring[(d + D - 1) % D]);
      uint32_t x = acc;
#pragma unroll
      for (int j = 0; j < 4; j++) x ^= ring[d][j][0] ^ ring[d][j][1] ^ ring[d][j][2] ^ ring[d][j][3];
      acc = x;
#pragma unroll
      for (int i = 0; i < N; i++) asm volatile("v_add_u32 %0, 7, %0" : "+v"(c));
      if (ST == 1) {  // 64 B per tile written (lanes 0-3, 16 B each, the wave's output contiguous): the scan's ~1.5 %
        if (lane < 4) ((u32x4*)out)[(k + d) * 4 + lane] = u32x4{x, c, x ^ c, acc};
      } else if (ST == 2) {  // the same bytes, 192 B by lanes 0-11 every third tile (a store point per ring round)
        if (d == D - 1 && lane < 12) ((u32x4*)out)[(k + d) * 4 - 8 + lane] = u32x4{x, c, x ^ c, acc};
      } else if (ST == 3) {  // the same bytes, 4 KiB (every lane 64 B) every 64 tiles
        if (((k + d - k0) & 63) == 63) {
          u32x4* o = (u32x4*)out + (k + d - 63) * 4 + 4 * lane;
#pragma unroll
          for (int j = 0; j < 4; j++) o[j] = u32x4{x, c, x ^ c, acc + j};
        }
      } else if (ST == 4) {  // 64 B per tile as nontemporal stores
        if (lane < 4) __builtin_nontemporal_store(u32x4{x, c, x ^ c, acc}, (u32x4*)out + (k + d) * 4 + lane);
      } else if (ST == 5) {  // 16 KiB (every lane 256 B) every 256 tiles
        if (((k + d - k0) & 255) == 255) {
          u32x4* o = (u32x4*)out + (k + d - 255) * 4 + 16 * lane;
#pragma unroll
          for (int j = 0; j < 16; j++) o[j] = u32x4{x, c, x ^ c, acc + j};
        }
      }
      if (R) {  // R rounds of 16 data-dependent LDS lookups (4 chains x 4), like the CRC's slice-by-4 levels
        uint32_t a4[4] = {x, x * 3u, x * 5u, x * 7u};
#pragma unroll
        for (int r = 0; r < R; r++) {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint32_t v = a4[q];
            a4[q] = tab[(v & 0x1FFF)] ^ tab[((v >> 8) & 0x1FFF)] ^ tab[((v >> 16) & 0x1FFF)] ^ tab[((v >> 19) & 0x1FFF)];
          }
        }
        c ^= a4[0] ^ a4[1] ^ a4[2] ^ a4[3];
      }
    }
  }
  if ((acc ^ c) == 0x9E3779B9u) out[w] = acc;
}

template <int MAP, int N, int D = 3, int R = 0, int ST = 0, int LD = 0>
static float run(const uint8_t* f, uint64_t nt, uint32_t* out, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> v;
  for (int r = 0; r < 7; r++) {
    hipEventRecord(a);
    probe<MAP, N, D, R, ST, LD><<<blocks, 1024>>>(f, nt, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

template <int N, int LD>
static void row(const uint8_t* f, uint64_t nt, uint32_t* out, int blocks, double bytes) {
  const float m0 = run<0, N, 3, 0, 0, LD>(f, nt, out, blocks), m1 = run<0, N, 3, 0, 1, LD>(f, nt, out, blocks),
              m3 = run<0, N, 3, 0, 3, LD>(f, nt, out, blocks), m4 = run<0, N, 3, 0, 4, LD>(f, nt, out, blocks),
              m5 = run<0, N, 3, 0, 5, LD>(f, nt, out, blocks);
  printf("N=%4d LD=%3d  no stores %.4f ms | 64 B/tile %+.1f %% | 4 KiB / 64 tiles %+.1f %% | 64 B/tile nt %+.1f %% | 16 KiB / 256 tiles %+.1f %%\n",
         N, LD, m0, 100.0 * (m1 / m0 - 1), 100.0 * (m3 / m0 - 1), 100.0 * (m4 / m0 - 1), 100.0 * (m5 / m0 - 1));
  fflush(stdout);
}

template <int N, int LD>
static void rowp(const uint8_t* f, uint64_t nt, uint32_t* out, int blocks, double bytes) {
  const float m0 = run<0, N, 3, 0, 0, LD>(f, nt, out, blocks);
  printf("N=%4d LD=%3d  %.4f ms (%.0f GB/s)\n", N, LD, m0, bytes / m0 / 1e6);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const uint64_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4362076116ull, nt = (bytes + TILE - 1) / TILE;
  uint8_t* f;
  uint32_t* out;
  if (hipMalloc(&f, nt * TILE + 3 * TILE) != hipSuccess || hipMalloc(&out, (nt + 64) * 64) != hipSuccess) return 1;
  hipMemset(f, 0x5a, nt * TILE + 3 * TILE);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount;
  printf("CUs %d, tiles %llu, bytes %llu\n", blocks, (unsigned long long)nt, (unsigned long long)(nt * TILE));
  const double b = (double)(nt * TILE);
  {  // distinct bytes per position, then the transpose check
    std::vector<uint32_t> h(1 << 20);
    for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
    hipMemcpy(f, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    unsigned long long* bad;
    hipMalloc(&bad, 16);
    for (unsigned long long mode = 0; mode < 3; mode++) {
      unsigned long long hb[2] = {0, mode};
      hipMemcpy(bad, hb, 16, hipMemcpyHostToDevice);
      verify_transpose<<<256, 256>>>(f, 1024, bad);
      hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost);
      printf("transpose %s check over 1024 tiles: %llu mismatching dwords\n", mode == 2 ? "permlane-only" : mode ? "2-swap" : "3-swap", hb[0]);
    }
  }
  rowp<0, 0>(f, nt, out, blocks, b);
  rowp<0, 3>(f, nt, out, blocks, b);
  rowp<0, 301>(f, nt, out, blocks, b);
  rowp<0, 302>(f, nt, out, blocks, b);
  rowp<0, 303>(f, nt, out, blocks, b);
  rowp<256, 0>(f, nt, out, blocks, b);
  rowp<256, 3>(f, nt, out, blocks, b);
  rowp<256, 301>(f, nt, out, blocks, b);
  rowp<256, 302>(f, nt, out, blocks, b);
  rowp<256, 303>(f, nt, out, blocks, b);
  rowp<512, 0>(f, nt, out, blocks, b);
  rowp<512, 3>(f, nt, out, blocks, b);
  rowp<512, 301>(f, nt, out, blocks, b);
  rowp<512, 302>(f, nt, out, blocks, b);
  rowp<512, 303>(f, nt, out, blocks, b);
  return 0;
}

// smfmac_rate.hip — cycles per v_smfmac_i32_32x32x64_i8 per SIMD in the scan's
// shape: KS-step accumulation chains over KS distinct random B fragments
// (registers), three waves per SIMD, with and without the per-tile zeroing
// and min-test of the accumulator.  Diagnostic only (s_memtime: shader
// cycles, clock-independent).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/smfmac_rate tools/smfmac_rate.hip && ./tools/smfmac_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int KS = 13;
constexpr int TILES = 4096;

// MODE 0: one long chain over the KS B fragments (no per-tile work)
// MODE 1: per tile: zero the accumulator, KS steps, min of the 16 sums + ballot
// MODE 2: as 1 with two accumulators (tile t+1's chain beside tile t's test)
// MODE 3: as 1 with the operands read from the scan's two 16-entry LDS
//         tables by random code bytes (3 reads in flight), as in the scan
// MODE 4: v_smfmac_i32_16x16x128_i8 (the 16-slot tiles), two chains in turn
//         as in the 16-slot scan, operands in registers (one long chain)
template <int MODE>
__global__ void __launch_bounds__(768) rate(const int* __restrict__ rnd, long long* cycles,
                                            int* sink) {
  const int lane = threadIdx.x & 63;
  v8i b[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) b[s][j] = rnd[(s * 8 + j) * 64 + lane];
  v4i a = {rnd[lane] & 0x00010001, rnd[64 + lane] & 0x00010001, 0x00010000, 0x1};
  int ix = rnd[128 + lane];
  v16i acc = v16i{0}, acc2 = v16i{0};
  unsigned long long hits = 0;
  __shared__ __align__(256) v4i grp_tab[16];
  __shared__ int pos_tab[16];
  if (threadIdx.x < 16) {
    const uint32_t g0 = threadIdx.x & 3u, g1 = threadIdx.x >> 2;
    v4i tt = {0, 0, 0, 0};
    tt[g0 >> 1] = int(1u << (16 * (g0 & 1u)));
    tt[2 + (g1 >> 1)] = int(1u << (16 * (g1 & 1u)));
    grp_tab[threadIdx.x] = tt;
    pos_tab[threadIdx.x] = int((threadIdx.x & 3u) * 0x5555u | ((threadIdx.x >> 2) * 0x5555u) << 16);
  }
  __syncthreads();
  uint32_t codes[4] = {uint32_t(rnd[lane]), uint32_t(rnd[64 + lane]), uint32_t(rnd[128 + lane]),
                       uint32_t(rnd[192 + lane])};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < TILES; ++t) {
    if (MODE >= 1) acc = v16i{0};
    if (MODE == 3) {
      constexpr int R = 3;
      auto grp = [&](int q) { return (codes[q >> 2] >> ((q & 3) * 8)) & 0xFu; };
      auto pos = [&](int q) { return (codes[q >> 2] >> ((q & 3) * 8 + 4)) & 0xFu; };
      v4i o[R];
      int ixr[R];
#pragma unroll
      for (int q = 0; q < R; ++q) {
        o[q] = grp_tab[grp(q)];
        ixr[q] = pos_tab[pos(q)];
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc = __builtin_amdgcn_smfmac_i32_32x32x64_i8(o[s % R], b[s], acc, ixr[s % R], 0, 0);
        if (s + R < KS) {
          o[s % R] = grp_tab[grp(s + R)];
          ixr[s % R] = pos_tab[pos(s + R)];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) codes[q] = codes[q] * 1664525u + 1013904223u;
    } else if (MODE == 4) {
      v4i acc_a = {acc[0], acc[1], acc[2], acc[3]}, acc_b = {acc[4], acc[5], acc[6], acc[7]};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc_a = __builtin_amdgcn_smfmac_i32_16x16x128_i8(a, b[s], acc_a, ix, 0, 0);
        // (chain B on other B fragments: identical chains would be merged)
        acc_b = __builtin_amdgcn_smfmac_i32_16x16x128_i8(a, b[KS - 1 - s], acc_b, ix, 0, 0);
        a[0] += 0x00010000;
      }
      acc[0] = acc_a[0]; acc[1] = acc_a[1]; acc[2] = acc_a[2]; acc[3] = acc_a[3];
      acc[4] = acc_b[0]; acc[5] = acc_b[1]; acc[6] = acc_b[2]; acc[7] = acc_b[3];
    } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      acc = __builtin_amdgcn_smfmac_i32_32x32x64_i8(a, b[s], acc, ix, 0, 0);
      a[0] += 0x00010000;
    }
    }
    if (MODE >= 1) {
      int m = acc[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) m = min(m, acc[i]);
      hits += __popcll(__builtin_amdgcn_ballot_w64(m < -1000));
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  int x = int(hits);
#pragma unroll
  for (int j = 0; j < 16; ++j) x ^= acc[j] ^ acc2[j];
  if (lane == 0) cycles[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
  if (x == 0x12345) sink[0] = x;
}

template <int MODE>
void run(const int* d_rnd, int waves_per_simd, const char* name) {
  long long* d;
  int* s;
  const int blocks = 256;
  const int threads = 64 * 4 * waves_per_simd;
  CHECK(hipMalloc(&d, sizeof(long long) * blocks * threads / 64));
  CHECK(hipMalloc(&s, 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(rate<MODE>, dim3(blocks), dim3(threads), 0, 0, d_rnd, d, s);
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(rate<MODE>, dim3(blocks), dim3(threads), 0, 0, d_rnd, d, s);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 3;
  static long long h[8192];
  const int nw = blocks * threads / 64;
  CHECK(hipMemcpy(h, d, sizeof(long long) * nw, hipMemcpyDeviceToHost));
  double m = 0;
  for (int i = 0; i < nw; ++i) m += double(h[i]) / nw;
  const int per_tile = MODE == 4 ? 2 * KS : KS;   // smfmacs per tile
  const double per = m / (double(TILES) * per_tile);
  // wall: the smfmacs of a CU's waves over its 4 SIMDs, at the in-kernel clock
  const double per_simd_smfmac = double(TILES) * per_tile * waves_per_simd;
  const double wall_cyc = per / waves_per_simd;   // memtime basis
  printf("%-34s %d wave(s)/SIMD: %6.1f memtime cycles per smfmac per wave, %6.1f per SIMD; "
         "wall %.3f ms = %.2f ns per smfmac per SIMD (%.0f smfmac/SIMD)\n", name,
         waves_per_simd, per, wall_cyc, ms, ms * 1e6 / per_simd_smfmac, per_simd_smfmac);
  CHECK(hipFree(d));
  CHECK(hipFree(s));
}

int main() {
  int* d_rnd;
  const int n = 64 * 8 * KS + 256;
  int* h = new int[n];
  unsigned x = 2463534242u;
  for (int i = 0; i < n; ++i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; h[i] = int(x); }
  CHECK(hipMalloc(&d_rnd, n * 4));
  CHECK(hipMemcpy(d_rnd, h, n * 4, hipMemcpyHostToDevice));
  for (int w = 1; w <= 3; ++w) {
    run<0>(d_rnd, w, "chain, 13 random B");
    run<1>(d_rnd, w, "per-tile zero + min test");
    run<3>(d_rnd, w, "+ LDS operand tables (scan)");
    run<4>(d_rnd, w, "16x16x128 chains A/B, 26 per tile");
  }
  return 0;
}

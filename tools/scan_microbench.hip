// scan_microbench.hip — ablation of the LUT16 scan inner loop on MI355X.
//
// Glove-shaped synthetic work: 4000 work items, each = 32 query LUTs (K=25
// steps of 2 blocks) x 37 consecutive 32-datapoint code tiles (1 KiB each).
// Variants (template bit mask) remove one component at a time so the time of
// each is visible:  LOAD (code tiles from HBM/L2), ONEHOT (VALU expansion),
// MFMA (i32_32x32x32_i8), EPI (threshold compare of the 16 sums per lane).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/smb tools/scan_microbench.hip && /tmp/smb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int K = 25;
constexpr int NW = 4;
constexpr int W = 16;
enum { LOAD = 1, ONEHOT = 2, MFMA = 4, EPI = 8, ALL = 15, TWOACC = 16, M16 = 32 };

__device__ __forceinline__ v4i OneHot64(uint32_t sh) {
  const uint64_t x = 1ull << (sh & 63u);
  const uint32_t lo = uint32_t(x), hi = uint32_t(x >> 32);
  const uint32_t m = 0u - ((sh >> 6) & 1u);
  v4i r;
  r[0] = int(lo & ~m);
  r[1] = int(hi & ~m);
  r[2] = int(lo & m);
  r[3] = int(hi & m);
  return r;
}

template <int V>
__global__ void __launch_bounds__(256) scan(const uint8_t* __restrict__ tiles, const uint32_t* __restrict__ item_tile,
                                           const int8_t* __restrict__ lut, unsigned* counter, unsigned items,
                                           int ntile, int* out) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  int sink = 0;
  for (;;) {
    unsigned w = 0;
    if (lane == 0) w = atomicAdd(counter, 1u);
    w = __builtin_amdgcn_readfirstlane(__shfl(w, 0));
    if (w >= items) break;
    const int q = (w * 32 + (lane & 31)) % 1000;
    v4i frag[K];
    const v4i* lrow = reinterpret_cast<const v4i*>(lut + size_t(q) * 2 * K * 16);
#pragma unroll
    for (int s = 0; s < K; ++s) frag[s] = lrow[2 * s + h];
    const uint8_t* tb = tiles + size_t(item_tile[w]) * 64 * W + lane * W;
    uint32_t codes[NW], next[NW];
    if (V & LOAD) {
      const uint4 v = *reinterpret_cast<const uint4*>(tb);
      codes[0] = v.x; codes[1] = v.y; codes[2] = v.z; codes[3] = v.w;
    } else {
      for (int i = 0; i < NW; ++i) codes[i] = lane * 0x9E3779B9u + i;
    }
    const int amax = -100000 + (w & 1);
    for (int j = 0; j < ntile; ++j) {
      if ((V & LOAD) && j + 1 < ntile) {
        const uint4 v = *reinterpret_cast<const uint4*>(tb + size_t(j + 1) * 64 * W);
        next[0] = v.x; next[1] = v.y; next[2] = v.z; next[3] = v.w;
      } else {
        for (int i = 0; i < NW; ++i) next[i] = codes[i] * 3u + j;
      }
      v16i acc = {0}, acc2 = {0};
      typedef int v4 __attribute__((ext_vector_type(4)));
      v4 c16[4] = {{0}, {0}, {0}, {0}};
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int sh = (s & 7) * 4;
        const uint32_t wv = codes[s >> 3];
        const uint32_t e8 = sh >= 3 ? ((wv >> (sh - 3)) & 0x78u) : ((wv << 3) & 0x78u);
        v4i a;
        if (V & ONEHOT) {
          a = OneHot64(e8);
        } else {
          a[0] = int(wv); a[1] = int(wv >> 1); a[2] = int(wv >> 2); a[3] = int(wv >> 3);
        }
        if ((V & MFMA) && (V & M16)) {
          // same op count: 4 x 16x16x64 per 32x32x32 (16 dps x 16 queries x 4 blocks each)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            c16[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, frag[(s + t) % K], c16[t], 0, 0, 0);
        } else if ((V & MFMA) && (V & TWOACC) && (s & 1)) {
          acc2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, frag[s], acc2, 0, 0, 0);
        } else if (V & MFMA) {
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, frag[s], acc, 0, 0, 0);
        } else {
          acc[s & 15] += a[0] ^ a[1] ^ a[2] ^ a[3] ^ frag[s][s & 3];
        }
      }
      if (V & TWOACC) acc += acc2;
      if (V & M16) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] += c16[t][0] + c16[t][1] + c16[t][2] + c16[t][3];
      }
      if (V & EPI) {
        uint32_t pass = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) pass |= uint32_t(acc[i] <= amax) << i;
        if (pass) sink += __popc(pass);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) sink ^= acc[i];
      }
      for (int i = 0; i < NW; ++i) codes[i] = next[i];
    }
  }
  if (sink == 0x7fffffff) out[0] = sink;
}

template <int V>
float Run(const char* name, const uint8_t* tiles, const uint32_t* item_tile, const int8_t* lut, unsigned* counter,
          unsigned items, int ntile, int* out, int grid, double flops) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipMemset(counter, 0, 4));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(scan<V>, dim3(grid), dim3(256), 0, 0, tiles, item_tile, lut, counter, items, ntile, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  printf("%-28s %8.1f us   %7.1f TOPS(i8 mfma-equivalent)\n", name, best * 1000.0f, flops / (best * 1e-3) / 1e12);
  return best;
}

int main(int argc, char** argv) {
  const unsigned items = argc > 1 ? atoi(argv[1]) : 4000;
  const int ntile = argc > 2 ? atoi(argv[2]) : 37;
  const int total_tiles = 37000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  std::vector<uint8_t> h_tiles(size_t(total_tiles) * 64 * W);
  for (size_t i = 0; i < h_tiles.size(); ++i) h_tiles[i] = uint8_t(i * 2654435761u >> 13);
  std::vector<uint32_t> h_item(items);
  for (unsigned i = 0; i < items; ++i) h_item[i] = (i * 7919u) % (total_tiles - ntile);
  std::vector<int8_t> h_lut(1000 * 2 * K * 16);
  for (size_t i = 0; i < h_lut.size(); ++i) h_lut[i] = int8_t((i * 31) % 255 - 127);
  uint8_t* tiles;
  uint32_t* item;
  int8_t* lut;
  unsigned* counter;
  int* out;
  CHECK(hipMalloc(&tiles, h_tiles.size()));
  CHECK(hipMalloc(&item, 4 * items));
  CHECK(hipMalloc(&lut, h_lut.size()));
  CHECK(hipMalloc(&counter, 4));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemcpy(tiles, h_tiles.data(), h_tiles.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(item, h_item.data(), 4 * items, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(lut, h_lut.data(), h_lut.size(), hipMemcpyHostToDevice));
  const double flops = double(items) * ntile * K * 2.0 * 32 * 32 * 32;
  const int cus = prop.multiProcessorCount;
  printf("CUs %d, items %u x %d tiles x K=%d: %.2e MFMA ops; ideal @5 POPS = %.1f us\n", cus, items, ntile, K,
         flops, flops / 5.0e15 * 1e6);
  for (int grid : {cus * 2, cus * 4}) {
    printf("-- grid %d blocks of 4 waves\n", grid);
    Run<ALL>("full", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<ALL & ~EPI>("no epilogue", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<ALL & ~LOAD>("no code loads", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<ALL & ~ONEHOT>("no one-hot", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<ALL & ~MFMA>("no mfma (VALU stand-in)", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<MFMA>("mfma only", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<MFMA | ONEHOT>("mfma + one-hot", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<MFMA | TWOACC>("mfma only, 2 accumulators", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<MFMA | M16>("mfma only, 16x16x64 (4 acc)", tiles, item, lut, counter, items, ntile, out, grid, flops);
    Run<ALL | TWOACC>("full, 2 accumulators", tiles, item, lut, counter, items, ntile, out, grid, flops);
  }
  return 0;
}

// smfmac_chain.hip — cycles per v_smfmac_i32_32x32x64_i8 on one dependent
// accumulator chain vs two and four interleaved chains, one wave per SIMD and
// three waves per SIMD (the scan kernel's tile is one 13-long chain).
// Diagnostic only; s_memtime inside the kernel (clock-independent).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/smfmac_chain tools/smfmac_chain.hip && ./tools/smfmac_chain
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

constexpr int N = 1024;

template <int NACC>
__global__ void __launch_bounds__(256) chain(int seed, long long* cycles, int* sink) {
  const int lane = threadIdx.x & 63;
  v4i a = {lane + seed, 1, 0, 0};
  v8i b = {1, 2, 3, 4, 5, 6, 7, lane};
  const int ix = 0x5555 * (lane & 3);
  v16i acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = v16i{0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N / NACC; ++i) {
#pragma unroll
    for (int k = 0; k < NACC; ++k)
      acc[k] = __builtin_amdgcn_smfmac_i32_32x32x64_i8(a, b, acc[k], ix, 0, 0);
  }
  int x = 0;
#pragma unroll
  for (int k = 0; k < NACC; ++k)
#pragma unroll
    for (int j = 0; j < 16; ++j) x ^= acc[k][j];
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cycles[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
  if (x == 0x12345) sink[0] = x;
}

template <int NACC>
void run(int waves_per_simd) {
  long long* d;
  int* s;
  const int blocks = 256;   // one per CU
  const int threads = 64 * 4 * waves_per_simd;
  CHECK(hipMalloc(&d, sizeof(long long) * blocks * threads / 64));
  CHECK(hipMalloc(&s, 4));
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(threads), 0, 0, 1, d, s);
  CHECK(hipDeviceSynchronize());
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(threads), 0, 0, 2, d, s);
  CHECK(hipDeviceSynchronize());
  long long h[4096];
  const int nw = blocks * threads / 64;
  CHECK(hipMemcpy(h, d, sizeof(long long) * nw, hipMemcpyDeviceToHost));
  double m = 0;
  for (int i = 0; i < nw; ++i) m += double(h[i]) / nw;
  printf("smfmac_i32_32x32x64_i8: %d chain(s), %d wave(s)/SIMD: %.1f cycles per instruction per wave, "
         "%.1f per SIMD\n", NACC, waves_per_simd, m / N, m / N / waves_per_simd);
  CHECK(hipFree(d));
  CHECK(hipFree(s));
}

int main() {
  run<1>(1);
  run<2>(1);
  run<4>(1);
  run<1>(3);
  run<2>(3);
  return 0;
}

// mfma_rate.hip — cycles per v_mfma_i32_32x32x32_i8 on one SIMD (s_memtime
// inside the kernel, so the number is independent of the DVFS clock), for 1
// and 4 independent accumulators, 1..4 waves per SIMD, one-hot-like sparse vs
// dense operands.  Diagnostic only.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_rate tools/mfma_rate.hip && ./tools/mfma_rate
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

constexpr int N = 2048;

template <int NACC, bool BF16>
__global__ void __launch_bounds__(256) rate(int dense, long long* cycles, int* sink) {
  const int lane = threadIdx.x & 63;
  v4i a, b;
  if (dense) {
    a = v4i{lane * 0x01030507, lane * 0x0b0d1113, lane ^ 0x55aa55aa, lane * 77};
    b = v4i{lane * 0x13110d0b, lane + 0x07050301, lane * 0x3f3f3f3f, lane ^ 0x7f7f7f7f};
  } else {
    a = v4i{0, 0, 0, 0};
    a[lane & 3] = 1 << (8 * ((lane >> 2) & 3));
    b = v4i{lane * 0x13110d0b, lane + 0x07050301, lane * 0x3f3f3f3f, lane ^ 0x7f7f7f7f};
  }
  v16i acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = v16i{0};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < N / NACC; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if (BF16) {
        typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
        typedef float f16v __attribute__((ext_vector_type(16)));
        f16v* fa = reinterpret_cast<f16v*>(&acc[i]);
        *fa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b),
                                                     *fa, 0, 0, 0);
      } else {
        acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
      }
    }
  }
  int x = 0;
  for (int i = 0; i < NACC; ++i)
    for (int j = 0; j < 16; ++j) x ^= acc[i][j];
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cycles[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
  if (x == 0x12345) sink[0] = x;
}

template <int NACC, bool BF16>
void Run(const char* name, int waves_per_simd, int dense, long long* d_cyc, int* sink, int cus) {
  // one block of 4*w waves per CU: w waves on each SIMD
  const int threads = 256 * waves_per_simd > 1024 ? 1024 : 256 * waves_per_simd;
  const int nw = threads / 64;
  hipLaunchKernelGGL((rate<NACC, BF16>), dim3(cus), dim3(threads), 0, 0, dense, d_cyc, sink);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((rate<NACC, BF16>), dim3(cus), dim3(threads), 0, 0, dense, d_cyc, sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> c(size_t(cus) * nw);
  CHECK(hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost));
  double avg = 0;
  for (auto v : c) avg += double(v);
  avg /= double(c.size());
  // s_memtime counts shader-clock cycles; each SIMD ran waves_per_simd * N MFMAs
  const double per_mfma_simd = avg / (double(N) * waves_per_simd);
  printf("%-34s waves/SIMD %d %-6s: %7.1f cyc per MFMA per SIMD   (%.1f us wall, %.2f GHz implied)\n",
         name, waves_per_simd, dense ? "dense" : "sparse", per_mfma_simd, ms * 1000.0,
         avg / (ms * 1e-3) / 1e9);
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  long long* d_cyc;
  int* sink;
  CHECK(hipMalloc(&d_cyc, 8 * size_t(cus) * 16));
  CHECK(hipMalloc(&sink, 4));
  for (int dense = 0; dense < 2; ++dense)
    for (int w : {1, 2, 4}) {
      Run<1, false>("i8 32x32x32, 1 accumulator", w, dense, d_cyc, sink, cus);
      Run<4, false>("i8 32x32x32, 4 accumulators", w, dense, d_cyc, sink, cus);
      Run<4, true>("bf16 32x32x16, 4 accumulators", w, dense, d_cyc, sink, cus);
    }
  return 0;
}

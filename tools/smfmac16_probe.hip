// Layout probe for v_smfmac_i32_16x16x128_i8 (the 16-query-slot scan tile).
// For every A lane la, compressed value j and index setting t (every 2-bit
// field of the index VGPR = t), A = a single 1 at (la, j); B = its lane id + 1
// (pass "L") or its byte id + 1 (pass "B").  Every non-zero output element
// (lane ld, element e) names the B lane and byte the value was paired with.
// A second part sets random index words and checks that value j follows
// field j only.  Prints CSV rows:
//   map,la,j,t,ld,e,blane,bbyte
//   field,j,word,bbyte
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/smfmac16_probe tools/smfmac16_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));

__global__ void one(const v4i* a, const v8i* b, const int* idx, v4i* out) {
  v4i acc = v4i{0, 0, 0, 0};
  acc = __builtin_amdgcn_smfmac_i32_16x16x128_i8(a[threadIdx.x], b[threadIdx.x], acc,
                                                 idx[threadIdx.x], 0, 0);
  out[threadIdx.x] = acc;
}

static v4i *da, *dout;
static v8i* db;
static int* di;

static void run(const int8_t (&A)[64][16], const int8_t (&B)[64][32], const uint32_t (&I)[64],
                int (&D)[64][4]) {
  (void)hipMemcpy(da, A, sizeof(A), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, B, sizeof(B), hipMemcpyHostToDevice);
  (void)hipMemcpy(di, I, sizeof(I), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(one, dim3(1), dim3(64), 0, 0, da, db, di, dout);
  (void)hipMemcpy(D, dout, sizeof(int) * 64 * 4, hipMemcpyDeviceToHost);
}

int main() {
  (void)hipMalloc(&da, 64 * sizeof(v4i));
  (void)hipMalloc(&db, 64 * sizeof(v8i));
  (void)hipMalloc(&di, 64 * sizeof(int));
  (void)hipMalloc(&dout, 64 * sizeof(v4i));
  int8_t BL[64][32], BB[64][32];
  for (int l = 0; l < 64; ++l)
    for (int k = 0; k < 32; ++k) {
      BL[l][k] = int8_t(l + 1);
      BB[l][k] = int8_t(k + 1);
    }
  for (int la = 0; la < 64; ++la)
    for (int j = 0; j < 16; ++j)
      for (int t = 0; t < 4; ++t) {
        int8_t A[64][16];
        std::memset(A, 0, sizeof(A));
        A[la][j] = 1;
        uint32_t I[64];
        for (int l = 0; l < 64; ++l) I[l] = uint32_t(t) * 0x55555555u;
        int DL[64][4], DB[64][4];
        run(A, BL, I, DL);
        run(A, BB, I, DB);
        for (int ld = 0; ld < 64; ++ld)
          for (int e = 0; e < 4; ++e)
            if (DL[ld][e] || DB[ld][e])
              std::printf("map,%d,%d,%d,%d,%d,%d,%d\n", la, j, t, ld, e, DL[ld][e] - 1,
                          DB[ld][e] - 1);
      }
  std::mt19937 rng(7);
  for (int j = 0; j < 16; ++j)
    for (int rep = 0; rep < 8; ++rep) {
      int8_t A[64][16];
      std::memset(A, 0, sizeof(A));
      A[0][j] = 1;
      uint32_t I[64];
      const uint32_t w = uint32_t(rng());
      for (int l = 0; l < 64; ++l) I[l] = w;
      int DB[64][4];
      run(A, BB, I, DB);
      int v = -1;
      for (int ld = 0; ld < 64; ++ld)
        for (int e = 0; e < 4; ++e)
          if (DB[ld][e]) v = DB[ld][e] - 1;
      std::printf("field,%d,%u,%d\n", j, w, v);
    }
  return 0;
}

// Layout probe 2 for v_smfmac_i32_32x32x64_i8: one non-zero A value
// (lane la, compressed value ja, index bits p for every value of that lane)
// against B = lane id (pass 0) / byte id (pass 1); prints where D is
// non-zero: (output lane, acc element) and the B lane/byte it picked.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void one(const v4i* a, const v8i* b, const int* idx, v16i* out) {
  v16i acc = v16i{0};
  acc = __builtin_amdgcn_smfmac_i32_32x32x64_i8(a[threadIdx.x], b[threadIdx.x], acc,
                                                idx[threadIdx.x], 0, 0);
  out[threadIdx.x] = acc;
}

int main() {
  v4i *da; v8i *db; int *di; v16i *dout;
  (void)hipMalloc(&da, 64 * sizeof(v4i)); (void)hipMalloc(&db, 64 * sizeof(v8i));
  (void)hipMalloc(&di, 64 * sizeof(int)); (void)hipMalloc(&dout, 64 * sizeof(v16i));
  const int las[] = {0, 1, 5, 32, 33};
  const int jas[] = {0, 1, 2, 3, 4, 7, 8, 15};
  for (int la : las)
    for (int ja : jas)
      for (int p = 0; p < 4; ++p) {
        int8_t A[64][16];
        memset(A, 0, sizeof(A));
        A[la][ja] = 1;
        uint32_t I[64];
        for (int l = 0; l < 64; ++l) {
          uint32_t x = 0;
          for (int j = 0; j < 16; ++j) x |= uint32_t(p) << (2 * j);
          I[l] = x;
        }
        (void)hipMemcpy(da, A, sizeof(A), hipMemcpyHostToDevice);
        (void)hipMemcpy(di, I, sizeof(I), hipMemcpyHostToDevice);
        int D0[64][16], D1[64][16];
        for (int pass = 0; pass < 2; ++pass) {
          int8_t B[64][32];
          for (int l = 0; l < 64; ++l)
            for (int k = 0; k < 32; ++k) B[l][k] = int8_t(pass ? k + 1 : l + 1);
          (void)hipMemcpy(db, B, sizeof(B), hipMemcpyHostToDevice);
          hipLaunchKernelGGL(one, dim3(1), dim3(64), 0, 0, da, db, di, dout);
          (void)hipMemcpy(pass ? D1 : D0, dout, sizeof(D0), hipMemcpyDeviceToHost);
        }
        printf("la=%2d ja=%2d p=%d:", la, ja, p);
        int shown = 0;
        for (int l = 0; l < 64 && shown < 4; ++l)
          for (int i = 0; i < 16 && shown < 4; ++i)
            if (D0[l][i] || D1[l][i]) {
              printf(" [out lane %d acc %d: B lane %d byte %d]", l, i, D0[l][i] - 1, D1[l][i] - 1);
              ++shown;
            }
        int nz = 0;
        for (int l = 0; l < 64; ++l)
          for (int i = 0; i < 16; ++i) nz += D0[l][i] != 0;
        printf(" nonzero=%d\n", nz);
      }
  return 0;
}

// Layout probe 3 for v_smfmac_i32_32x32x64_i8: which 2-bit field of the
// index VGPR belongs to compressed A value j.  One A value j = 1 (lane 0),
// index field f = 3 and every other field 0; B = byte id.  Prints, per j, the
// field f whose setting moves the picked B byte by +3.
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
  int8_t B[64][32];
  for (int l = 0; l < 64; ++l)
    for (int k = 0; k < 32; ++k) B[l][k] = int8_t(k + 1);
  (void)hipMemcpy(db, B, sizeof(B), hipMemcpyHostToDevice);
  for (int la : {0, 32}) {
    for (int j = 0; j < 16; ++j) {
      int8_t A[64][16];
      memset(A, 0, sizeof(A));
      A[la][j] = 1;
      (void)hipMemcpy(da, A, sizeof(A), hipMemcpyHostToDevice);
      int base = -1;
      printf("la=%d j=%2d:", la, j);
      for (int f = -1; f < 16; ++f) {
        uint32_t I[64];
        for (int l = 0; l < 64; ++l) I[l] = f < 0 ? 0u : (3u << (2 * f));
        (void)hipMemcpy(di, I, sizeof(I), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(one, dim3(1), dim3(64), 0, 0, da, db, di, dout);
        int D[64][16];
        (void)hipMemcpy(D, dout, sizeof(D), hipMemcpyDeviceToHost);
        int v = 0;
        for (int l = 0; l < 64; ++l)
          for (int i = 0; i < 16; ++i)
            if (D[l][i]) v = D[l][i];
        if (f < 0) { base = v; printf(" base byte %d;", base - 1); }
        else if (v != base) printf(" field %d -> byte %d", f, v - 1);
      }
      printf("\n");
    }
  }
  return 0;
}

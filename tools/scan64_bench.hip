// scan64_bench.hip — the LUT16 scan's main loop in two shapes, timed alone
// and checked against a host computation of the same sums.
//
//   cur : the product's shape (smx_kernels.hip lut16_scan_kernel): 32 query
//         slots per wave, B fragments (13 x v8i) in VGPRs, 3 waves per SIMD,
//         one accumulator, codes one tile ahead.
//   q64 : 64 query slots per wave sharing each one-hot A operand (two smfmac
//         per LDS lookup), one wave per SIMD, B fragments of both halves in
//         AGPRs (26 x v8i: the smfmac is an asm statement with an "a" operand,
//         so the compiler keeps them there), two accumulator pairs (tile t's
//         epilogue runs beside tile t+1's MFMAs), codes two tiles ahead.
//
// Synthetic glove-shaped work: `tiles` 32-datapoint code tiles (64 lanes x 16
// B, EncodeCodePair bytes), int8 LUTs [nq][2K][16]; each wave runs segments of
// SEG consecutive tiles with one set of query slots.  A first small launch of
// each kernel dumps every tile's sums and the host recomputes them.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/scan64_bench tools/scan64_bench.hip
//   tools/scan64_bench [tiles] [seg]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int K = 26;           // nibble steps (glove: 50 blocks -> 26)
constexpr int KS = K / 2;       // sparse MFMA steps per tile
constexpr int W = 16;           // code bytes per lane per tile

__device__ __forceinline__ uint32_t Grp(const uint32_t* c, int t) { return (c[t >> 2] >> ((t & 3) * 8)) & 0xFu; }
__device__ __forceinline__ uint32_t Pos(const uint32_t* c, int t) { return (c[t >> 2] >> ((t & 3) * 8 + 4)) & 0xFu; }

__device__ __forceinline__ void Tables(v4i* grp_tab, int* pos_tab) {
  if (threadIdx.x < 16) {
    const uint32_t g0 = threadIdx.x & 3u, g1 = threadIdx.x >> 2;
    v4i t = {0, 0, 0, 0};
    t[g0 >> 1] = int(1u << (16 * (g0 & 1u)));
    t[2 + (g1 >> 1)] = int(1u << (16 * (g1 & 1u)));
    grp_tab[threadIdx.x] = t;
    pos_tab[threadIdx.x] = int((threadIdx.x & 3u) * 0x5555u | ((threadIdx.x >> 2) * 0x5555u) << 16);
  }
  __syncthreads();
}

// 8 x v_mov_b64, then the 2 wait states a VALU write needs before an MFMA
// reads the register (the smfmac below is an asm statement: nothing pads it)
__device__ __forceinline__ v16i Zero16();
__device__ __forceinline__ void ZeroAcc(v16i& a) {
  a = Zero16();
  asm volatile("s_nop 1" : "+v"(a));
}

__device__ __forceinline__ v16i Zero16() {
  typedef long long v8l __attribute__((ext_vector_type(8)));
  v8l z;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    long long t;
    asm volatile("v_mov_b64 %0, 0" : "=v"(t));
    z[k] = t;
  }
  return __builtin_bit_cast(v16i, z);
}

__device__ __forceinline__ int Min16(const v16i& a) {
  int m = min(min(a[0], a[1]), a[2]);
#pragma unroll
  for (int i = 3; i < 15; i += 2) m = min(min(m, a[i]), a[i + 1]);
  return min(m, a[15]);
}

// acc += sparse(A, idx) x B, B in AGPRs
#define SMFMAC_AB(acc, a, b, ix) \
  asm volatile("v_smfmac_i32_32x32x64_i8 %0, %1, %2, %3" : "+v"(acc) : "v"(a), "a"(b), "v"(ix))
// the wait states between a 16-pass XDL write and any other reader (19 >= 18)
#define XDL_READ_PAD(acc) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 2" : "+v"(acc))

// ---------------------------------------------------------------------------
// cur: 32 slots, 12 waves per CU
// ---------------------------------------------------------------------------
// MODE bits (timing ablations, results invalid): 1 = no code loads after the
// first tile, 2 = no one-hot lookups in the loop, 4 = B fragments loaded once
// per wave instead of once per segment
template <int NB, int MODE = 0>
__global__ void __launch_bounds__(768, 1) scan_cur(const uint8_t* __restrict__ tiles, uint32_t ntiles,
                                                   const int8_t* __restrict__ lut, int nq, int seg,
                                                   int amax, unsigned long long* __restrict__ out,
                                                   int* __restrict__ dump) {
  __shared__ __align__(256) v4i grp_tab[16];
  __shared__ int pos_tab[16];
  Tables(grp_tab, pos_tab);
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const uint32_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  const uint32_t nseg = (ntiles + seg - 1) / seg;
  unsigned long long hits = 0;
  v8i b[KS];
  v16i acc;
  const uint64_t ck0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t sg = wave; sg < nseg; sg += nwaves) {
    const uint32_t q = (sg * 32 + c) % uint32_t(nq);
    const v8i* bp = reinterpret_cast<const v8i*>(lut + (size_t(q) * K + h) * 32);
    if (!(MODE & 4) || sg == wave) {
#pragma unroll
      for (int s = 0; s < KS; ++s) b[s] = bp[2 * s];
    }
    const uint32_t t0 = sg * seg, t1 = min(ntiles, t0 + seg);
    uint32_t codes[4], nxt[4];
    if (MODE & 8) acc = Zero16();
    {
      const uint4 v = *reinterpret_cast<const uint4*>(tiles + (size_t(t0) * 64 + lane) * W);
      codes[0] = v.x; codes[1] = v.y; codes[2] = v.z; codes[3] = v.w;
    }
    for (uint32_t t = t0; t < t1; ++t) {
      const uint32_t tn = t + 1 < t1 ? t + 1 : t;
      uint4 v;
      if (MODE & 1) {
        v = make_uint4(codes[0] ^ t, codes[1], codes[2], codes[3]);
      } else {
        v = *reinterpret_cast<const uint4*>(tiles + (size_t(tn) * 64 + lane) * W);
      }
      constexpr int R = 3;
      v4i o[NB];
      int ix[NB];
#pragma unroll
      for (int p = 0; p < R; ++p) {
        o[p] = grp_tab[Grp(codes, p)];
        ix[p] = pos_tab[Pos(codes, p)];
      }
      if (!(MODE & 8)) acc = Zero16();
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc = __builtin_amdgcn_smfmac_i32_32x32x64_i8(o[(MODE & 2) ? 0 : s % NB], b[s], acc,
                                                      ix[(MODE & 2) ? 0 : s % NB], 0, 0);
        if (!(MODE & 2) && s + R < KS) {
          o[(s + R) % NB] = grp_tab[Grp(codes, s + R)];
          ix[(s + R) % NB] = pos_tab[Pos(codes, s + R)];
        }
      }
      if (dump) {   // dump[t][slot][dp]: lane (c, h) holds dps (i&3) + 8(i>>2) + 4h of query slot c
#pragma unroll
        for (int i = 0; i < 16; ++i)
          dump[(size_t(t) * 64 + c) * 32 + (i & 3) + 8 * (i >> 2) + 4 * h] = acc[i];
      }
      if (!(MODE & 8)) {
        const int m = Min16(acc);
        const unsigned long long hb = __builtin_amdgcn_ballot_w64(m <= amax);
        hits += __popcll(hb);
      }
      nxt[0] = v.x; nxt[1] = v.y; nxt[2] = v.z; nxt[3] = v.w;
#pragma unroll
      for (int i = 0; i < 4; ++i) codes[i] = nxt[i];
    }
    if (MODE & 8) hits += __popcll(__builtin_amdgcn_ballot_w64(Min16(acc) <= amax));
  }
  if (lane == 0) {
    out[wave] = hits;
    // in-kernel clock: shader cycles over 100 MHz realtime ticks
    const uint64_t ck1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    out[4096 + wave] = ((ck1 - ck0) << 24) | ((rt1 - rt0) & 0xFFFFFFull);
  }
}

// ---------------------------------------------------------------------------
// q64: 64 slots (two B halves share each A), one wave per SIMD
// ---------------------------------------------------------------------------
#ifndef Q64_R
#define Q64_R 2
#endif
#ifndef Q64_EPI_STEP
#define Q64_EPI_STEP 2   // the previous tile's epilogue after this many steps
#endif
template <int NWV, int R, int NB, bool ONLY>
__global__ void __launch_bounds__(64 * NWV, 1) scan_q64(const uint8_t* __restrict__ tiles,
                                                        uint32_t ntiles,
                                                        const int8_t* __restrict__ lut, int nq,
                                                        int seg, int amax,
                                                        unsigned long long* __restrict__ out,
                                                        int* __restrict__ dump) {
  __shared__ __align__(256) v4i grp_tab[16];
  __shared__ int pos_tab[16];
  Tables(grp_tab, pos_tab);
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const uint32_t wave = blockIdx.x * NWV + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * NWV;
  const uint32_t nseg = (ntiles + seg - 1) / seg;
  unsigned long long hits = 0;
  for (uint32_t sg = wave; sg < nseg; sg += nwaves) {
    const uint32_t qa = (sg * 64 + c) % uint32_t(nq), qb = (sg * 64 + 32 + c) % uint32_t(nq);
    const v8i* bpa = reinterpret_cast<const v8i*>(lut + (size_t(qa) * K + h) * 32);
    const v8i* bpb = reinterpret_cast<const v8i*>(lut + (size_t(qb) * K + h) * 32);
    v8i ba[KS], bb[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      ba[s] = bpa[2 * s];
      bb[s] = bpb[2 * s];
    }
    const uint32_t t0 = sg * seg, t1 = min(ntiles, t0 + seg);
    auto ld = [&](uint32_t t, uint32_t* cd) {
      const uint4 v = *reinterpret_cast<const uint4*>(tiles + (size_t(min(t, t1 - 1)) * 64 + lane) * W);
      cd[0] = v.x; cd[1] = v.y; cd[2] = v.z; cd[3] = v.w;
    };
    uint32_t c0[4], c1[4];
    ld(t0, c0);
    ld(t0 + 1, c1);
    v16i x0, x1, y0, y1;       // accumulator pairs of even / odd tiles
    bool pend = false;          // the other pair holds an untested tile
    uint32_t pt = 0;
    // the test of a finished tile's sums (and the dump)
    auto epilogue = [&](v16i& p0, v16i& p1, uint32_t t) {
      XDL_READ_PAD(p0);
      XDL_READ_PAD(p1);
      if (dump) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          dump[(size_t(t) * 64 + c) * 32 + (i & 3) + 8 * (i >> 2) + 4 * h] = p0[i];
          dump[(size_t(t) * 64 + 32 + c) * 32 + (i & 3) + 8 * (i >> 2) + 4 * h] = p1[i];
        }
      }
      const unsigned long long hb = __builtin_amdgcn_ballot_w64(min(Min16(p0), Min16(p1)) <= amax);
      hits += __popcll(hb);
    };
    auto tile = [&](uint32_t* cd, uint32_t t, v16i& a0, v16i& a1, v16i& p0, v16i& p1) {
      uint32_t cn[4];
      ld(t + 2, cn);   // two tiles ahead
      v4i o[NB];
      int ix[NB];
#pragma unroll
      for (int p = 0; p < R; ++p) {
        o[p] = grp_tab[Grp(cd, p)];
        ix[p] = pos_tab[Pos(cd, p)];
      }
      ZeroAcc(a0);
      ZeroAcc(a1);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (ONLY) {
          SMFMAC_AB(a0, o[0], ba[s], ix[0]);
          SMFMAC_AB(a1, o[0], bb[s], ix[0]);
        } else {
          SMFMAC_AB(a0, o[s % NB], ba[s], ix[s % NB]);
          SMFMAC_AB(a1, o[s % NB], bb[s], ix[s % NB]);
          if (s + R < KS) {
            o[(s + R) % NB] = grp_tab[Grp(cd, s + R)];
            ix[(s + R) % NB] = pos_tab[Pos(cd, s + R)];
          }
        }
        if (s == Q64_EPI_STEP && pend) epilogue(p0, p1, pt);
      }
      pend = true;
      pt = t;
#pragma unroll
      for (int i = 0; i < 4; ++i) cd[i] = cn[i];
    };
    uint32_t t = t0;
    for (; t + 1 < t1; t += 2) {
      tile(c0, t, x0, x1, y0, y1);
      tile(c1, t + 1, y0, y1, x0, x1);
    }
    if (t < t1) {
      tile(c0, t, x0, x1, y0, y1);
      epilogue(x0, x1, t);
    } else if (pend) {
      epilogue(y0, y1, t - 1);
    }
    pend = false;
  }
  if (lane == 0) out[wave] = hits;
}

// ---------------------------------------------------------------------------
// p32: 32 slots, two accumulators in turn (tile t's test while tile t+1's
// MFMAs run), codes two tiles ahead, NWV waves per CU
// ---------------------------------------------------------------------------
template <int NWV, int R, int NB, int EPI>
__global__ void __launch_bounds__(64 * NWV, 1) scan_p32(const uint8_t* __restrict__ tiles,
                                                        uint32_t ntiles,
                                                        const int8_t* __restrict__ lut, int nq,
                                                        int seg, int amax,
                                                        unsigned long long* __restrict__ out,
                                                        int* __restrict__ dump) {
  __shared__ __align__(256) v4i grp_tab[16];
  __shared__ int pos_tab[16];
  Tables(grp_tab, pos_tab);
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const uint32_t wave = blockIdx.x * NWV + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * NWV;
  const uint32_t nseg = (ntiles + seg - 1) / seg;
  unsigned long long hits = 0;
  for (uint32_t sg = wave; sg < nseg; sg += nwaves) {
    const uint32_t qa = (sg * 32 + c) % uint32_t(nq);
    const v8i* bpa = reinterpret_cast<const v8i*>(lut + (size_t(qa) * K + h) * 32);
    v8i ba[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) ba[s] = bpa[2 * s];
    const uint32_t t0 = sg * seg, t1 = min(ntiles, t0 + seg);
    auto ld = [&](uint32_t t, uint32_t* cd) {
      const uint4 v = *reinterpret_cast<const uint4*>(tiles + (size_t(min(t, t1 - 1)) * 64 + lane) * W);
      cd[0] = v.x; cd[1] = v.y; cd[2] = v.z; cd[3] = v.w;
    };
    uint32_t c0[4], c1[4];
    ld(t0, c0);
    ld(t0 + 1, c1);
    v16i x0, y0;
    bool pend = false;
    uint32_t pt = 0;
    auto epilogue = [&](v16i& p0, uint32_t t) {
      XDL_READ_PAD(p0);
      if (dump) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          dump[(size_t(t) * 64 + c) * 32 + (i & 3) + 8 * (i >> 2) + 4 * h] = p0[i];
      }
      const unsigned long long hb = __builtin_amdgcn_ballot_w64(Min16(p0) <= amax);
      hits += __popcll(hb);
    };
    auto tile = [&](uint32_t* cd, uint32_t t, v16i& a0, v16i& p0) {
      uint32_t cn[4];
      ld(t + 2, cn);
      v4i o[NB];
      int ix[NB];
#pragma unroll
      for (int p = 0; p < R; ++p) {
        o[p] = grp_tab[Grp(cd, p)];
        ix[p] = pos_tab[Pos(cd, p)];
      }
      ZeroAcc(a0);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        SMFMAC_AB(a0, o[s % NB], ba[s], ix[s % NB]);
        if (s + R < KS) {
          o[(s + R) % NB] = grp_tab[Grp(cd, s + R)];
          ix[(s + R) % NB] = pos_tab[Pos(cd, s + R)];
        }
        if (s == EPI && pend) epilogue(p0, pt);
      }
      pend = true;
      pt = t;
#pragma unroll
      for (int i = 0; i < 4; ++i) cd[i] = cn[i];
    };
    uint32_t t = t0;
    for (; t + 1 < t1; t += 2) {
      tile(c0, t, x0, y0);
      tile(c1, t + 1, y0, x0);
    }
    if (t < t1) {
      tile(c0, t, x0, y0);
      epilogue(x0, t);
    } else if (pend) {
      epilogue(y0, t - 1);
    }
    pend = false;
  }
  if (lane == 0) out[wave] = hits;
}

static uint32_t Enc(uint32_t x0, uint32_t x1) {
  return ((x0 >> 2) | ((x1 >> 2) << 2)) | (((x0 & 3u) | ((x1 & 3u) << 2)) << 4);
}

int main(int argc, char** argv) {
  const uint32_t ntiles = argc > 1 ? uint32_t(std::atoi(argv[1])) : 114000u;
  const int seg = argc > 2 ? std::atoi(argv[2]) : 20;
  const int nq = 1000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::vector<uint8_t> h_tiles(size_t(ntiles) * 64 * W);
  uint64_t x = 88172645463325252ull;
  auto rnd = [&] { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  for (auto& b : h_tiles) b = uint8_t(rnd());
  std::vector<int8_t> h_lut(size_t(nq) * 2 * K * 16);
  for (auto& b : h_lut) b = int8_t(int(rnd() % 255) - 127);
  uint8_t* d_tiles;
  int8_t* d_lut;
  unsigned long long* d_out;
  int* d_dump;
  const uint32_t vt = 64;   // tiles verified
  CHECK(hipMalloc(&d_tiles, h_tiles.size()));
  CHECK(hipMalloc(&d_lut, h_lut.size()));
  CHECK(hipMalloc(&d_out, sizeof(unsigned long long) * 8192));
  CHECK(hipMemset(d_out, 0, sizeof(unsigned long long) * 8192));
  CHECK(hipMalloc(&d_dump, sizeof(int) * vt * 64 * 32));
  CHECK(hipMemcpy(d_tiles, h_tiles.data(), h_tiles.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_lut, h_lut.data(), h_lut.size(), hipMemcpyHostToDevice));
  // host sums of tile t, slot `slot` (query = segment's slot mapping), dp r
  auto host_sum = [&](uint32_t t, int slot, int r, int slots_per_seg) {
    const uint32_t sg = t / uint32_t(seg);
    const uint32_t q = (sg * slots_per_seg + slot) % uint32_t(nq);
    int sum = 0;
    for (int s = 0; s < KS; ++s)
      for (int hh = 0; hh < 2; ++hh) {
        const uint8_t by = h_tiles[(size_t(t) * 64 + hh * 32 + r) * W + s];
        // decode (inverse of Enc)
        uint32_t x0 = 0, x1 = 0;
        for (uint32_t a = 0; a < 16; ++a)
          for (uint32_t b = 0; b < 16; ++b)
            if (Enc(a, b) == by) { x0 = a; x1 = b; }
        const int blk0 = 4 * s + hh, blk1 = 4 * s + 2 + hh;
        sum += h_lut[(size_t(q) * 2 * K + blk0) * 16 + x0] + h_lut[(size_t(q) * 2 * K + blk1) * 16 + x1];
      }
    return sum;
  };
  auto verify = [&](const char* name, int slots) {
    std::vector<int> dump(size_t(vt) * 64 * 32);
    CHECK(hipMemcpy(dump.data(), d_dump, dump.size() * sizeof(int), hipMemcpyDeviceToHost));
    int bad = 0;
    for (uint32_t t = 0; t < vt; ++t)
      for (int slot = 0; slot < slots; ++slot)
        for (int r = 0; r < 32; ++r)
          if (dump[(size_t(t) * 64 + slot) * 32 + r] != host_sum(t, slot, r, slots)) ++bad;
    std::printf("%-4s verify over %u tiles: %d mismatches\n", name, vt, bad);
    return bad;
  };
  int bad = 0;
  CHECK(hipMemset(d_dump, 0, sizeof(int) * vt * 64 * 32));
  hipLaunchKernelGGL(scan_cur<3>, dim3(cus), dim3(768), 0, 0, d_tiles, vt, d_lut, nq, seg, 0, d_out,
                     d_dump);
  CHECK(hipDeviceSynchronize());
  bad += verify("cur", 32);
  CHECK(hipMemset(d_dump, 0, sizeof(int) * vt * 64 * 32));
  hipLaunchKernelGGL((scan_q64<4, 2, 3, false>), dim3(cus), dim3(256), 0, 0, d_tiles, vt, d_lut,
                     nq, seg, 0, d_out, d_dump);
  CHECK(hipDeviceSynchronize());
  bad += verify("q64", 64);
  CHECK(hipMemset(d_dump, 0, sizeof(int) * vt * 64 * 32));
  hipLaunchKernelGGL((scan_p32<8, 3, 4, 3>), dim3(cus), dim3(512), 0, 0, d_tiles, vt, d_lut, nq,
                     seg, 0, d_out, d_dump);
  CHECK(hipDeviceSynchronize());
  bad += verify("p32", 32);

  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int amax = -1500;   // a few hits per tile on random data
  auto timeit = [&](const char* name, auto launch, double smfmac) {
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    // MFMA-bound time: smfmac x 32 cycles over 4 * cus SIMDs at 2.4 GHz
    const double bound_ms = smfmac * 32.0 / (4.0 * cus) / 2.4e9 * 1e3;
    // median in-kernel clock of the last launch's waves (scan_cur only)
    std::vector<unsigned long long> ck(4096);
    CHECK(hipMemcpy(ck.data(), d_out + 4096, 4096 * 8, hipMemcpyDeviceToHost));
    std::vector<double> mhz;
    for (auto v : ck) {
      const double cyc = double(v >> 24), rt = double(v & 0xFFFFFFull);
      if (rt > 0) mhz.push_back(cyc / rt * 100.0);
    }
    std::sort(mhz.begin(), mhz.end());
    const double clk = mhz.empty() ? 0.0 : mhz[mhz.size() / 2];
    std::printf("%-26s %8.2f us  %.1f cycles per smfmac per SIMD at 2.4 GHz  MFMA bound %.2f us  "
                "frac %.3f  in-kernel clock %.0f MHz (%.1f cycles per smfmac)\n",
                name, ms * 1e3, ms * 1e-3 * 2.4e9 * 4.0 * cus / smfmac, bound_ms * 1e3,
                bound_ms / ms, clk, ms * 1e-3 * clk * 1e6 * 4.0 * cus / smfmac);
    CHECK(hipMemset(d_out + 4096, 0, 4096 * 8));
  };
  const double sm = double(ntiles) * KS;   // cur: ntiles x 32 slots; q64: ntiles/2 x 64
#define CUR(NB, NAME)                                                                         \
  timeit(NAME, [&] {                                                                          \
    hipLaunchKernelGGL(scan_cur<NB>, dim3(cus), dim3(768), 0, 0, d_tiles, ntiles, d_lut, nq, seg, \
                       amax, d_out, nullptr);                                                 \
  }, sm)
#define CURM(MODE, NAME)                                                                      \
  timeit(NAME, [&] {                                                                          \
    hipLaunchKernelGGL((scan_cur<3, MODE>), dim3(cus), dim3(768), 0, 0, d_tiles, ntiles, d_lut, nq, \
                       seg, amax, d_out, nullptr);                                            \
  }, sm)
#define CUR1(NB, NAME)                                                                        \
  timeit(NAME, [&] {                                                                          \
    hipLaunchKernelGGL(scan_cur<NB>, dim3(cus), dim3(256), 0, 0, d_tiles, ntiles, d_lut, nq, seg, \
                       amax, d_out, nullptr);                                                 \
  }, sm)
#define Q64(R, NB, ONLY, NAME)                                                               \
  timeit(NAME, [&] {                                                                          \
    hipLaunchKernelGGL((scan_q64<4, R, NB, ONLY>), dim3(cus), dim3(256), 0, 0, d_tiles, ntiles / 2, \
                       d_lut, nq, seg, amax, d_out, nullptr);                                 \
  }, sm)
#define P32(NWV, R, NB, EPI, NAME)                                                            \
  timeit(NAME, [&] {                                                                          \
    hipLaunchKernelGGL((scan_p32<NWV, R, NB, EPI>), dim3(cus), dim3(64 * NWV), 0, 0, d_tiles,   \
                       ntiles, d_lut, nq, seg, amax, d_out, nullptr);                         \
  }, sm)
  CUR(3, "cur R3 NB3 (product)");
  P32(8, 3, 4, 3, "p32 2/SIMD R3 NB4 E3");
  P32(8, 4, 5, 3, "p32 2/SIMD R4 NB5 E3");
  P32(8, 2, 3, 2, "p32 2/SIMD R2 NB3 E2");
  P32(8, 3, 4, 6, "p32 2/SIMD R3 NB4 E6");
  P32(12, 2, 3, 2, "p32 3/SIMD R2 NB3 E2");
  P32(4, 4, 5, 3, "p32 1/SIMD R4 NB5 E3");
  CURM(7, "cur MFMA only");
  CURM(15, "cur MFMA chain, no test");
  CURM(8, "cur no per-tile test");
  Q64(2, 2, false, "q64 R2 NB2");
  Q64(2, 2, true, "q64 mfma only");
  CHECK(hipGetLastError());
  std::printf("tiles %u seg %d CUs %d\n", ntiles, seg, cus);
  return bad ? 1 : 0;
}

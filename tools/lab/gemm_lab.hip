// Main-loop lab for the conv GEMMs (measurement only; not linked into the product).
//
// Plain bf16 GEMM C[M][N] = A[M][K] * B[N][K]^T (both operands k-contiguous, as
// the implicit-GEMM forward sees im2col rows and KRSC weights), fp32 accumulation.
//   intake<NW, DEPTH, REG>: LDS-DMA (REG=0) or buffer loads to VGPRs (REG=1) of a
//       256x256 tile's operands per 64-deep k-step, DEPTH k-steps in flight, no math:
//       the per-CU operand intake a 256x256 tile gets.
//   gemm<WM, WN, SCHED>: 256x256 tile, WM x WN waves, 2-stage LDS-DMA ring, BK 64,
//       XOR-swizzled 128-B k-rows, 16x16x32 MFMA, LDS-staged 16-B epilogue.
//       SCHED 0: DMA burst then fragment reads then MFMAs; 1: DMA interleaved
//       among the MFMAs (sched_group_barrier).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm_lab.hip -o gemm_lab
// run:   ./gemm_lab            (prints one line per case)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ int ktile_off(int row, int slot) { return row * 128 + ((slot ^ ((row >> 1) & 7)) << 4); }

// XCD-aware tile order (bijective): each XCD takes a contiguous run of tiles
__device__ __forceinline__ int xcd_tile(int lin, int nb) {
  const int xcd = lin & 7, q = nb >> 3, r = nb & 7;
  return xcd * q + min(xcd, r) + (lin >> 3);
}

// ---------------------------------------------------------------------------
// intake: 256-row A panel per workgroup + shared 256-row B panel, 64 KiB per k-step
// ---------------------------------------------------------------------------
template <int NW, int DEPTH, int REG>
__global__ void __launch_bounds__(64 * NW, 1) intake_kernel(const __bf16* A, const __bf16* B, int K, int ksteps,
                                                             int* sink) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 65536];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = xcd_tile(blockIdx.x, gridDim.x);
  constexpr int PER = 64 / NW / 2;  // instructions per operand per wave per k-step
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A + (long)t * 256 * K, 256u * K * 2);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(B, 256u * K * 2);
  const int row0 = 8 * wave + (lane >> 3);
  const uint32_t off = (uint32_t)((row0 * K + (((lane & 7) ^ ((row0 >> 1) & 7)) * 8)) * 2);
  i32x4 acc = {0, 0, 0, 0};
  for (int ks = 0; ks < ksteps; ++ks) {
    char* st = smem + (ks & 1) * 65536;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t so = (uint32_t)((8 * NW * i) * K * 2 + ks * 128);
      if (REG) {
        acc ^= __builtin_amdgcn_raw_buffer_load_b128(rsA, off, so, 0);
        acc ^= __builtin_amdgcn_raw_buffer_load_b128(rsB, off, so, 0);
      } else {
        blds16(rsA, off, so, st + (wave + NW * i) * 1024);
        blds16(rsB, off, so, st + 32768 + (wave + NW * i) * 1024);
      }
    }
    if (ks >= DEPTH - 1) {
      // leave DEPTH-1 k-steps of this wave's loads in flight
      if constexpr (DEPTH == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (DEPTH == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
      else if constexpr (DEPTH == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * PER) : "memory");
    }
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc[0] == 0x12345 && acc[1] == 7) sink[0] = acc[2];
}

// ---------------------------------------------------------------------------
// GEMM 256x256 tile, 2-stage LDS-DMA ring
// ---------------------------------------------------------------------------
constexpr int lab_waves(int bm, int bn, int nw) {
  return ((163840 / (2 * (bm + bn) * 128)) * nw) / 4 > 8 ? 8 : ((163840 / (2 * (bm + bn) * 128)) * nw) / 4;
}
template <int WM, int WN, int SCHED, bool L2MODE = false, int BM = 256, int BN = 256>
__global__ void __launch_bounds__(64 * WM * WN, lab_waves(BM, BN, WM * WN)) gemm_kernel(const __bf16* A,
                                                                                         const __bf16* B, __bf16* C,
                                                                                         int M, int N, int K) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;  // 1-KiB instructions per operand per wave per k-step
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int EROW = BN * 2 + 16;  // epilogue staging row (bf16 + pad)
  __shared__ __attribute__((aligned(16))) char smem[BM * EROW > 2 * STAGE ? BM * EROW : 2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = N / BN;
  const int t = xcd_tile(blockIdx.x, gridDim.x);
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // L2MODE: every XCD's run of tiles re-reads two 256-row A panels (~2.4 MB
  // per XCD at K 2304, L2-resident like the implicit GEMM's im2col rows);
  // otherwise each tile streams its own rows (HBM)
  const long arow = L2MODE ? (long)(((t / 32) * 2 + (t & 1)) % (M / 256)) * BM : (long)m0;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A + arow * K, (uint32_t)(min(BM, M - m0) * K * 2));
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(B + (long)n0 * K, (uint32_t)(BN * K * 2));
  const int row0 = 8 * wave + (lane >> 3);
  const uint32_t off = (uint32_t)((row0 * K + (((lane & 7) ^ ((row0 >> 1) & 7)) * 8)) * 2);
  const int nk = K / 64;

  // (SCHED & 8: issued every k-step, the one past the end reading zeros
  // (out-of-extent offsets) into the idle slot, so it sits in the MFMA block)
  auto issue = [&](int ks) {
    char* st = smem + (ks & 1) * STAGE;
    const bool past = ks >= nk;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const uint32_t so = (uint32_t)((8 * NW * i) * K * 2 + ks * 128);
      blds16(rsA, past ? 0xFFFFFFF0u : off, past ? 0u : so, st + (wave + NW * i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const uint32_t so = (uint32_t)((8 * NW * i) * K * 2 + ks * 128);
      blds16(rsB, past ? 0xFFFFFFF0u : off, past ? 0u : so, st + BM * 128 + (wave + NW * i) * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if constexpr ((SCHED & 4) != 0) {
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  issue(0);
  for (int ks = 0; ks < nk; ++ks) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const char* As = smem + (ks & 1) * STAGE;
    const char* Bs = As + BM * 128;
    if constexpr ((SCHED & 8) == 0) {
      if (ks + 1 < nk) issue(ks + 1);
    }
    bf16x8 fa[2][FM], fb[2][FN];
    auto readh = [&](int h) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * WTM + i * 16 + (lane & 15);
        fa[h][i] = *reinterpret_cast<const bf16x8*>(As + ktile_off(r, 4 * h + (lane >> 4)));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * WTN + j * 16 + (lane & 15);
        fb[h][j] = *reinterpret_cast<const bf16x8*>(Bs + ktile_off(r, 4 * h + (lane >> 4)));
      }
    };
    auto mmah = [&](int h) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[h][i], fb[h][j], acc[i][j], 0, 0, 0);
    };
    if constexpr ((SCHED & 8) != 0) {  // reads, then the DMA (source order lets it sink among the MFMAs)
      readh(0);
      readh(1);
      issue(ks + 1);
      mmah(0);
      mmah(1);
    } else if constexpr ((SCHED & 2) != 0) {  // both halves' fragments requested before the first MFMA
      readh(0);
      readh(1);
      mmah(0);
      mmah(1);
    } else {  // the production order: half 0 read, its MFMAs, half 1 read, its MFMAs
      readh(0);
      mmah(0);
      readh(1);
      mmah(1);
    }
    if constexpr ((SCHED & 1) != 0) {
      // every fragment read first, then the MFMAs, the DMA issue (SCHED & 8:
      // in this block) spread over them: one 1-KiB piece per MFMA group
      constexpr int NDMA = PA + PB, NMF = 2 * FM * FN;
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (FM + FN), 0);  // fragment reads first
#pragma unroll
      for (int g = 0; g < NDMA; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, NMF / NDMA, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    }
  }
  // epilogue: each wave stages its tile as bf16 in LDS, then 16-B row stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = wm * WTM + i * 16 + (lane >> 4) * 4 + e;
        const int c = wn * WTN + j * 16 + (lane & 15);
        *reinterpret_cast<__bf16*>(smem + r * EROW + c * 2) = (__bf16)acc[i][j][e];
      }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B chunks per row
  for (int idx = tid; idx < BM * CPR; idx += 64 * NW) {
    const int r = idx / CPR, c = idx % CPR;
    if (m0 + r < M)
      *reinterpret_cast<i32x4*>(C + (long)(m0 + r) * N + n0 + c * 8) =
          *reinterpret_cast<const i32x4*>(smem + r * EROW + c * 16);
  }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
static float bf2f(__bf16 v) { return (float)v; }

template <typename F>
static float time_ms(F launch, int iters) {
  for (int i = 0; i < 3; ++i) launch();
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int WM, int WN, int SCHED, bool L2MODE = false, int BM = 256, int BN = 256>
static void run_gemm(const char* name, const __bf16* dA, const __bf16* dB, __bf16* dC, int M, int N, int K,
                     const std::vector<__bf16>& hA, const std::vector<__bf16>& hB, int iters) {
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  auto go = [&] {
    hipLaunchKernelGGL((gemm_kernel<WM, WN, SCHED, L2MODE, BM, BN>), dim3(tiles), dim3(64 * WM * WN), 0, 0, dA, dB,
                       dC, M, N, K);
  };
  go();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  // spot check 512 outputs against a double-precision host product
  std::vector<__bf16> hC((size_t)M * N);
  CK(hipMemcpy(hC.data(), dC, hC.size() * 2, hipMemcpyDeviceToHost));
  double maxrel = 0;
  for (int s = 0; s < 512; ++s) {
    const int m = (int)((s * 2654435761u) % (unsigned)M), n = (int)((s * 40503u + 17) % (unsigned)N);
    int am = m;
    if (L2MODE) {  // the A row this output row read: tile t's panel (t = the remapped tile index)
      const int tiles_n = N / BN;
      const int t = (m / BM) * tiles_n + n / BN;
      am = (((t / 32) * 2 + (t & 1)) % (M / 256)) * BM + m % BM;
    }
    double ref = 0, mag = 0;
    for (int k = 0; k < K; ++k) {
      const double p = (double)bf2f(hA[(size_t)am * K + k]) * bf2f(hB[(size_t)n * K + k]);
      ref += p;
      mag += fabs(p);
    }
    maxrel = fmax(maxrel, fabs(bf2f(hC[(size_t)m * N + n]) - ref) / (mag + 1e-30));
  }
  const float ms = time_ms(go, iters);
  printf("%-28s M=%6d N=%4d K=%5d  %8.1f us  %6.0f TF/s  check %.2e %s\n", name, M, N, K, ms * 1e3,
         2.0 * M * N * K / (ms * 1e-3) / 1e12, maxrel, maxrel < 1e-2 ? "ok" : "BAD");
  fflush(stdout);
}

template <int NW, int DEPTH, int REG>
static void run_intake(const __bf16* dA, const __bf16* dB, int K, int blocks, int* sink, int iters) {
  const int ks = K / 64;
  auto go = [&] {
    hipLaunchKernelGGL((intake_kernel<NW, DEPTH, REG>), dim3(blocks), dim3(64 * NW), 0, 0, dA, dB, K, ks, sink);
  };
  go();
  CK(hipGetLastError());
  const float ms = time_ms(go, iters);
  const double bytes = (double)blocks * ks * 65536;
  printf("intake %-4s waves=%d depth=%d blocks=%4d  %8.1f us  %7.1f GB/s/CU (%d CU busy)  chip %6.2f TB/s\n",
         REG ? "reg" : "lds", NW, DEPTH, blocks, ms * 1e3, bytes / (ms * 1e-3) / 1e9 / (blocks < 256 ? blocks : 256),
         blocks < 256 ? blocks : 256, bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const int M = 65536, N = 256, K = 2304;
  std::vector<__bf16> hA((size_t)M * K), hB((size_t)N * K);
  uint32_t s = 12345;
  auto rnd = [&] { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f; };
  for (auto& v : hA) v = (__bf16)rnd();
  for (auto& v : hB) v = (__bf16)(rnd() * 0.05f);
  __bf16 *dA, *dB, *dC;
  int* sink;
  CK(hipMalloc(&dA, hA.size() * 2));
  CK(hipMalloc(&dB, hB.size() * 2));
  CK(hipMalloc(&dC, (size_t)M * N * 2));
  CK(hipMalloc(&sink, 64));
  CK(hipMemcpy(dA, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));

  // L2-resident A (two panels per XCD), the implicit GEMM's regime.  Layer-2-like
  // shape (N 128, K 1152): 128x128 (2 per CU) against 256x128 (1 per CU)
  run_gemm<4, 2, 0, true, 128, 128>("128x128 prod  N128", dA, dB, dC, M, 128, K / 2, hA, hB, iters);
  run_gemm<4, 2, 1, true, 128, 128>("128x128 rf    N128", dA, dB, dC, M, 128, K / 2, hA, hB, iters);
  run_gemm<4, 2, 0, true, 256, 128>("256x128 prod  N128", dA, dB, dC, M, 128, K / 2, hA, hB, iters);
  run_gemm<4, 2, 1, true, 256, 128>("256x128 rf    N128", dA, dB, dC, M, 128, K / 2, hA, hB, iters);
  run_gemm<2, 4, 1, true, 256, 128>("256x128 2x4rf N128", dA, dB, dC, M, 128, K / 2, hA, hB, iters);
  // layer-3-like (N 256, K 2304) at 196 tiles
  run_gemm<4, 2, 1, true>("256x256 rf l3 M", dA, dB, dC, 50176, N, K, hA, hB, iters);
  run_gemm<4, 2, 1, true, 128, 128>("128x128 rf l3 M", dA, dB, dC, 50176, N, K, hA, hB, iters);
  run_gemm<4, 2, 1, true, 256, 128>("256x128 rf l3 M", dA, dB, dC, 50176, N, K, hA, hB, iters);
  return 0;
}

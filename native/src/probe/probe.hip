// mi355x-probe: per-device readiness check for gfx950 (MI355X), the MI355X-native replacement for
// the reference's GPU smoke test (`kubectl run ... nvidia-smi`, GPU调度平台搭建.md:134-138).
//
// A device passes only if
//   1. HBM: two complementary pseudo-random patterns written over `hbmBytes` of HBM3E and read
//      back bit-exactly (stuck-at / coupling faults in both polarities), with the achieved
//      write+read bandwidth reported;
//   2. MFMA: a bf16 GEMM on the matrix cores (`v_mfma_f32_16x16x32_bf16`) is bit-exact against
//      (a) a full VALU fp32 reference on a 256^3 problem with an asymmetric B (catches fragment
//      layout / row<->col faults) and (b) exact u32 (mod 2^32) ABFT row+column checksums on an N^3 problem
//      whose operands are small integers (all partial sums exact in fp32), with TFLOP/s reported.
//
// Design for CDNA4: 64-wide waves; 16-byte vector loads/stores everywhere (Guideline 13);
// HBM kernels grid-stride with ~8 workgroups per CU and 4 independent 16-B accesses in flight per
// lane; the GEMM (gemm_bf16_mfma_256p) uses a 256x256x64 tile, 8 waves each owning a 64x32 block of
// every 128x128 quadrant, operands DMA'd HBM->LDS with global_load_lds (two stages, XOR-swizzled) in
// half-tiles that stay in flight across barriers (counted vmcnt), the two wave groups one barrier
// apart, and an XCD-aware bijective workgroup remap (T1) so neighbouring tiles share an XCD's L2.
// The 2-phase loop (gemm_bf16_mfma_256) stays selectable ("gemmPipe":0). The older 128x128 register-staged
// kernel stays selectable ("gemmTile":128) for in-process A/B comparisons. Host side: one arena
// allocation per probe (the HBM pattern region is reused for the GEMM operands), pinned result
// slots and one stream sync per phase.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <type_traits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "mi355x/probe.h"

#define PROBE_CHECK(expr)                                                                 \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      throw ProbeError(std::string(#expr) + " -> " + hipGetErrorString(e_));             \
    }                                                                                     \
  } while (0)

namespace {

struct ProbeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;  // native vector: 16-B global ops
using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;

// ------------------------------------------------------------------ HBM pattern test
__device__ __forceinline__ uint32_t pattern_word(uint64_t idx, uint32_t seed) {
  // Cheap invertible mix of the word index: distinct per address, dense in both bit values.
  uint32_t x = static_cast<uint32_t>(idx) * 0x9E3779B1u ^ static_cast<uint32_t>(idx >> 32) * 0x85EBCA77u;
  x ^= seed;
  x ^= x >> 15;
  x *= 0x2C1B3C6Du;
  x ^= x >> 12;
  return x;
}

// Pattern of one 16-byte chunk. kPat 0: an independent mix per 32-bit word (3 integer multiplies
// per word; v_mul_lo_u32 is quarter rate, so 12 of them per 16 B). kPat 1: one multiply per 16 B —
// a bijective mix of the chunk index, its 4 words byte rotations of it XOR fixed masks. Both keep
// every chunk distinct from every other (an aliased address line reads another chunk's pattern)
// and both bit values dense; the complementary pass (flip) drives every bit to 0 and 1 either way.
template <int kPat>
__device__ __forceinline__ u32x4 pattern16(uint64_t i16, uint32_t seed, uint32_t flip) {
  u32x4 v;
  if constexpr (kPat == 0) {
    uint64_t w = i16 * 4;
    v.x = pattern_word(w, seed) ^ flip;
    v.y = pattern_word(w + 1, seed) ^ flip;
    v.z = pattern_word(w + 2, seed) ^ flip;
    v.w = pattern_word(w + 3, seed) ^ flip;
  } else {
    uint32_t h = (static_cast<uint32_t>(i16) ^ seed) * 0x9E3779B1u;
    h ^= __builtin_rotateleft32(static_cast<uint32_t>(i16 >> 32), 7);
    h ^= h >> 15;
    v.x = h ^ flip;
    v.y = __builtin_rotateleft32(h, 8) ^ 0xA5A5A5A5u ^ flip;
    v.z = __builtin_rotateleft32(h, 16) ^ 0x3C96C396u ^ flip;
    v.w = __builtin_rotateleft32(h, 24) ^ 0x5A0FF05Au ^ flip;
  }
  return v;
}
// Default pattern (probe option "hbmPattern" selects per run, for in-process A/B). Measured on
// MI355X, 9 interleaved rounds (profiles/r3h_probe_pattern_ab.json): 1 GiB test 6.16 -> 6.41 TB/s
// (write 5.77 -> 6.06, read 6.64 -> 6.76), claim-time probe (beside the MFMA phase) 0.98 -> 0.91 ms.
constexpr int kHbmPattern = 1;
// Grid-stride (0) measured faster than tiled (1) for the fill (6.03 vs 5.51 TB/s) and within 4 % for
// the verify: claim-time probe 0.757 vs 0.772 ms (profiles/r4h_probe_hbm_layout_ab_rejected.json).
constexpr int kHbmLayout = 0;

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

constexpr int kHbmThreads = 256;
constexpr int kHbmUnroll = 4;

// Layouts (probe option "hbmLayout", in-process A/B): 0 grid-stride — each unrolled access of a
// thread is a whole grid (MiBs) apart; 1 tiled — a workgroup's kHbmUnroll accesses per iteration
// cover one contiguous 16 KiB tile (more row-buffer locality per workgroup).
constexpr uint64_t kHbmTile = static_cast<uint64_t>(kHbmThreads) * kHbmUnroll;  // 16-B vectors

// Resets the first ``nreset`` result-counter pairs [bad bits = 0, first bad = all-ones] from block
// 0 on its way (null/0: none), so the claim-time probe enqueues no memsets ahead of its first fill.
__device__ __forceinline__ void reset_pairs(unsigned long long* __restrict__ cnt, int nreset) {
  if (blockIdx.x == 0 && static_cast<int>(threadIdx.x) < 2 * nreset)
    cnt[threadIdx.x] = (threadIdx.x & 1) ? ~0ull : 0ull;
}

template <int kPat = kHbmPattern, int kLayout = 0>
__global__ __launch_bounds__(kHbmThreads) void hbm_fill(u32x4* __restrict__ p, uint64_t n16,
                                                        uint32_t seed, uint32_t flip,
                                                        unsigned long long* __restrict__ reset, int nreset) {
  reset_pairs(reset, nreset);
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kHbmThreads;
  if constexpr (kLayout == 1) {
    const uint64_t tiles = n16 / kHbmTile;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
      const uint64_t base = t * kHbmTile + threadIdx.x;
#pragma unroll
      for (int u = 0; u < kHbmUnroll; ++u) {
        const uint64_t j = base + static_cast<uint64_t>(u) * kHbmThreads;
        __builtin_nontemporal_store(pattern16<kPat>(j, seed, flip), &p[j]);
      }
    }
    for (uint64_t i = tiles * kHbmTile + static_cast<uint64_t>(blockIdx.x) * kHbmThreads + threadIdx.x; i < n16;
         i += stride)
      __builtin_nontemporal_store(pattern16<kPat>(i, seed, flip), &p[i]);
    return;
  }
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * kHbmThreads + threadIdx.x;
  for (; i + (kHbmUnroll - 1) * stride < n16; i += kHbmUnroll * stride) {
#pragma unroll
    for (int u = 0; u < kHbmUnroll; ++u) {
      uint64_t j = i + u * stride;
      __builtin_nontemporal_store(pattern16<kPat>(j, seed, flip), &p[j]);
    }
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(pattern16<kPat>(i, seed, flip), &p[i]);
}

__device__ __forceinline__ uint32_t mismatches16(u32x4 v, u32x4 e) {
  return __builtin_popcount(v.x ^ e.x) + __builtin_popcount(v.y ^ e.y) +
         __builtin_popcount(v.z ^ e.z) + __builtin_popcount(v.w ^ e.w);
}

// Counts flipped BITS; records the lowest faulting 16-byte index. One atomic per wave.
template <int kPat = kHbmPattern, int kLayout = 0>
__global__ __launch_bounds__(kHbmThreads) void hbm_verify(const u32x4* __restrict__ p, uint64_t n16,
                                                          uint32_t seed, uint32_t flip,
                                                          unsigned long long* __restrict__ bad_bits,
                                                          unsigned long long* __restrict__ first_bad) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kHbmThreads;
  uint32_t bad = 0;
  uint64_t first = ~0ull;
  auto check = [&](u32x4 v, uint64_t j) {
    uint32_t m = mismatches16(v, pattern16<kPat>(j, seed, flip));
    if (m) {
      bad += m;
      first = umin64(first, j);
    }
  };
  if constexpr (kLayout == 1) {
    const uint64_t tiles = n16 / kHbmTile;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
      const uint64_t base = t * kHbmTile + threadIdx.x;
      u32x4 v[kHbmUnroll];
#pragma unroll
      for (int u = 0; u < kHbmUnroll; ++u) v[u] = __builtin_nontemporal_load(&p[base + static_cast<uint64_t>(u) * kHbmThreads]);
#pragma unroll
      for (int u = 0; u < kHbmUnroll; ++u) check(v[u], base + static_cast<uint64_t>(u) * kHbmThreads);
    }
    for (uint64_t i = tiles * kHbmTile + static_cast<uint64_t>(blockIdx.x) * kHbmThreads + threadIdx.x; i < n16;
         i += stride)
      check(__builtin_nontemporal_load(&p[i]), i);
  } else {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * kHbmThreads + threadIdx.x;
    for (; i + (kHbmUnroll - 1) * stride < n16; i += kHbmUnroll * stride) {
      u32x4 v[kHbmUnroll];
#pragma unroll
      for (int u = 0; u < kHbmUnroll; ++u) v[u] = __builtin_nontemporal_load(&p[i + u * stride]);
#pragma unroll
      for (int u = 0; u < kHbmUnroll; ++u) check(v[u], i + u * stride);
    }
    for (; i < n16; i += stride) check(__builtin_nontemporal_load(&p[i]), i);
  }
  // wave64 reduction
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    bad += __shfl_xor(bad, off, 64);
    first = umin64(first, static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(first), off, 64)));
  }
  if ((threadIdx.x & 63) == 0 && bad) {
    atomicAdd(bad_bits, static_cast<unsigned long long>(bad));
    atomicMin(first_bad, static_cast<unsigned long long>(first));
  }
}

// ------------------------------------------------------------------ operand generation
__device__ __forceinline__ short small_int_bf16(uint32_t h, int span) {
  // Integer in [-span, span] encoded as bf16 (exact).
  float v = static_cast<float>(static_cast<int>(h % static_cast<uint32_t>(2 * span + 1)) - span);
  return static_cast<short>(__float_as_uint(v) >> 16);
}

// ``zero``/``nzero``: the grid also zeroes nzero words (the MFMA phase's result slots, its ABFT
// accumulators), so that phase's stream needs no memsets and no hand-off from the HBM stream.
__global__ void gen_operand(short* __restrict__ out, uint64_t n, uint32_t seed, int span,
                            uint32_t* __restrict__ zero, uint64_t nzero) {
  for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < nzero;
       j += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    zero[j] = 0u;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i < n; i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = small_int_bf16(pattern_word(i, seed), span);
}

__device__ __forceinline__ float bf16_to_f32(short s) {
  return __uint_as_float(static_cast<uint32_t>(static_cast<uint16_t>(s)) << 16);
}

// ------------------------------------------------------------------ CU identity + MFMA census
// The hardware identity of the CU a wave runs on: XCC_ID (which XCD) and HW_ID's SE/SH/CU fields
// (CDNA3/4 ISA "HW_ID": CU_ID [11:8], SH_ID [12], SE_ID [15:13]). Both are read-only hardware
// registers (s_getreg), packed into an 11-bit key: xcc[10:8] se[7:5] sh[4] cu[3:0].
constexpr int kCuKeys = 2048, kCuMapWords = kCuKeys / 64;

__device__ __forceinline__ int cu_key() {
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return static_cast<int>(((xcc & 7u) << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u));
}

__device__ __forceinline__ void mark_cu(unsigned long long* map) {
  const int k = cu_key();
  atomicOr(&map[k >> 6], 1ull << (k & 63));
}

// Every CU must prove its matrix cores: each wave chains ``iters`` v_mfma_f32_16x16x32_bf16 on
// operands A[r][k] = fa(r), B[c][k] = gb(c) (small integers from the runtime seed, so nothing folds
// at compile time) and checks every accumulator against iters * 32 * fa(r) * gb(c), exact in fp32.
// A wave whose result is exact sets its CU's bit; a wrong result counts into ``bad``. The grid is
// several waves per CU slot so the dispatcher places work on every CU of every XCD.
constexpr int kCensusThreads = 256;
__global__ __launch_bounds__(kCensusThreads) void cu_census(unsigned long long* __restrict__ map,
                                                            unsigned long long* __restrict__ bad, int iters,
                                                            uint32_t seed, int fault_xcc) {
  const int lane = threadIdx.x & 63;
  const uint32_t h = seed ^ (blockIdx.x * 0x9E3779B1u);
  const int fa = 1 + static_cast<int>((h + (lane & 15)) & 3);          // row value of this lane's A fragment
  const int gb = 1 + static_cast<int>(((h >> 8) + (lane & 15)) & 3);   // col value of this lane's B fragment
  const short a16 = static_cast<short>(__float_as_uint(static_cast<float>(fa)) >> 16);
  const short b16 = static_cast<short>(__float_as_uint(static_cast<float>(gb)) >> 16);
  bf16x8 av, bv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a16;
    bv[j] = b16;
  }
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < iters; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  if (fault_xcc >= 0 && (cu_key() >> 8) == fault_xcc) acc[0] += 1.0f;  // test hook: a "bad" XCD
  // C/D layout of 16x16x32: col = lane&15, row = 4*(lane>>4) + j; fa of row r is held by lane r
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 4 * (lane >> 4) + j;
    const int far = 1 + static_cast<int>((h + r) & 3);
    ok = ok && acc[j] == static_cast<float>(iters * 32 * far * gb);
  }
  const bool wave_ok = __all(ok);
  if (lane == 0) {
    if (wave_ok) mark_cu(map);
    else atomicAdd(bad, 1ull);
  }
}

// ------------------------------------------------------------------ MFMA GEMM  C = A * Bt^T
// A: [M][K] bf16 row-major, Bt: [N][K] bf16 row-major (the "NT" layout: both operands are read
// along K, so every MFMA fragment is one contiguous 16-byte LDS read), C: [M][N] fp32.
constexpr int BM = 128, BN = 128, BK = 32;
constexpr int LDS_STRIDE = BK + 8;  // +16 B pad per row: 80-B rows spread ds_read_b128 lane groups
constexpr int kGemmThreads = 256;

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  // Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
  // consecutive logical tiles land on the same XCD (shared L2) under round-robin dispatch.
  int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__global__ __launch_bounds__(kGemmThreads, 2) void gemm_bf16_mfma_nt(const short* __restrict__ A,
                                                                      const short* __restrict__ Bt,
                                                                      float* __restrict__ C, int M,
                                                                      int N, int K) {
  __shared__ __attribute__((aligned(16))) short smem[2 * (BM + BN) * LDS_STRIDE];
  short* As = smem;
  short* Bs = smem + BM * LDS_STRIDE;

  const int tiles_n = N / BN;
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tile_m = wg / tiles_n, tile_n = wg % tiles_n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;  // 2x2 waves, each 64x64

  // global->register staging: 128 rows x 32 bf16 = 512 x 16 B per operand, 2 per thread
  const int ld_row = tid >> 2, ld_col = (tid & 3) * 8;
  const short* a_src = A + static_cast<int64_t>(tile_m * BM + ld_row) * K + ld_col;
  const short* b_src = Bt + static_cast<int64_t>(tile_n * BN + ld_row) * K + ld_col;
  const int64_t row64 = static_cast<int64_t>(64) * K;

  bf16x8 ra0, ra1, rb0, rb1;
  auto gload = [&](int k0) {
    ra0 = *reinterpret_cast<const bf16x8*>(a_src + k0);
    ra1 = *reinterpret_cast<const bf16x8*>(a_src + row64 + k0);
    rb0 = *reinterpret_cast<const bf16x8*>(b_src + k0);
    rb1 = *reinterpret_cast<const bf16x8*>(b_src + row64 + k0);
  };
  auto swrite = [&](int buf) {
    short* as = As + buf * (BM + BN) * LDS_STRIDE;
    short* bs = as + BM * LDS_STRIDE;
    *reinterpret_cast<bf16x8*>(as + ld_row * LDS_STRIDE + ld_col) = ra0;
    *reinterpret_cast<bf16x8*>(as + (ld_row + 64) * LDS_STRIDE + ld_col) = ra1;
    *reinterpret_cast<bf16x8*>(bs + ld_row * LDS_STRIDE + ld_col) = rb0;
    *reinterpret_cast<bf16x8*>(bs + (ld_row + 64) * LDS_STRIDE + ld_col) = rb1;
  };
  (void)Bs;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;  // fragment row/col and k-half
  gload(0);
  swrite(0);
  __syncthreads();
  const int ksteps = K / BK;
  for (int kt = 0; kt < ksteps; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ksteps) gload((kt + 1) * BK);  // next tile in flight under this tile's MFMAs
    const short* as = As + buf * (BM + BN) * LDS_STRIDE;
    const short* bs = as + BM * LDS_STRIDE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(as + (wr * 64 + i * 32 + fr) * LDS_STRIDE + ks * 16 + fh * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(bs + (wc * 64 + j * 32 + fr) * LDS_STRIDE + ks * 16 + fh * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < ksteps) swrite(buf ^ 1);  // other buffer: last read one iteration ago
    __syncthreads();
  }
  // C/D layout of 32x32x16: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = tile_n * BN + wc * 64 + j * 32 + fr;
      const int row0 = tile_m * BM + wr * 64 + i * 32 + 4 * fh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + (r & 3) + 8 * (r >> 2);
        C[static_cast<int64_t>(row) * N + col] = acc[i][j][r];
      }
    }
}

// ------------------------------------------------------------------ MFMA GEMM, 256x256 tile
// The probe's main GEMM (cdna_hip_programming.md §5 "glds, 2 LDS buffers, BK=64" row and the
// T3/T4 "minimum 2-phase" loop), C = A * Bt^T with the same NT layout as above:
//   * 256x256x64 block tile, 8 waves as 2(M) x 4(N), each wave 128x64 = 8x4 tiles of
//     v_mfma_f32_16x16x32_bf16 (64 MFMAs per wave per K-step, 128 accumulator registers);
//   * operands staged HBM -> LDS by global_load_lds_dwordx4 (no VGPR round trip, 8 per thread per
//     K-step), two 64 KiB LDS stages: the next K-tile's DMA is issued before this tile's
//     ds_reads + MFMAs and retired by one vmcnt(0) + barrier per K-step;
//   * st_16x32-style XOR swizzle so each 16-lane ds_read_b128 group hits 16 distinct 16-B bank
//     slots: glds writes LDS lane-linearly, so the permutation is applied to the per-lane GLOBAL
//     source address and the same involution on the read (rule 21);
//   * one block per CU at N=4096 (256 tiles), XCD-aware bijective remap (T1).
constexpr int G2_BM = 256, G2_BN = 256, G2_BK = 64;
// Tile order of gemm_bf16_mfma_256: 0 row-major, > 1 grouped. Groups of 4 tile rows: 8192^3 1331 vs
// 1118 TFLOP/s (+19 %), 4096^3 unchanged (1366 vs 1372) (profiles/r4q_probe_gemm_group_ab.json).
constexpr int kGemmGroupM = 4;
// K-loop of the 256x256 GEMM ("gemmPipe" selects per probe): 0 the 2-phase loop, 1 the half-tile
// pipeline, 2 the half-tile pipeline with staggered wave groups and a static s_setprio(1) for waves
// 4-7 (default: 4096^3 1411 vs 1276 TFLOP/s for 0, 8192^3 1459 vs 1339, profiles/r6v_gemm_prio_ab.json),
// 21 the same with s_setprio flips around every MFMA cluster instead (1358 / 1430; r6q, r6s), 22 with
// no s_setprio, 3 the 32x32x16 fragment-ring variant (measured slower, r6t: A/B only). Also measured
// and dropped: the phase reads as inline-asm ds_read_b128 in k-sub order with counted lgkmcnt, so a
// quadrant's first MFMAs start on half its fragments (4096^3 1354 vs 1411, 8192^3 1420 vs 1456,
// profiles/r6za_gemm_counted_reads_ab_rejected.json), and tile-row groups of 2/8/16 instead of 4
// (r6z_gemm_group_ab.json).
constexpr int kGemmPipe = 2;
constexpr int kGemm2Threads = 512;
constexpr int G2_STAGE_SHORTS = (G2_BM + G2_BN) * G2_BK;  // one stage: A then B, 64 KiB
typedef __attribute__((address_space(3))) void lds_void_t;

// byte offset, inside a [rows][64] bf16 tile (128-B rows), of logical 16-B chunk c of row r
__device__ __forceinline__ int g2_swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// kPrio: s_setprio(1) around each K-step's MFMA block (cdna_hip_programming.md T5). Measured null on
// this 2-phase loop (4096^3 1246 vs 1236, 8192^3 1315 vs 1312 TFLOP/s, profiles/
// r4u_gemm_setprio_ab_rejected.json): off by default, selectable for A/B ("gemmPrio").
// kVecC: the MFMA computes each 16x16 tile transposed (B fragment as the first operand), so a lane
// holds 4 consecutive columns of one C row and the epilogue writes them as one 16-byte store
// instead of four 4-byte ones (same MFMAs, same C). Measured no faster (4096^3 1322 vs 1322, 2048^3
// 315 vs 337 TFLOP/s, profiles/r4v_gemm_vecc_ab_rejected.json): off, selectable ("gemmVecC").
template <bool kPrio = false, bool kVecC = false>
__global__ __launch_bounds__(kGemm2Threads, 1) void gemm_bf16_mfma_256(const short* __restrict__ A,
                                                                       const short* __restrict__ Bt,
                                                                       float* __restrict__ C, int M,
                                                                       int N, int K,
                                                                       unsigned long long* __restrict__ cu_map,
                                                                       int group_m) {
  __shared__ __attribute__((aligned(16))) short smem[2 * G2_STAGE_SHORTS];  // 128 KiB, the only LDS object
  if (cu_map && threadIdx.x == 0) mark_cu(cu_map);  // which CUs ran GEMM tiles (probe report)
  const int tiles_n = N / G2_BN, tiles_m = M / G2_BM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  // Tile order inside each XCD's contiguous range of wg (xcd_remap): row-major (group_m <= 1) walks
  // whole tile rows, so the tiles an XCD runs at once share one or two A panels but need a B panel
  // each; grouped (group_m rows at a time, column-major inside a group) makes them a group_m x k
  // block that shares both, less operand traffic into the XCD's 4 MB L2 per K-step. Bijective.
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n, first_m = (wg / per_group) * group_m;
    const int gm = min(tiles_m - first_m, group_m), r = wg % per_group;
    tile_m = first_m + r % gm;
    tile_n = r / gm;
  } else {
    tile_m = wg / tiles_n;
    tile_n = wg % tiles_n;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  // glds source addresses. Chunk q = i*512 + tid (i = 0..3) of a 256x8-chunk operand tile lands at
  // LDS byte q*16 (lane-linear per wave: q = i*512 + wave*64 + lane): LDS row q>>3, slot q&7. The
  // slot holds logical chunk (slot ^ swz(row)), so that is the chunk we fetch.
  const short* a_src[4];
  const short* b_src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * kGemm2Threads + tid, row = q >> 3, slot = q & 7;
    const int chunk = slot ^ ((row >> 1) & 7);
    a_src[i] = A + static_cast<int64_t>(tile_m * G2_BM + row) * K + chunk * 8;
    b_src[i] = Bt + static_cast<int64_t>(tile_n * G2_BN + row) * K + chunk * 8;
  }
  // wave-uniform LDS destinations (M0) for instruction i of this wave: byte (i*512 + wave*64)*16
  auto stage = [&](int buf, int k0) {
    char* base = reinterpret_cast<char*>(smem) + buf * G2_STAGE_SHORTS * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = (i * kGemm2Threads + wave * 64) * 16;
      __builtin_amdgcn_global_load_lds(a_src[i] + k0, (lds_void_t*)(base + off), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(b_src[i] + k0, (lds_void_t*)(base + G2_BM * 128 + off), 16,
                                       0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;  // fragment row and k-quarter (8 elements)
  const int ksteps = K / G2_BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < ksteps; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ksteps) stage(cur ^ 1, (kt + 1) * G2_BK);  // next tile's DMA under this tile's MFMAs
    const char* as = reinterpret_cast<const char*>(smem) + cur * G2_STAGE_SHORTS * 2;
    const char* bs = as + G2_BM * 128;
#pragma unroll
    for (int ks = 0; ks < G2_BK / 32; ++ks) {
      const int c = ks * 4 + fq;
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int n = 0; n < 4; ++n)
        bfr[n] = *reinterpret_cast<const bf16x8*>(bs + g2_swz(wc * 64 + n * 16 + fr, c));
#pragma unroll
      for (int m = 0; m < 8; ++m)
        af[m] = *reinterpret_cast<const bf16x8*>(as + g2_swz(wr * 128 + m * 16 + fr, c));
      if constexpr (kPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          if constexpr (kVecC)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[n], af[m], acc[m][n], 0, 0, 0);
          else
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
        }
      if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile kt+1 has landed
    __syncthreads();                                   // ...and every other wave's; reads of kt done
  }
  if constexpr (kVecC) {
    // transposed tile: lane holds C[m*16 + (lane&15)][n*16 + 4*(lane>>4) + j], j = 0..3
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = tile_m * G2_BM + wr * 128 + m * 16 + fr;
        const int col0 = tile_n * G2_BN + wc * 64 + n * 16 + 4 * fq;
        *reinterpret_cast<f32x4*>(C + static_cast<int64_t>(row) * N + col0) = acc[m][n];
      }
  } else {
    // C/D layout of 16x16x32: col = lane&15, row = 4*(lane>>4) + j
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = tile_n * G2_BN + wc * 64 + n * 16 + fr;
        const int row0 = tile_m * G2_BM + wr * 128 + m * 16 + 4 * fq;
#pragma unroll
        for (int j = 0; j < 4; ++j) C[static_cast<int64_t>(row0 + j) * N + col] = acc[m][n][j];
      }
  }
}

// ------------------------------------------------------------------ MFMA GEMM, 256x256, half-tile pipeline
// Same tile, LDS image, swizzle and tile order as gemm_bf16_mfma_256, but the K-loop no longer
// drains its DMA at every K-step (cdna_hip_programming.md §5 "Pipelining across barriers", T3+T4):
//   * a K-tile is four half-tiles (A rows 0-127 "A0", B rows 0-127 "B0", "B1", "A1"), each 16 KiB,
//     two global_load_lds per thread; K-tile t+1's half h is issued in phase h of K-tile t;
//   * each wave owns a 64x32 sub-block in each of the block tile's four 128x128 quadrants, so
//     phase 0 needs only A0+B0, phase 1 B1, phase 2 A1 (phase 3 computes from registers): the
//     wait before a phase retires just the halves it reads — counted vmcnt(4), i.e. two halves
//     stay in flight across every barrier — and a raw s_barrier (no __syncthreads: its fence
//     would drain the DMA) publishes them to every wave;
//   * WAR: half h of K-tile t+1 lands in K-tile t-1's buffer, whose half h was last read in a
//     phase <= h of K-tile t-1, at least one barrier earlier;
//   * s_setprio(1) around each 16-MFMA quadrant keeps hipcc from moving the cluster across the
//     barriers (T5).
// All LDS is the one __shared__ array (a second LDS object makes hipcc wait vmcnt(0) before ds_reads).
// kStagger: waves 4-7 run one phase (one barrier) behind waves 0-3, so on each SIMD one wave reads
// LDS while the other runs its MFMAs. Every wave then retires a half one phase BEFORE the phase that
// reads it (a reader one barrier behind the writer needs one barrier more: §5 "Read a staged buffer
// one phase AFTER the wait that retires it"), every phase has a barrier, and both groups execute
// the same number of barriers (group 1 one extra before the loop, group 0 one extra after it).
// kAblate (timing experiments only, wrong C): 1 = no DMA inside the K-loop, 2 = no MFMAs.
// kPrio: 0 s_setprio(1) around every quadrant's MFMAs, 1 one static s_setprio(1) for waves 4-7 and
// no flips (MI355X_MICROARCH.md §Two waves per SIMD item 4), 2 none.
template <bool kStagger, int kAblate = 0, int kPrio = 0>
__global__ __launch_bounds__(kGemm2Threads, 1) void gemm_bf16_mfma_256p(const short* __restrict__ A,
                                                                        const short* __restrict__ Bt,
                                                                        float* __restrict__ C, int M,
                                                                        int N, int K,
                                                                        unsigned long long* __restrict__ cu_map,
                                                                        int group_m) {
  __shared__ __attribute__((aligned(16))) short smem[2 * G2_STAGE_SHORTS];  // 128 KiB
  if (cu_map && threadIdx.x == 0) mark_cu(cu_map);
  const int tiles_n = N / G2_BN, tiles_m = M / G2_BM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n, first_m = (wg / per_group) * group_m;
    const int gm = min(tiles_m - first_m, group_m), r = wg % per_group;
    tile_m = first_m + r % gm;
    tile_n = r / gm;
  } else {
    tile_m = wg / tiles_n;
    tile_n = wg % tiles_n;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  // half-tile h (0 A0, 1 B0, 2 B1, 3 A1): operand and row half
  // chunk q = i*512 + tid (i = 0, 1) of a 128x8-chunk half lands at byte q*16 of the half's LDS
  // image: row q>>3, slot q&7 holding logical chunk slot ^ ((row>>1)&7) (the full-tile row has
  // the same bits 1..3, so the swizzle matches g2_swz on the 256-row image)
  const short* src[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const bool is_a = (h == 0 || h == 3);
    const int half = (h == 0 || h == 1) ? 0 : 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = i * kGemm2Threads + tid, row = q >> 3, slot = q & 7;
      const int chunk = slot ^ ((row >> 1) & 7);
      const int grow = (is_a ? tile_m * G2_BM : tile_n * G2_BN) + half * 128 + row;
      src[h][i] = (is_a ? A : Bt) + static_cast<int64_t>(grow) * K + chunk * 8;
    }
  }
  auto stage_half = [&](int buf, int h, int k0) {
    if (kAblate == 1 && k0 > 0) return;
    const bool is_a = (h == 0 || h == 3);
    const int half = (h == 0 || h == 1) ? 0 : 1;
    char* base = reinterpret_cast<char*>(smem) + buf * G2_STAGE_SHORTS * 2 + (is_a ? 0 : G2_BM * 128) +
                 half * 128 * 128;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds(src[h][i] + k0, (lds_void_t*)(base + (i * kGemm2Threads + wave * 64) * 16),
                                       16, 0, 0);
  };

  f32x4 acc[4][4][2];  // [quadrant i*2+j][m][n]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[q][m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int ksteps = K / G2_BK;
  bf16x8 af[2][4], b0f[2][2], b1f[2][2];  // [k-sub][m|n]
  auto read_a = [&](const char* as, int half) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        af[ks][m] = *reinterpret_cast<const bf16x8*>(as + g2_swz(half * 128 + wr * 64 + m * 16 + fr, ks * 4 + fq));
  };
  auto read_b = [&](const char* bs, int half, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        bf[ks][n] = *reinterpret_cast<const bf16x8*>(bs + g2_swz(half * 128 + wc * 32 + n * 16 + fr, ks * 4 + fq));
  };
  auto quadrant = [&](f32x4 (&c)[4][2], const bf16x8 (&bf)[2][2]) {
    if constexpr (kAblate == 2) {  // keep the fragment reads alive without the matrix work
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int m = 0; m < 4; ++m) asm volatile("" ::"v"(af[ks][m]));
#pragma unroll
        for (int n = 0; n < 2; ++n) asm volatile("" ::"v"(bf[ks][n]));
      }
      return;
    }
    if constexpr (kPrio == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][m], bf[ks][n], c[m][n], 0, 0, 0);
    if constexpr (kPrio == 0) __builtin_amdgcn_s_setprio(0);
  };
  auto sync = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS read moves above the barrier
  };

#pragma unroll
  for (int h = 0; h < 4; ++h) stage_half(0, h, 0);
  // group 1 = waves 4-7; readfirstlane makes the branch scalar (a divergent-looking `if` would
  // run the s_barrier for every wave: balanced, but no stagger)
  const bool group1 = __builtin_amdgcn_readfirstlane(wave) >= 4;
  if constexpr (kPrio == 1) {
    if (group1) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr (kStagger) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A0, B0 of tile 0
    sync();
    if (group1) sync();
  }
  // one K-tile: kLast drops the prefetch and retires the tail with smaller counts
  auto ktile = [&](int t, auto last_tag) {
    constexpr bool kLast = decltype(last_tag)::value;
    const int cur = t & 1, k1 = (t + 1) * G2_BK;
    const char* as = reinterpret_cast<const char*>(smem) + cur * G2_STAGE_SHORTS * 2;
    const char* bs = as + G2_BM * 128;
    if constexpr (kStagger) {
      // waits retire what the NEXT phase reads: outstanding before phase 0 = B1, A1 of this tile
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // B1 (read in phase 1)
      sync();
      if constexpr (!kLast) stage_half(cur ^ 1, 0, k1);
      read_a(as, 0);
      read_b(bs, 0, b0f);
      quadrant(acc[0], b0f);
      if constexpr (kLast) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // A1 (read in phase 2); A0' in flight
      sync();
      if constexpr (!kLast) stage_half(cur ^ 1, 1, k1);
      read_b(bs, 1, b1f);
      quadrant(acc[1], b1f);
      sync();
      if constexpr (!kLast) stage_half(cur ^ 1, 2, k1);
      read_a(as, 1);
      quadrant(acc[3], b1f);
      if constexpr (!kLast) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // A0', B0' (next tile's phase 0)
      sync();
      if constexpr (!kLast) stage_half(cur ^ 1, 3, k1);
      quadrant(acc[2], b0f);
    } else {
      // phase 0: A0 + B0 of this tile (A1, B1 may still be in flight)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      sync();
      if constexpr (!kLast) stage_half(cur ^ 1, 0, k1);
      read_a(as, 0);
      read_b(bs, 0, b0f);
      quadrant(acc[0], b0f);
      // phase 1: B1
      if constexpr (kLast) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      sync();
      if constexpr (!kLast) stage_half(cur ^ 1, 1, k1);
      read_b(bs, 1, b1f);
      quadrant(acc[1], b1f);
      // phase 2: A1
      if constexpr (kLast) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      sync();
      if constexpr (!kLast) stage_half(cur ^ 1, 2, k1);
      read_a(as, 1);
      quadrant(acc[3], b1f);
      // phase 3: registers only (A1 x B0); A1 of the next tile goes out
      if constexpr (!kLast) stage_half(cur ^ 1, 3, k1);
      quadrant(acc[2], b0f);
    }
  };
  for (int t = 0; t + 1 < ksteps; ++t) ktile(t, std::false_type{});
  ktile(ksteps - 1, std::true_type{});
  if constexpr (kStagger) {
    if (!group1) sync();  // balance group 1's extra barrier: every wave ran 4*ksteps + 2
  }

  // C/D layout of 16x16x32: col = lane&15, row = 4*(lane>>4) + j; quadrant q = i*2 + j
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = tile_n * G2_BN + (q & 1) * 128 + wc * 32 + n * 16 + fr;
        const int row0 = tile_m * G2_BM + (q >> 1) * 128 + wr * 64 + m * 16 + 4 * fq;
#pragma unroll
        for (int j = 0; j < 4; ++j) C[static_cast<int64_t>(row0 + j) * N + col] = acc[q][m][n][j];
      }
}

// ------------------------------------------------------------------ MFMA GEMM, 256x256, 32x32x16 + fragment ring
// The same tile, LDS image and DMA as gemm_bf16_mfma_256 (one 64 KiB K-tile per stage, two stages,
// one barrier per K-tile), with the fragment reads pipelined instead of issued in a burst:
//   * v_mfma_f32_32x32x16_bf16: a wave's 128x64 is 4x2 tiles of 32x32, a K-tile 4 k-steps of 16,
//     8 MFMAs (256 matrix cycles) per k-step;
//   * two fragment register sets (A 4 x 16 B, B 2 x 16 B each): while k-step s runs its MFMAs from
//     one set, the 6 ds_read_b128 of k-step s+1 fill the other — the reads sit in the MFMA gaps
//     (2 per 32-cycle gap cost ~nothing, MI355X_MICROARCH.md §LDS) instead of in front of them;
//   * k-step 0 of the next K-tile is read during k-step 3 of this one, so the K-tile's barrier sits
//     between k-steps 2 and 3: vmcnt(0) (this wave's DMA of the next tile, issued a K-tile ago) +
//     lgkmcnt(0) (its reads of this tile's last k-step, so the stage can be overwritten) + barrier,
//     then the DMA of the tile after next goes into this tile's stage.
// 32x32x16 operand map: lane l holds A[row l&31][k 8*(l>>5) + j], B likewise; C: col = l&31,
// row = (reg&3) + 8*(reg>>2) + 4*(l>>5).
__global__ __launch_bounds__(kGemm2Threads, 1) void gemm_bf16_mfma_256x(const short* __restrict__ A,
                                                                        const short* __restrict__ Bt,
                                                                        float* __restrict__ C, int M,
                                                                        int N, int K,
                                                                        unsigned long long* __restrict__ cu_map,
                                                                        int group_m) {
  __shared__ __attribute__((aligned(16))) short smem[2 * G2_STAGE_SHORTS];  // 128 KiB
  if (cu_map && threadIdx.x == 0) mark_cu(cu_map);
  const int tiles_n = N / G2_BN, tiles_m = M / G2_BM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n, first_m = (wg / per_group) * group_m;
    const int gm = min(tiles_m - first_m, group_m), r = wg % per_group;
    tile_m = first_m + r % gm;
    tile_n = r / gm;
  } else {
    tile_m = wg / tiles_n;
    tile_n = wg % tiles_n;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const short* a_src[4];
  const short* b_src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * kGemm2Threads + tid, row = q >> 3, slot = q & 7;
    const int chunk = slot ^ ((row >> 1) & 7);
    a_src[i] = A + static_cast<int64_t>(tile_m * G2_BM + row) * K + chunk * 8;
    b_src[i] = Bt + static_cast<int64_t>(tile_n * G2_BN + row) * K + chunk * 8;
  }
  auto stage = [&](int buf, int k0) {
    char* base = reinterpret_cast<char*>(smem) + buf * G2_STAGE_SHORTS * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = (i * kGemm2Threads + wave * 64) * 16;
      __builtin_amdgcn_global_load_lds(a_src[i] + k0, (lds_void_t*)(base + off), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(b_src[i] + k0, (lds_void_t*)(base + G2_BM * 128 + off), 16, 0, 0);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[m][n][j] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  bf16x8 ra0[4], rb0[2], ra1[4], rb1[2];  // the two fragment sets
  // Fragment reads are inline-asm ds_read_b128 with hand-counted lgkmcnt: hipcc waits lgkmcnt(0)
  // for its own reads before every MFMA group here, which serialises the ring. hipcc neither
  // tracks nor waits for these, so every use sits behind an explicit wait + sched_barrier
  // (cdna_hip_programming.md §5.4 rule 18).
  typedef __attribute__((address_space(3))) char lds_char_t;
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_char_t*)smem));
  // per-lane byte offset of k-step s inside a stage, A rows (wr*128 + fr) and B rows (wc*64 + fr);
  // the m / n tiles add 32 rows = 4096 B (the swizzle depends on row bits 1..3 only)
  uint32_t a_off[4], b_off[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    a_off[st] = lds0 + g2_swz(wr * 128 + fr, 2 * st + fh);
    b_off[st] = lds0 + G2_BM * 128 + g2_swz(wc * 64 + fr, 2 * st + fh);
  }
  auto ds16 = [](uint32_t addr) {
    bf16x8 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
    return r;
  };
  auto read = [&](int buf, int st, bf16x8 (&ra)[4], bf16x8 (&rb)[2]) {
    const uint32_t bo = static_cast<uint32_t>(buf) * (G2_STAGE_SHORTS * 2);
#pragma unroll
    for (int n = 0; n < 2; ++n) rb[n] = ds16(b_off[st] + bo + n * 4096);
#pragma unroll
    for (int m = 0; m < 4; ++m) ra[m] = ds16(a_off[st] + bo + m * 4096);
  };
  auto wait_lgkm6 = [] {
    asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto wait_lgkm0 = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma = [&](const bf16x8 (&ra)[4], const bf16x8 (&rb)[2]) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[m], rb[n], acc[m][n], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  const int ksteps = K / G2_BK;
  stage(0, 0);
  if (ksteps > 1) stage(1, G2_BK);
  if (ksteps > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // stage 0 (stage 1 in flight)
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read(0, 0, ra0, rb0);
  for (int t = 0; t < ksteps; ++t) {
    const int cur = t & 1;
    read(cur, 1, ra1, rb1);
    wait_lgkm6();  // k-step 0's six reads are in, k-step 1's six may be in flight
    mfma(ra0, rb0);
    read(cur, 2, ra0, rb0);
    wait_lgkm6();
    mfma(ra1, rb1);
    read(cur, 3, ra1, rb1);
    wait_lgkm6();
    mfma(ra0, rb0);
    if (t + 1 < ksteps) {
      // the next tile's stage has landed (this wave's part; the barrier makes it everyone's) and
      // this wave's reads of this stage are done, so the tile after next may overwrite it
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < ksteps) stage(cur, (t + 2) * G2_BK);
      __builtin_amdgcn_sched_barrier(0);
      read(cur ^ 1, 0, ra0, rb0);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      wait_lgkm0();
    }
    mfma(ra1, rb1);
  }

#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int col = tile_n * G2_BN + wc * 64 + n * 32 + fr;
      const int rbase = tile_m * G2_BM + wr * 128 + m * 32 + 4 * fh;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        C[static_cast<int64_t>(rbase + (j & 3) + 8 * (j >> 2)) * N + col] = acc[m][n][j];
    }
}

// Full VALU reference (independent of the matrix cores), fp32, k-ordered.
// One thread per output; both operand rows read with 16-byte loads (K % 8 == 0).
__global__ void gemm_ref_valu(const short* __restrict__ A, const short* __restrict__ Bt,
                              float* __restrict__ C, int M, int N, int K) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  int m = blockIdx.y;
  if (n >= N || m >= M) return;
  const bf16x8* a = reinterpret_cast<const bf16x8*>(A + static_cast<int64_t>(m) * K);
  const bf16x8* b = reinterpret_cast<const bf16x8*>(Bt + static_cast<int64_t>(n) * K);
  float s = 0.f;
  for (int k8 = 0; k8 < K / 8; ++k8) {
    const bf16x8 av = a[k8], bv = b[k8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf(bf16_to_f32(av[j]), bf16_to_f32(bv[j]), s);
  }
  C[static_cast<int64_t>(m) * N + n] = s;
}

__global__ void count_diff(const float* __restrict__ x, const float* __restrict__ y, uint64_t n,
                           unsigned long long* __restrict__ bad) {
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint32_t b = 0;
  for (; i < n; i += static_cast<uint64_t>(gridDim.x) * blockDim.x) b += x[i] != y[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) b += __shfl_xor(b, off, 64);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(bad, static_cast<unsigned long long>(b));
}

// ABFT (algorithm-based fault tolerance) checks. Every operand is a small integer, so with
// C = A * Bt^T these identities hold over the integers, and therefore modulo 2^32:
//   column checksum  sum_m C[m][n] == sum_k (sum_m A[m][k]) * Bt[n][k]
//   row checksum     sum_n C[m][n] == sum_k A[m][k] * (sum_n Bt[n][k])
// All arithmetic is unsigned 32-bit (wraps exactly; a corrupted element changes a sum by a
// non-multiple of 2^32). Two memory-bound primitives with 16-byte loads per lane and four loads in
// flight (profiles/r1q: the former 2-byte-load / int64 versions took ~0.5 ms per probe, 4-5x the
// GEMM they check).
__device__ __forceinline__ uint32_t to_u32(short v) { return static_cast<uint32_t>(static_cast<int>(bf16_to_f32(v))); }
__device__ __forceinline__ uint32_t to_u32(float v) {
  // clamp first: an out-of-range float-to-int conversion is undefined (colsum_partial flags it)
  return static_cast<uint32_t>(static_cast<int>(fminf(fmaxf(v, -2.0e9f), 2.0e9f)));
}

constexpr int kColRows = 64;  // rows per colsum_partial block (4 waves x 16 interleaved rows)
constexpr int kUnroll = 4;    // independent 16-byte loads in flight per lane

// Column sums: a lane owns V = 16/sizeof(T) adjacent columns (one 16-byte load per row); the
// block's 4 waves take interleaved rows of a kColRows chunk, combine through LDS, and add one
// 32-bit atomic per column. cols % V == 0.
// For the fp32 product C the same pass also flags any element that is not an exact integer, is
// not finite, or exceeds ``bound`` (= K * span^2): a corrupted element that keeps its integer part
// (a low-mantissa flip) or wraps the int cast would otherwise leave the mod-2^32 sums intact.
template <class T>
__global__ __launch_bounds__(256) void colsum_partial(const T* __restrict__ X, int rows, int cols,
                                                      uint32_t* __restrict__ out, float bound,
                                                      unsigned long long* __restrict__ bad) {
  constexpr int V = 16 / sizeof(T);
  using vec = __attribute__((ext_vector_type(V))) T;
  __shared__ uint32_t part[4][64 * V];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cb = blockIdx.x * 64 * V;
  const int c0 = cb + lane * V;
  const int r0 = blockIdx.y * kColRows;
  const int r1 = min(rows, r0 + kColRows);
  uint32_t acc[V] = {};
  uint32_t odd = 0;
  if (c0 < cols) {
    for (int r = r0 + wave; r < r1; r += 4 * kUnroll) {
      vec v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        if (r + 4 * u < r1) v[u] = *reinterpret_cast<const vec*>(X + static_cast<int64_t>(r + 4 * u) * cols + c0);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        if (r + 4 * u < r1) {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const T x = static_cast<T>(v[u][j]);
            if constexpr (sizeof(T) == 4) odd += !(x == rintf(x) && fabsf(x) <= bound);  // NaN fails both
            acc[j] += to_u32(x);
          }
        }
    }
  }
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) odd += __shfl_xor(odd, off, 64);
    if (lane == 0 && odd && bad) atomicAdd(bad, static_cast<unsigned long long>(odd));
  }
#pragma unroll
  for (int j = 0; j < V; ++j) part[wave][lane * V + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * V && cb + i < cols; i += 256)
    atomicAdd(&out[cb + i], part[0][i] + part[1][i] + part[2][i] + part[3][i]);
}

// out[r] = sum_k X[r][k] * w[k] mod 2^32 (w = nullptr: plain row sums); one wave64 per row, 4 rows
// per block. The 32-bit weights (colsum_partial's output) are read with 16-byte loads and stay in
// L1/L2 (K * 4 bytes). K % V == 0.
template <class T>
__global__ __launch_bounds__(256) void rowdot(const T* __restrict__ X, int rows, int K, const uint32_t* __restrict__ w,
                                              uint32_t* __restrict__ out) {
  constexpr int V = 16 / sizeof(T);
  using vec = __attribute__((ext_vector_type(V))) T;
  using wvec = __attribute__((ext_vector_type(V))) uint32_t;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* x = X + static_cast<int64_t>(row) * K;
  uint32_t s = 0;
  for (int k0 = lane * V; k0 < K; k0 += 64 * V * kUnroll) {
    vec v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      if (k0 + u * 64 * V < K) v[u] = *reinterpret_cast<const vec*>(x + k0 + u * 64 * V);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = k0 + u * 64 * V;
      if (k >= K) break;
      if (w) {
        const wvec wv = *reinterpret_cast<const wvec*>(w + k);
#pragma unroll
        for (int j = 0; j < V; ++j) s += to_u32(static_cast<T>(v[u][j])) * wv[j];
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) s += to_u32(static_cast<T>(v[u][j]));
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[row] = s;
}

// ---- fault injection (test hooks: prove the checkers catch corruption on real hardware)
// Flips bit (i % 32) of word i*stride for i < count: distinct words, so exactly ``count`` bits.
__global__ void inject_bit_flips(unsigned int* __restrict__ p, uint64_t nwords, int count) {
  const uint64_t stride = nwords / static_cast<uint64_t>(count + 1);
  for (int i = threadIdx.x; i < count; i += blockDim.x) p[static_cast<uint64_t>(i + 1) * stride] ^= 1u << (i % 32);
}

// mode 1: +1.0 (an integer error: caught by the mod-2^32 checksums); mode 2: +0.25 (the integer
// part survives: caught only by the integrality check); mode 3: NaN.
__global__ void inject_gemm_fault(float* __restrict__ c, int64_t idx, int mode) {
  if (mode == 1) c[idx] += 1.0f;
  else if (mode == 2) c[idx] += 0.25f;
  else c[idx] = __int_as_float(0x7fc00000);
}

__global__ void count_ne_u32(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, int n,
                             unsigned long long* __restrict__ bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t d = (i < n && a[i] != b[i]) ? 1u : 0u;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
  if ((threadIdx.x & 63) == 0 && d) atomicAdd(bad, static_cast<unsigned long long>(d));
}

// ------------------------------------------------------------------ host side
constexpr long long kMaxPatterns = 4;
// device counter / pinned host result slots: 2 per HBM pattern, then the two GEMM check counters
constexpr int kSlotSmall = 2 * kMaxPatterns, kSlotAbft = kSlotSmall + 1, kSlotCensusBad = kSlotAbft + 1,
              kSlotCensusMap = kSlotCensusBad + 1, kSlotGemmMap = kSlotCensusMap + kCuMapWords,
              kResSlots = kSlotGemmMap + kCuMapWords;
constexpr int kCensusIters = 128;
static_assert(2 * kMaxPatterns <= kHbmThreads, "hbm_fill resets the HBM pairs from one block");

// The HBM sweep buffer is allocated as kSweepChunk pieces, not one ~282 GiB allocation: freeing
// one huge mapping held the process's address-space lock for ~2.5 s, and every thread of the agent
// that mapped memory meanwhile (a thread start, a large malloc) stalled behind it — a claim issued
// right after a scrub waited 2.46 s (profiles/r2o_scrub_claim_diag.txt). Per chunk the stall is
// bounded by one chunk's unmap. 1 GiB: VRAM that an earlier process used is cleared as it is mapped
// again, at ~35 GB/s — 121 ms per 4 GiB chunk on a box whose last tenant left 90 GiB dirty
// (profiles/r4r_sweep_chunks.txt) — and a claim-time probe that arrives mid-chunk waits for it.
constexpr uint64_t kSweepChunk = 1ull << 30;

struct SweepBuf {
  std::vector<void*> chunks;  // kSweepChunk bytes each, the last one possibly shorter
  uint64_t span = 0;
  bool empty() const { return chunks.empty(); }
};

struct DeviceCtx {
  hipStream_t stream = nullptr;   // HBM pattern test
  hipStream_t stream2 = nullptr;  // MFMA checks, overlapped with the bandwidth-bound HBM test
  hipEvent_t ev[1 + 2 * kMaxPatterns] = {};
  hipEvent_t gev[3] = {};         // GEMM timing + "counters zeroed" hand-off between the streams
  hipDeviceProp_t prop{};
  unsigned long long* host_res = nullptr;
  // The probe arena is kept between probes (a hipMalloc of ~1.2 GiB costs ~0.25 ms, a fifth of a
  // probe) and freed by mi355x_probe_trim once idle, so a pod on the GPU gets the memory back.
  void* arena = nullptr;
  size_t arena_bytes = 0;
  std::chrono::steady_clock::time_point arena_used{};
  // HBM sweep buffer (mi355x_probe_hbm_sweep): nearly all free HBM, held only for a scrub pass
  SweepBuf sweep;
  unsigned long long* sweep_cnt = nullptr;
  // Freed VRAM is cleared by the driver before it is handed out again (~6 s for ~282 GiB measured,
  // profiles/r2h_sweep_claim_diag.txt): an arena hipMalloc issued in that window waits for it. The
  // arena is therefore allocated before the sweep buffer and not trimmed while a sweep is held or
  // for kSweepClearGrace after its release, so a claim-time probe never allocates behind a clear.
  std::chrono::steady_clock::time_point sweep_released{};
  // xGMI ring check (mi355x_probe_peer_ring): send / receive windows kept between claims like the
  // arena (a 64 MiB hipMalloc + hipFree pair per link per claim cost more than the copy), freed by
  // the same idle trim
  void* peer_send = nullptr;
  void* peer_recv = nullptr;
  uint64_t peer_bytes = 0;
  unsigned long long* peer_cnt = nullptr;
  std::chrono::steady_clock::time_point peer_used{};
  std::string uuid;  // hip_uuid(), cached: the runtime query is not free on a cold CPU
  bool ready = false;
};

constexpr std::chrono::seconds kSweepClearGrace{30};

std::mutex g_mu;
std::vector<DeviceCtx> g_ctx;
int g_count = -1;

std::mutex& device_mutex(int dev) {
  static std::vector<std::mutex> mu(64);
  return mu[static_cast<size_t>(dev) % mu.size()];
}

std::string jnum(double v) {
  char b[64];
  std::snprintf(b, sizeof b, "%.6g", v);
  return b;
}

std::string jstr(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o.push_back('\\');
    if (static_cast<unsigned char>(c) < 0x20) continue;
    o.push_back(c);
  }
  return o + "\"";
}

long long opt_int(const char* json, const char* key, long long def) {
  if (!json) return def;
  std::string pat = std::string("\"") + key + "\"";
  const char* p = std::strstr(json, pat.c_str());
  if (!p) return def;
  p = std::strchr(p + pat.size(), ':');
  if (!p) return def;
  ++p;
  while (*p == ' ') ++p;
  if (std::strncmp(p, "true", 4) == 0) return 1;
  if (std::strncmp(p, "false", 5) == 0) return 0;
  return std::strtoll(p, nullptr, 10);
}

char* dup(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

std::string hip_uuid(int dev) {
  hipUUID u{};
  if (hipDeviceGetUuid(&u, dev) != hipSuccess) return "";
  std::string s(u.bytes, u.bytes + 16);
  // ROCm reports the ASIC serial as ASCII hex: "GPU-<serial>" is the ROCR_VISIBLE_DEVICES form.
  bool ascii = true;
  for (char c : s) ascii = ascii && ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'));
  if (ascii) return "GPU-" + s;
  char buf[40];
  std::string hex;
  for (int i = 0; i < 16; ++i) {
    std::snprintf(buf, sizeof buf, "%02x", static_cast<unsigned char>(u.bytes[i]));
    hex += buf;
  }
  return "GPU-" + hex;
}

// Enqueues the whole MFMA phase on stream s (no host sync): (a) a 256^3 GEMM checked element by
// element against the VALU reference with asymmetric operands, (b) the timed N^3 GEMM (events
// ctx.gev[0..1]) with exact u32 (mod 2^32) ABFT row/column checksums, then copies the two mismatch
// counters to hres[kSlotSmall..kSlotAbft]. Operands are carved from ``gbase``. zero_mfma: the operand
// kernels zero the phase's counters cnt[kSlotSmall..kResSlots) and ABFT accumulators themselves.
void launch_mfma_phase(char* gbase, int gemm_n, bool tile256, int pipe, bool prio, bool vec_c, int group_m, int reps, int inject_gemm,
                       int census_fault_xcc, bool zero_mfma, bool poison_c, unsigned long long* cnt,
                       unsigned long long* hres, DeviceCtx& ctx, hipStream_t s) {
  const size_t n = static_cast<size_t>(gemm_n), n0 = 256;
  auto align = [](size_t x) { return (x + 4095) & ~static_cast<size_t>(4095); };
  char* p = gbase;
  auto carve = [&](size_t bytes) {
    char* q = p;
    p += align(bytes);
    return q;
  };
  auto* a0 = reinterpret_cast<short*>(carve(n0 * n0 * 2));
  auto* b0 = reinterpret_cast<short*>(carve(n0 * n0 * 2));
  auto* c0 = reinterpret_cast<float*>(carve(n0 * n0 * 4));
  auto* r0 = reinterpret_cast<float*>(carve(n0 * n0 * 4));
  auto* a = reinterpret_cast<short*>(carve(n * n * 2));
  auto* b = reinterpret_cast<short*>(carve(n * n * 2));
  auto* c = reinterpret_cast<float*>(carve(n * n * 4));
  auto* v = reinterpret_cast<unsigned long long*>(carve(6 * n * 8));
  auto gemm = [&](const short* a_, const short* b_, float* c_, int nn, unsigned long long* cu_map) {
    const dim3 grid((nn / G2_BM) * (nn / G2_BN));
    if (tile256 && pipe == 1)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<false>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn, cu_map,
                         group_m);
    else if (tile256 && pipe == 2)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<true, 0, 1>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn, cu_map,
                         group_m);
    else if (tile256 && pipe == 3)
      hipLaunchKernelGGL(gemm_bf16_mfma_256x, grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn, cu_map, group_m);
    else if (tile256 && pipe == 21)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<true, 0, 0>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn,
                         cu_map, group_m);
    else if (tile256 && pipe == 22)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<true, 0, 2>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn,
                         cu_map, group_m);
    else if (tile256 && pipe == 11)  // ablations (timing only; the checks fail)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<true, 1, 1>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn,
                         cu_map, group_m);
    else if (tile256 && pipe == 12)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<true, 2, 1>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn,
                         cu_map, group_m);
    else if (tile256 && prio)
      hipLaunchKernelGGL((gemm_bf16_mfma_256<true, false>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn,
                         cu_map, group_m);
    else if (tile256 && vec_c)
      hipLaunchKernelGGL((gemm_bf16_mfma_256<false, true>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn,
                         cu_map, group_m);
    else if (tile256)
      hipLaunchKernelGGL((gemm_bf16_mfma_256<false, false>), grid, dim3(kGemm2Threads), 0, s, a_, b_, c_, nn, nn, nn,
                         cu_map, group_m);
    else
      hipLaunchKernelGGL(gemm_bf16_mfma_nt, dim3((nn / BM) * (nn / BN)), dim3(kGemmThreads), 0, s, a_, b_, c_, nn, nn, nn);
  };
  // (a) 256^3 full-element check vs the VALU reference; asymmetric operands
  const uint64_t e0 = static_cast<uint64_t>(n0) * n0;
  hipLaunchKernelGGL(gen_operand, dim3(256), dim3(256), 0, s, a0, e0, 0x1234u, 3,
                     zero_mfma ? reinterpret_cast<uint32_t*>(cnt + kSlotSmall) : nullptr,
                     zero_mfma ? static_cast<uint64_t>(kResSlots - kSlotSmall) * 2 : 0);
  hipLaunchKernelGGL(gen_operand, dim3(256), dim3(256), 0, s, b0, e0, 0xBEEFu, 3, static_cast<uint32_t*>(nullptr), 0);
  gemm(a0, b0, c0, static_cast<int>(n0), nullptr);
  hipLaunchKernelGGL(gemm_ref_valu, dim3(n0 / 256, n0), dim3(256), 0, s, a0, b0, r0, static_cast<int>(n0),
                     static_cast<int>(n0), static_cast<int>(n0));
  hipLaunchKernelGGL(count_diff, dim3(64), dim3(256), 0, s, static_cast<const float*>(c0), static_cast<const float*>(r0),
                     e0, cnt + kSlotSmall);
  PROBE_CHECK(hipGetLastError());

  // (b) N^3 timed GEMM + exact ABFT checksums
  const uint64_t e = static_cast<uint64_t>(n) * n;
  // ABFT checksums: 6 uint32 vectors [acol | bcol | colsumC | expCol | rowsumC | expRow]; the first
  // three accumulate atomically and start from zero (zeroed by the operand kernel, or a memset)
  uint32_t* v32 = reinterpret_cast<uint32_t*>(v);
  hipLaunchKernelGGL(gen_operand, dim3(2048), dim3(256), 0, s, a, e, 0x51u, 2, zero_mfma ? v32 : nullptr,
                     zero_mfma ? 3 * n : 0);
  hipLaunchKernelGGL(gen_operand, dim3(2048), dim3(256), 0, s, b, e, 0x77u, 2, static_cast<uint32_t*>(nullptr), 0);
  // test hook: C starts as all-ones words (NaN) so a tile the GEMM never writes fails the checks
  // instead of passing on the previous run's identical result (the arena is reused)
  if (poison_c) PROBE_CHECK(hipMemsetAsync(c, 0xFF, n * n * sizeof(float), s));
  // the 256^3 check above already ran this kernel's code object: time the first launch
  PROBE_CHECK(hipEventRecord(ctx.gev[0], s));
  for (int rep = 0; rep < reps; ++rep) gemm(a, b, c, gemm_n, cnt + kSlotGemmMap);  // reps 0: test hook
  PROBE_CHECK(hipEventRecord(ctx.gev[1], s));
  PROBE_CHECK(hipGetLastError());
  if (inject_gemm)
    hipLaunchKernelGGL(inject_gemm_fault, dim3(1), dim3(1), 0, s, c, static_cast<int64_t>(gemm_n / 3) * gemm_n + gemm_n / 5,
                       inject_gemm);
  uint32_t *vacol = v32, *vbcol = v32 + n, *vcolC = v32 + 2 * n, *vexpC = v32 + 3 * n, *vrowC = v32 + 4 * n,
           *vexpR = v32 + 5 * n;
  if (!zero_mfma) PROBE_CHECK(hipMemsetAsync(v32, 0, 3 * n * sizeof(uint32_t), s));
  const int rows_y = (gemm_n + kColRows - 1) / kColRows;
  const dim3 cgrid_h((gemm_n + 511) / 512, rows_y), cgrid_f((gemm_n + 255) / 256, rows_y);
  const float bound = static_cast<float>(gemm_n) * 4.0f;  // |C| <= K * span^2, span 2
  hipLaunchKernelGGL(colsum_partial<short>, cgrid_h, dim3(256), 0, s, static_cast<const short*>(a), gemm_n, gemm_n, vacol,
                     0.f, static_cast<unsigned long long*>(nullptr));
  hipLaunchKernelGGL(colsum_partial<short>, cgrid_h, dim3(256), 0, s, static_cast<const short*>(b), gemm_n, gemm_n, vbcol,
                     0.f, static_cast<unsigned long long*>(nullptr));
  hipLaunchKernelGGL(colsum_partial<float>, cgrid_f, dim3(256), 0, s, static_cast<const float*>(c), gemm_n, gemm_n, vcolC,
                     bound, cnt + kSlotAbft);
  const dim3 rgrid((gemm_n + 3) / 4);
  hipLaunchKernelGGL(rowdot<short>, rgrid, dim3(256), 0, s, static_cast<const short*>(b), gemm_n, gemm_n,
                     static_cast<const uint32_t*>(vacol), vexpC);
  hipLaunchKernelGGL(rowdot<float>, rgrid, dim3(256), 0, s, static_cast<const float*>(c), gemm_n, gemm_n,
                     static_cast<const uint32_t*>(nullptr), vrowC);
  hipLaunchKernelGGL(rowdot<short>, rgrid, dim3(256), 0, s, static_cast<const short*>(a), gemm_n, gemm_n,
                     static_cast<const uint32_t*>(vbcol), vexpR);
  hipLaunchKernelGGL(count_ne_u32, dim3((gemm_n + 255) / 256), dim3(256), 0, s, vcolC, vexpC, gemm_n, cnt + kSlotAbft);
  hipLaunchKernelGGL(count_ne_u32, dim3((gemm_n + 255) / 256), dim3(256), 0, s, vrowC, vexpR, gemm_n, cnt + kSlotAbft);
  // (c) every CU's matrix cores: the census (the GEMM above marked the CUs that ran its tiles)
  hipLaunchKernelGGL(cu_census, dim3(8 * ctx.prop.multiProcessorCount), dim3(kCensusThreads), 0, s, cnt + kSlotCensusMap,
                     cnt + kSlotCensusBad, kCensusIters, 0xC0FFEEu ^ static_cast<uint32_t>(gemm_n), census_fault_xcc);
  PROBE_CHECK(hipGetLastError());
  PROBE_CHECK(hipMemcpyAsync(hres + kSlotSmall, cnt + kSlotSmall, (kResSlots - kSlotSmall) * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, s));
}

struct CuCount {
  int total = 0;
  int per_xcc[8] = {};
};

CuCount count_cus(const unsigned long long* map) {
  CuCount c;
  for (int w = 0; w < kCuMapWords; ++w) {
    const int n = __builtin_popcountll(map[w]);
    c.total += n;
    c.per_xcc[(w * 64) >> 8] += n;
  }
  return c;
}

std::string run_probe(int dev, const char* opts) {
  const uint64_t hbm_bytes = static_cast<uint64_t>(opt_int(opts, "hbmBytes", 1LL << 30));
  const bool do_mfma = opt_int(opts, "mfma", 1) != 0;
  int gemm_n = static_cast<int>(opt_int(opts, "gemmN", 4096));
  gemm_n = std::max(256, (gemm_n / 256) * 256);
  const int patterns = static_cast<int>(std::min(kMaxPatterns, std::max(1LL, opt_int(opts, "patterns", 2))));
  const int inject_flips = static_cast<int>(std::min(4096LL, std::max(0LL, opt_int(opts, "injectBitFlips", 0))));
  const int inject_gemm = static_cast<int>(opt_int(opts, "injectGemmFault", 0));
  const bool tile256 = opt_int(opts, "gemmTile", 256) != 128;  // 128 = the older 128x128 kernel (A/B)
  const int group_m = static_cast<int>(opt_int(opts, "gemmGroupM", kGemmGroupM));  // tile order (A/B)
  const int gemm_pipe = static_cast<int>(opt_int(opts, "gemmPipe", kGemmPipe));      // 1, 2: half-tile pipeline
  const bool gemm_prio = opt_int(opts, "gemmPrio", 0) != 0;                        // s_setprio (A/B)
  const bool gemm_vec_c = opt_int(opts, "gemmVecC", 0) != 0;                       // 16-B C stores (A/B)
  const bool poison_c = opt_int(opts, "poisonC", 0) != 0;                           // test hook
  // The HBM test is bandwidth-bound with few waves per CU; the MFMA phase is compute-bound and
  // touches ~130 MiB: run them concurrently on two streams (overlap=0: one stream, serial).
  const bool overlap = opt_int(opts, "overlap", 1) != 0;
  auto t0 = std::chrono::steady_clock::now();
  PROBE_CHECK(hipSetDevice(dev));
  DeviceCtx& ctx = g_ctx[static_cast<size_t>(dev)];
  if (!ctx.ready) {
    PROBE_CHECK(hipStreamCreateWithFlags(&ctx.stream, hipStreamNonBlocking));
    PROBE_CHECK(hipStreamCreateWithFlags(&ctx.stream2, hipStreamNonBlocking));
    for (auto& e : ctx.ev) PROBE_CHECK(hipEventCreate(&e));
    for (auto& e : ctx.gev) PROBE_CHECK(hipEventCreate(&e));
    PROBE_CHECK(hipGetDeviceProperties(&ctx.prop, dev));
    // pinned result slots: device->host copies of the counters are truly async (one sync per phase)
    PROBE_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ctx.host_res), kResSlots * sizeof(unsigned long long)));
    ctx.uuid = hip_uuid(dev);
    ctx.ready = true;
  }
  hipStream_t s = ctx.stream;
  const hipDeviceProp_t& prop = ctx.prop;
  const int cus = prop.multiProcessorCount;
  auto ms_since = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  const double setup_ms = ms_since(t0);

  // ---------------- one arena for the whole probe: [HBM pattern region | GEMM operands | counters],
  // so a probe costs one hipMalloc/hipFree instead of a dozen.
  auto t_alloc = std::chrono::steady_clock::now();
  const uint64_t n16 = hbm_bytes / 16;
  const size_t n = static_cast<size_t>(gemm_n), n0 = 256;
  auto align = [](size_t x) { return (x + 4095) & ~static_cast<size_t>(4095); };
  const size_t sz_a0 = align(n0 * n0 * 2), sz_c0 = align(n0 * n0 * 4), sz_a = align(n * n * 2), sz_c = align(n * n * 4),
               sz_v = align(6 * n * 8);
  const size_t gemm_bytes = do_mfma ? 2 * sz_a0 + 2 * sz_c0 + 2 * sz_a + sz_c + sz_v : 0;
  const size_t hbm_region = align(n16 * 16);
  const size_t region = hbm_region + gemm_bytes;
  const size_t need = region + align(kResSlots * sizeof(unsigned long long));
  const bool keep = opt_int(opts, "keepArena", 1) != 0;
  if (ctx.arena && (ctx.arena_bytes < need || ctx.arena_bytes > 2 * need)) {
    (void)hipFree(ctx.arena);
    ctx.arena = nullptr;
    ctx.arena_bytes = 0;
  }
  const bool reused = ctx.arena != nullptr;
  if (!ctx.arena) {
    PROBE_CHECK(hipMalloc(&ctx.arena, need));
    ctx.arena_bytes = need;
  }
  ctx.arena_used = std::chrono::steady_clock::now();
  DevBuf transient;  // owns the arena for this probe only when it is not kept
  if (!keep) {
    transient.p = ctx.arena;
    ctx.arena = nullptr;
    ctx.arena_bytes = 0;
  }
  char* base = static_cast<char*>(keep ? ctx.arena : transient.p);
  auto* cnt = reinterpret_cast<unsigned long long*>(base + region);
  unsigned long long* hres = ctx.host_res;
  const double alloc_ms = ms_since(t_alloc);
  auto t_run = std::chrono::steady_clock::now();

  // counters: [2p] = flipped bits, [2p+1] = first bad 16-B index (init all-ones) of pattern p,
  // then the MFMA phase's counters. zeroInKernel (default): the first fill resets the HBM pairs and
  // the MFMA phase's first kernel its own slots, so neither stream starts behind memsets or waits
  // on the other — after an idle gap each API call ahead of the first fill costs tens of us
  // (profiles/r4i_probe_idle_gap_ab.json). 0: memsets on s, s2 waits for them (the older path).
  const bool zero_in_kernel = opt_int(opts, "zeroInKernel", 1) != 0;
  hipStream_t s2 = overlap ? ctx.stream2 : s;
  if (!zero_in_kernel) {
    PROBE_CHECK(hipMemsetAsync(cnt, 0, kResSlots * sizeof(unsigned long long), s));
    for (int pi = 0; pi < patterns; ++pi)
      PROBE_CHECK(hipMemsetAsync(cnt + 2 * pi + 1, 0xFF, sizeof(unsigned long long), s));
    if (overlap) {
      PROBE_CHECK(hipEventRecord(ctx.gev[2], s));
      PROBE_CHECK(hipStreamWaitEvent(s2, ctx.gev[2], 0));
    }
  }

  // ---------------- MFMA phase (launched first so it starts beside the HBM fill)
  bool mfma_ok = true;
  unsigned long long small_bad = 0, abft_bad = 0, census_bad = 0;
  CuCount census, gemm_cus;
  const bool require_all_cus = opt_int(opts, "requireAllCUs", 1) != 0;
  double tflops = 0, gemm_ms = 0;
  // gemmSkip (test hook, with poisonC): no timed GEMM at all, so C keeps the poison
  const int reps = opt_int(opts, "gemmSkip", 0) ? 0 : static_cast<int>(std::max(1LL, opt_int(opts, "gemmReps", 1)));
  const int census_fault_xcc = static_cast<int>(opt_int(opts, "injectCensusFaultXcc", -1));
  const bool want_keys = opt_int(opts, "cuKeys", 0) != 0;
  std::vector<int> cu_keys;
  // Launch order: the HBM test is the probe's critical path (~0.68 ms of kernels for 1 GiB x 2
  // patterns); the MFMA phase (~0.1 ms of GPU time beside it) costs ~20 API calls to enqueue. With
  // hbmFirst (default) the HBM kernels are enqueued first, so the fill starts ~20 launches earlier
  // and the MFMA phase is enqueued while it runs (profiles/r4e_probe_launch_order_ab.json).
  // hbmFirst=2: the MFMA phase is enqueued right after the first fill (in-process A/B), so it starts
  // earlier on the GPU while the rest of the HBM test is still enqueued well ahead of need.
  const int hbm_first = static_cast<int>(opt_int(opts, "hbmFirst", 1));
  if (do_mfma && hbm_first == 0)
    launch_mfma_phase(base + hbm_region, gemm_n, tile256, gemm_pipe, gemm_prio, gemm_vec_c, group_m, reps, inject_gemm, census_fault_xcc, zero_in_kernel, poison_c, cnt, hres,
                      ctx, s2);

  // ---------------- HBM: all patterns back to back, per-pattern counters
  auto* hbm = reinterpret_cast<u32x4*>(base);
  // Grid per HBM kernel (workgroups per CU). Measured on MI355X (scripts/probe_hbm_sweep.py):
  // the streaming store kernel is fastest with few long-running waves per CU, the verify kernel
  // with a few more loads in flight; the old 8/CU for both was among the slowest settings.
  auto hbm_grid_for = [&](const char* key, long long def) {
    const uint64_t per_cu = static_cast<uint64_t>(std::max(1LL, opt_int(opts, key, def)));
    return static_cast<int>(std::min<uint64_t>(static_cast<uint64_t>(cus) * per_cu,
                                               (n16 + kHbmThreads - 1) / kHbmThreads));
  };
  const int fill_grid = hbm_grid_for("hbmFillBlocksPerCU", opt_int(opts, "hbmBlocksPerCU", 1));
  const int verify_grid = hbm_grid_for("hbmVerifyBlocksPerCU", opt_int(opts, "hbmBlocksPerCU", 3));
  const uint32_t seed = 0xA5A50000u + static_cast<uint32_t>(dev);
  const bool cheap_pattern = opt_int(opts, "hbmPattern", kHbmPattern) == 1;  // in-process A/B
  const bool tiled = cheap_pattern && opt_int(opts, "hbmLayout", kHbmLayout) == 1;
  PROBE_CHECK(hipEventRecord(ctx.ev[0], s));
  for (int pi = 0; pi < patterns; ++pi) {
    const uint32_t flip = (pi & 1) ? 0xFFFFFFFFu : 0u;  // complementary polarity on odd passes
    unsigned long long* reset = zero_in_kernel && pi == 0 ? cnt : nullptr;
    const int nreset = reset ? patterns : 0;
    if (tiled)
      hipLaunchKernelGGL((hbm_fill<1, 1>), dim3(fill_grid), dim3(kHbmThreads), 0, s, hbm, n16, seed, flip, reset, nreset);
    else if (cheap_pattern)
      hipLaunchKernelGGL(hbm_fill<1>, dim3(fill_grid), dim3(kHbmThreads), 0, s, hbm, n16, seed, flip, reset, nreset);
    else
      hipLaunchKernelGGL(hbm_fill<0>, dim3(fill_grid), dim3(kHbmThreads), 0, s, hbm, n16, seed, flip, reset, nreset);
    PROBE_CHECK(hipEventRecord(ctx.ev[1 + 2 * pi], s));
    if (pi == 0 && do_mfma && hbm_first == 2)
      launch_mfma_phase(base + hbm_region, gemm_n, tile256, gemm_pipe, gemm_prio, gemm_vec_c, group_m, reps, inject_gemm, census_fault_xcc, zero_in_kernel, poison_c, cnt, hres,
                        ctx, s2);
    if (pi == 0 && inject_flips > 0)
      hipLaunchKernelGGL(inject_bit_flips, dim3(1), dim3(256), 0, s, reinterpret_cast<unsigned int*>(hbm), n16 * 4,
                         inject_flips);
    if (tiled)
      hipLaunchKernelGGL((hbm_verify<1, 1>), dim3(verify_grid), dim3(kHbmThreads), 0, s, static_cast<const u32x4*>(hbm),
                         n16, seed, flip, cnt + 2 * pi, cnt + 2 * pi + 1);
    else if (cheap_pattern)
      hipLaunchKernelGGL(hbm_verify<1>, dim3(verify_grid), dim3(kHbmThreads), 0, s, static_cast<const u32x4*>(hbm), n16,
                         seed, flip, cnt + 2 * pi, cnt + 2 * pi + 1);
    else
      hipLaunchKernelGGL(hbm_verify<0>, dim3(verify_grid), dim3(kHbmThreads), 0, s, static_cast<const u32x4*>(hbm), n16,
                         seed, flip, cnt + 2 * pi, cnt + 2 * pi + 1);
    PROBE_CHECK(hipEventRecord(ctx.ev[2 + 2 * pi], s));
  }
  PROBE_CHECK(hipGetLastError());
  PROBE_CHECK(hipMemcpyAsync(hres, cnt, 2 * patterns * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  if (do_mfma && hbm_first == 1)
    launch_mfma_phase(base + hbm_region, gemm_n, tile256, gemm_pipe, gemm_prio, gemm_vec_c, group_m, reps, inject_gemm, census_fault_xcc, zero_in_kernel, poison_c, cnt, hres,
                      ctx, s2);
  const double launch_ms = ms_since(t_run);  // host time to enqueue the whole probe
  PROBE_CHECK(hipStreamSynchronize(s));
  const double hbm_wall_ms = ms_since(t_run);
  if (do_mfma) {
    PROBE_CHECK(hipStreamSynchronize(s2));
    float ms;
    PROBE_CHECK(hipEventElapsedTime(&ms, ctx.gev[0], ctx.gev[1]));
    gemm_ms = reps > 0 ? ms / reps : 0.0;
    tflops = gemm_ms > 0 ? 2.0 * gemm_n * static_cast<double>(gemm_n) * gemm_n / (gemm_ms * 1e-3) / 1e12 : 0.0;
    small_bad = hres[kSlotSmall];
    abft_bad = hres[kSlotAbft];
    census_bad = hres[kSlotCensusBad];
    census = count_cus(hres + kSlotCensusMap);
    if (want_keys)  // the (xcc, se, sh, cu) key of every CU that proved its MFMA (isolation tests)
      for (int k = 0; k < kCuKeys; ++k)
        if (hres[kSlotCensusMap + k / 64] >> (k % 64) & 1ull) cu_keys.push_back(k);
    gemm_cus = count_cus(hres + kSlotGemmMap);
    // every CU the runtime reports must have proven its matrix cores (requireAllCUs, default on)
    const bool cus_ok = !require_all_cus || census.total >= cus;
    mfma_ok = small_bad == 0 && abft_bad == 0 && census_bad == 0 && cus_ok;
  }
  const double mfma_wall_ms = do_mfma ? ms_since(t_run) : 0.0;
  unsigned long long bad_bits = 0, first_bad = ~0ull;
  float write_ms = 0, read_ms = 0;
  for (int pi = 0; pi < patterns; ++pi) {
    float w, r;
    PROBE_CHECK(hipEventElapsedTime(&w, pi == 0 ? ctx.ev[0] : ctx.ev[2 * pi], ctx.ev[1 + 2 * pi]));
    PROBE_CHECK(hipEventElapsedTime(&r, ctx.ev[1 + 2 * pi], ctx.ev[2 + 2 * pi]));
    write_ms += w;
    read_ms += r;
    bad_bits += hres[2 * pi];
    first_bad = std::min(first_bad, hres[2 * pi + 1]);
  }
  const double bytes_moved = static_cast<double>(n16) * 16.0 * patterns;
  const double write_gbps = bytes_moved / (write_ms * 1e-3) / 1e9;
  const double read_gbps = bytes_moved / (read_ms * 1e-3) / 1e9;
  const double hbm_gbps = 2.0 * bytes_moved / ((write_ms + read_ms) * 1e-3) / 1e9;
  const bool hbm_ok = bad_bits == 0;
  auto t_free = std::chrono::steady_clock::now();
  if (transient.p) {
    (void)hipFree(transient.p);
    transient.p = nullptr;
  }
  const double free_ms = ms_since(t_free);
  double total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const auto t_report = std::chrono::steady_clock::now();
  std::string out;
  out.reserve(2048);  // one allocation for the whole report
  out += "{\"device\":" + std::to_string(dev);
  out += ",\"hipUUID\":" + jstr(ctx.uuid);
  out += ",\"gcnArch\":" + jstr(prop.gcnArchName);
  out += ",\"passed\":" + std::string(hbm_ok && mfma_ok ? "true" : "false");
  out += ",\"hbm\":{\"ok\":" + std::string(hbm_ok ? "true" : "false") + ",\"bytes\":" + std::to_string(n16 * 16) +
         ",\"patterns\":" + std::to_string(patterns) + ",\"badBits\":" + std::to_string(bad_bits) +
         ",\"firstBadOffset\":" + (first_bad == ~0ull ? std::string("null") : std::to_string(first_bad * 16)) +
         ",\"writeGBps\":" + jnum(write_gbps) + ",\"readGBps\":" + jnum(read_gbps) + ",\"GBps\":" + jnum(hbm_gbps) +
         ",\"ms\":" + jnum(write_ms + read_ms) + "}";
  out += ",\"mfma\":{\"ok\":" + std::string(mfma_ok ? "true" : "false") + ",\"enabled\":" + (do_mfma ? "true" : "false") +
         ",\"n\":" + std::to_string(gemm_n) + ",\"tile\":" + (tile256 ? "256" : "128") + ",\"pipe\":" + std::to_string(tile256 ? gemm_pipe : 0) +
         ",\"elementMismatches\":" + std::to_string(small_bad) + ",\"abftMismatches\":" + std::to_string(abft_bad) +
         ",\"tflops\":" + jnum(tflops) + ",\"ms\":" + jnum(gemm_ms) + "}";
  if (do_mfma) {
    std::string per = "[";
    for (int x = 0; x < 8; ++x) per += (x ? "," : "") + std::to_string(census.per_xcc[x]);
    out += ",\"cus\":{\"expected\":" + std::to_string(cus) + ",\"mfmaVerified\":" + std::to_string(census.total) +
           ",\"perXcd\":" + per + "]" + ",\"gemmTiles\":" + std::to_string(gemm_cus.total) +
           ",\"badWaves\":" + std::to_string(census_bad) + ",\"ok\":" +
           (census_bad == 0 && census.total >= cus ? "true" : "false");
    if (want_keys) {
      out += ",\"cuKeys\":[";
      for (size_t i = 0; i < cu_keys.size(); ++i) out += (i ? "," : "") + std::to_string(cu_keys[i]);
      out += "]";
    }
    out += "}";
  }
  out += ",\"ms\":" + jnum(total_ms);
  out += ",\"phases\":{\"arenaReused\":" + std::string(reused ? "true" : "false") +
         ",\"setupMs\":" + jnum(setup_ms) + ",\"allocMs\":" + jnum(alloc_ms) + ",\"launchMs\":" + jnum(launch_ms) +
         ",\"hbmFirst\":" + std::to_string(hbm_first) +
         ",\"hbmWallMs\":" + jnum(hbm_wall_ms) + ",\"mfmaWallMs\":" + jnum(mfma_wall_ms) + ",\"freeMs\":" + jnum(free_ms) +
         "}";
  // host time spent building this report after the clock above stopped (timing of the binding)
  out += ",\"reportMs\":" + jnum(ms_since(t_report)) + "}";
  return out;
}

// One direction of the xGMI peer check (see mi355x_probe_peer in probe.h). Serialised against
// probes of either device by the caller.
std::string run_peer(int src, int dst, const char* opts) {
  const uint64_t bytes = static_cast<uint64_t>(std::max(1LL << 20, opt_int(opts, "bytes", 256LL << 20)));
  const uint64_t n16 = bytes / 16;
  for (int d : {src, dst}) {
    DeviceCtx& c = g_ctx[static_cast<size_t>(d)];
    if (!c.ready) (void)run_probe(d, "{\"hbmBytes\":1048576,\"patterns\":1,\"mfma\":false}");  // create streams/events
  }
  int can = src == dst ? 1 : 0;
  if (src != dst) PROBE_CHECK(hipDeviceCanAccessPeer(&can, src, dst));
  if (!can)
    return "{\"src\":" + std::to_string(src) + ",\"dst\":" + std::to_string(dst) +
           ",\"canAccessPeer\":false,\"passed\":false,\"error\":\"hipDeviceCanAccessPeer=0\"}";
  DeviceCtx& cs = g_ctx[static_cast<size_t>(src)];
  DeviceCtx& cd = g_ctx[static_cast<size_t>(dst)];
  if (src != dst) {
    PROBE_CHECK(hipSetDevice(src));
    hipError_t e = hipDeviceEnablePeerAccess(dst, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) PROBE_CHECK(e);
    (void)hipGetLastError();  // clear a sticky "already enabled"
  }
  DevBuf sbuf, dbuf, cnt_buf;
  PROBE_CHECK(hipSetDevice(src));
  PROBE_CHECK(hipMalloc(&sbuf.p, n16 * 16));
  PROBE_CHECK(hipSetDevice(dst));
  PROBE_CHECK(hipMalloc(&dbuf.p, n16 * 16));
  PROBE_CHECK(hipMalloc(&cnt_buf.p, 2 * sizeof(unsigned long long)));
  auto* cnt = static_cast<unsigned long long*>(cnt_buf.p);
  const uint32_t seed = 0x5EED0000u + static_cast<uint32_t>(src * 16 + dst);
  // src: write the pattern
  PROBE_CHECK(hipSetDevice(src));
  const int sgrid = std::min<int>(cs.prop.multiProcessorCount, static_cast<int>((n16 + kHbmThreads - 1) / kHbmThreads));
  hipLaunchKernelGGL(hbm_fill<>, dim3(sgrid), dim3(kHbmThreads), 0, cs.stream, static_cast<u32x4*>(sbuf.p), n16, seed, 0u,
                     static_cast<unsigned long long*>(nullptr), 0);
  PROBE_CHECK(hipGetLastError());
  // the copy over the peer link, timed on src's stream
  PROBE_CHECK(hipEventRecord(cs.gev[0], cs.stream));
  PROBE_CHECK(hipMemcpyPeerAsync(dbuf.p, dst, sbuf.p, src, n16 * 16, cs.stream));
  PROBE_CHECK(hipEventRecord(cs.gev[1], cs.stream));
  PROBE_CHECK(hipStreamSynchronize(cs.stream));
  float ms = 0;
  PROBE_CHECK(hipEventElapsedTime(&ms, cs.gev[0], cs.gev[1]));
  // dst: verify every bit that arrived
  PROBE_CHECK(hipSetDevice(dst));
  PROBE_CHECK(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), cd.stream));
  PROBE_CHECK(hipMemsetAsync(cnt + 1, 0xFF, sizeof(unsigned long long), cd.stream));
  const int dgrid = std::min<int>(3 * cd.prop.multiProcessorCount, static_cast<int>((n16 + kHbmThreads - 1) / kHbmThreads));
  hipLaunchKernelGGL(hbm_verify<>, dim3(dgrid), dim3(kHbmThreads), 0, cd.stream, static_cast<const u32x4*>(dbuf.p), n16,
                     seed, 0u, cnt, cnt + 1);
  PROBE_CHECK(hipGetLastError());
  PROBE_CHECK(hipMemcpyAsync(cd.host_res, cnt, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, cd.stream));
  PROBE_CHECK(hipStreamSynchronize(cd.stream));
  const unsigned long long bad = cd.host_res[0];
  const double gbps = ms > 0 ? static_cast<double>(n16 * 16) / (ms * 1e-3) / 1e9 : 0.0;
  return "{\"src\":" + std::to_string(src) + ",\"dst\":" + std::to_string(dst) + ",\"canAccessPeer\":true" +
         ",\"passed\":" + (bad == 0 ? "true" : "false") + ",\"badBits\":" + std::to_string(bad) +
         ",\"bytes\":" + std::to_string(n16 * 16) + ",\"GBps\":" + jnum(gbps) + ",\"ms\":" + jnum(ms) + "}";
}

// Cached peer windows of one device (caller holds its lock, device selected).
void ensure_peer_bufs(DeviceCtx& c, uint64_t bytes) {
  if (c.peer_bytes != bytes) {
    if (c.peer_send) (void)hipFree(c.peer_send);
    if (c.peer_recv) (void)hipFree(c.peer_recv);
    c.peer_send = c.peer_recv = nullptr;
    c.peer_bytes = 0;
    PROBE_CHECK(hipMalloc(&c.peer_send, bytes));
    PROBE_CHECK(hipMalloc(&c.peer_recv, bytes));
    c.peer_bytes = bytes;
  }
  if (!c.peer_cnt) PROBE_CHECK(hipMalloc(&c.peer_cnt, 2 * sizeof(unsigned long long)));
}

void free_peer_bufs(DeviceCtx& c) {
  if (c.peer_send) (void)hipFree(c.peer_send);
  if (c.peer_recv) (void)hipFree(c.peer_recv);
  c.peer_send = c.peer_recv = nullptr;
  c.peer_bytes = 0;
}

// The whole xGMI ring at once (see mi355x_probe_peer_ring in probe.h): link i copies devs[i]'s send
// window into devs[i+1]'s receive window. On an MI355X node every GPU pair has its own xGMI link, so
// the n copies of a ring use n distinct links and run concurrently, one per source stream: the check
// costs one copy time instead of n (a pair-at-a-time check also serialised pairs sharing a device).
// Phases: every source fills its window (one pattern per source device), every link copies, the host
// waits for all copies, every receiver verifies the bits that arrived. A device may appear more than
// once (a 1-GPU box runs [0, 0]: local copies through the same code). Caller holds every device's lock.
std::string run_peer_ring(const std::vector<int>& devs, const char* opts) {
  const uint64_t bytes = static_cast<uint64_t>(std::max(1LL << 20, opt_int(opts, "bytes", 64LL << 20))) / 16 * 16;
  const uint64_t n16 = bytes / 16;
  const size_t n = devs.size();
  std::vector<int> uniq(devs);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  for (int d : uniq) {
    DeviceCtx& c = g_ctx[static_cast<size_t>(d)];
    if (!c.ready) (void)run_probe(d, "{\"hbmBytes\":1048576,\"patterns\":1,\"mfma\":false}");  // streams/events
    PROBE_CHECK(hipSetDevice(d));
    ensure_peer_bufs(c, bytes);
    c.peer_used = std::chrono::steady_clock::now();
  }
  std::vector<std::string> errs(n);
  for (size_t i = 0; i < n; ++i) {  // peer access for every link (idempotent)
    const int src = devs[i], dst = devs[(i + 1) % n];
    if (src == dst) continue;
    int can = 0;
    PROBE_CHECK(hipDeviceCanAccessPeer(&can, src, dst));
    if (!can) {
      errs[i] = "hipDeviceCanAccessPeer=0";
      continue;
    }
    PROBE_CHECK(hipSetDevice(src));
    hipError_t e = hipDeviceEnablePeerAccess(dst, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) PROBE_CHECK(e);
    (void)hipGetLastError();  // clear a sticky "already enabled"
  }
  auto seed_of = [](int dev) { return 0x5EED0000u + static_cast<uint32_t>(dev) * 0x9E37u; };
  for (int d : uniq) {  // 1. each source device writes its pattern once, all devices at once
    DeviceCtx& c = g_ctx[static_cast<size_t>(d)];
    PROBE_CHECK(hipSetDevice(d));
    const int grid = std::min<int>(c.prop.multiProcessorCount, static_cast<int>((n16 + kHbmThreads - 1) / kHbmThreads));
    hipLaunchKernelGGL(hbm_fill<>, dim3(grid), dim3(kHbmThreads), 0, c.stream, static_cast<u32x4*>(c.peer_send), n16,
                       seed_of(d), 0u, static_cast<unsigned long long*>(nullptr), 0);
    PROBE_CHECK(hipGetLastError());
  }
  for (int d : uniq) {  // the copies below read other devices' windows: every fill must be done
    PROBE_CHECK(hipSetDevice(d));
    PROBE_CHECK(hipStreamSynchronize(g_ctx[static_cast<size_t>(d)].stream));
  }
  // 2. all links at once, each timed on its source's stream. A source with two outgoing links
  // (only with repeated devices) times them back to back on its one stream.
  std::vector<hipEvent_t> t0(n, nullptr), t1(n, nullptr);
  struct EvGuard {
    std::vector<hipEvent_t>& a;
    std::vector<hipEvent_t>& b;
    ~EvGuard() {
      for (auto* v : {&a, &b})
        for (hipEvent_t e : *v)
          if (e) (void)hipEventDestroy(e);
    }
  } guard{t0, t1};
  for (size_t i = 0; i < n; ++i) {
    if (!errs[i].empty()) continue;
    const int src = devs[i], dst = devs[(i + 1) % n];
    DeviceCtx& cs = g_ctx[static_cast<size_t>(src)];
    DeviceCtx& cd = g_ctx[static_cast<size_t>(dst)];
    PROBE_CHECK(hipSetDevice(src));
    PROBE_CHECK(hipEventCreate(&t0[i]));
    PROBE_CHECK(hipEventCreate(&t1[i]));
    PROBE_CHECK(hipEventRecord(t0[i], cs.stream));
    PROBE_CHECK(hipMemcpyPeerAsync(cd.peer_recv, dst, cs.peer_send, src, bytes, cs.stream));
    PROBE_CHECK(hipEventRecord(t1[i], cs.stream));
  }
  for (int d : uniq) {
    PROBE_CHECK(hipSetDevice(d));
    PROBE_CHECK(hipStreamSynchronize(g_ctx[static_cast<size_t>(d)].stream));
  }
  // 3. every receiving link verifies what arrived. The receivers of a batch of consecutive links
  // are distinct devices (each has one counter pair and one result slot), so the batch's verifies
  // run concurrently, one per receiver, and the host waits once per receiver; a receiver named
  // again (only with repeated devices, e.g. [0, 0] on a 1-GPU box) starts the next batch and is
  // verified against that link's source pattern in turn.
  std::vector<unsigned long long> bad(n, 0);
  for (size_t i = 0; i < n;) {
    std::vector<size_t> batch;
    std::vector<int> used;
    for (; i < n; ++i) {
      const int dst = devs[(i + 1) % n];
      if (errs[i].empty()) {
        if (std::find(used.begin(), used.end(), dst) != used.end()) break;
        used.push_back(dst);
      }
      batch.push_back(i);
    }
    for (size_t j : batch) {
      if (!errs[j].empty()) continue;
      const int src = devs[j], dst = devs[(j + 1) % n];
      DeviceCtx& cd = g_ctx[static_cast<size_t>(dst)];
      PROBE_CHECK(hipSetDevice(dst));
      PROBE_CHECK(hipMemsetAsync(cd.peer_cnt, 0, sizeof(unsigned long long), cd.stream));
      PROBE_CHECK(hipMemsetAsync(cd.peer_cnt + 1, 0xFF, sizeof(unsigned long long), cd.stream));
      const int grid = std::min<int>(3 * cd.prop.multiProcessorCount, static_cast<int>((n16 + kHbmThreads - 1) / kHbmThreads));
      hipLaunchKernelGGL(hbm_verify<>, dim3(grid), dim3(kHbmThreads), 0, cd.stream,
                         static_cast<const u32x4*>(cd.peer_recv), n16, seed_of(src), 0u, cd.peer_cnt, cd.peer_cnt + 1);
      PROBE_CHECK(hipGetLastError());
      PROBE_CHECK(hipMemcpyAsync(cd.host_res, cd.peer_cnt, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                 cd.stream));
    }
    for (size_t j : batch) {
      if (!errs[j].empty()) continue;
      const int dst = devs[(j + 1) % n];
      DeviceCtx& cd = g_ctx[static_cast<size_t>(dst)];
      PROBE_CHECK(hipSetDevice(dst));
      PROBE_CHECK(hipStreamSynchronize(cd.stream));
      bad[j] = cd.host_res[0];
    }
  }
  std::string out = "{\"bytes\":" + std::to_string(bytes) + ",\"links\":[";
  bool all_ok = true;
  for (size_t i = 0; i < n; ++i) {
    const int src = devs[i], dst = devs[(i + 1) % n];
    std::string link = "{\"src\":" + std::to_string(src) + ",\"dst\":" + std::to_string(dst);
    if (!errs[i].empty()) {
      link += ",\"canAccessPeer\":false,\"passed\":false,\"error\":" + jstr(errs[i]) + "}";
      all_ok = false;
    } else {
      float ms = 0;
      PROBE_CHECK(hipSetDevice(src));
      PROBE_CHECK(hipEventElapsedTime(&ms, t0[i], t1[i]));
      const double gbps = ms > 0 ? static_cast<double>(bytes) / (ms * 1e-3) / 1e9 : 0.0;
      all_ok = all_ok && bad[i] == 0;
      link += ",\"canAccessPeer\":true,\"passed\":" + std::string(bad[i] == 0 ? "true" : "false") +
              ",\"badBits\":" + std::to_string(bad[i]) + ",\"bytes\":" + std::to_string(bytes) +
              ",\"GBps\":" + jnum(gbps) + ",\"ms\":" + jnum(ms) + "}";
    }
    out += (i ? "," : "") + link;
  }
  return out + "],\"passed\":" + (all_ok ? "true" : "false") + "}";
}

// All free HBM minus ``reserve``, 2 MiB granular, as kSweepChunk pieces. Measured on MI355X
// (profiles/r2h_sweep_claim_diag.txt): ~0.2 s to allocate ~282 GiB of fresh VRAM, ~6 s once the
// driver must clear previously used VRAM; neither runs under the device lock a probe takes.
// Claim-time probes running per device (mi355x_probe_run). Mapping or unmapping the sweep buffer
// stalls a probe that runs beside it — up to the whole 6 s allocation when the driver is still
// clearing the previous buffer, 5-211 ms per chunk otherwise (profiles/r4p_probe_during_sweep_free.json)
// — so the lock-free sweep alloc / free paths wait between chunks while a probe runs: a probe then
// shares the device with at most one chunk operation (the scrubber avoids the pending clear).
// Counted over all devices: the HIP runtime serialises parts of an allocation process-wide, so a
// chunk mapped on one GPU can hold up a probe launching on another (an 8-GPU node scrubs idle GPUs
// while claims probe the others).
std::atomic<int> g_probes_active{0};

struct ProbeActive {
  ProbeActive() { g_probes_active.fetch_add(1); }
  ~ProbeActive() { g_probes_active.fetch_sub(1); }
};

// Wait until no claim-time probe runs in this process; dev -1: never wait (callers holding a
// device lock). Bounded twice: at most 2 s before one chunk, and at most ``budget`` (what is left of
// the whole alloc / free call's 3 s) over all its chunks — ~282 chunks under steady claim traffic
// must not turn a free into minutes while the pod's Allocate waits for it. In the agent's probe
// helpers a process holds one GPU, so only probes of that GPU are waited for. Returns the seconds
// spent waiting (the sweep trace reports them).
double yield_to_probes(int dev, double* budget) {
  static const bool off = std::getenv("GPUPOOL_SWEEP_NO_YIELD") != nullptr;  // in-process A/B only
  if (dev < 0 || off || !budget || *budget <= 0) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  const auto deadline = t0 + std::chrono::duration<double>(std::min(2.0, *budget));
  while (g_probes_active.load() > 0 && std::chrono::steady_clock::now() < deadline)
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *budget -= waited;
  return waited;
}

constexpr double kYieldBudgetS = 3.0;  // per sweep-buffer alloc / free call, over all its chunks

SweepBuf sweep_alloc_raw(uint64_t reserve, int yield_dev = -1) {
  size_t free_b = 0, total_b = 0;
  PROBE_CHECK(hipMemGetInfo(&free_b, &total_b));
  const uint64_t gran = 2ull << 20;
  if (free_b <= reserve + gran) throw ProbeError("not enough free HBM for a sweep window");
  SweepBuf b;
  const uint64_t span = ((free_b - reserve) / gran) * gran;
  double budget = kYieldBudgetS, yielded = 0;
  static const bool trace = std::getenv("GPUPOOL_SWEEP_TRACE") != nullptr;  // chunk timings
  for (uint64_t at = 0; at < span; at += kSweepChunk) {
    void* p = nullptr;
    yielded += yield_to_probes(yield_dev, &budget);
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipMalloc(&p, std::min<uint64_t>(kSweepChunk, span - at));
    if (e != hipSuccess) {
      for (void* q : b.chunks) (void)hipFree(q);
      (void)hipGetLastError();
      throw ProbeError(std::string("sweep chunk hipMalloc: ") + hipGetErrorString(e));
    }
    b.chunks.push_back(p);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (trace) std::fprintf(stderr, "sweep chunk %zu: %.3f ms\n", b.chunks.size() - 1, ms);
  }
  if (trace) std::fprintf(stderr, "sweep alloc: %zu chunks, %.1f ms yielded to probes\n", b.chunks.size(), yielded * 1e3);
  b.span = span;
  return b;
}

void sweep_free(SweepBuf& b, int yield_dev = -1) {
  double budget = kYieldBudgetS, yielded = 0;
  for (void* p : b.chunks) {  // one bounded unmap per chunk
    yielded += yield_to_probes(yield_dev, &budget);
    (void)hipFree(p);
  }
  static const bool trace = std::getenv("GPUPOOL_SWEEP_TRACE") != nullptr;
  if (trace) std::fprintf(stderr, "sweep free: %zu chunks, %.1f ms yielded to probes\n", b.chunks.size(), yielded * 1e3);
  b.chunks.clear();
  b.span = 0;
}

// One window of the rotating HBM sweep (see mi355x_probe_hbm_sweep in probe.h). The claim-time
// probe always tests the same ~1 GiB arena; this walks the rest of the 288 GB: a buffer of all free
// HBM minus ``reserve`` is allocated once per scrub pass (kept while ``keep``), and each call
// pattern-tests [offset, offset+bytes) of it with the same fill/verify kernels and both polarities.
std::string run_sweep(int dev, const char* opts) {
  const uint64_t want = static_cast<uint64_t>(std::max(1LL << 20, opt_int(opts, "bytes", 16LL << 30)));
  const uint64_t reserve = static_cast<uint64_t>(std::max(0LL, opt_int(opts, "reserve", 4LL << 30)));
  const uint64_t offset_in = static_cast<uint64_t>(std::max(0LL, opt_int(opts, "offset", 0)));
  const bool keep = opt_int(opts, "keep", 0) != 0;
  const int inject_flips = static_cast<int>(std::min(4096LL, std::max(0LL, opt_int(opts, "injectBitFlips", 0))));
  DeviceCtx& ctx = g_ctx[static_cast<size_t>(dev)];
  if (!ctx.ready) (void)run_probe(dev, "{\"hbmBytes\":1048576,\"patterns\":1,\"mfma\":false}");
  PROBE_CHECK(hipSetDevice(dev));
  auto t0 = std::chrono::steady_clock::now();
  double alloc_ms = 0;
  if (ctx.sweep.empty()) {  // normally pre-allocated by mi355x_probe_sweep_alloc outside the device lock
    ctx.sweep = sweep_alloc_raw(reserve);
    alloc_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  const uint64_t span = ctx.sweep.span;
  const uint64_t offset = (offset_in % span) & ~static_cast<uint64_t>(15);
  const uint64_t bytes = std::min<uint64_t>(want, span - offset) & ~static_cast<uint64_t>(15);
  if (!ctx.sweep_cnt) PROBE_CHECK(hipMalloc(reinterpret_cast<void**>(&ctx.sweep_cnt), 4 * sizeof(unsigned long long)));
  unsigned long long* cnt = ctx.sweep_cnt;
  hipStream_t s = ctx.stream;
  const int cus = ctx.prop.multiProcessorCount;
  unsigned long long bad = 0, first = ~0ull;
  float ms = 0;
  // the window may straddle chunks: test it piece by piece (both polarities per piece)
  for (uint64_t pos = offset; pos < offset + bytes;) {
    const size_t ci = static_cast<size_t>(pos / kSweepChunk);
    const uint64_t in = pos % kSweepChunk;
    const uint64_t clen = std::min<uint64_t>(kSweepChunk, span - ci * kSweepChunk);
    const uint64_t n = std::min<uint64_t>(offset + bytes - pos, clen - in) & ~static_cast<uint64_t>(15);
    if (n == 0) break;
    const uint64_t n16 = n / 16;
    auto* win = reinterpret_cast<u32x4*>(static_cast<char*>(ctx.sweep.chunks[ci]) + in);
    const int fill_grid = static_cast<int>(std::min<uint64_t>(static_cast<uint64_t>(cus), (n16 + kHbmThreads - 1) / kHbmThreads));
    const int verify_grid = static_cast<int>(std::min<uint64_t>(3ull * cus, (n16 + kHbmThreads - 1) / kHbmThreads));
    const uint32_t seed = 0x5CAB0000u ^ static_cast<uint32_t>(pos >> 20);
    PROBE_CHECK(hipMemsetAsync(cnt, 0, 4 * sizeof(unsigned long long), s));
    PROBE_CHECK(hipMemsetAsync(cnt + 1, 0xFF, sizeof(unsigned long long), s));
    PROBE_CHECK(hipMemsetAsync(cnt + 3, 0xFF, sizeof(unsigned long long), s));
    PROBE_CHECK(hipEventRecord(ctx.ev[0], s));
    for (int pi = 0; pi < 2; ++pi) {
      const uint32_t flip = pi ? 0xFFFFFFFFu : 0u;
      hipLaunchKernelGGL(hbm_fill<>, dim3(fill_grid), dim3(kHbmThreads), 0, s, win, n16, seed, flip,
                         static_cast<unsigned long long*>(nullptr), 0);
      if (pi == 0 && inject_flips > 0 && pos == offset)
        hipLaunchKernelGGL(inject_bit_flips, dim3(1), dim3(256), 0, s, reinterpret_cast<unsigned int*>(win), n16 * 4,
                           inject_flips);
      hipLaunchKernelGGL(hbm_verify<>, dim3(verify_grid), dim3(kHbmThreads), 0, s, static_cast<const u32x4*>(win), n16,
                         seed, flip, cnt + 2 * pi, cnt + 2 * pi + 1);
    }
    PROBE_CHECK(hipEventRecord(ctx.ev[1], s));
    PROBE_CHECK(hipGetLastError());
    PROBE_CHECK(hipMemcpyAsync(ctx.host_res, cnt, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    PROBE_CHECK(hipStreamSynchronize(s));
    float piece_ms = 0;
    PROBE_CHECK(hipEventElapsedTime(&piece_ms, ctx.ev[0], ctx.ev[1]));
    ms += piece_ms;
    bad += ctx.host_res[0] + ctx.host_res[2];
    const unsigned long long f = std::min(ctx.host_res[1], ctx.host_res[3]);
    if (f != ~0ull) first = std::min(first, (pos - offset) / 16 + f);
    pos += n;
  }
  if (!keep) sweep_free(ctx.sweep);
  const double gbps = ms > 0 ? 4.0 * static_cast<double>(bytes) / (ms * 1e-3) / 1e9 : 0.0;
  return "{\"device\":" + std::to_string(dev) + ",\"passed\":" + (bad == 0 ? "true" : "false") +
         ",\"offset\":" + std::to_string(offset) + ",\"bytes\":" + std::to_string(bytes) +
         ",\"span\":" + std::to_string(span) + ",\"badBits\":" + std::to_string(bad) +
         ",\"firstBadOffset\":" + (first == ~0ull ? std::string("null") : std::to_string(offset + first * 16)) +
         ",\"GBps\":" + jnum(gbps) + ",\"ms\":" + jnum(ms) + ",\"allocMs\":" + jnum(alloc_ms) + "}";
}

}  // namespace

extern "C" {

int mi355x_probe_init(char* err, size_t errlen) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_count >= 0) return g_count;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    if (err && errlen) std::snprintf(err, errlen, "hipGetDeviceCount: %s", hipGetErrorString(e));
    return -1;
  }
  g_ctx.resize(static_cast<size_t>(n));
  // Warm every context now so a claim-time probe pays no runtime/context initialisation.
  g_count = n;
  for (int d = 0; d < n; ++d) {
    if (hipSetDevice(d) != hipSuccess) continue;
    (void)hipFree(nullptr);
    try {
      (void)run_probe(d, "{\"hbmBytes\":1048576,\"patterns\":1,\"gemmN\":256,\"gemmReps\":1,\"keepArena\":0}");
    } catch (const std::exception&) {
      // a broken device fails its real probe later with the actual error
    }
  }
  return n;
}

int mi355x_probe_device_count(void) { return g_count; }

char* mi355x_probe_identify(int dev) {
  if (g_count < 0 || dev < 0 || dev >= g_count) return dup("{\"error\":\"bad device\"}");
  hipDeviceProp_t prop{};
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return dup("{\"error\":\"hipGetDeviceProperties failed\"}");
  char bdf[32];
  std::snprintf(bdf, sizeof bdf, "%04x:%02x:%02x.0", prop.pciDomainID, prop.pciBusID, prop.pciDeviceID);
  std::string out = "{\"device\":" + std::to_string(dev) + ",\"hipUUID\":" + jstr(hip_uuid(dev)) +
                    ",\"name\":" + jstr(prop.name) + ",\"gcnArch\":" + jstr(prop.gcnArchName) +
                    ",\"bdf\":" + jstr(bdf) + ",\"totalMem\":" + std::to_string(prop.totalGlobalMem) +
                    ",\"computeUnits\":" + std::to_string(prop.multiProcessorCount) + "}";
  return dup(out);
}

char* mi355x_probe_run(int dev, const char* opts_json) {
  if (g_count < 0 || dev < 0 || dev >= g_count) return dup("{\"passed\":false,\"error\":\"bad device index\"}");
  ProbeActive active;  // the sweep buffer's chunk (un)mapping waits while this runs
  // Per-device serialisation: concurrent probes of DIFFERENT devices run in parallel.
  std::lock_guard<std::mutex> g(device_mutex(dev));
  try {
    return dup(run_probe(dev, opts_json));
  } catch (const std::exception& e) {
    (void)hipGetLastError();
    return dup(std::string("{\"device\":") + std::to_string(dev) + ",\"passed\":false,\"error\":" + jstr(e.what()) + "}");
  }
}

char* mi355x_probe_peer(int src, int dst, const char* opts_json) {
  if (g_count < 0 || src < 0 || dst < 0 || src >= g_count || dst >= g_count)
    return dup("{\"passed\":false,\"error\":\"bad device index\"}");
  // both devices' probe locks, in index order (no deadlock against a concurrent pair)
  std::lock_guard<std::mutex> a(device_mutex(std::min(src, dst)));
  std::unique_lock<std::mutex> b;
  if (src != dst) b = std::unique_lock<std::mutex>(device_mutex(std::max(src, dst)));
  try {
    return dup(run_peer(src, dst, opts_json));
  } catch (const std::exception& e) {
    (void)hipGetLastError();
    return dup(std::string("{\"src\":") + std::to_string(src) + ",\"dst\":" + std::to_string(dst) +
               ",\"passed\":false,\"error\":" + jstr(e.what()) + "}");
  }
}

char* mi355x_probe_peer_ring(const int* devs, int n, const char* opts_json) {
  if (g_count < 0 || !devs || n < 2 || n > 64) return dup("{\"passed\":false,\"error\":\"bad ring\"}");
  std::vector<int> ring(devs, devs + n);
  for (int d : ring)
    if (d < 0 || d >= g_count) return dup("{\"passed\":false,\"error\":\"bad device index\"}");
  // every distinct device's probe lock, in index order (no deadlock against probes or pairs)
  std::vector<int> uniq(ring);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  std::vector<std::unique_lock<std::mutex>> locks;
  for (int d : uniq) locks.emplace_back(device_mutex(d));
  try {
    return dup(run_peer_ring(ring, opts_json));
  } catch (const std::exception& e) {
    (void)hipGetLastError();
    return dup(std::string("{\"passed\":false,\"error\":") + jstr(e.what()) + "}");
  }
}

// Frees the probe arenas idle for at least ``idle_ms`` (0: all, unconditionally); returns how many
// were freed. With idle_ms > 0 an arena stays while its device holds an HBM sweep buffer or freed one
// less than kSweepClearGrace ago.
int mi355x_probe_trim(int idle_ms) {
  if (g_count <= 0) return 0;
  int freed = 0;
  const auto now = std::chrono::steady_clock::now();
  for (int d = 0; d < g_count; ++d) {
    std::lock_guard<std::mutex> g(device_mutex(d));
    DeviceCtx& ctx = g_ctx[static_cast<size_t>(d)];
    const auto idle = std::chrono::milliseconds(idle_ms);
    bool arena = ctx.arena && now - ctx.arena_used >= idle;
    if (idle_ms > 0 && (!ctx.sweep.empty() || now - ctx.sweep_released < kSweepClearGrace)) arena = false;  // 0 = forced
    const bool peer = ctx.peer_bytes && now - ctx.peer_used >= idle;  // the xGMI ring windows
    if (!arena && !peer) continue;
    if (hipSetDevice(d) != hipSuccess) continue;
    if (peer) free_peer_bufs(ctx);
    if (!arena) continue;
    (void)hipFree(ctx.arena);
    ctx.arena = nullptr;
    ctx.arena_bytes = 0;
    ++freed;
  }
  return freed;
}

char* mi355x_probe_hbm_sweep(int dev, const char* opts_json) {
  if (g_count < 0 || dev < 0 || dev >= g_count) return dup("{\"passed\":false,\"error\":\"bad device index\"}");
  std::lock_guard<std::mutex> g(device_mutex(dev));
  try {
    return dup(run_sweep(dev, opts_json));
  } catch (const std::exception& e) {
    (void)hipGetLastError();
    return dup(std::string("{\"device\":") + std::to_string(dev) + ",\"passed\":false,\"error\":" + jstr(e.what()) + "}");
  }
}

int mi355x_probe_sweep_alloc(int dev, long long reserve) {
  if (g_count < 0 || dev < 0 || dev >= g_count) return -1;
  {
    std::lock_guard<std::mutex> g(device_mutex(dev));
    if (!g_ctx[static_cast<size_t>(dev)].sweep.empty()) return 0;
  }
  SweepBuf b;
  try {
    if (hipSetDevice(dev) != hipSuccess) return -1;
    b = sweep_alloc_raw(static_cast<uint64_t>(std::max(0LL, reserve)), dev);
  } catch (const std::exception&) {
    (void)hipGetLastError();
    return -2;
  }
  std::lock_guard<std::mutex> g(device_mutex(dev));
  DeviceCtx& ctx = g_ctx[static_cast<size_t>(dev)];
  if (!ctx.sweep.empty()) {  // lost a race with another allocator: keep theirs
    sweep_free(b);
    return 0;
  }
  ctx.sweep = std::move(b);
  return 1;
}

int mi355x_probe_sweep_release(int dev) {
  if (g_count < 0 || dev < 0 || dev >= g_count) return -1;
  SweepBuf b;
  {
    std::lock_guard<std::mutex> g(device_mutex(dev));
    DeviceCtx& ctx = g_ctx[static_cast<size_t>(dev)];
    b = std::move(ctx.sweep);
    ctx.sweep = SweepBuf{};
    ctx.sweep_released = std::chrono::steady_clock::now();
  }
  if (b.empty()) return 0;
  if (hipSetDevice(dev) != hipSuccess) return -1;
  sweep_free(b, dev);  // outside the device lock, chunk by chunk, between probes
  return 1;
}

int mi355x_probe_gemm_bf16(int dev, const void* A, const void* Bt, void* C, int m, int n, int k) {
  if (g_count < 0 || dev < 0 || dev >= g_count) return -1;
  if (m <= 0 || n <= 0 || k <= 0 || m % G2_BM || n % G2_BN || k % G2_BK || !A || !Bt || !C) return -2;
  std::lock_guard<std::mutex> g(device_mutex(dev));
  try {
    PROBE_CHECK(hipSetDevice(dev));
    const size_t sa = static_cast<size_t>(m) * k * 2, sb = static_cast<size_t>(n) * k * 2,
                 sc = static_cast<size_t>(m) * n * 4;
    DevBuf da, db, dc;
    PROBE_CHECK(hipMalloc(&da.p, sa));
    PROBE_CHECK(hipMalloc(&db.p, sb));
    PROBE_CHECK(hipMalloc(&dc.p, sc));
    PROBE_CHECK(hipMemcpy(da.p, A, sa, hipMemcpyHostToDevice));
    PROBE_CHECK(hipMemcpy(db.p, Bt, sb, hipMemcpyHostToDevice));
    const dim3 grid((m / G2_BM) * (n / G2_BN));
    if (kGemmPipe == 2)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<true, 0, 1>), grid, dim3(kGemm2Threads), 0, nullptr,
                         static_cast<const short*>(da.p), static_cast<const short*>(db.p), static_cast<float*>(dc.p), m,
                         n, k, static_cast<unsigned long long*>(nullptr), kGemmGroupM);
    else if (kGemmPipe == 1)
      hipLaunchKernelGGL((gemm_bf16_mfma_256p<false>), grid, dim3(kGemm2Threads), 0, nullptr, static_cast<const short*>(da.p),
                         static_cast<const short*>(db.p), static_cast<float*>(dc.p), m, n, k,
                         static_cast<unsigned long long*>(nullptr), kGemmGroupM);
    else
      hipLaunchKernelGGL((gemm_bf16_mfma_256<false, false>), grid, dim3(kGemm2Threads), 0, nullptr,
                         static_cast<const short*>(da.p), static_cast<const short*>(db.p), static_cast<float*>(dc.p), m,
                         n, k, static_cast<unsigned long long*>(nullptr), kGemmGroupM);
    PROBE_CHECK(hipGetLastError());
    PROBE_CHECK(hipMemcpy(C, dc.p, sc, hipMemcpyDeviceToHost));
    return 0;
  } catch (const std::exception&) {
    (void)hipGetLastError();
    return -4;
  }
}

void mi355x_probe_free(char* p) { std::free(p); }

}  // extern "C"

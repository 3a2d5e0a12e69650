// GPU self-test for the probe's MFMA fragment mapping, independent of the probe's own checks:
// A = identity, B asymmetric (B[k][n] = k*1000 + n) — per cdna_hip_programming.md §3 "Always A=I
// check with ASYMMETRIC B" — so a row<->col swap in the C-write cannot pass.
// Built as part of `make native`; run by tests/gpu/test_probe_gpu.py on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x16 = __attribute__((ext_vector_type(16))) float;

static short f2bf(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  return static_cast<short>(u >> 16);
}

// One wave computes C[32][32] = A[32][16] * B[16][32] (B given as Bt[n][k]).
__global__ void one_tile(const short* A, const short* Bt, float* C) {
  int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[r * 16 + 8 * h + j];
    b[j] = Bt[r * 16 + 8 * h + j];
  }
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) {
    int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    C[row * 32 + r] = acc[i];
  }
}

// One wave computes C[16][16] = A[16][32] * B[32][16] with v_mfma_f32_16x16x32_bf16 (the probe's
// main GEMM instruction): lane l holds A[l&15][8(l>>4)+j], Bt[l&15][8(l>>4)+j]; C/D col = l&15,
// row = 4(l>>4) + reg.
using f32x4 = __attribute__((ext_vector_type(4))) float;
__global__ void one_tile16(const short* A, const short* Bt, float* C) {
  int lane = threadIdx.x, r = lane & 15, q = lane >> 4;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[r * 32 + 8 * q + j];
    b[j] = Bt[r * 32 + 8 * q + j];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[(4 * q + i) * 16 + r] = acc[i];
}

static int check16() {
  // A[16][32]: A[i][i] = 1, A[i][i+16] = 3 (both k-halves used); Bt asymmetric: Bt[n][k] = 4k + n%4.
  std::vector<short> A(16 * 32, 0), Bt(16 * 32);
  std::vector<float> ref(16 * 16, 0.f);
  for (int i = 0; i < 16; ++i) {
    A[i * 32 + i] = f2bf(1.f);
    A[i * 32 + i + 16] = f2bf(3.f);
  }
  for (int n = 0; n < 16; ++n)
    for (int k = 0; k < 32; ++k) Bt[n * 32 + k] = f2bf(static_cast<float>(4 * k + (n % 4)));
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) ref[m * 16 + n] = 1.f * (4 * m + n % 4) + 3.f * (4 * (m + 16) + n % 4);
  short *dA, *dB;
  float* dC;
  if (hipMalloc(&dA, A.size() * 2) || hipMalloc(&dB, Bt.size() * 2) || hipMalloc(&dC, 16 * 16 * 4)) return -1;
  (void)hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, Bt.data(), Bt.size() * 2, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(one_tile16, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  std::vector<float> C(16 * 16);
  (void)hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16 * 16; ++i) bad += C[i] != ref[i];
  (void)hipFree(dA);
  (void)hipFree(dB);
  (void)hipFree(dC);
  return bad;
}

int main() {
  // A: 32x16 "identity" (A[i][i%16] = 1 for i<16, A[i][i-16]=2 for i>=16): rows pick rows of B.
  std::vector<short> A(32 * 16, 0), Bt(32 * 16);
  std::vector<float> ref(32 * 32, 0.f);
  for (int i = 0; i < 32; ++i) A[i * 16 + (i % 16)] = f2bf(i < 16 ? 1.f : 2.f);
  for (int n = 0; n < 32; ++n)
    for (int k = 0; k < 16; ++k) Bt[n * 16 + k] = f2bf(static_cast<float>(k * 8 + (n % 8)));  // exact in bf16
  for (int m = 0; m < 32; ++m)
    for (int n = 0; n < 32; ++n) {
      float s = 0;
      for (int k = 0; k < 16; ++k) {
        unsigned ua = static_cast<unsigned>(static_cast<unsigned short>(A[m * 16 + k])) << 16;
        unsigned ub = static_cast<unsigned>(static_cast<unsigned short>(Bt[n * 16 + k])) << 16;
        float fa, fb;
        std::memcpy(&fa, &ua, 4);
        std::memcpy(&fb, &ub, 4);
        s += fa * fb;
      }
      ref[m * 32 + n] = s;
    }
  short *dA, *dB;
  float* dC;
  if (hipMalloc(&dA, A.size() * 2) || hipMalloc(&dB, Bt.size() * 2) || hipMalloc(&dC, 32 * 32 * 4)) return 3;
  (void)hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, Bt.data(), Bt.size() * 2, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(one_tile, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  std::vector<float> C(32 * 32);
  (void)hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32 * 32; ++i) bad += C[i] != ref[i];
  (void)hipFree(dA);
  (void)hipFree(dB);
  (void)hipFree(dC);
  const int bad16 = check16();
  std::printf("{\"mfma_layout_mismatches\": %d, \"mfma16_layout_mismatches\": %d}\n", bad, bad16);
  return bad == 0 && bad16 == 0 ? 0 : 1;
}

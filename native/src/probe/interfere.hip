// libmi355x_interfere.so — the two load shapes of the slot-interference A/B
// (scripts/xcd_interference_ab.py): does a slot that streams HBM slow down a sibling slot on the
// same GPU, under a striped CU mask (every slot on every XCD, so every slot shares all eight 4 MB
// L2s) versus an XCD-aligned one (each slot owns whole XCDs and so their L2s)?
//
//   * mi355x_interfere_l2     — the L2-resident victim: every block re-reads a small buffer (sized
//     to fit one XCD's L2) `iters` times per launch; reported as the read bandwidth it sustains.
//   * mi355x_interfere_stream — the aggressor: a read+write copy over a large buffer (far beyond the
//     256 MB MALL) for a wall-clock duration, i.e. a continuous L2-thrashing HBM stream.
//
// Both run whatever CU mask the process was given (libgpupool_share.so via HSA_TOOLS_LIB), so the
// grid is sized for the whole GPU and the dispatcher confines it to the slot's CUs. The kernels
// only read/write through vector memory ops; no bounds can be exceeded (grid-stride loops with
// power-of-two masks checked on the host).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <vector>

namespace {

using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
constexpr int kThreads = 256;

// Each pass starts at a different offset so the compiler cannot fold passes into one load.
__global__ __launch_bounds__(kThreads) void l2_reread(const u32x4* __restrict__ p, uint64_t mask16,
                                                      int iters, u32x4* __restrict__ sink) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int it = 0; it < iters; ++it) {
    const uint64_t base = static_cast<uint64_t>(it) * 4099u;
    for (uint64_t i = tid; i <= mask16; i += stride) acc += p[(i + base) & mask16];
  }
  sink[tid] = acc;  // one vector store per thread keeps the loads live
}

__global__ __launch_bounds__(kThreads) void stream_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                        uint64_t n16) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n16; i += stride)
    dst[i] = src[i] + 1u;
}

struct Buf {
  void* p = nullptr;
  ~Buf() { if (p) (void)hipFree(p); }
};

bool pow2(uint64_t x) { return x && !(x & (x - 1)); }

}  // namespace

extern "C" {

// Median read bandwidth (GB/s) of `reps` launches, each re-reading `bytes` `iters` times.
// Returns 0 on success, <0 on a bad argument or HIP error.
int mi355x_interfere_l2(int dev, unsigned long long bytes, int iters, int reps, double* gbps) {
  if (!gbps || bytes < 4096 || !pow2(bytes) || iters <= 0 || reps <= 0) return -1;
  if (hipSetDevice(dev) != hipSuccess) return -2;
  // one vector per thread per pass: a 2 MB buffer is 512 blocks, 8 per CU of a 64-CU slot
  const int blocks = static_cast<int>(std::min<uint64_t>(4096, std::max<uint64_t>(1, bytes / sizeof(u32x4) / kThreads)));
  Buf buf, sink;
  if (hipMalloc(&buf.p, bytes) != hipSuccess) return -3;
  if (hipMalloc(&sink.p, static_cast<size_t>(blocks) * kThreads * sizeof(u32x4)) != hipSuccess) return -3;
  if (hipMemset(buf.p, 0x5a, bytes) != hipSuccess) return -4;
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -4;
  const uint64_t mask16 = bytes / sizeof(u32x4) - 1;
  std::vector<double> gb;
  int rc = 0;
  for (int r = 0; r <= reps && rc == 0; ++r) {  // launch 0 warms the L2 and is not counted
    (void)hipEventRecord(a, nullptr);
    hipLaunchKernelGGL(l2_reread, dim3(blocks), dim3(kThreads), 0, nullptr, static_cast<const u32x4*>(buf.p),
                       mask16, iters, static_cast<u32x4*>(sink.p));
    (void)hipEventRecord(b, nullptr);
    if (hipEventSynchronize(b) != hipSuccess) { rc = -5; break; }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r > 0 && ms > 0) gb.push_back(static_cast<double>(bytes) * iters / (ms * 1e6));
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (rc || gb.empty()) return rc ? rc : -5;
  std::sort(gb.begin(), gb.end());
  *gbps = gb[gb.size() / 2];
  return 0;
}

// Copy a `bytes` buffer into another (read + write) back to back for `seconds` of wall clock.
// *gbps = bytes moved (read + written) per second over the whole run.
int mi355x_interfere_stream(int dev, unsigned long long bytes, double seconds, double* gbps) {
  if (!gbps || bytes < (1ull << 20) || !pow2(bytes) || !(seconds > 0)) return -1;
  if (hipSetDevice(dev) != hipSuccess) return -2;
  Buf src, dst;
  if (hipMalloc(&src.p, bytes) != hipSuccess || hipMalloc(&dst.p, bytes) != hipSuccess) return -3;
  if (hipMemset(src.p, 1, bytes) != hipSuccess) return -4;
  const uint64_t n16 = bytes / sizeof(u32x4);
  const auto t0 = std::chrono::steady_clock::now();
  double elapsed = 0;
  uint64_t passes = 0;
  while (elapsed < seconds) {
    for (int k = 0; k < 8; ++k, ++passes)
      hipLaunchKernelGGL(stream_copy, dim3(8192), dim3(kThreads), 0, nullptr, static_cast<const u32x4*>(src.p),
                         static_cast<u32x4*>(dst.p), n16);
    if (hipDeviceSynchronize() != hipSuccess) return -5;
    elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  *gbps = 2.0 * static_cast<double>(bytes) * passes / (elapsed * 1e9);
  return 0;
}

}  // extern "C"

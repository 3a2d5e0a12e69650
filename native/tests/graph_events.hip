// Feasibility + cost of replaying a two-stream kernel sequence as a hipGraph on gfx950: captures
// a fork (stream A) / join (stream B) sequence of streaming kernels with timing events recorded
// inside the capture, replays it, and checks that hipEventElapsedTime works on events recorded by
// the graph. Then times the host enqueue + completion of the same sequence issued eagerly vs as one
// graph launch, interleaved, after an idle gap and back to back.
//
//   graph_events [MiB=1024] [rounds=15]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                   hipGetErrorString(e_));                                    \
      std::exit(2);                                                           \
    }                                                                         \
  } while (0)

namespace {

__global__ void fill(uint4* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    p[i] = make_uint4(seed ^ unsigned(i), seed + unsigned(i), ~unsigned(i), seed);
}

__global__ void verify(const uint4* p, size_t n, unsigned seed, unsigned long long* bad) {
  unsigned long long b = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    uint4 v = p[i];
    b += (v.x != (seed ^ unsigned(i))) + (v.y != seed + unsigned(i)) + (v.z != ~unsigned(i)) + (v.w != seed);
  }
  if (b) atomicAdd(bad, b);
}

__global__ void small_work(float* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 1.0001f + 1.0f;
}

struct Ctx {
  hipStream_t a, b;
  hipEvent_t fork, join, t[5];
  uint4* buf;
  size_t n16;
  float* sm;
  unsigned long long* bad;
  unsigned long long* host;
  int cus;
};

// the sequence: A: t0 fill t1 verify t2 fill t3 verify t4 -> D2H; B: 12 small kernels
void enqueue(Ctx& c) {
  CHECK(hipEventRecord(c.fork, c.a));
  CHECK(hipStreamWaitEvent(c.b, c.fork, 0));
  CHECK(hipMemsetAsync(c.bad, 0, 8, c.a));
  CHECK(hipEventRecord(c.t[0], c.a));
  for (int p = 0; p < 2; ++p) {
    hipLaunchKernelGGL(fill, dim3(c.cus), dim3(1024), 0, c.a, c.buf, c.n16, 0x1234u + p);
    CHECK(hipEventRecord(c.t[1 + 2 * p], c.a));
    hipLaunchKernelGGL(verify, dim3(3 * c.cus), dim3(1024), 0, c.a, c.buf, c.n16, 0x1234u + p, c.bad);
    CHECK(hipEventRecord(c.t[2 + 2 * p], c.a));
  }
  for (int k = 0; k < 12; ++k) hipLaunchKernelGGL(small_work, dim3(64), dim3(256), 0, c.b, c.sm, 64 * 256);
  CHECK(hipEventRecord(c.join, c.b));
  CHECK(hipStreamWaitEvent(c.a, c.join, 0));
  CHECK(hipMemcpyAsync(c.host, c.bad, 8, hipMemcpyDeviceToHost, c.a));
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

}  // namespace

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 15;
  Ctx c{};
  CHECK(hipSetDevice(0));
  hipDeviceProp_t prop{};
  CHECK(hipGetDeviceProperties(&prop, 0));
  c.cus = prop.multiProcessorCount;
  CHECK(hipStreamCreateWithFlags(&c.a, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&c.b, hipStreamNonBlocking));
  CHECK(hipEventCreate(&c.fork));
  CHECK(hipEventCreate(&c.join));
  for (auto& e : c.t) CHECK(hipEventCreate(&e));
  c.n16 = (mib << 20) / 16;
  CHECK(hipMalloc(&c.buf, c.n16 * 16));
  CHECK(hipMalloc(&c.sm, 64 * 256 * 4));
  CHECK(hipMalloc(&c.bad, 8));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&c.host), 8));

  // capture
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  CHECK(hipStreamBeginCapture(c.a, hipStreamCaptureModeThreadLocal));
  enqueue(c);
  CHECK(hipStreamEndCapture(c.a, &g));
  size_t nodes = 0;
  CHECK(hipGraphGetNodes(g, nullptr, &nodes));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));

  // correctness + events from the graph
  CHECK(hipGraphLaunch(ge, c.a));
  CHECK(hipStreamSynchronize(c.a));
  float w = -1, r = -1;
  hipError_t ew = hipEventElapsedTime(&w, c.t[0], c.t[1]);
  hipError_t er = hipEventElapsedTime(&r, c.t[1], c.t[2]);
  std::printf("{\"graphNodes\":%zu,\"badAfterGraph\":%llu,\"eventsInGraph\":{\"write\":\"%s\",\"writeMs\":%.4f,"
              "\"read\":\"%s\",\"readMs\":%.4f}}\n",
              nodes, *c.host, hipGetErrorString(ew), w, hipGetErrorString(er), r);

  // interleaved timing: eager vs graph, after a 300 ms idle gap and back to back
  std::vector<double> eager_idle, graph_idle, eager_warm, graph_warm, eager_enq, graph_enq;
  for (int i = 0; i < rounds; ++i) {
    for (int mode = 0; mode < 2; ++mode) {
      std::this_thread::sleep_for(std::chrono::milliseconds(300));
      for (int warm = 0; warm < 2; ++warm) {
        auto t0 = std::chrono::steady_clock::now();
        if (mode == 0)
          enqueue(c);
        else
          CHECK(hipGraphLaunch(ge, c.a));
        double enq = ms_since(t0);
        CHECK(hipStreamSynchronize(c.a));
        double tot = ms_since(t0);
        if (*c.host != 0) std::fprintf(stderr, "verify mismatch %llu\n", *c.host);
        auto& v = mode == 0 ? (warm ? eager_warm : eager_idle) : (warm ? graph_warm : graph_idle);
        v.push_back(tot);
        if (!warm) (mode == 0 ? eager_enq : graph_enq).push_back(enq);
      }
    }
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  std::printf("{\"rounds\":%d,\"MiB\":%zu,\"eagerIdleMs\":%.4f,\"graphIdleMs\":%.4f,\"eagerWarmMs\":%.4f,"
              "\"graphWarmMs\":%.4f,\"eagerEnqueueIdleMs\":%.4f,\"graphEnqueueIdleMs\":%.4f}\n",
              rounds, mib, med(eager_idle), med(graph_idle), med(eager_warm), med(graph_warm), med(eager_enq),
              med(graph_enq));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return 0;
}

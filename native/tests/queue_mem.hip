// Host memory per HIP hardware queue on this GPU: RSS of the process and the large anonymous
// "do not copy" regions (VmFlags dc) the runtime maps, after each step of bringing up streams.
// Each HW queue of a gfx950 device carries a context-save area sized for all of its CUs' waves.
//
//   queue_mem [streams=3] [devices=1]     (GPU_MAX_HW_QUEUES in the environment caps HW queues)
//
// scripts/hip_host_memory.py runs it under several settings.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

namespace {

__global__ void touch(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

struct Mem {
  double rss_mib = 0;
  int regions = 0;        // anonymous dc regions >= 64 MiB
  double region_mib = 0;  // their RSS together
};

Mem measure() {
  Mem m;
  std::ifstream f("/proc/self/smaps");
  std::string line;
  bool big = false, anon = false;
  double cur_rss = 0;
  auto close_region = [&](const std::string& flags) {
    if (big && anon && flags.find(" dc") != std::string::npos) {
      ++m.regions;
      m.region_mib += cur_rss;
    }
  };
  while (std::getline(f, line)) {
    unsigned long a = 0, b = 0;
    char perm[8] = {0};
    if (std::sscanf(line.c_str(), "%lx-%lx %7s", &a, &b, perm) == 3 && line.find(':') > 8) {
      big = (b - a) >= (64ul << 20);
      // the pathname column is empty for an anonymous mapping
      size_t n = 0;
      int fields = 0;
      bool in = false;
      for (; n < line.size(); ++n) {
        bool sp = line[n] == ' ';
        if (!sp && !in) ++fields;
        in = !sp;
      }
      anon = fields <= 5;
      cur_rss = 0;
    } else if (line.rfind("Rss:", 0) == 0) {
      cur_rss = std::atof(line.c_str() + 4) / 1024.0;
    } else if (line.rfind("VmFlags:", 0) == 0) {
      close_region(line);
    }
  }
  std::ifstream s("/proc/self/status");
  while (std::getline(s, line))
    if (line.rfind("VmRSS:", 0) == 0) m.rss_mib = std::atof(line.c_str() + 6) / 1024.0;
  return m;
}

void report(const char* step) {
  Mem m = measure();
  std::printf("{\"step\":\"%s\",\"rssMiB\":%.1f,\"dcRegions\":%d,\"dcRegionMiB\":%.1f}\n", step, m.rss_mib,
              m.regions, m.region_mib);
  std::fflush(stdout);
}

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(2);                                                                \
    }                                                                              \
  } while (0)

}  // namespace

int main(int argc, char** argv) {
  const int nstreams = argc > 1 ? std::atoi(argv[1]) : 3;
  int ndev = argc > 2 ? std::atoi(argv[2]) : 1;
  report("start");
  CHECK(hipInit(0));
  report("hipInit");
  int have = 0;
  CHECK(hipGetDeviceCount(&have));
  if (ndev > have) ndev = have;
  std::vector<int*> buf(ndev, nullptr);
  for (int d = 0; d < ndev; ++d) {
    CHECK(hipSetDevice(d));
    CHECK(hipMalloc(&buf[d], 4096));
    CHECK(hipMemset(buf[d], 0, 4096));
    CHECK(hipDeviceSynchronize());
  }
  report("context+null-stream memset");
  for (int d = 0; d < ndev; ++d) {
    CHECK(hipSetDevice(d));
    hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, nullptr, buf[d]);
    CHECK(hipDeviceSynchronize());
  }
  report("kernel on the null stream");
  std::vector<hipStream_t> st;
  for (int i = 0; i < nstreams; ++i) {
    for (int d = 0; d < ndev; ++d) {
      CHECK(hipSetDevice(d));
      hipStream_t s = nullptr;
      CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, buf[d]);
      CHECK(hipStreamSynchronize(s));
      st.push_back(s);
    }
    char name[64];
    std::snprintf(name, sizeof name, "stream %d (+kernel)", i + 1);
    report(name);
  }
  for (hipStream_t s : st) CHECK(hipStreamDestroy(s));
  report("streams destroyed");
  return 0;
}

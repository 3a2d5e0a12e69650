// mi355x-probe CLI: `mi355x-probe [--device N|--all] [--hbm-bytes B] [--gemm-n N] [--no-mfma]
// [--list]`. Prints one JSON object per probed device and exits 0 iff every probe passed.
// Equivalent of the reference's in-pod `nvidia-smi` smoke check (GPU调度平台搭建.md:134-138),
// but it exercises HBM and the matrix cores instead of only enumerating the device.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mi355x/probe.h"

int main(int argc, char** argv) {
  long long hbm = 1LL << 30;
  int gemm_n = 4096;
  bool mfma = true, all = true, list = false;
  int device = -1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--device") {
      device = std::atoi(next());
      all = false;
    } else if (a == "--all") {
      all = true;
    } else if (a == "--hbm-bytes") {
      hbm = std::atoll(next());
    } else if (a == "--gemm-n") {
      gemm_n = std::atoi(next());
    } else if (a == "--no-mfma") {
      mfma = false;
    } else if (a == "--list") {
      list = true;
    } else if (a == "-h" || a == "--help") {
      std::printf("usage: mi355x-probe [--device N|--all] [--hbm-bytes B] [--gemm-n N] [--no-mfma] [--list]\n");
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  char err[256] = {0};
  int n = mi355x_probe_init(err, sizeof err);
  if (n < 0) {
    std::fprintf(stderr, "probe init failed: %s\n", err);
    return 3;
  }
  if (n == 0) {
    std::fprintf(stderr, "no HIP devices visible\n");
    return 3;
  }
  std::vector<int> devs;
  if (all) {
    for (int d = 0; d < n; ++d) devs.push_back(d);
  } else {
    if (device < 0 || device >= n) {
      std::fprintf(stderr, "device %d out of range [0,%d)\n", device, n);
      return 2;
    }
    devs.push_back(device);
  }
  if (list) {
    for (int d : devs) {
      char* s = mi355x_probe_identify(d);
      std::printf("%s\n", s);
      mi355x_probe_free(s);
    }
    return 0;
  }
  char opts[256];
  std::snprintf(opts, sizeof opts, "{\"hbmBytes\":%lld,\"mfma\":%s,\"gemmN\":%d}", hbm, mfma ? "true" : "false", gemm_n);
  std::vector<std::string> results(devs.size());
  std::vector<std::thread> ths;
  for (size_t i = 0; i < devs.size(); ++i) {
    ths.emplace_back([&, i] {
      char* s = mi355x_probe_run(devs[i], opts);
      results[i] = s;
      mi355x_probe_free(s);
    });
  }
  for (auto& t : ths) t.join();
  int rc = 0;
  for (const auto& r : results) {
    std::printf("%s\n", r.c_str());
    if (r.find("\"passed\":true") == std::string::npos) rc = 1;
  }
  return rc;
}

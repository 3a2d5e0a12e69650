// Runner: `gpupool_tests [filter]` runs every registered case whose name contains ``filter``.
#include <chrono>
#include <cstring>

#include "testing.h"

int main(int argc, char** argv) {
  const char* filter = argc > 1 ? argv[1] : "";
  int pass = 0, fail = 0;
  for (auto& c : gtest_lite::registry()) {
    if (*filter && !std::strstr(c.name, filter)) continue;
    auto t0 = std::chrono::steady_clock::now();
    try {
      c.fn();
      ++pass;
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      std::printf("[ OK ] %s (%.1f ms)\n", c.name, ms);
    } catch (const std::exception& e) {
      ++fail;
      std::printf("[FAIL] %s: %s\n", c.name, e.what());
    }
  }
  std::printf("%d passed, %d failed\n", pass, fail);
  return fail ? 1 : 0;
}

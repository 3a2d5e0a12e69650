// Runner: `gpupool_tests [filter]` runs every registered case whose name contains ``filter``.
#include <chrono>
#include <cstring>

#include "gpupool/agentauth.h"
#include "testing.h"

int main(int argc, char** argv) {
  // `gpupool_tests --sign KEY METHOD TARGET NODE BODY`: print the manager's signature header for
  // one request (tests/unit/test_edsig.py checks it against the agent's Python verifier)
  // (with an 8th argument, the agent's base64url X25519 key: the v2 per-node MAC header)
  if ((argc == 7 || argc == 8) && std::strcmp(argv[1], "--sign") == 0) {
    gpupool::AgentSigner s(argv[2]);
    std::fputs(s.header(argv[3], argv[4], argv[5], argv[6], argc == 8 ? argv[7] : "").c_str(), stdout);
    return 0;
  }
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

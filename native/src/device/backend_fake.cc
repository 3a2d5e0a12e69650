// Fake backend: a node snapshot loaded from a JSON fixture (CPU-only tests, SURVEY.md §4.2
// "Device layer" row). The default fixture tests/fixtures/node_8x_mi355x.json models an
// 8x MI355X OAM node after the shapes captured from real hardware (tests/fixtures/real_mi355x/).
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "model.h"

namespace mi355x {

namespace {

Json load_json_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open fixture " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return Json::parse(ss.str());
}

uint32_t fnv1a(const std::string& s) {
  uint32_t h = 2166136261u;
  for (unsigned char c : s) {
    h ^= c;
    h *= 16777619u;
  }
  return h;
}

class FakeBackend : public Backend {
 public:
  explicit FakeBackend(const Json& cfg) {
    std::string path = cfg["fixture"].as_string();
    if (path.empty()) throw std::runtime_error("fake backend needs config.fixture");
    base_ = load_json_file(path);
    if (!base_["devices"].is_array()) throw std::runtime_error("fixture has no devices[]");
    std::string node = cfg["node"].as_string();
    int64_t limit = cfg["count"].as_int(-1);
    if (limit >= 0) {
      auto& devs = base_["devices"].elements();
      if (static_cast<size_t>(limit) < devs.size()) devs.resize(static_cast<size_t>(limit));
    }
    // Distinct nodes must not share device identities: salt UUIDs with the node name.
    if (!node.empty() && cfg["saltUUIDs"].as_bool(true)) {
      uint32_t h = fnv1a(node);
      for (auto& d : base_["devices"].elements()) {
        char buf[16];
        std::snprintf(buf, sizeof buf, "%08x", h ^ static_cast<uint32_t>(d["index"].as_int()));
        std::string u = d["uuid"].as_string();
        if (u.size() >= 8) d["uuid"] = u.substr(0, u.size() - 8) + buf;
        std::string hu = d["hipUUID"].as_string();
        if (hu.size() >= 8) d["hipUUID"] = hu.substr(0, hu.size() - 8) + buf;
      }
    }
    if (!node.empty()) base_["node"] = node;
  }
  std::string name() const override { return "fake"; }
  Json snapshot() override {
    Json s = base_;
    s["backend"] = "fake";
    return s;
  }

 private:
  Json base_;
};

}  // namespace

std::unique_ptr<Backend> make_fake_backend(const Json& cfg) { return std::make_unique<FakeBackend>(cfg); }

}  // namespace mi355x

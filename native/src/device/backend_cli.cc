// CLI backend: parses `amd-smi {list,static,metric,xgmi,partition} --json`. It is deliberately
// independent of libamd_smi (subprocess + text) so the bench/tests can cross-check the operator's
// amdsmi path against it. With config {"cliDir": dir} it reads previously captured outputs
// (<dir>/amdsmi_<cmd>.json) instead — used on CPU with the shapes frozen from real MI355X
// hardware in tests/fixtures/real_mi355x/.
#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

#include "model.h"

namespace mi355x {

namespace {

std::string run_cmd(const std::string& cmd) {
  FILE* p = popen(cmd.c_str(), "r");
  if (!p) throw std::runtime_error("popen failed: " + cmd);
  std::string out;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, p)) > 0) out.append(buf, n);
  int rc = pclose(p);
  if (rc != 0) throw std::runtime_error("command failed (" + std::to_string(rc) + "): " + cmd);
  return out;
}

Json val_unit(const Json& v) {  // {"value": 46, "unit": "C"} | "N/A" | 46
  if (v.is_object()) return v["value"];
  if (v.is_number()) return v;
  return Json();
}

std::string to_lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}

class CliBackend : public Backend {
 public:
  explicit CliBackend(const Json& cfg) {
    bin_ = cfg["amdsmiBin"].str_or("amd-smi");
    dir_ = cfg["cliDir"].as_string();
    node_ = cfg["node"].as_string();
    (void)fetch("list");  // fail fast if amd-smi is unusable
  }

  std::string name() const override { return "cli"; }

  Json fetch(const std::string& cmd) {
    std::string text;
    if (!dir_.empty()) {
      std::ifstream f(dir_ + "/amdsmi_" + cmd + ".json");
      if (!f) throw std::runtime_error("missing captured amd-smi output " + dir_ + "/amdsmi_" + cmd + ".json");
      std::stringstream ss;
      ss << f.rdbuf();
      text = ss.str();
    } else {
      text = run_cmd(bin_ + " " + cmd + " --json 2>/dev/null");
    }
    return Json::parse(text);
  }

  Json snapshot() override {
    Json list = fetch("list");
    Json st = fetch("static");
    Json me = fetch("metric");
    Json xg;
    Json part;
    try { xg = fetch("xgmi"); } catch (const std::exception&) {}
    try { part = fetch("partition"); } catch (const std::exception&) {}
    auto by_gpu = [](const Json& arr) {
      std::map<int64_t, Json> m;
      for (const auto& e : arr.elements()) m[e["gpu"].as_int(e["gpu_id"].as_int(-1))] = e;
      return m;
    };
    const Json& st_arr = st["gpu_data"].is_array() ? st["gpu_data"] : st;
    const Json& me_arr = me["gpu_data"].is_array() ? me["gpu_data"] : me;
    auto sm = by_gpu(st_arr), mm = by_gpu(me_arr);
    auto links = by_gpu(xg["link_port_status"]);
    auto parts = by_gpu(part["current_partition"]);
    Json devs = Json::array();
    for (const auto& l : list.elements()) {
      int64_t g = l["gpu"].as_int();
      Json d = Json::object();
      d["index"] = g;
      d["uuid"] = l["uuid"];
      d["bdf"] = l["bdf"];
      d["kfdNode"] = l["node_id"];
      d["kfdId"] = l["kfd_id"];
      const Json& s = sm[g];
      std::string serial = s.path("asic.asic_serial").as_string();
      if (serial.rfind("0x", 0) == 0 || serial.rfind("0X", 0) == 0) serial = serial.substr(2);
      if (!serial.empty()) d["hipUUID"] = "GPU-" + to_lower(serial);
      d["asic"]["marketName"] = s.path("asic.market_name");
      d["asic"]["deviceId"] = s.path("asic.device_id");
      d["asic"]["gfx"] = s.path("asic.target_graphics_version");
      d["asic"]["computeUnits"] = s.path("asic.num_compute_units");
      d["asic"]["serial"] = s.path("asic.asic_serial");
      Json vram_mb = val_unit(s.path("vram.size"));
      if (vram_mb.is_number()) d["memTotalBytes"] = vram_mb.as_int() * 1024LL * 1024LL;
      d["numa"] = s.path("numa.node");
      const Json& m = mm[g];
      d["ecc"]["correctable"] = m.path("ecc.total_correctable_count").as_int(0);
      d["ecc"]["uncorrectable"] = m.path("ecc.total_uncorrectable_count").as_int(0);
      d["ecc"]["deferred"] = m.path("ecc.total_deferred_count").as_int(0);
      Json temps = Json::object();
      struct S {
        const char* ours;
        const char* cli;
        const char* slow;
        const char* shut;
      } sensors[] = {{"edge", "edge", "slowdown_edge_temperature", "shutdown_edge_temperature"},
                     {"hotspot", "hotspot", "slowdown_hotspot_temperature", "shutdown_hotspot_temperature"},
                     {"vram", "mem", "slowdown_vram_temperature", "shutdown_vram_temperature"}};
      for (const auto& sn : sensors) {
        Json cur = val_unit(m["temperature"][sn.cli]);
        if (!cur.is_number()) continue;
        Json t = Json::object();
        t["current"] = cur;
        Json crit = val_unit(s["limit"][sn.slow]);
        Json emer = val_unit(s["limit"][sn.shut]);
        if (crit.is_number()) t["critical"] = crit;
        if (emer.is_number()) t["emergency"] = emer;
        temps[sn.ours] = t;
      }
      d["temps"] = temps;
      Json sock = val_unit(m.path("power.socket_power"));
      if (sock.is_number()) d["power"]["socketW"] = sock;
      Json lk = links[g]["link_status"];
      if (lk.is_array()) {
        d["xgmi"]["links"] = lk;
        int up, down;
        count_links(lk, &up, &down);
        d["xgmi"]["up"] = up;
        d["xgmi"]["down"] = down;
      }
      const Json& p = parts[g];
      if (p.is_object()) {
        d["partition"]["compute"] = p["accelerator_type"];
        d["partition"]["memory"] = p["memory"];
      }
      d["present"] = true;
      devs.push_back(d);
    }
    Json out = Json::object();
    out["backend"] = "cli";
    out["node"] = node_;
    out["devices"] = devs;
    return out;
  }

 private:
  std::string bin_, dir_, node_;
};

}  // namespace

std::unique_ptr<Backend> make_cli_backend(const Json& cfg) { return std::make_unique<CliBackend>(cfg); }

}  // namespace mi355x

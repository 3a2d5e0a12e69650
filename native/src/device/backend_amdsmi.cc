// amdsmi backend: libamd_smi.so, dlopen'ed so libmi355x_dev still loads (fake/cli backends) on
// hosts without ROCm. Static identity (uuid, bdf, render node, kfd node, asic, topology) is read
// once at open; dynamic telemetry (ECC, xGMI link state, temperatures, power, activity,
// partition) on every snapshot. API references: /opt/rocm/include/amd_smi/amdsmi.h
// (amdsmi_init :2440, ..._xgmi_link_status :5501, ..._total_ecc_count :4851,
// amdsmi_get_temp_metric :6386, ..._compute_partition :5768, ..._memory_partition :5844).
#include <amd_smi/amdsmi.h>
#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "model.h"

namespace mi355x {

namespace {

struct Api {
  void* lib = nullptr;
#define AMDSMI_FN(name) decltype(&::name) name = nullptr
  AMDSMI_FN(amdsmi_init);
  AMDSMI_FN(amdsmi_shut_down);
  AMDSMI_FN(amdsmi_get_socket_handles);
  AMDSMI_FN(amdsmi_get_processor_handles);
  AMDSMI_FN(amdsmi_get_processor_type);
  AMDSMI_FN(amdsmi_get_gpu_device_bdf);
  AMDSMI_FN(amdsmi_get_gpu_device_uuid);
  AMDSMI_FN(amdsmi_get_gpu_enumeration_info);
  AMDSMI_FN(amdsmi_get_gpu_memory_total);
  AMDSMI_FN(amdsmi_get_gpu_total_ecc_count);
  AMDSMI_FN(amdsmi_get_gpu_xgmi_link_status);
  AMDSMI_FN(amdsmi_topo_get_link_weight);
  AMDSMI_FN(amdsmi_topo_get_link_type);
  AMDSMI_FN(amdsmi_topo_get_numa_node_number);
  AMDSMI_FN(amdsmi_get_gpu_compute_partition);
  AMDSMI_FN(amdsmi_get_gpu_memory_partition);
  AMDSMI_FN(amdsmi_get_gpu_asic_info);
  AMDSMI_FN(amdsmi_get_gpu_kfd_info);
  AMDSMI_FN(amdsmi_get_temp_metric);
  AMDSMI_FN(amdsmi_get_gpu_activity);
  AMDSMI_FN(amdsmi_get_power_info);
  // optional: bound when present, features degrade to "unsupported" otherwise
  AMDSMI_FN(amdsmi_get_gpu_bad_page_info);
  AMDSMI_FN(amdsmi_get_gpu_ecc_count);
  AMDSMI_FN(amdsmi_get_gpu_memory_usage);
  AMDSMI_FN(amdsmi_get_gpu_process_list);
  AMDSMI_FN(amdsmi_init_gpu_event_notification);
  AMDSMI_FN(amdsmi_set_gpu_event_notification_mask);
  AMDSMI_FN(amdsmi_get_gpu_event_notification);
  AMDSMI_FN(amdsmi_stop_gpu_event_notification);
#undef AMDSMI_FN
};

template <class F>
void bind(void* lib, F& fn, const char* name) {
  fn = reinterpret_cast<F>(dlsym(lib, name));
  if (!fn) throw std::runtime_error(std::string("libamd_smi missing symbol ") + name);
}

template <class F>
void bind_optional(void* lib, F& fn, const char* name) {
  fn = reinterpret_cast<F>(dlsym(lib, name));
}

const char* event_name(amdsmi_evt_notification_type_t t) {
  switch (t) {
    case AMDSMI_EVT_NOTIF_VMFAULT: return "VMFault";
    case AMDSMI_EVT_NOTIF_THERMAL_THROTTLE: return "ThermalThrottle";
    case AMDSMI_EVT_NOTIF_GPU_PRE_RESET: return "GPUPreReset";
    case AMDSMI_EVT_NOTIF_GPU_POST_RESET: return "GPUPostReset";
    default: return "Other";
  }
}

std::string bdf_str(const amdsmi_bdf_t& b) {
  char buf[32];
  std::snprintf(buf, sizeof buf, "%04llx:%02llx:%02llx.%llx",
                static_cast<unsigned long long>(b.domain_number), static_cast<unsigned long long>(b.bus_number),
                static_cast<unsigned long long>(b.device_number), static_cast<unsigned long long>(b.function_number));
  return buf;
}

class AmdSmiBackend : public Backend {
 public:
  explicit AmdSmiBackend(const Json& cfg) {
    std::string path = cfg["libamd_smi"].str_or("");
    const char* candidates[] = {"libamd_smi.so.26", "libamd_smi.so", "/opt/rocm/lib/libamd_smi.so"};
    if (!path.empty()) api_.lib = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    for (const char* c : candidates) {
      if (api_.lib) break;
      api_.lib = dlopen(c, RTLD_NOW | RTLD_LOCAL);
    }
    if (!api_.lib) throw std::runtime_error(std::string("dlopen libamd_smi failed: ") + dlerror());
    bind(api_.lib, api_.amdsmi_init, "amdsmi_init");
    bind(api_.lib, api_.amdsmi_shut_down, "amdsmi_shut_down");
    bind(api_.lib, api_.amdsmi_get_socket_handles, "amdsmi_get_socket_handles");
    bind(api_.lib, api_.amdsmi_get_processor_handles, "amdsmi_get_processor_handles");
    bind(api_.lib, api_.amdsmi_get_processor_type, "amdsmi_get_processor_type");
    bind(api_.lib, api_.amdsmi_get_gpu_device_bdf, "amdsmi_get_gpu_device_bdf");
    bind(api_.lib, api_.amdsmi_get_gpu_device_uuid, "amdsmi_get_gpu_device_uuid");
    bind(api_.lib, api_.amdsmi_get_gpu_enumeration_info, "amdsmi_get_gpu_enumeration_info");
    bind(api_.lib, api_.amdsmi_get_gpu_memory_total, "amdsmi_get_gpu_memory_total");
    bind(api_.lib, api_.amdsmi_get_gpu_total_ecc_count, "amdsmi_get_gpu_total_ecc_count");
    bind(api_.lib, api_.amdsmi_get_gpu_xgmi_link_status, "amdsmi_get_gpu_xgmi_link_status");
    bind(api_.lib, api_.amdsmi_topo_get_link_weight, "amdsmi_topo_get_link_weight");
    bind(api_.lib, api_.amdsmi_topo_get_link_type, "amdsmi_topo_get_link_type");
    bind(api_.lib, api_.amdsmi_topo_get_numa_node_number, "amdsmi_topo_get_numa_node_number");
    bind(api_.lib, api_.amdsmi_get_gpu_compute_partition, "amdsmi_get_gpu_compute_partition");
    bind(api_.lib, api_.amdsmi_get_gpu_memory_partition, "amdsmi_get_gpu_memory_partition");
    bind(api_.lib, api_.amdsmi_get_gpu_asic_info, "amdsmi_get_gpu_asic_info");
    bind(api_.lib, api_.amdsmi_get_gpu_kfd_info, "amdsmi_get_gpu_kfd_info");
    bind(api_.lib, api_.amdsmi_get_temp_metric, "amdsmi_get_temp_metric");
    bind(api_.lib, api_.amdsmi_get_gpu_activity, "amdsmi_get_gpu_activity");
    bind(api_.lib, api_.amdsmi_get_power_info, "amdsmi_get_power_info");
    bind_optional(api_.lib, api_.amdsmi_get_gpu_bad_page_info, "amdsmi_get_gpu_bad_page_info");
    bind_optional(api_.lib, api_.amdsmi_get_gpu_ecc_count, "amdsmi_get_gpu_ecc_count");
    bind_optional(api_.lib, api_.amdsmi_get_gpu_memory_usage, "amdsmi_get_gpu_memory_usage");
    bind_optional(api_.lib, api_.amdsmi_get_gpu_process_list, "amdsmi_get_gpu_process_list");
    bind_optional(api_.lib, api_.amdsmi_init_gpu_event_notification, "amdsmi_init_gpu_event_notification");
    bind_optional(api_.lib, api_.amdsmi_set_gpu_event_notification_mask, "amdsmi_set_gpu_event_notification_mask");
    bind_optional(api_.lib, api_.amdsmi_get_gpu_event_notification, "amdsmi_get_gpu_event_notification");
    bind_optional(api_.lib, api_.amdsmi_stop_gpu_event_notification, "amdsmi_stop_gpu_event_notification");

    amdsmi_status_t st = api_.amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_init failed: status " + std::to_string(st));
    inited_ = true;
    uint32_t nsock = 0;
    if (api_.amdsmi_get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS)
      throw std::runtime_error("amdsmi_get_socket_handles failed");
    std::vector<amdsmi_socket_handle> socks(nsock);
    api_.amdsmi_get_socket_handles(&nsock, socks.data());
    for (auto s : socks) {
      uint32_t np = 0;
      if (api_.amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ps(np);
      api_.amdsmi_get_processor_handles(s, &np, ps.data());
      for (auto p : ps) {
        processor_type_t t;
        if (api_.amdsmi_get_processor_type(p, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          handles_.push_back(p);
      }
    }
    if (handles_.empty()) throw std::runtime_error("amdsmi: no AMD GPUs found");
    node_ = cfg["node"].as_string();
    read_static_();
    if (cfg["events"].as_bool(true)) init_events_();
  }

  ~AmdSmiBackend() override {
    for (auto h : evt_handles_) api_.amdsmi_stop_gpu_event_notification(h);
    if (inited_) api_.amdsmi_shut_down();
    // libamd_smi is left loaded: unloading it while its threads wind down is not safe.
  }

  std::string name() const override { return "amdsmi"; }

  Json health_snapshot() override {
    std::lock_guard<std::mutex> g(mu_);
    Json s = Json::object();
    s["backend"] = "amdsmi";
    s["node"] = node_;
    Json devs = Json::array();
    for (size_t i = 0; i < handles_.size(); ++i) {
      Json d = Json::object();
      d["index"] = static_[i]["index"];
      d["uuid"] = static_[i]["uuid"];
      read_health_(i, d, /*limits=*/false);
      d["present"] = true;
      devs.push_back(d);
    }
    s["devices"] = devs;
    return s;
  }

  Json snapshot() override {
    std::lock_guard<std::mutex> g(mu_);
    Json s = Json::object();
    s["backend"] = "amdsmi";
    s["node"] = node_;
    Json devs = Json::array();
    for (size_t i = 0; i < handles_.size(); ++i) {
      Json d = static_[i];
      auto h = handles_[i];
      read_health_(i, d, /*limits=*/true);
      amdsmi_power_info_t pw{};
      if (api_.amdsmi_get_power_info(h, &pw) == AMDSMI_STATUS_SUCCESS) {
        d["power"]["socketW"] = static_cast<long long>(pw.current_socket_power ? pw.current_socket_power : pw.socket_power);
        d["power"]["limitW"] = static_cast<long long>(pw.power_limit > 100000 ? pw.power_limit / 1000000 : pw.power_limit);
      }
      amdsmi_engine_usage_t eu{};
      if (api_.amdsmi_get_gpu_activity(h, &eu) == AMDSMI_STATUS_SUCCESS) {
        d["activity"]["gfx"] = static_cast<long long>(eu.gfx_activity);
        d["activity"]["umc"] = static_cast<long long>(eu.umc_activity);
      }
      uint64_t used = 0;
      if (api_.amdsmi_get_gpu_memory_usage &&
          api_.amdsmi_get_gpu_memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &used) == AMDSMI_STATUS_SUCCESS)
        d["memUsedBytes"] = static_cast<long long>(used);
      d["ras"] = bad_pages_(h);
      d["processes"] = processes_(h);
      char buf[64] = {0};
      if (api_.amdsmi_get_gpu_compute_partition(h, buf, sizeof buf) == AMDSMI_STATUS_SUCCESS) d["partition"]["compute"] = std::string(buf);
      char mbuf[64] = {0};
      if (api_.amdsmi_get_gpu_memory_partition(h, mbuf, sizeof mbuf) == AMDSMI_STATUS_SUCCESS) d["partition"]["memory"] = std::string(mbuf);
      d["present"] = true;
      devs.push_back(d);
    }
    s["devices"] = devs;
    s["topology"] = topology_;
    return s;
  }

 private:
  // Processes holding this GPU (amdsmi_get_gpu_process_list, KFD's per-process accounting):
  // pid, VRAM, cumulative gfx-engine time, CUs occupied — what the agent attributes to pods.
  Json processes_(amdsmi_processor_handle h) {
    Json out = Json::array();
    if (!api_.amdsmi_get_gpu_process_list) return out;
    uint32_t n = 64;
    std::vector<amdsmi_proc_info_t> list(n);
    amdsmi_status_t st = api_.amdsmi_get_gpu_process_list(h, &n, list.data());
    if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return out;
    for (uint32_t i = 0; i < std::min<uint32_t>(n, 64); ++i) {
      const amdsmi_proc_info_t& p = list[i];
      Json j = Json::object();
      j["pid"] = static_cast<long long>(p.pid);
      j["name"] = std::string(p.name, strnlen(p.name, sizeof p.name));
      j["vramBytes"] = static_cast<long long>(p.memory_usage.vram_mem);
      j["memBytes"] = static_cast<long long>(p.mem);
      j["gfxNs"] = static_cast<long long>(p.engine_usage.gfx);
      j["cuOccupancy"] = static_cast<long long>(p.cu_occupancy);
      out.push_back(j);
    }
    return out;
  }

  void read_static_() {
    size_t n = handles_.size();
    Json weights = Json::array(), types = Json::array();
    for (size_t i = 0; i < n; ++i) {
      auto h = handles_[i];
      Json d = Json::object();
      d["index"] = static_cast<long long>(i);
      char uuid[AMDSMI_GPU_UUID_SIZE + 2] = {0};
      unsigned int ulen = sizeof uuid;
      if (api_.amdsmi_get_gpu_device_uuid(h, &ulen, uuid) == AMDSMI_STATUS_SUCCESS) d["uuid"] = std::string(uuid);
      amdsmi_bdf_t bdf{};
      if (api_.amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) d["bdf"] = bdf_str(bdf);
      amdsmi_enumeration_info_t en{};
      if (api_.amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
        d["hipUUID"] = std::string(en.hip_uuid);
        d["renderMinor"] = static_cast<long long>(en.drm_render);
        d["renderNode"] = "/dev/dri/renderD" + std::to_string(en.drm_render);
        d["cardIndex"] = static_cast<long long>(en.drm_card);
        d["kfdNode"] = static_cast<long long>(en.hsa_id);
        d["hipId"] = static_cast<long long>(en.hip_id);
      }
      amdsmi_kfd_info_t kfd{};
      if (api_.amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS) d["kfdId"] = static_cast<long long>(kfd.kfd_id);
      amdsmi_asic_info_t asic{};
      if (api_.amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS) {
        d["asic"]["marketName"] = std::string(asic.market_name);
        char id[32];
        std::snprintf(id, sizeof id, "0x%llx", static_cast<unsigned long long>(asic.device_id));
        d["asic"]["deviceId"] = std::string(id);
        d["asic"]["serial"] = std::string(asic.asic_serial);
        d["asic"]["computeUnits"] = static_cast<long long>(asic.num_of_compute_units);
        d["asic"]["oamId"] = static_cast<long long>(asic.oam_id);
        unsigned long long gv = asic.target_graphics_version;
        char gfx[32];
        std::snprintf(gfx, sizeof gfx, "gfx%llx", gv);
        d["asic"]["gfx"] = std::string(gfx);
      }
      uint64_t mem = 0;
      if (api_.amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &mem) == AMDSMI_STATUS_SUCCESS)
        d["memTotalBytes"] = static_cast<long long>(mem);
      uint32_t numa = 0;
      if (api_.amdsmi_topo_get_numa_node_number(h, &numa) == AMDSMI_STATUS_SUCCESS) d["numa"] = static_cast<long long>(numa);
      static_.push_back(d);
      limits_.push_back(Json::object());
      Json wrow = Json::array(), trow = Json::array();
      for (size_t j = 0; j < n; ++j) {
        if (i == j) {
          wrow.push_back(0);
          trow.push_back("SELF");
          continue;
        }
        uint64_t w = 0, hops = 0;
        amdsmi_link_type_t lt{};
        wrow.push_back(api_.amdsmi_topo_get_link_weight(h, handles_[j], &w) == AMDSMI_STATUS_SUCCESS ? Json(static_cast<long long>(w)) : Json());
        if (api_.amdsmi_topo_get_link_type(h, handles_[j], &hops, &lt) == AMDSMI_STATUS_SUCCESS) {
          trow.push_back(lt == AMDSMI_LINK_TYPE_XGMI ? "XGMI" : lt == AMDSMI_LINK_TYPE_PCIE ? "PCIE" : "OTHER");
        } else {
          trow.push_back(Json());
        }
      }
      weights.push_back(wrow);
      types.push_back(trow);
    }
    topology_ = Json::object();
    topology_["weights"] = weights;
    topology_["types"] = types;
  }

  // ECC counts, xGMI link state and temperatures of device i into d. Temperature limits are read
  // with the full snapshot only (they are static); the health poll reads current values.
  //
  // Measured on MI355X (profiles/r2m_amdsmi_call_costs_real.json): the all-blocks ECC total costs
  // ~0.5-0.7 ms per GPU, the UMC (HBM) block alone ~60 us, xGMI link status ~130 us, a temperature
  // ~10 us. The full sample reads both ECC forms; the 10 Hz health poll reads only the UMC count
  // ("eccUmc", checked as its own delta), so HBM errors are seen within the poll period and errors
  // of the other blocks within the sample period.
  void read_health_(size_t i, Json& d, bool limits) {
    auto h = handles_[i];
    amdsmi_error_count_t ec{};
    if (limits && api_.amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
      d["ecc"]["correctable"] = static_cast<long long>(ec.correctable_count);
      d["ecc"]["uncorrectable"] = static_cast<long long>(ec.uncorrectable_count);
      d["ecc"]["deferred"] = static_cast<long long>(ec.deferred_count);
    }
    amdsmi_error_count_t um{};
    if (api_.amdsmi_get_gpu_ecc_count && api_.amdsmi_get_gpu_ecc_count(h, AMDSMI_GPU_BLOCK_UMC, &um) == AMDSMI_STATUS_SUCCESS) {
      d["eccUmc"]["correctable"] = static_cast<long long>(um.correctable_count);
      d["eccUmc"]["uncorrectable"] = static_cast<long long>(um.uncorrectable_count);
      d["eccUmc"]["deferred"] = static_cast<long long>(um.deferred_count);
    }
    amdsmi_xgmi_link_status_t ls{};
    if (api_.amdsmi_get_gpu_xgmi_link_status(h, &ls) == AMDSMI_STATUS_SUCCESS) {
      Json links = Json::array();
      for (uint32_t l = 0; l < ls.total_links && l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
        links.push_back(ls.status[l] == AMDSMI_XGMI_LINK_UP ? "U" : ls.status[l] == AMDSMI_XGMI_LINK_DOWN ? "D" : "X");
      }
      d["xgmi"]["links"] = links;
      int up, down;
      count_links(links, &up, &down);
      d["xgmi"]["up"] = up;
      d["xgmi"]["down"] = down;
    }
    struct Sensor {
      const char* name;
      amdsmi_temperature_type_t t;
    } sensors[] = {{"edge", AMDSMI_TEMPERATURE_TYPE_EDGE},
                   {"hotspot", AMDSMI_TEMPERATURE_TYPE_HOTSPOT},
                   {"vram", AMDSMI_TEMPERATURE_TYPE_VRAM}};
    Json temps = Json::object();
    for (const auto& sn : sensors) {
      int64_t cur = 0, crit = 0, emer = 0;
      if (!limits && !limits_[i].contains(sn.name)) continue;  // unsupported sensor (edge on MI355X)
      if (api_.amdsmi_get_temp_metric(h, sn.t, AMDSMI_TEMP_CURRENT, &cur) != AMDSMI_STATUS_SUCCESS) continue;
      Json t = Json::object();
      t["current"] = static_cast<long long>(cur);
      if (limits) {
        if (api_.amdsmi_get_temp_metric(h, sn.t, AMDSMI_TEMP_CRITICAL, &crit) == AMDSMI_STATUS_SUCCESS)
          t["critical"] = static_cast<long long>(crit);
        if (api_.amdsmi_get_temp_metric(h, sn.t, AMDSMI_TEMP_EMERGENCY, &emer) == AMDSMI_STATUS_SUCCESS)
          t["emergency"] = static_cast<long long>(emer);
        limits_[i][sn.name] = t;
      } else if (limits_[i][sn.name].is_object()) {
        t["critical"] = limits_[i][sn.name]["critical"];
        t["emergency"] = limits_[i][sn.name]["emergency"];
      }
      temps[sn.name] = t;
    }
    d["temps"] = temps;
  }

  // amdsmi_get_gpu_bad_page_info: {badPagesSupported, retiredPages, pendingPages, unreservablePages}
  Json bad_pages_(amdsmi_processor_handle h) {
    Json r = Json::object();
    uint32_t n = 0;
    if (!api_.amdsmi_get_gpu_bad_page_info || api_.amdsmi_get_gpu_bad_page_info(h, &n, nullptr) != AMDSMI_STATUS_SUCCESS) {
      r["badPagesSupported"] = false;
      return r;
    }
    long long retired = 0, pending = 0, unres = 0;
    if (n > 0) {
      std::vector<amdsmi_retired_page_record_t> recs(n);
      uint32_t m = n;
      if (api_.amdsmi_get_gpu_bad_page_info(h, &m, recs.data()) == AMDSMI_STATUS_SUCCESS) {
        for (uint32_t i = 0; i < m && i < n; ++i) {
          if (recs[i].status == AMDSMI_MEM_PAGE_STATUS_RESERVED) ++retired;
          else if (recs[i].status == AMDSMI_MEM_PAGE_STATUS_PENDING) ++pending;
          else ++unres;
        }
      } else {
        retired = n;
      }
    }
    r["badPagesSupported"] = true;
    r["retiredPages"] = retired;
    r["pendingPages"] = pending;
    r["unreservablePages"] = unres;
    return r;
  }

  void init_events_() {
    if (!api_.amdsmi_init_gpu_event_notification || !api_.amdsmi_set_gpu_event_notification_mask ||
        !api_.amdsmi_get_gpu_event_notification || !api_.amdsmi_stop_gpu_event_notification)
      return;
    const uint64_t mask = AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_THERMAL_THROTTLE) |
                          AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_PRE_RESET) |
                          AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_POST_RESET) |
                          AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_VMFAULT);
    for (auto h : handles_) {
      if (api_.amdsmi_init_gpu_event_notification(h) != AMDSMI_STATUS_SUCCESS) {
        evt_error_ = "amdsmi_init_gpu_event_notification failed";
        continue;
      }
      if (api_.amdsmi_set_gpu_event_notification_mask(h, mask) != AMDSMI_STATUS_SUCCESS) {
        api_.amdsmi_stop_gpu_event_notification(h);
        evt_error_ = "amdsmi_set_gpu_event_notification_mask failed";
        continue;
      }
      evt_handles_.push_back(h);
    }
  }

 public:
  Json wait_events(int timeout_ms) override {
    Json out = Json::object();
    Json evs = Json::array();
    out["supported"] = !evt_handles_.empty();
    if (evt_handles_.empty()) {
      if (!evt_error_.empty()) out["error"] = evt_error_;
      out["events"] = evs;
      return out;
    }
    amdsmi_evt_notification_data_t data[16];
    uint32_t n = 16;
    // not under mu_: this blocks for up to timeout_ms while snapshots continue
    amdsmi_status_t st = api_.amdsmi_get_gpu_event_notification(timeout_ms, &n, data);
    if (st == AMDSMI_STATUS_SUCCESS) {
      for (uint32_t i = 0; i < n && i < 16; ++i) {
        Json e = Json::object();
        long long idx = -1;
        for (size_t k = 0; k < handles_.size(); ++k)
          if (handles_[k] == data[i].processor_handle) idx = static_cast<long long>(k);
        e["index"] = idx;
        e["type"] = event_name(data[i].event);
        e["message"] = std::string(data[i].message);
        evs.push_back(e);
      }
    } else if (st != AMDSMI_STATUS_NO_DATA && st != AMDSMI_STATUS_TIMEOUT) {
      out["status"] = static_cast<long long>(st);
    }
    out["events"] = evs;
    return out;
  }

 private:
  Api api_;
  std::vector<amdsmi_processor_handle> evt_handles_;
  std::string evt_error_;
  bool inited_ = false;
  std::vector<amdsmi_processor_handle> handles_;
  std::vector<Json> static_;
  std::vector<Json> limits_;  // per device: sensor -> {critical, emergency}
  Json topology_;
  std::string node_;
  std::mutex mu_;
};

}  // namespace

std::unique_ptr<Backend> make_amdsmi_backend(const Json& cfg) { return std::make_unique<AmdSmiBackend>(cfg); }

}  // namespace mi355x

#include "model.h"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <limits>
#include <set>
#include <tuple>

namespace mi355x {

Json Backend::wait_events(int /*timeout_ms*/) {
  Json out = Json::object();
  out["supported"] = false;
  out["events"] = Json::array();
  return out;
}

void deep_merge(Json& dst, const Json& src) {
  if (!src.is_object() || !dst.is_object()) {
    dst = src;
    return;
  }
  for (const auto& kv : src.members()) {
    if (kv.second.is_object() && dst[kv.first].is_object()) {
      deep_merge(dst[kv.first], kv.second);
    } else {
      dst[kv.first] = kv.second;
    }
  }
}

void apply_overlay(Json& snapshot, const Json& overlay) {
  const Json& faults = overlay["devices"];
  if (!faults.is_object()) return;
  auto& devs = snapshot["devices"].elements();
  for (const auto& kv : faults.members()) {
    for (auto& d : devs) {
      bool match = d["uuid"].as_string() == kv.first || d["hipUUID"].as_string() == kv.first ||
                   std::to_string(d["index"].as_int(-1)) == kv.first;
      if (!match) continue;
      deep_merge(d, kv.second);
      d["faultInjected"] = true;
    }
  }
}

void count_links(const Json& links, int* up, int* down) {
  *up = *down = 0;
  for (const auto& l : links.elements()) {
    const std::string& s = l.as_string();
    if (s == "U" || s == "UP" || s == "Up") ++*up;
    else if (s == "D" || s == "DOWN" || s == "Down") ++*down;
  }
}

static std::string fmt(const char* f, long long a, long long b = 0) {
  char buf[160];
  std::snprintf(buf, sizeof buf, f, a, b);
  return buf;
}

Json evaluate(const Json& dev, const Json& baseline, const Json& policy) {
  Json v = Json::object();
  Json reasons = Json::array();
  bool present = dev["present"].as_bool(true);
  const Json& health = policy["health"].is_object() ? policy["health"] : policy;

  // ---- xGMI links (amdsmi_get_gpu_xgmi_link_status: U/D/X per link)
  bool xgmi_ok = true;
  const Json& links = dev.path("xgmi.links");
  bool require_all = health["requireAllXGMILinks"].as_bool(true);
  int64_t min_up = health["minXGMILinksUp"].as_int(7);
  if (!links.is_array()) {
    if (require_all || min_up > 0) {
      xgmi_ok = false;
      reasons.push_back("XGMIStatusUnavailable: no xGMI link status reported");
    }
  } else {
    int up, down;
    count_links(links, &up, &down);
    if (require_all && down > 0) {
      xgmi_ok = false;
      reasons.push_back(fmt("XGMILinkDown: %lld link(s) down, %lld up", down, up));
    }
    if (up < min_up) {
      xgmi_ok = false;
      reasons.push_back(fmt("XGMILinksBelowMinimum: %lld up < %lld required", up, min_up));
    }
  }

  // ---- HBM ECC: deltas since the claim-time baseline (historic counts are not new faults)
  bool ecc_ok = true;
  int64_t unc = dev.path("ecc.uncorrectable").as_int(0);
  int64_t cor = dev.path("ecc.correctable").as_int(0);
  int64_t unc0 = baseline.path("ecc.uncorrectable").as_int(unc);
  int64_t cor0 = baseline.path("ecc.correctable").as_int(cor);
  int64_t d_unc = unc - unc0, d_cor = cor - cor0;
  if (d_unc > health["maxUncorrectableECC"].as_int(0)) {
    ecc_ok = false;
    reasons.push_back(fmt("HBMUncorrectableECC: +%lld uncorrectable since claim (max %lld)", d_unc,
                          health["maxUncorrectableECC"].as_int(0)));
  }
  // the UMC (HBM) block's own count, read by the fast health poll; checked as its own delta so a
  // poll-only reading never mixes with the all-blocks total
  const Json& umc = dev["eccUmc"];
  if (ecc_ok && umc.is_object()) {
    int64_t u = umc["uncorrectable"].as_int(0);
    int64_t d_umc = u - baseline.path("eccUmc.uncorrectable").as_int(u);
    if (d_umc > health["maxUncorrectableECC"].as_int(0)) {
      ecc_ok = false;
      reasons.push_back(fmt("HBMUncorrectableECC: +%lld uncorrectable in HBM (UMC) since claim (max %lld)", d_umc,
                            health["maxUncorrectableECC"].as_int(0)));
    }
  }
  if (d_cor > health["maxCorrectableECC"].as_int(100000)) {
    ecc_ok = false;
    reasons.push_back(fmt("HBMCorrectableECCExceeded: +%lld correctable since claim (max %lld)", d_cor,
                          health["maxCorrectableECC"].as_int(100000)));
  }

  // ---- HBM page retirement (amdsmi_get_gpu_bad_page_info): the driver's persistent record of HBM
  // pages retired after uncorrectable errors. Absolute, not a delta: it is what makes a GPU with a
  // failing HBM stack unclaimable even when no new error happens while it is claimed. Pending pages
  // (marked bad, not yet retired) and pages the driver could not reserve are worse still.
  const Json& ras = dev["ras"];
  if (ras.is_object() && ras["badPagesSupported"].as_bool(true)) {
    int64_t retired = ras["retiredPages"].as_int(0), pending = ras["pendingPages"].as_int(0),
            unres = ras["unreservablePages"].as_int(0);
    int64_t max_ret = health["maxRetiredPages"].as_int(64), max_pend = health["maxPendingPages"].as_int(0);
    if (retired > max_ret) {
      ecc_ok = false;
      reasons.push_back(fmt("HBMRetiredPages: %lld HBM page(s) retired (max %lld)", retired, max_ret));
    }
    if (pending > max_pend) {
      ecc_ok = false;
      reasons.push_back(fmt("HBMPendingRetirement: %lld bad HBM page(s) awaiting retirement (max %lld)",
                            pending, max_pend));
    }
    if (unres > 0) {
      ecc_ok = false;
      reasons.push_back(fmt("HBMUnreservablePages: %lld bad HBM page(s) could not be retired", unres));
    }
  }
  // lifetime (absolute) uncorrectable count, when the pool sets a limit (unset: only the delta
  // since claim counts, since retired pages already cover historic errors)
  if (health.contains("maxLifetimeUncorrectableECC") && unc > health["maxLifetimeUncorrectableECC"].as_int(0)) {
    ecc_ok = false;
    reasons.push_back(fmt("HBMUncorrectableECCHistory: %lld uncorrectable error(s) over the device lifetime (max %lld)",
                          unc, health["maxLifetimeUncorrectableECC"].as_int(0)));
  }

  // ---- thermals against the device's own limits (AMDSMI_TEMP_CRITICAL / _EMERGENCY)
  bool thermal_ok = true;
  std::string mode = health["thermal"].str_or("belowCritical");
  int64_t margin = health["thermalMarginC"].as_int(0);
  if (mode != "ignore") {
    const char* limit_key = mode == "belowEmergency" ? "emergency" : "critical";
    for (const auto& kv : dev["temps"].members()) {
      const Json& cur = kv.second["current"];
      const Json& lim = kv.second[limit_key];
      if (!cur.is_number() || !lim.is_number()) continue;
      if (cur.as_double() + static_cast<double>(margin) >= lim.as_double()) {
        thermal_ok = false;
        char buf[160];
        std::snprintf(buf, sizeof buf, "Thermal%s: %s %.0fC >= %s %.0fC (margin %lldC)",
                      mode == "belowEmergency" ? "Emergency" : "Critical", kv.first.c_str(),
                      cur.as_double(), limit_key, lim.as_double(), static_cast<long long>(margin));
        reasons.push_back(buf);
      }
    }
  }

  // ---- partition mode (observed, never mutated)
  bool part_ok = true;
  const Json& want = policy["partition"];
  for (const char* k : {"compute", "memory"}) {
    std::string w = want[k].str_or("Any");
    std::string have = dev.path(std::string("partition.") + k).as_string();
    if (w != "Any" && !have.empty() && have != w) {
      part_ok = false;
      reasons.push_back("PartitionMismatch: " + std::string(k) + " is " + have + ", pool requires " + w);
    }
  }

  if (!present) reasons.push_back("DeviceMissing: device no longer enumerated");
  v["present"] = present;
  v["xgmiOk"] = xgmi_ok;
  v["eccOk"] = ecc_ok;
  v["thermalOk"] = thermal_ok;
  v["partitionOk"] = part_ok;
  v["healthy"] = present && xgmi_ok && ecc_ok && thermal_ok && part_ok;
  v["eccDelta"]["uncorrectable"] = d_unc;
  v["eccDelta"]["correctable"] = d_cor;
  v["reasons"] = reasons;
  return v;
}

std::vector<int> select_devices(const Json& req) {
  int64_t k = req["count"].as_int(0);
  std::vector<int> cand;
  for (const auto& c : req["candidates"].elements()) cand.push_back(static_cast<int>(c.as_int()));
  std::sort(cand.begin(), cand.end());
  cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
  if (k <= 0) return {};
  if (static_cast<int64_t>(cand.size()) < k) return {};
  std::vector<int> owned;
  for (const auto& o : req["owned"].elements()) owned.push_back(static_cast<int>(o.as_int()));
  std::string policy = req["policy"].str_or("xgmi-packed");
  if (policy == "any") return std::vector<int>(cand.begin(), cand.begin() + k);

  const Json& W = req["weights"];
  const Json& numa = req["numa"];
  auto weight = [&](int a, int b) -> int64_t {
    const Json& w = W[static_cast<size_t>(a)][static_cast<size_t>(b)];
    return w.is_number() ? w.as_int() : 1000;  // unknown link: treat as far
  };
  auto numa_of = [&](int a) -> int64_t { return numa[static_cast<size_t>(a)].as_int(0); };

  using Score = std::tuple<int64_t, int64_t, int64_t>;  // (link weight sum, #numa nodes, index sum)
  auto score = [&](const std::vector<int>& chosen) -> Score {
    std::vector<int> all = owned;
    all.insert(all.end(), chosen.begin(), chosen.end());
    int64_t ws = 0, is = 0;
    std::set<int64_t> nodes;
    for (size_t i = 0; i < all.size(); ++i) {
      nodes.insert(numa_of(all[i]));
      for (size_t j = i + 1; j < all.size(); ++j) ws += weight(all[i], all[j]);
    }
    for (int c : chosen) is += c;
    return {ws, static_cast<int64_t>(nodes.size()), is};
  };

  // Exhaustive search when small (8 GPUs choose k <= 70 subsets), greedy otherwise.
  double combos = 1;
  for (int64_t i = 0; i < k; ++i) combos = combos * static_cast<double>(cand.size() - static_cast<size_t>(i)) / static_cast<double>(i + 1);
  std::vector<int> best;
  if (combos <= 20000) {
    Score best_s{std::numeric_limits<int64_t>::max(), 0, 0};
    std::vector<int> cur;
    std::function<void(size_t)> rec = [&](size_t start) {
      if (static_cast<int64_t>(cur.size()) == k) {
        Score s = score(cur);
        if (best.empty() || s < best_s) {
          best_s = s;
          best = cur;
        }
        return;
      }
      for (size_t i = start; i < cand.size(); ++i) {
        if (cand.size() - i < static_cast<size_t>(k) - cur.size()) break;
        cur.push_back(cand[i]);
        rec(i + 1);
        cur.pop_back();
      }
    };
    rec(0);
    return best;
  }
  std::vector<int> pool = cand;
  while (static_cast<int64_t>(best.size()) < k) {
    size_t bi = 0;
    Score bs{std::numeric_limits<int64_t>::max(), 0, 0};
    for (size_t i = 0; i < pool.size(); ++i) {
      std::vector<int> trial = best;
      trial.push_back(pool[i]);
      Score s = score(trial);
      if (s < bs) {
        bs = s;
        bi = i;
      }
    }
    best.push_back(pool[bi]);
    pool.erase(pool.begin() + static_cast<long>(bi));
  }
  std::sort(best.begin(), best.end());
  return best;
}

}  // namespace mi355x

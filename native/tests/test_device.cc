// Unit tests of the device model (health evaluation, topology-aware selection, fault overlay)
// and the fake cloud provider.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <thread>

#include "mi355x/dev.h"

#include "gpupool/provider.h"
#include "model.h"
#include "testing.h"

using namespace gpupool;

namespace {
Json healthy_dev() {
  return Json::parse(R"({"index":0,"uuid":"u0","present":true,
    "xgmi":{"links":["X","U","U","U","U","U","U","U"]},
    "ecc":{"correctable":5,"uncorrectable":1},
    "temps":{"hotspot":{"current":46,"critical":100,"emergency":112},"vram":{"current":33,"critical":115,"emergency":125}},
    "partition":{"compute":"SPX","memory":"NPS1"}})");
}
Json policy() { return Json::parse(R"({"health":{},"partition":{"compute":"Any","memory":"Any"}})"); }
}  // namespace

TEST(evaluate_healthy_real_shape) {
  Json v = mi355x::evaluate(healthy_dev(), healthy_dev(), policy());
  EXPECT_TRUE(v["healthy"].as_bool());
  EXPECT_EQ(v["reasons"].size(), 0u);
}

TEST(evaluate_xgmi_down) {
  Json d = healthy_dev();
  d["xgmi"]["links"] = Json::parse(R"(["X","U","D","U","U","U","U","U"])");
  Json v = mi355x::evaluate(d, healthy_dev(), policy());
  EXPECT_TRUE(!v["healthy"].as_bool());
  EXPECT_TRUE(!v["xgmiOk"].as_bool());
  EXPECT_TRUE(v["reasons"][0].as_string().rfind("XGMILinkDown", 0) == 0);
  // A pool that tolerates a down link but needs >= 6 up is fine with 6 up.
  Json p = Json::parse(R"({"health":{"requireAllXGMILinks":false,"minXGMILinksUp":6}})");
  EXPECT_TRUE(mi355x::evaluate(d, healthy_dev(), p)["xgmiOk"].as_bool());
}

TEST(evaluate_ecc_is_delta_since_claim) {
  Json d = healthy_dev();
  // absolute uncorrectable=1 existed at claim: not a new fault
  EXPECT_TRUE(mi355x::evaluate(d, healthy_dev(), policy())["eccOk"].as_bool());
  d["ecc"]["uncorrectable"] = 3;
  Json v = mi355x::evaluate(d, healthy_dev(), policy());
  EXPECT_TRUE(!v["eccOk"].as_bool());
  EXPECT_EQ(v["eccDelta"]["uncorrectable"].as_int(), 2);
  Json p = Json::parse(R"({"health":{"maxUncorrectableECC":2}})");
  EXPECT_TRUE(mi355x::evaluate(d, healthy_dev(), p)["eccOk"].as_bool());
}

TEST(evaluate_thermal_uses_device_limits) {
  Json d = healthy_dev();
  d["temps"]["hotspot"]["current"] = 100;  // == critical
  EXPECT_TRUE(!mi355x::evaluate(d, d, policy())["thermalOk"].as_bool());
  Json p = Json::parse(R"({"health":{"thermal":"belowEmergency"}})");
  EXPECT_TRUE(mi355x::evaluate(d, d, p)["thermalOk"].as_bool());
  Json m = Json::parse(R"({"health":{"thermalMarginC":60}})");
  EXPECT_TRUE(!mi355x::evaluate(healthy_dev(), healthy_dev(), m)["thermalOk"].as_bool());
  Json ig = Json::parse(R"({"health":{"thermal":"ignore"}})");
  EXPECT_TRUE(mi355x::evaluate(d, d, ig)["thermalOk"].as_bool());
}

TEST(evaluate_partition_and_missing) {
  Json p = Json::parse(R"({"health":{},"partition":{"compute":"CPX","memory":"Any"}})");
  EXPECT_TRUE(!mi355x::evaluate(healthy_dev(), healthy_dev(), p)["partitionOk"].as_bool());
  Json d = healthy_dev();
  d["present"] = false;
  EXPECT_TRUE(!mi355x::evaluate(d, d, policy())["healthy"].as_bool());
}

TEST(select_prefers_numa_locality_and_is_all_or_nothing) {
  // 8 GPUs fully xGMI-connected (weight 15); NUMA 0 = 0..3, NUMA 1 = 4..7.
  Json req = Json::object();
  Json w = Json::array(), numa = Json::array(), cand = Json::array();
  for (int i = 0; i < 8; ++i) {
    Json row = Json::array();
    for (int j = 0; j < 8; ++j) row.push_back(i == j ? 0 : 15);
    w.push_back(row);
    numa.push_back(i < 4 ? 0 : 1);
  }
  for (int i : {1, 2, 4, 5, 6, 7}) cand.push_back(i);
  req["weights"] = w;
  req["numa"] = numa;
  req["candidates"] = cand;
  req["count"] = 3;
  auto sel = mi355x::select_devices(req);
  EXPECT_EQ(sel.size(), 3u);
  for (int s : sel) EXPECT_TRUE(s >= 4);  // only NUMA 1 has 3 free
  req["count"] = 2;
  sel = mi355x::select_devices(req);
  EXPECT_EQ(sel[0], 1);
  EXPECT_EQ(sel[1], 2);
  req["owned"] = Json::parse("[7]");  // grow next to what the pool already holds
  sel = mi355x::select_devices(req);
  EXPECT_TRUE(sel[0] >= 4 && sel[1] >= 4);
  req["count"] = 7;
  EXPECT_TRUE(mi355x::select_devices(req).empty());
}

TEST(evaluate_retired_pages_pending_and_umc_delta) {
  Json d = healthy_dev();
  d["ras"] = Json::parse(R"({"badPagesSupported":true,"retiredPages":65,"pendingPages":0,"unreservablePages":0})");
  Json v = mi355x::evaluate(d, d, policy());
  EXPECT_TRUE(!v["eccOk"].as_bool());
  EXPECT_TRUE(v["reasons"][0].as_string().rfind("HBMRetiredPages: 65", 0) == 0);
  EXPECT_TRUE(mi355x::evaluate(d, d, Json::parse(R"({"health":{"maxRetiredPages":100}})"))["healthy"].as_bool());
  d["ras"]["pendingPages"] = 1;
  v = mi355x::evaluate(d, d, Json::parse(R"({"health":{"maxRetiredPages":100}})"));
  EXPECT_TRUE(!v["healthy"].as_bool());
  EXPECT_TRUE(v["reasons"][0].as_string().rfind("HBMPendingRetirement", 0) == 0);
  // the poll's UMC count is its own delta
  Json base = healthy_dev();
  base["eccUmc"] = Json::parse(R"({"uncorrectable":2})");
  Json now = base;
  now["eccUmc"]["uncorrectable"] = 3;
  EXPECT_TRUE(!mi355x::evaluate(now, base, policy())["eccOk"].as_bool());
  EXPECT_TRUE(mi355x::evaluate(base, base, policy())["eccOk"].as_bool());
}

TEST(c_api_evaluate_batch_and_fault_watch) {
  // batched verdicts, in order, baseline defaulting to the device
  Json items = Json::array();
  Json a = Json::object();
  a["device"] = healthy_dev();
  items.push_back(a);
  Json b = Json::object();
  Json bad = healthy_dev();
  bad["ras"] = Json::parse(R"({"retiredPages":1000})");
  b["device"] = bad;
  b["policy"] = policy();
  items.push_back(b);
  char* out = mi355x_dev_evaluate_batch(items.dump().c_str());
  Json vs = Json::parse(out);
  mi355x_free(out);
  EXPECT_EQ(vs.size(), 2u);
  EXPECT_TRUE(vs[0]["healthy"].as_bool());
  EXPECT_TRUE(!vs[1]["healthy"].as_bool());
  // fault-overlay watch: a rename into place wakes the waiter
  char dir[] = "/tmp/gpdevXXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  const std::string faults = std::string(dir) + "/faults.json", fixture = std::string(dir) + "/node.json";
  {
    std::ofstream f(fixture);
    f << R"({"devices":[{"index":0,"uuid":"u0","hipUUID":"GPU-0","present":true}]})";
  }
  Json cfg = Json::object();
  cfg["fixture"] = fixture;
  cfg["faults"] = faults;
  char err[256] = {0};
  mi355x_dev* dv = mi355x_dev_open("fake", cfg.dump().c_str(), err, sizeof err);
  EXPECT_TRUE(dv != nullptr);
  char* ev = mi355x_dev_wait_events(dv, 10);
  EXPECT_TRUE(!Json::parse(ev)["supported"].as_bool(true));  // fake: no hardware event source
  mi355x_free(ev);
  char* w0 = mi355x_dev_wait_faults(dv, 20);  // arms the watch; nothing changed yet
  EXPECT_TRUE(!Json::parse(w0)["changed"].as_bool(true));
  mi355x_free(w0);
  std::thread writer([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    {
      std::ofstream f(faults + ".tmp");
      f << R"({"devices":{"0":{"ecc":{"uncorrectable":3}}}})";
    }
    std::rename((faults + ".tmp").c_str(), faults.c_str());
  });
  auto t0 = std::chrono::steady_clock::now();
  char* w = mi355x_dev_wait_faults(dv, 2000);
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  writer.join();
  EXPECT_TRUE(Json::parse(w)["changed"].as_bool());
  EXPECT_TRUE(ms < 1500);
  mi355x_free(w);
  char* snap = mi355x_dev_health_snapshot(dv);  // the overlay applies to the health poll too
  EXPECT_EQ(Json::parse(snap)["devices"][0]["ecc"]["uncorrectable"].as_int(), 3);
  mi355x_free(snap);
  mi355x_dev_close(dv);
  std::remove(faults.c_str());
  std::remove(fixture.c_str());
  rmdir(dir);
}

TEST(overlay_merges_by_uuid_and_index) {
  Json snap = Json::parse(R"({"devices":[{"index":0,"uuid":"a","ecc":{"uncorrectable":0}},{"index":1,"uuid":"b"}]})");
  Json ov = Json::parse(R"({"devices":{"a":{"ecc":{"uncorrectable":4}},"1":{"present":false}}})");
  mi355x::apply_overlay(snap, ov);
  EXPECT_EQ(snap["devices"][0]["ecc"]["uncorrectable"].as_int(), 4);
  EXPECT_TRUE(!snap["devices"][1]["present"].as_bool(true));
  EXPECT_TRUE(snap["devices"][1]["faultInjected"].as_bool());
}

TEST(cli_backend_parses_real_captures) {
  // Shapes frozen from a real MI355X (tests/fixtures/real_mi355x, gpurun M0 capture).
  const char* dir = std::getenv("GPUPOOL_REAL_FIXTURES");
  std::string d = dir ? dir : "tests/fixtures/real_mi355x";
  std::ifstream probe(d + "/amdsmi_list.json");
  if (!probe) return;  // run from repo root in CI
  Json cfg = Json::object();
  cfg["cliDir"] = d;
  auto be = mi355x::make_cli_backend(cfg);
  Json s = be->snapshot();
  EXPECT_EQ(s["devices"].size(), 1u);
  const Json& dev = s["devices"][0];
  EXPECT_EQ(dev["hipUUID"].as_string(), std::string("GPU-be288b252f0d032c"));
  EXPECT_EQ(dev["xgmi"]["up"].as_int(), 7);
  EXPECT_EQ(dev["temps"]["hotspot"]["critical"].as_int(), 100);
  EXPECT_EQ(dev["partition"]["compute"].as_string(), std::string("SPX"));
  Json v = mi355x::evaluate(dev, dev, policy());
  EXPECT_TRUE(v["healthy"].as_bool());
}

TEST(fakecloud_lifecycle_and_cleanup) {
  FakeCloudOptions o;
  o.provision = std::chrono::milliseconds(30);
  FakeCloudProvider cloud(o);
  Credentials c;
  c.values = {{"AZURE_CLIENT_ID", "1"}, {"AZURE_CLIENT_SECRET", "2"}, {"AZURE_TENANT_ID", "3"}, {"AZURE_SUBSCRIPTION_ID", "4"}};
  AzureVmPoolSpec spec;
  spec.resource_group = "rg";
  spec.vm_size = "Standard_NC4as_T4_v3";
  auto r = cloud.create(c, spec, "default-p", "p-1");
  EXPECT_EQ(r.state, std::string("Creating"));
  auto again = cloud.create(c, spec, "default-p", "p-1");  // idempotent
  EXPECT_EQ(cloud.list(c, "rg", "default-p").size(), 1u);
  (void)again;
  EXPECT_EQ(cloud.list(c, "rg", "other").size(), 0u);  // tag isolation
  std::this_thread::sleep_for(std::chrono::milliseconds(40));
  EXPECT_EQ(cloud.list(c, "rg", "default-p")[0].state, std::string("Succeeded"));
  cloud.destroy(c, "rg", "p-1");
  EXPECT_EQ(cloud.list(c, "rg", "default-p").size(), 0u);
  EXPECT_EQ(cloud.orphans(c, "rg", "default-p", "p-").size(), 0u);  // NIC + disk gone too
  Credentials bad;
  EXPECT_THROW(cloud.list(bad, "rg", "default-p"));
}

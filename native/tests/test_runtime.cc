// Unit tests: JSON DOM/parser (incl. a randomized fuzz loop), chunked decoding, work queue
// semantics, metrics, conditions, validation. Run under ASan/UBSan and TSan via `make SAN=...`.
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <set>
#include <thread>

#include "gpupool/api.h"
#include "gpupool/http.h"
#include "gpupool/json.h"
#include "gpupool/kube.h"
#include "gpupool/log.h"
#include "gpupool/metrics.h"
#include "gpupool/reconciler.h"
#include "gpupool/trace.h"
#include "gpupool/workqueue.h"
#include "gpupool/yaml.h"
#include "testing.h"

using namespace gpupool;

TEST(json_roundtrip) {
  const char* doc = R"({"a":1,"b":[true,false,null,-2.5e3,"x\"y\\z\n"],"c":{"d":{}, "e":[]},"u":"\u00e9\ud83d\ude00"})";
  Json j = Json::parse(doc);
  EXPECT_EQ(j["a"].as_int(), 1);
  EXPECT_EQ(j["b"].size(), 5u);
  EXPECT_EQ(j["b"][3].as_double(), -2500.0);
  EXPECT_EQ(j["b"][4].as_string(), std::string("x\"y\\z\n"));
  EXPECT_EQ(j["u"].as_string(), std::string("\xc3\xa9\xf0\x9f\x98\x80"));
  Json k = Json::parse(j.dump());
  EXPECT_TRUE(j == k);
  Json p = Json::parse(j.dump(2));
  EXPECT_TRUE(j == p);
  EXPECT_TRUE(j.path("c.d").is_object());
  EXPECT_TRUE(j.path("c.missing.deeper").is_null());
}

TEST(json_key_order_and_mutation) {
  Json j = Json::object();
  j["z"] = 1;
  j["a"] = 2;
  j["m"]["n"] = "x";
  EXPECT_EQ(j.dump(), std::string(R"({"z":1,"a":2,"m":{"n":"x"}})"));
  EXPECT_TRUE(j.erase("a"));
  EXPECT_EQ(j.dump(), std::string(R"({"z":1,"m":{"n":"x"}})"));
  Json arr;
  arr.push_back(1);
  arr.push_back("two");
  EXPECT_EQ(arr.dump(), std::string(R"([1,"two"])"));
  EXPECT_TRUE(Json(3) == Json(3.0));
}

TEST(json_rejects_malformed) {
  const char* bad[] = {"", "{", "[1,]", "{\"a\" 1}", "tru", "\"\\x\"", "01", "1.", "-", "\"\x01\"",
                       "{\"a\":1}}", "\"\\ud800\"", "[1 2]"};
  for (const char* b : bad) EXPECT_TRUE(!Json::try_parse(b).has_value());
  std::string deep(100000, '[');
  EXPECT_TRUE(!Json::try_parse(deep).has_value());  // depth limit, no stack overflow
}

TEST(json_fuzz_no_crash) {
  // Mutational fuzz: random byte flips of valid documents must never crash (ASan/UBSan build).
  std::mt19937 rng(12345);
  std::vector<std::string> seeds = {R"({"type":"ADDED","object":{"metadata":{"name":"p","resourceVersion":"12"}}})",
                                    R"([1,2.5,-3e-2,"a\u0041",{"x":[null,true]}])"};
  for (int it = 0; it < 20000; ++it) {
    std::string s = seeds[static_cast<size_t>(it) % seeds.size()];
    int flips = 1 + static_cast<int>(rng() % 4);
    for (int f = 0; f < flips; ++f) s[rng() % s.size()] = static_cast<char>(rng() % 256);
    if (rng() % 5 == 0) s = s.substr(0, rng() % s.size());
    auto j = Json::try_parse(s);
    if (j) (void)j->dump();
  }
}

TEST(chunked_decoder_basic_and_split) {
  std::string wire = "4\r\nWiki\r\n5;ext=1\r\npedia\r\nE\r\n in\r\n\r\nchunks.\r\n0\r\n\r\n";
  for (size_t split = 0; split <= wire.size(); ++split) {
    ChunkedDecoder d;
    std::string out;
    EXPECT_TRUE(d.feed(std::string_view(wire).substr(0, split), out));
    EXPECT_TRUE(d.feed(std::string_view(wire).substr(split), out));
    EXPECT_TRUE(d.done());
    EXPECT_EQ(out, std::string("Wikipedia in\r\n\r\nchunks."));
  }
}

TEST(chunked_decoder_rejects_garbage) {
  const char* bad[] = {"zz\r\n", "4\r\nabcdX", "\r\n", "4\rX", "ffffffffffffffffff\r\n"};
  for (const char* b : bad) {
    ChunkedDecoder d;
    std::string out;
    EXPECT_TRUE(!d.feed(b, out));
  }
  std::mt19937 rng(7);
  for (int it = 0; it < 5000; ++it) {  // fuzz: never crash / over-read
    std::string s(1 + rng() % 64, '\0');
    for (auto& c : s) c = "0123456789abcdef\r\n;x"[rng() % 21];
    ChunkedDecoder d;
    std::string out;
    (void)d.feed(s, out);
  }
}

TEST(url_parse) {
  Url u = Url::parse("http://127.0.0.1:6443");
  EXPECT_EQ(u.host, std::string("127.0.0.1"));
  EXPECT_EQ(u.port, 6443);
  Url x = Url::parse("unix:///tmp/agent.sock");
  EXPECT_EQ(x.unix_path, std::string("/tmp/agent.sock"));
  EXPECT_THROW(Url::parse("ftp://x"));
  Url s = Url::parse("https://kubernetes.default.svc");
  EXPECT_EQ(s.scheme, std::string("https"));
  EXPECT_EQ(s.port, 443);
}

TEST(trace_spans_ring_and_scoping) {
  trace::reset();
  trace::add_span("orphan", 1.0);  // no active trace: no-op
  EXPECT_EQ(trace::current_id(), std::string());
  std::string outer_id;
  {
    trace::Trace t("Mi355xPool/default/p");
    outer_id = t.id();
    EXPECT_EQ(trace::current_id(), outer_id);
    { trace::Span s("observe"); }
    trace::add_span("agent.claim.probe", 2.5);
    {
      trace::Trace inner("AzureVmPool/default/q");  // nested: restores the outer on close
      EXPECT_TRUE(trace::current_id() != outer_id);
    }
    EXPECT_EQ(trace::current_id(), outer_id);
    t.attr("reason", "ScalingUp");
    t.finish("requeue");
  }
  EXPECT_EQ(trace::current_id(), std::string());
  Json r = trace::recent(10);
  EXPECT_EQ(r.size(), static_cast<size_t>(2));
  const Json& last = r.elements()[0];  // newest first: the outer finished last
  EXPECT_EQ(last["reconcileID"].as_string(), outer_id);
  EXPECT_EQ(last["result"].as_string(), std::string("requeue"));
  EXPECT_EQ(last["spans"].size(), static_cast<size_t>(2));
  EXPECT_EQ(last["spans"].elements()[0]["name"].as_string(), std::string("observe"));
  EXPECT_EQ(last["spans"].elements()[1]["ms"].as_double(), 2.5);
  EXPECT_EQ(last.path("attrs.reason").as_string(), std::string("ScalingUp"));
  for (int i = 0; i < 4200; ++i) trace::Trace t("X/y/" + std::to_string(i));
  EXPECT_EQ(trace::recent(5000).size(), static_cast<size_t>(4096));
  EXPECT_EQ(url_decode("Mi355xPool%2Fdefault%2Fa+b"), std::string("Mi355xPool/default/a b"));
  trace::reset();
}

TEST(base64_decode_long_and_urlsafe) {
  EXPECT_EQ(base64_decode("aGVsbG8gd29ybGQ="), std::string("hello world"));
  EXPECT_EQ(base64_decode("aGVs\nbG8=\n"), std::string("hello"));
  std::string big(3000, '\0');
  for (size_t i = 0; i < big.size(); ++i) big[i] = static_cast<char>(i * 7);
  static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string enc;
  for (size_t i = 0; i < big.size(); i += 3) {
    uint32_t v = (static_cast<uint8_t>(big[i]) << 16) | (static_cast<uint8_t>(big[i + 1]) << 8) | static_cast<uint8_t>(big[i + 2]);
    for (int s = 18; s >= 0; s -= 6) enc.push_back(tbl[(v >> s) & 63]);
  }
  EXPECT_TRUE(base64_decode(enc) == big);  // no overflow on long inputs (UBSan build)
  EXPECT_EQ(base64_decode("-_8="), base64_decode("+/8="));
}

TEST(yaml_subset) {
  const char* doc = R"(# kubeconfig-like
apiVersion: v1
clusters:
- cluster:
    server: https://10.0.0.1:6443   # trailing comment
    insecure-skip-tls-verify: true
  name: "c1"
contexts:
- context: {cluster: c1, user: u1, namespace: team-a}
  name: ctx1
list:
  - 1
  - -2.5
  - 'it''s'
  - "a\tb \u00e9"
  - [x, "y, z", {k: v}]
  - ~
nested:
  - - a
    - b
empty_map: {}
seq_at_parent_indent:
- k: v
  k2: null
block: |
  line one
    indented
tail: end
---
ignored: second document
)";
  Json j = yaml_parse(doc);
  EXPECT_EQ(j["apiVersion"].as_string(), std::string("v1"));
  EXPECT_EQ(j["clusters"][0]["name"].as_string(), std::string("c1"));
  EXPECT_EQ(j["clusters"][0]["cluster"]["server"].as_string(), std::string("https://10.0.0.1:6443"));
  EXPECT_TRUE(j["clusters"][0]["cluster"]["insecure-skip-tls-verify"].as_bool(false));
  EXPECT_EQ(j["contexts"][0]["context"]["namespace"].as_string(), std::string("team-a"));
  EXPECT_EQ(j["list"][0].as_int(), 1);
  EXPECT_EQ(j["list"][1].as_double(), -2.5);
  EXPECT_EQ(j["list"][2].as_string(), std::string("it's"));
  EXPECT_EQ(j["list"][3].as_string(), std::string("a\tb \xc3\xa9"));
  EXPECT_EQ(j["list"][4][1].as_string(), std::string("y, z"));
  EXPECT_EQ(j["list"][4][2]["k"].as_string(), std::string("v"));
  EXPECT_TRUE(j["list"][5].is_null());
  EXPECT_EQ(j["nested"][0][1].as_string(), std::string("b"));
  EXPECT_TRUE(j["empty_map"].is_object());
  EXPECT_EQ(j["seq_at_parent_indent"][0]["k"].as_string(), std::string("v"));
  EXPECT_EQ(j["block"].as_string(), std::string("line one\n  indented\n"));
  EXPECT_EQ(j["tail"].as_string(), std::string("end"));
  EXPECT_TRUE(!j.contains("ignored"));
  EXPECT_THROW(yaml_parse("a: [1, 2"));
  EXPECT_THROW(yaml_parse("a:\n\t- 1"));
  EXPECT_THROW(yaml_parse("a: &x 1"));
  std::mt19937 rng(99);  // fuzz: malformed input must throw or parse, never crash (ASan build)
  std::string seed = doc;
  for (int it = 0; it < 3000; ++it) {
    std::string s = seed.substr(0, rng() % seed.size());
    if (s.empty()) continue;
    for (int f = 0; f < 3; ++f) s[rng() % s.size()] = "-: \n'\"[{#|"[rng() % 11];
    try {
      (void)yaml_parse(s);
    } catch (const YamlError&) {
    }
  }
}

TEST(kubeconfig_resolution) {
  char tmpl[] = "/tmp/gp-kc-XXXXXX";
  std::string dir = mkdtemp(tmpl);
  { std::ofstream(dir + "/ca.pem") << "PEM"; }
  { std::ofstream(dir + "/tok") << "file-token\n"; }
  {
    std::ofstream(dir + "/config") << R"(apiVersion: v1
kind: Config
current-context: dev
clusters:
- name: prod
  cluster:
    server: https://prod:6443
    certificate-authority-data: UEVNLURBVEE=
- name: dev
  cluster:
    server: https://127.0.0.1:7443
    certificate-authority: ca.pem
contexts:
- name: dev
  context: {cluster: dev, user: dev-user, namespace: ns1}
- name: prod
  context:
    cluster: prod
    user: prod-user
- name: broken
  context: {cluster: dev, user: exec-user}
users:
- name: dev-user
  user:
    tokenFile: tok
- name: prod-user
  user:
    token: abc
    client-certificate-data: Q0VSVA==
    client-key-data: S0VZ
- name: exec-user
  user:
    exec: {command: aws}
)";
  }
  KubeConfig d = load_kubeconfig(dir + "/config");
  EXPECT_EQ(d.context, std::string("dev"));
  EXPECT_EQ(d.server, std::string("https://127.0.0.1:7443"));
  EXPECT_EQ(d.tls.ca_file, dir + "/ca.pem");
  EXPECT_EQ(d.token, std::string("file-token"));
  EXPECT_EQ(d.ns, std::string("ns1"));
  KubeConfig p = load_kubeconfig(dir + "/config", "prod");
  EXPECT_EQ(p.tls.ca_pem, std::string("PEM-DATA"));
  EXPECT_EQ(p.tls.cert_pem, std::string("CERT"));
  EXPECT_EQ(p.tls.key_pem, std::string("KEY"));
  EXPECT_EQ(p.token, std::string("abc"));
  EXPECT_THROW(load_kubeconfig(dir + "/config", "broken"));
  EXPECT_THROW(load_kubeconfig(dir + "/config", "missing"));
  EXPECT_THROW(load_kubeconfig(dir + "/nope"));
  for (const char* f : {"/config", "/ca.pem", "/tok"}) std::remove((dir + f).c_str());
  rmdir(dir.c_str());
}

TEST(kube_in_cluster_config) {
  char tmpl[] = "/tmp/gp-sa-XXXXXX";
  std::string dir = mkdtemp(tmpl);
  { std::ofstream(dir + "/token") << "abc.def\n"; }
  { std::ofstream(dir + "/ca.crt") << "-----BEGIN CERTIFICATE-----\n"; }
  std::string server, token;
  TlsOptions tls;
  unsetenv("KUBERNETES_SERVICE_HOST");
  EXPECT_TRUE(!KubeClient::in_cluster(&server, &token, &tls, dir));
  setenv("KUBERNETES_SERVICE_HOST", "10.96.0.1", 1);
  setenv("KUBERNETES_SERVICE_PORT", "6443", 1);
  EXPECT_TRUE(KubeClient::in_cluster(&server, &token, &tls, dir));
  EXPECT_EQ(server, std::string("https://10.96.0.1:6443"));
  EXPECT_EQ(token, std::string("abc.def"));
  EXPECT_EQ(tls.ca_file, dir + "/ca.crt");
  setenv("KUBERNETES_SERVICE_HOST", "fd00::1", 1);
  EXPECT_TRUE(KubeClient::in_cluster(&server, &token, &tls, dir));
  EXPECT_EQ(server, std::string("https://[fd00::1]:6443"));
  unsetenv("KUBERNETES_SERVICE_HOST");
  unsetenv("KUBERNETES_SERVICE_PORT");
  std::remove((dir + "/token").c_str());
  std::remove((dir + "/ca.crt").c_str());
  rmdir(dir.c_str());
}

TEST(workqueue_dedup_and_processing) {
  WorkQueue q;
  q.add("a");
  q.add("a");
  q.add("b");
  EXPECT_EQ(q.len(), 2u);
  std::string k;
  EXPECT_TRUE(q.get_for(&k, std::chrono::milliseconds(10)));
  EXPECT_EQ(k, std::string("a"));
  q.add("a");  // while processing: marked dirty, not queued twice
  EXPECT_EQ(q.len(), 1u);
  q.done("a");  // re-queued now
  EXPECT_EQ(q.len(), 2u);
  // time spent ready in the queue (the reconcile trace's queueWaitMs)
  double waited = -1;
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  EXPECT_TRUE(q.get_for(&k, std::chrono::milliseconds(10), &waited));
  EXPECT_EQ(k, std::string("b"));
  EXPECT_TRUE(waited >= 15.0 && waited < 5000.0);
  q.done("b");
  q.add("c");
  EXPECT_TRUE(q.get_for(&k, std::chrono::milliseconds(10), &waited));  // "a", re-queued by done()
  EXPECT_TRUE(waited >= 15.0);
  EXPECT_TRUE(q.get_for(&k, std::chrono::milliseconds(10), &waited));
  EXPECT_EQ(k, std::string("c"));
  EXPECT_TRUE(waited >= 0.0 && waited < 15.0);
}

TEST(workqueue_delay_and_backoff) {
  WorkQueue q(std::chrono::milliseconds(5), std::chrono::milliseconds(40));
  q.add_after("x", std::chrono::milliseconds(30));
  std::string k;
  EXPECT_TRUE(!q.get_for(&k, std::chrono::milliseconds(5)));
  EXPECT_TRUE(q.get_for(&k, std::chrono::milliseconds(200)));
  EXPECT_EQ(k, std::string("x"));
  q.done("x");
  EXPECT_EQ(q.backoff_for("y").count(), 5);
  q.add_rate_limited("y");
  EXPECT_EQ(q.backoff_for("y").count(), 10);
  q.add_rate_limited("y");
  q.add_rate_limited("y");
  q.add_rate_limited("y");
  EXPECT_EQ(q.backoff_for("y").count(), 40);  // capped
  EXPECT_EQ(q.num_requeues("y"), 4);
  q.forget("y");
  EXPECT_EQ(q.num_requeues("y"), 0);
}

TEST(workqueue_concurrent_exclusive) {
  // Many producers, 4 workers: a key is never processed by two workers at once.
  WorkQueue q;
  std::atomic<int> inflight_a{0}, violations{0}, processed{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> workers;
  for (int w = 0; w < 4; ++w) {
    workers.emplace_back([&] {
      std::string k;
      while (q.get(&k)) {
        if (k == "a" && inflight_a.fetch_add(1) != 0) violations++;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (k == "a") inflight_a--;
        processed++;
        q.done(k);
      }
    });
  }
  std::vector<std::thread> producers;
  for (int p = 0; p < 4; ++p)
    producers.emplace_back([&, p] {
      for (int i = 0; i < 500; ++i) q.add(i % 3 == 0 ? "a" : "k" + std::to_string((i + p) % 17));
    });
  for (auto& t : producers) t.join();
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  q.shutdown();
  for (auto& t : workers) t.join();
  EXPECT_EQ(violations.load(), 0);
  EXPECT_TRUE(processed.load() > 0);
}

TEST(metrics_render_and_quantile) {
  Registry& r = Registry::global();
  auto& c = r.counter("test_total", "help");
  c.inc({{"k", "v"}});
  c.inc({{"k", "v"}}, 2);
  EXPECT_EQ(c.get({{"k", "v"}}), 3.0);
  auto& h = r.histogram("test_seconds", "help", {0.1, 0.2, 0.4});
  for (int i = 0; i < 10; ++i) h.observe({}, 0.15);
  EXPECT_EQ(h.count(), 10u);
  double q = h.quantile({}, 0.5);
  EXPECT_TRUE(q > 0.1 && q <= 0.2);
  std::string txt = r.render();
  EXPECT_TRUE(txt.find("test_total{k=\"v\"} 3") != std::string::npos);
  EXPECT_TRUE(txt.find("test_seconds_bucket{le=\"+Inf\"} 10") != std::string::npos);
}

TEST(conditions_transition_time_only_on_flip) {
  Json conds;
  EXPECT_TRUE(set_condition(conds, "Ready", "False", "ScalingUp", "0/1", 1, "T1"));
  EXPECT_TRUE(!set_condition(conds, "Ready", "False", "ScalingUp", "0/1", 1, "T2"));
  EXPECT_EQ(find_condition(conds, "Ready")["lastTransitionTime"].as_string(), std::string("T1"));
  EXPECT_TRUE(set_condition(conds, "Ready", "False", "Probing", "0/1", 1, "T3"));
  EXPECT_EQ(find_condition(conds, "Ready")["lastTransitionTime"].as_string(), std::string("T1"));
  EXPECT_TRUE(set_condition(conds, "Ready", "True", "AllReplicasReady", "1/1", 2, "T4"));
  EXPECT_EQ(find_condition(conds, "Ready")["lastTransitionTime"].as_string(), std::string("T4"));
  EXPECT_EQ(find_condition(conds, "Ready")["observedGeneration"].as_int(), 2);
  EXPECT_TRUE(condition_true(conds, "Ready"));
  EXPECT_EQ(conds.size(), 1u);
}

TEST(validation_matches_crd) {
  Json ok = Json::parse(R"({"kind":"Mi355xPool","spec":{"replicas":2}})");
  EXPECT_TRUE(validate_mi355x(ok).empty());
  Json neg = Json::parse(R"({"kind":"Mi355xPool","spec":{"replicas":-1}})");
  EXPECT_EQ(validate_mi355x(neg).size(), 1u);
  Json badres = Json::parse(R"({"kind":"Mi355xPool","spec":{"replicas":1,"resourceName":"BAD"}})");
  EXPECT_EQ(validate_mi355x(badres).size(), 1u);
  // the cross-field rules the CRD states in CEL (x-kubernetes-validations), checked again here
  for (const char* bad : {R"({"replicas":1,"sharing":{"replicasPerGPU":4,"cuPerSlot":128}})",
                          R"({"replicas":1,"sharing":{"replicasPerGPU":4,"cuPerSlot":4}})",
                          R"({"replicas":1,"partition":{"compute":"DPX"},"sharing":{"cuPerSlot":2}})",
                          R"({"replicas":1,"autoscale":{"minReplicas":5,"maxReplicas":2}})"}) {
    Json o = Json::parse(std::string(R"({"kind":"Mi355xPool","spec":)") + bad + "}");
    EXPECT_EQ(validate_mi355x(o).size(), 1u);
  }
  for (const char* good : {R"({"replicas":1,"sharing":{"replicasPerGPU":4,"cuPerSlot":64}})",
                           R"({"replicas":1,"partition":{"compute":"CPX"},"sharing":{"cuPerSlot":1}})",
                           R"({"replicas":1,"autoscale":{"minReplicas":2,"maxReplicas":2}})"}) {
    Json o = Json::parse(std::string(R"({"kind":"Mi355xPool","spec":)") + good + "}");
    EXPECT_TRUE(validate_mi355x(o).empty());
  }
  Json az = Json::parse(R"({"kind":"AzureVmPool","spec":{"replicas":0,"resourceGroupName":"rg","location":"eastus",
    "vmSize":"s","vnetName":"v","subnetName":"s","azureCredentialSecret":"c",
    "imageReference":{"publisher":"p","offer":"o","sku":"s","version":"v"}}})");
  EXPECT_TRUE(validate_azure(az).empty());
  az["spec"].erase("location");
  EXPECT_EQ(validate_azure(az).size(), 1u);
}

TEST(rfc3339_roundtrip) {
  auto now = std::chrono::system_clock::now();
  std::chrono::system_clock::time_point t;
  EXPECT_TRUE(parse_rfc3339(rfc3339(now), &t));
  EXPECT_TRUE(std::chrono::abs(std::chrono::duration_cast<std::chrono::seconds>(t - now)).count() <= 1);
  EXPECT_TRUE(parse_rfc3339(microtime_now(), &t));
  EXPECT_TRUE(!parse_rfc3339("garbage", &t));
}

// ---------------------------------------------------------------- Mi355xJob gang placement
TEST(job_gang_placement) {
  using gpupool::Mi355xJobReconciler;
  using F = std::vector<std::pair<std::string, int64_t>>;
  // whole gang fits one node: the tightest such node (keeps the roomy node for bigger gangs)
  auto s = Mi355xJobReconciler::place(F{{"a", 8}, {"b", 4}, {"c", 2}}, 2, 2);
  EXPECT_EQ(s.size(), 2u);
  EXPECT_TRUE(s[0].node == "b" && s[1].node == "b" && s[0].index == 0 && s[1].index == 1);
  // spans nodes: fewest nodes, roomiest first, rank 0 on the first
  s = Mi355xJobReconciler::place(F{{"a", 2}, {"b", 5}, {"c", 3}}, 4, 2);
  EXPECT_EQ(s.size(), 4u);
  EXPECT_TRUE(s[0].node == "b" && s[1].node == "b" && s[2].node == "c" && s[3].node == "a");
  // all-or-nothing: 3 x 2 GPUs do not fit 5 free GPUs split 3+1+1
  EXPECT_TRUE(Mi355xJobReconciler::place(F{{"a", 3}, {"b", 1}, {"c", 1}}, 3, 2).empty());
  EXPECT_TRUE(Mi355xJobReconciler::place(F{}, 1, 1).empty());
  // CPU-only workers go together on the first candidate
  s = Mi355xJobReconciler::place(F{{"x", 0}, {"y", 0}}, 3, 0);
  EXPECT_TRUE(s.size() == 3 && s[2].node == "x");
}

TEST(autoscale_demand) {
  auto J = [](const char* s) { return gpupool::Json::parse(s); };
  std::vector<gpupool::Json> pods = {
      J(R"({"metadata":{},"spec":{"nodeName":"n","containers":[{"resources":{"limits":{"r/g":"2"}}}]},"status":{"phase":"Running"}})"),
      J(R"({"metadata":{},"spec":{"containers":[{"resources":{"limits":{"r/g":1}}}]}})"),  // pending, unbound
      J(R"({"metadata":{},"spec":{"containers":[{"resources":{"limits":{"r/g":1}}}]},"status":{"phase":"Succeeded"}})"),
      J(R"({"metadata":{"deletionTimestamp":"x"},"spec":{"containers":[{"resources":{"limits":{"r/g":1}}}]}})"),
      J(R"({"metadata":{},"spec":{"containers":[{"resources":{"limits":{"other/g":4}}}]}})"),
  };
  std::vector<gpupool::Json> jobs = {
      // waiting gang on this pool: 2 x 2
      J(R"({"metadata":{"namespace":"ns"},"spec":{"poolRef":"p","replicas":2,"gpusPerReplica":2}})"),
      // held back by admission: adds nothing
      J(R"({"metadata":{"namespace":"ns"},"spec":{"poolRef":"p","replicas":3},"status":{"conditions":[{"type":"Scheduled","status":"False","reason":"QueueClosed"}]}})"),
      // placed, one slot not created yet (its created pod is already among the pods)
      J(R"({"metadata":{"namespace":"ns"},"spec":{"resourceName":"r/g","replicas":2},"status":{"phase":"Pending","placement":[{"index":0,"node":"n","created":true},{"index":1,"node":"n","created":false}]}})"),
      J(R"({"metadata":{"namespace":"ns"},"spec":{"poolRef":"p","replicas":4,"suspend":true}})"),
      J(R"({"metadata":{"namespace":"ns"},"spec":{"poolRef":"p","replicas":4},"status":{"phase":"Succeeded"}})"),
      J(R"({"metadata":{"namespace":"other"},"spec":{"poolRef":"p","replicas":4,"resourceName":"x/y"}})"),
  };
  EXPECT_EQ(gpupool::Mi355xPoolAutoscaler::demand(pods, jobs, "ns", "p", "r/g"), 8);  // 2 + 1 + 4 + 1
  EXPECT_EQ(gpupool::Mi355xPoolAutoscaler::demand({}, {}, "ns", "p", "r/g"), 0);
  // a gang naming another pool is not this pool's demand
  std::vector<gpupool::Json> other = {J(R"({"metadata":{"namespace":"ns"},"spec":{"poolRef":"q","resourceName":"r/g","replicas":3}})")};
  EXPECT_EQ(gpupool::Mi355xPoolAutoscaler::demand({}, other, "ns", "p", "r/g"), 0);
}

TEST(autoscale_pool_demand_attribution) {
  auto J = [](const char* s) { return gpupool::Json::parse(s); };
  auto pod = [&](int n) {
    return J((std::string(R"({"metadata":{},"spec":{"containers":[{"resources":{"limits":{"r/g":)") +
              std::to_string(n) + "}}}]}}").c_str());
  };
  auto P = [&](const char* name, bool autoscale, int replicas, int maxr) {
    return J((std::string(R"({"metadata":{"namespace":"ns","name":")") + name + R"("},"spec":{"resourceName":"r/g","replicas":)" +
              std::to_string(replicas) + R"(,"autoscale":{"enabled":)" + (autoscale ? "true" : "false") +
              R"(,"minReplicas":0,"maxReplicas":)" + std::to_string(maxr) + "}}}")
                 .c_str());
  };
  using A = gpupool::Mi355xPoolAutoscaler;
  std::vector<gpupool::Json> pods = {pod(2), pod(2), pod(2)};  // 6 GPUs
  // two autoscaled pools: split in name order up to maxReplicas (4 + 2), never 6 + 6
  std::vector<gpupool::Json> pools = {P("b", true, 0, 4), P("a", true, 0, 4)};
  EXPECT_EQ(A::pool_demand(pods, {}, pools, "ns", "a", "r/g"), 4);
  EXPECT_EQ(A::pool_demand(pods, {}, pools, "ns", "b", "r/g"), 2);
  pools = {P("b", true, 0, 4), P("a", true, 0, 2)};  // overflow goes to the last pool
  EXPECT_EQ(A::pool_demand(pods, {}, pools, "ns", "a", "r/g"), 2);
  EXPECT_EQ(A::pool_demand(pods, {}, pools, "ns", "b", "r/g"), 4);
  // a fixed pool of 4 serves shared demand first: the autoscaled pool sees only 2
  pools = {P("a", true, 0, 8), P("fixed", false, 4, 0)};
  EXPECT_EQ(A::pool_demand(pods, {}, pools, "ns", "a", "r/g"), 2);
  // its own gang counts for it regardless of the shared split
  std::vector<gpupool::Json> jobs = {J(R"({"metadata":{"namespace":"ns"},"spec":{"poolRef":"a","replicas":3}})")};
  EXPECT_EQ(A::pool_demand(pods, jobs, pools, "ns", "a", "r/g"), 5);
  // a single pool gets exactly demand()
  pools = {P("a", true, 0, 16)};
  EXPECT_EQ(A::pool_demand(pods, jobs, pools, "ns", "a", "r/g"), A::demand(pods, jobs, "ns", "a", "r/g"));
  // two autoscaled pools, pods already running on the later one ("b"): their GPUs are b's
  // demand, not the first pool's in the split (a would grow idle, b would drain them)
  auto named = [&](const char* name, int n) {
    return J((std::string(R"({"metadata":{"namespace":"ns","name":")") + name +
              R"("},"status":{"phase":"Running"},"spec":{"containers":[{"resources":{"limits":{"r/g":)" +
              std::to_string(n) + "}}}]}}").c_str());
  };
  gpupool::Json b = P("b", true, 2, 4);
  b["status"] = J(R"({"devices":[{"uuid":"u1","pods":["ns/w1"]},{"uuid":"u2","pods":["ns/w2"]}]})");
  pools = {P("a", true, 0, 4), b};
  std::vector<gpupool::Json> running = {named("w1", 1), named("w2", 1), named("new", 1)};
  EXPECT_EQ(A::pool_demand(running, {}, pools, "ns", "b", "r/g"), 2);  // its two running pods
  EXPECT_EQ(A::pool_demand(running, {}, pools, "ns", "a", "r/g"), 1);  // only the pending one
}

TEST(job_validation) {
  using gpupool::Json;
  Json ok = Json::parse(R"({"spec":{"replicas":2,"template":{"spec":{}}}})");
  EXPECT_TRUE(gpupool::validate_job(ok).empty());
  Json bad = Json::parse(
      R"({"spec":{"replicas":0,"gpusPerReplica":-1,"restartPolicy":"Always","masterPort":70000}})");
  auto errs = gpupool::validate_job(bad);
  EXPECT_EQ(errs.size(), 5u);  // replicas, gpusPerReplica, masterPort, restartPolicy, template
  // minAvailable <= replicas (the CRD's CEL rule)
  EXPECT_EQ(gpupool::validate_job(Json::parse(
      R"({"spec":{"replicas":2,"minAvailable":3,"template":{}}})")).size(), 1u);
  EXPECT_TRUE(gpupool::validate_job(Json::parse(
      R"({"spec":{"replicas":2,"minAvailable":2,"template":{}}})")).empty());
  auto spec = gpupool::Mi355xJobSpec::from(ok["spec"]);
  EXPECT_TRUE(spec.gpus_per_replica == 1 && spec.restart_policy == "OnFailure" && spec.master_port == 29500);
}

TEST(token_source_rotates_from_file) {
  const std::string path = "/tmp/gpupool_token_test_" + std::to_string(::getpid());
  { std::ofstream(path) << "first\n"; }
  auto t = gpupool::TokenSource::file(path, std::chrono::hours(1));
  EXPECT_TRUE(t->token() == "first");
  { std::ofstream(path) << "second\n"; }
  EXPECT_TRUE(t->token() == "first");  // not due yet: the cached value
  EXPECT_TRUE(t->reload());            // what a 401 triggers
  EXPECT_TRUE(t->token() == "second");
  EXPECT_TRUE(!t->reload());           // unchanged
  EXPECT_TRUE(t->reloads() == 1);
  std::remove(path.c_str());
  EXPECT_TRUE(!t->reload() && t->token() == "second");  // mid-swap: keep the last value
  auto f = gpupool::TokenSource::fixed("x");
  EXPECT_TRUE(f->token() == "x" && !f->reload());
}

// The manager's per-request Ed25519 signature on node-agent RPCs (the Python side, verifier and
// test signer: gpupool/utils/edsig.py — the same canonical bytes).
//
// No reusable secret travels to an agent endpoint: each request carries a signature over
//   "gpupool-agent-rpc-v1" \n METHOD \n target(path+query) \n node \n ts_ms \n nonce \n sha256(body)
// so what any endpoint receives is good only for that request to that node within the agents'
// clock-skew window (and agents drop a nonce they have seen). The key file is re-read when it
// changes: rotate by adding the new public key to the agents' bundle first, then swapping this
// file, then removing the old public key.
#pragma once

#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>

namespace gpupool {

// v2 (the per-node MAC, edsig.py): with the agent's X25519 public key (its Node annotation
// gpupool.amd.com/agent-kx) the request carries HMAC-SHA256(K, canonical) instead, K derived once
// per (node, agent key) from X25519(this key's Ed25519 scalar, agent key) — ~2 us per request
// for the agent to check instead of an Ed25519 verification (~0.17 ms).
class AgentSigner {
 public:
  explicit AgentSigner(std::string key_file, std::chrono::milliseconds recheck = std::chrono::seconds(5));
  // "X-Gpupool-Signature: v1 keyId=.. node=.. ts=.. nonce=.. body=.. sig=..\r\n", or with
  // ``agent_kx`` (base64url X25519 public key) "v2 keyId=.. kx=.. node=.. ... mac=..\r\n"
  std::string header(const std::string& method, const std::string& target, const std::string& node,
                     const std::string& body, const std::string& agent_kx = "");
  std::string key_id();
  uint64_t reloads() const { return reloads_.load(); }

 private:
  void load_locked_(bool force);
  std::mutex mu_;
  std::string path_;
  std::chrono::milliseconds recheck_;
  std::chrono::steady_clock::time_point checked_at_{};
  long long mtime_ns_ = -1;
  std::shared_ptr<void> key_;  // EVP_PKEY* (Ed25519)
  std::shared_ptr<void> xkey_;  // EVP_PKEY* (X25519: the same secret scalar)
  std::string xpub_;            // its public key (32 bytes)
  std::string kid_;
  static constexpr size_t kMaxMacKeys = 4096;    // ~2 keys per node on a large cluster
  std::map<std::string, std::string> mac_keys_;  // node \n agent key -> K (cleared on reload / when full)
  std::atomic<uint64_t> reloads_{0};
};

// sha256 of ``data`` as lowercase hex
std::string sha256_hex(const std::string& data);

}  // namespace gpupool

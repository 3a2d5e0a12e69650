#include "gpupool/agentauth.h"

#include <sys/stat.h>

#include <array>
#include <cstdint>
#include <cstdio>
#include <stdexcept>

#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/pem.h>
#include <openssl/rand.h>
#include <openssl/sha.h>

namespace gpupool {

namespace {

std::string hex(const unsigned char* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string out(n * 2, '0');
  for (size_t i = 0; i < n; ++i) {
    out[2 * i] = d[p[i] >> 4];
    out[2 * i + 1] = d[p[i] & 15];
  }
  return out;
}

std::string b64url(const unsigned char* p, size_t n) {
  static const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
  std::string out;
  size_t i = 0;
  for (; i + 2 < n; i += 3) {
    unsigned v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
    out += a[v >> 18];
    out += a[(v >> 12) & 63];
    out += a[(v >> 6) & 63];
    out += a[v & 63];
  }
  if (i + 1 == n) {
    unsigned v = p[i] << 16;
    out += a[v >> 18];
    out += a[(v >> 12) & 63];
  } else if (i + 2 == n) {
    unsigned v = (p[i] << 16) | (p[i + 1] << 8);
    out += a[v >> 18];
    out += a[(v >> 12) & 63];
    out += a[(v >> 6) & 63];
  }
  return out;
}

std::string unb64url(const std::string& s) {
  static const std::array<int8_t, 256> rev = [] {
    std::array<int8_t, 256> r{};
    r.fill(-1);
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    for (int i = 0; i < 64; ++i) r[static_cast<unsigned char>(a[i])] = static_cast<int8_t>(i);
    return r;
  }();
  std::string out;
  unsigned v = 0;
  int bits = 0;
  for (unsigned char c : s) {
    if (c == '=') break;
    if (rev[c] < 0) return "";
    v = (v << 6) | static_cast<unsigned>(rev[c]);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out += static_cast<char>((v >> bits) & 0xff);
    }
  }
  return out;
}

std::string hmac_sha256(const std::string& key, const std::string& msg) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  if (!HMAC(EVP_sha256(), key.data(), static_cast<int>(key.size()),
            reinterpret_cast<const unsigned char*>(msg.data()), msg.size(), out, &n))
    throw std::runtime_error("HMAC-SHA256 failed");
  return std::string(reinterpret_cast<char*>(out), n);
}

// X25519(priv, peer) -> 32-byte shared secret ("" on failure: a low-order peer key, bad input)
std::string x25519(EVP_PKEY* priv, const std::string& peer) {
  EVP_PKEY* pk = EVP_PKEY_new_raw_public_key(EVP_PKEY_X25519, nullptr,
                                             reinterpret_cast<const unsigned char*>(peer.data()), peer.size());
  EVP_PKEY_CTX* ctx = EVP_PKEY_CTX_new(priv, nullptr);
  std::string out(32, '\0');
  size_t n = out.size();
  bool ok = pk && ctx && EVP_PKEY_derive_init(ctx) == 1 && EVP_PKEY_derive_set_peer(ctx, pk) == 1 &&
            EVP_PKEY_derive(ctx, reinterpret_cast<unsigned char*>(out.data()), &n) == 1 && n == 32;
  EVP_PKEY_CTX_free(ctx);
  EVP_PKEY_free(pk);
  return ok ? out : "";
}

}  // namespace

std::string sha256_hex(const std::string& data) {
  unsigned char md[SHA256_DIGEST_LENGTH];
  SHA256(reinterpret_cast<const unsigned char*>(data.data()), data.size(), md);
  return hex(md, sizeof md);
}

AgentSigner::AgentSigner(std::string key_file, std::chrono::milliseconds recheck)
    : path_(std::move(key_file)), recheck_(recheck) {
  std::lock_guard<std::mutex> g(mu_);
  load_locked_(true);
  if (!key_) throw std::runtime_error("agent signing key " + path_ + ": not an Ed25519 private key");
}

void AgentSigner::load_locked_(bool force) {
  const auto now = std::chrono::steady_clock::now();
  if (!force && now - checked_at_ < recheck_) return;
  checked_at_ = now;
  struct stat st {};
  if (::stat(path_.c_str(), &st) != 0) return;  // mid-swap: keep the current key
  const long long m = static_cast<long long>(st.st_mtim.tv_sec) * 1000000000LL + st.st_mtim.tv_nsec;
  if (!force && m == mtime_ns_) return;
  FILE* f = std::fopen(path_.c_str(), "r");
  if (!f) return;
  EVP_PKEY* k = PEM_read_PrivateKey(f, nullptr, nullptr, nullptr);
  std::fclose(f);
  if (!k || EVP_PKEY_id(k) != EVP_PKEY_ED25519) {
    if (k) EVP_PKEY_free(k);
    return;
  }
  unsigned char pub[32];
  size_t n = sizeof pub;
  if (EVP_PKEY_get_raw_public_key(k, pub, &n) != 1 || n != 32) {
    EVP_PKEY_free(k);
    return;
  }
  unsigned char md[SHA256_DIGEST_LENGTH];
  SHA256(pub, n, md);
  // the X25519 twin: the Ed25519 secret scalar is SHA-512(seed)[0:32] (X25519 clamps it alike)
  unsigned char seed[32], h[SHA512_DIGEST_LENGTH];
  size_t sn = sizeof seed;
  EVP_PKEY* xk = nullptr;
  std::string xpub;
  if (EVP_PKEY_get_raw_private_key(k, seed, &sn) == 1 && sn == 32) {
    SHA512(seed, sn, h);
    xk = EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, nullptr, h, 32);
    OPENSSL_cleanse(seed, sizeof seed);
    OPENSSL_cleanse(h, sizeof h);
    unsigned char xp[32];
    size_t xn = sizeof xp;
    if (xk && EVP_PKEY_get_raw_public_key(xk, xp, &xn) == 1 && xn == 32)
      xpub.assign(reinterpret_cast<char*>(xp), xn);
  }
  if (key_) reloads_.fetch_add(1);
  key_ = std::shared_ptr<void>(k, [](void* p) { EVP_PKEY_free(static_cast<EVP_PKEY*>(p)); });
  xkey_ = xk ? std::shared_ptr<void>(xk, [](void* p) { EVP_PKEY_free(static_cast<EVP_PKEY*>(p)); })
             : std::shared_ptr<void>();
  xpub_ = xpub;
  mac_keys_.clear();
  kid_ = hex(md, sizeof md).substr(0, 16);
  mtime_ns_ = m;
}

std::string AgentSigner::key_id() {
  std::lock_guard<std::mutex> g(mu_);
  return kid_;
}

std::string AgentSigner::header(const std::string& method, const std::string& target, const std::string& node,
                                const std::string& body, const std::string& agent_kx) {
  std::shared_ptr<void> key;
  std::string kid, mac_key, agent_x;
  {
    std::lock_guard<std::mutex> g(mu_);
    load_locked_(false);
    key = key_;
    kid = kid_;
    if (!agent_kx.empty() && xkey_) {
      agent_x = unb64url(agent_kx);
      if (agent_x.size() == 32) {
        const std::string ck = node + "\n" + agent_x;
        auto it = mac_keys_.find(ck);
        if (it == mac_keys_.end()) {
          const std::string shared = x25519(static_cast<EVP_PKEY*>(xkey_.get()), agent_x);
          // agents rotate their keys: stale node/key pairs would pile up for the manager's lifetime
          if (mac_keys_.size() >= kMaxMacKeys) mac_keys_.clear();
          if (!shared.empty())
            it = mac_keys_.emplace(ck, hmac_sha256(shared, "gpupool-agent-rpc-v2\n" + node + "\n" + xpub_ + agent_x))
                     .first;
        }
        if (it != mac_keys_.end()) mac_key = it->second;
      }
    }
  }
  const long long ts = std::chrono::duration_cast<std::chrono::milliseconds>(
                           std::chrono::system_clock::now().time_since_epoch())
                           .count();
  unsigned char rnd[16];
  if (RAND_bytes(rnd, sizeof rnd) != 1) throw std::runtime_error("RAND_bytes failed");
  const std::string nonce = hex(rnd, sizeof rnd);
  const std::string digest = sha256_hex(body);
  const std::string tail = method + "\n" + target + "\n" + node + "\n" + std::to_string(ts) + "\n" + nonce + "\n" + digest;
  if (!mac_key.empty()) {  // v2: the per-node MAC
    const std::string mac = hmac_sha256(mac_key, "gpupool-agent-rpc-v2\n" + tail);
    return "X-Gpupool-Signature: v2 keyId=" + kid + " kx=" + sha256_hex(agent_x).substr(0, 16) + " node=" + node +
           " ts=" + std::to_string(ts) + " nonce=" + nonce + " body=" + digest +
           " mac=" + b64url(reinterpret_cast<const unsigned char*>(mac.data()), mac.size()) + "\r\n";
  }
  const std::string msg = "gpupool-agent-rpc-v1\n" + tail;
  unsigned char sig[64];
  size_t slen = sizeof sig;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  bool ok = ctx && EVP_DigestSignInit(ctx, nullptr, nullptr, nullptr, static_cast<EVP_PKEY*>(key.get())) == 1 &&
            EVP_DigestSign(ctx, sig, &slen, reinterpret_cast<const unsigned char*>(msg.data()), msg.size()) == 1;
  EVP_MD_CTX_free(ctx);
  if (!ok) throw std::runtime_error("Ed25519 signing failed");
  return "X-Gpupool-Signature: v1 keyId=" + kid + " node=" + node + " ts=" + std::to_string(ts) +
         " nonce=" + nonce + " body=" + digest + " sig=" + b64url(sig, slen) + "\r\n";
}

}  // namespace gpupool

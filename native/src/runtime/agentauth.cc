#include "gpupool/agentauth.h"

#include <sys/stat.h>

#include <cstdio>
#include <stdexcept>

#include <openssl/evp.h>
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
  if (key_) reloads_.fetch_add(1);
  key_ = std::shared_ptr<void>(k, [](void* p) { EVP_PKEY_free(static_cast<EVP_PKEY*>(p)); });
  kid_ = hex(md, sizeof md).substr(0, 16);
  mtime_ns_ = m;
}

std::string AgentSigner::key_id() {
  std::lock_guard<std::mutex> g(mu_);
  return kid_;
}

std::string AgentSigner::header(const std::string& method, const std::string& target, const std::string& node,
                                const std::string& body) {
  std::shared_ptr<void> key;
  std::string kid;
  {
    std::lock_guard<std::mutex> g(mu_);
    load_locked_(false);
    key = key_;
    kid = kid_;
  }
  const long long ts = std::chrono::duration_cast<std::chrono::milliseconds>(
                           std::chrono::system_clock::now().time_since_epoch())
                           .count();
  unsigned char rnd[16];
  if (RAND_bytes(rnd, sizeof rnd) != 1) throw std::runtime_error("RAND_bytes failed");
  const std::string nonce = hex(rnd, sizeof rnd);
  const std::string digest = sha256_hex(body);
  const std::string msg = "gpupool-agent-rpc-v1\n" + method + "\n" + target + "\n" + node + "\n" +
                          std::to_string(ts) + "\n" + nonce + "\n" + digest;
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

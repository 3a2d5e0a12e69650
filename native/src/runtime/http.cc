#include "gpupool/http.h"

#include <algorithm>
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <fstream>
#include <sstream>

#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <stdexcept>

namespace gpupool {

// ------------------------------------------------------------------ Url
Url Url::parse(const std::string& s) {
  Url u;
  auto p = s.find("://");
  std::string rest;
  if (p == std::string::npos) {
    u.scheme = "http";
    rest = s;
  } else {
    u.scheme = s.substr(0, p);
    rest = s.substr(p + 3);
  }
  if (u.scheme == "unix") {
    u.unix_path = rest.empty() || rest[0] == '/' ? rest : "/" + rest;
    if (u.unix_path.empty()) throw std::invalid_argument("empty unix socket path");
    return u;
  }
  if (u.scheme != "http" && u.scheme != "https") throw std::invalid_argument("unsupported scheme: " + u.scheme);
  auto slash = rest.find('/');
  if (slash != std::string::npos) rest = rest.substr(0, slash);
  auto colon = rest.rfind(':');
  if (colon != std::string::npos && rest.find(']') == std::string::npos) {
    u.host = rest.substr(0, colon);
    u.port = std::stoi(rest.substr(colon + 1));
  } else {
    u.host = rest;
    u.port = u.scheme == "https" ? 443 : 80;
  }
  if (u.host.empty()) u.host = "127.0.0.1";
  return u;
}

std::string Url::str() const {
  if (scheme == "unix") return "unix://" + unix_path;
  return scheme + "://" + host + ":" + std::to_string(port);
}

std::string url_encode(std::string_view s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out.push_back(static_cast<char>(c));
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    }
  }
  return out;
}

std::string base64_decode(std::string_view in) {
  auto val = [](unsigned char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+' || c == '-') return 62;  // '-' '_': the URL-safe alphabet
    if (c == '/' || c == '_') return 63;
    return -1;
  };
  std::string out;
  out.reserve(in.size() * 3 / 4);
  uint32_t acc = 0;
  int bits = 0;
  for (unsigned char c : in) {
    if (c == '=') break;
    int v = val(c);
    if (v < 0) continue;
    acc = ((acc << 6) | static_cast<uint32_t>(v)) & 0xFFFFFFu;  // never more than 24 live bits
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back(static_cast<char>((acc >> bits) & 0xFFu));
    }
  }
  return out;
}

std::string url_decode(std::string_view s) {
  auto hexval = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && hexval(s[i + 1]) >= 0 && hexval(s[i + 2]) >= 0) {
      out.push_back(static_cast<char>(hexval(s[i + 1]) * 16 + hexval(s[i + 2])));
      i += 2;
    } else if (s[i] == '+') {
      out.push_back(' ');
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

// ------------------------------------------------------------------ chunked
bool ChunkedDecoder::feed(std::string_view in, std::string& out) {
  size_t i = 0;
  while (i < in.size()) {
    char c = in[i];
    switch (state_) {
      case State::Size: {
        int v = -1;
        if (c >= '0' && c <= '9') v = c - '0';
        else if (c >= 'a' && c <= 'f') v = c - 'a' + 10;
        else if (c >= 'A' && c <= 'F') v = c - 'A' + 10;
        if (v >= 0) {
          if (++size_digits_ > 15) return false;  // > 2^60: refuse
          remaining_ = remaining_ * 16 + static_cast<uint64_t>(v);
          ++i;
        } else if (c == ';' || c == ' ' || c == '\t') {
          if (size_digits_ == 0) return false;
          state_ = State::SizeExt;
          ++i;
        } else if (c == '\r') {
          if (size_digits_ == 0) return false;
          state_ = State::SizeLF;
          ++i;
        } else {
          return false;
        }
        break;
      }
      case State::SizeExt:
        if (c == '\r') state_ = State::SizeLF;
        ++i;
        break;
      case State::SizeLF:
        if (c != '\n') return false;
        ++i;
        size_digits_ = 0;
        if (remaining_ == 0) {
          state_ = State::Trailer;
          trailer_line_empty_ = true;
        } else {
          state_ = State::Data;
        }
        break;
      case State::Data: {
        size_t n = std::min<uint64_t>(remaining_, in.size() - i);
        out.append(in.data() + i, n);
        i += n;
        remaining_ -= n;
        if (remaining_ == 0) state_ = State::DataCR;
        break;
      }
      case State::DataCR:
        if (c != '\r') return false;
        state_ = State::DataLF;
        ++i;
        break;
      case State::DataLF:
        if (c != '\n') return false;
        state_ = State::Size;
        ++i;
        break;
      case State::Trailer:
        if (c == '\r') {
          state_ = State::TrailerLF;
        } else {
          trailer_line_empty_ = false;
        }
        ++i;
        break;
      case State::TrailerLF:
        if (c != '\n') return false;
        ++i;
        if (trailer_line_empty_) {
          state_ = State::Done;
        } else {
          state_ = State::Trailer;
          trailer_line_empty_ = true;
        }
        break;
      case State::Done:
        return true;  // ignore anything after the terminator
    }
  }
  return true;
}

// ------------------------------------------------------------------ connection
struct HttpClient::Conn {
  int fd = -1;
  SSL* ssl = nullptr;  // non-null for https
  std::string rbuf;
  ~Conn() {
    if (ssl) {
      SSL_shutdown(ssl);
      SSL_free(ssl);
    }
    if (fd >= 0) ::close(fd);
  }

  // Wait for readability; returns 1 ready, 0 timeout, -1 error.
  int wait_readable(int timeout_ms) const {
    if (ssl && SSL_pending(ssl) > 0) return 1;  // decrypted bytes already buffered
    pollfd p{fd, POLLIN, 0};
    int r;
    do {
      r = ::poll(&p, 1, timeout_ms);
    } while (r < 0 && errno == EINTR);
    if (r < 0) return -1;
    return r == 0 ? 0 : 1;
  }

  // Read more bytes into rbuf. Returns bytes read, 0 on EOF, -1 on error, -2 on timeout.
  ssize_t fill(int timeout_ms) {
    int w = wait_readable(timeout_ms);
    if (w == 0) return -2;
    if (w < 0) return -1;
    char buf[65536];
    ssize_t n;
    if (ssl) {
      for (;;) {
        int r = SSL_read(ssl, buf, sizeof buf);
        if (r > 0) {
          rbuf.append(buf, static_cast<size_t>(r));
          return r;
        }
        int e = SSL_get_error(ssl, r);
        if (e == SSL_ERROR_ZERO_RETURN) return 0;
        if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) {
          if (wait_readable(timeout_ms) <= 0) return -2;
          continue;
        }
        return e == SSL_ERROR_SYSCALL && r == 0 ? 0 : -1;
      }
    }
    do {
      n = ::recv(fd, buf, sizeof buf, 0);
    } while (n < 0 && errno == EINTR);
    if (n > 0) rbuf.append(buf, static_cast<size_t>(n));
    return n;
  }

  bool send_all(const std::string& data) const {
    if (ssl) {
      size_t off = 0;
      while (off < data.size()) {
        int r = SSL_write(ssl, data.data() + off, static_cast<int>(data.size() - off));
        if (r <= 0) {
          int e = SSL_get_error(ssl, r);
          if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) continue;
          return false;
        }
        off += static_cast<size_t>(r);
      }
      return true;
    }
    size_t off = 0;
    while (off < data.size()) {
      ssize_t n = ::send(fd, data.data() + off, data.size() - off, MSG_NOSIGNAL);
      if (n < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      off += static_cast<size_t>(n);
    }
    return true;
  }
};

namespace {
std::string ssl_errors() {
  std::string out;
  unsigned long e;
  char buf[256];
  while ((e = ERR_get_error()) != 0) {
    ERR_error_string_n(e, buf, sizeof buf);
    if (!out.empty()) out += "; ";
    out += buf;
  }
  return out.empty() ? "unknown TLS error" : out;
}
}  // namespace

std::shared_ptr<TokenSource> TokenSource::fixed(std::string token) {
  std::shared_ptr<TokenSource> t(new TokenSource());
  t->token_ = std::move(token);
  return t;
}

std::shared_ptr<TokenSource> TokenSource::file(std::string path, std::chrono::milliseconds reload_after) {
  std::shared_ptr<TokenSource> t(new TokenSource());
  t->path_ = std::move(path);
  t->reload_after_ = reload_after;
  std::lock_guard<std::mutex> g(t->mu_);
  t->read_locked_();
  if (t->token_.empty()) throw HttpError("token file " + t->path_ + " is missing or empty");
  return t;
}

void TokenSource::read_locked_() {
  read_at_ = std::chrono::steady_clock::now();
  std::ifstream f(path_, std::ios::binary);
  if (!f) return;  // mid-rotation (the kubelet swaps a symlink): keep the last value
  std::stringstream ss;
  ss << f.rdbuf();
  std::string t = ss.str();
  while (!t.empty() && (t.back() == '\n' || t.back() == '\r' || t.back() == ' ')) t.pop_back();
  if (!t.empty() && t != token_) {
    if (!token_.empty()) reloads_.fetch_add(1);
    token_ = std::move(t);
  }
}

std::string TokenSource::token() {
  std::lock_guard<std::mutex> g(mu_);
  if (!path_.empty() && std::chrono::steady_clock::now() - read_at_ >= reload_after_) read_locked_();
  return token_;
}

bool TokenSource::reload() {
  if (path_.empty()) return false;
  std::lock_guard<std::mutex> g(mu_);
  const std::string before = token_;
  read_locked_();
  return token_ != before;
}

HttpClient::HttpClient(Url url, std::shared_ptr<TokenSource> tokens, int timeout_ms, TlsOptions tls)
    : HttpClient(std::move(url), std::string(), timeout_ms, std::move(tls)) {
  tokens_ = std::move(tokens);
}

std::string HttpClient::auth_headers_(const std::string& method, const std::string& path, const std::string& body,
                                      const std::string* bearer) {
  std::string h;
  if (tokens_) {
    std::string t = bearer ? *bearer : tokens_->token();
    if (!t.empty()) h += "Authorization: Bearer " + t + "\r\n";
  } else if (!token_.empty()) {
    h += "Authorization: Bearer " + token_ + "\r\n";
  }
  if (signer_) h += signer_(method, path, body);
  return h;
}

// After a 401 sent with ``used``: worth one more try when the source now holds another token —
// re-read just now, or already by a concurrent request that got its 401 first.
bool HttpClient::reload_after_401_(const std::string& used) {
  if (!tokens_) return false;
  tokens_->reload();
  return tokens_->token() != used;
}

HttpClient::HttpClient(Url url, std::string bearer_token, int timeout_ms, TlsOptions tls)
    : url_(std::move(url)), token_(std::move(bearer_token)), timeout_ms_(timeout_ms), tls_(std::move(tls)) {
  if (url_.scheme != "https") return;
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) throw HttpError("SSL_CTX_new: " + ssl_errors());
  ssl_ctx_ = std::shared_ptr<void>(ctx, [](void* p) { SSL_CTX_free(static_cast<SSL_CTX*>(p)); });
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  if (tls_.insecure) {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_NONE, nullptr);
  } else {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
    if (!tls_.ca_pem.empty()) {
      // every certificate in the PEM bundle becomes a trust anchor
      std::unique_ptr<BIO, decltype(&BIO_free)> bio(BIO_new_mem_buf(tls_.ca_pem.data(), static_cast<int>(tls_.ca_pem.size())),
                                                    BIO_free);
      X509_STORE* store = SSL_CTX_get_cert_store(ctx);
      int added = 0;
      while (X509* x = PEM_read_bio_X509(bio.get(), nullptr, nullptr, nullptr)) {
        added += X509_STORE_add_cert(store, x) == 1;
        X509_free(x);
      }
      ERR_clear_error();  // PEM_read_bio_X509 leaves "no start line" at end of input
      if (added == 0) throw HttpError("certificate-authority-data: no usable certificate");
    } else {
      int ok = tls_.ca_file.empty() ? SSL_CTX_set_default_verify_paths(ctx)
                                    : SSL_CTX_load_verify_locations(ctx, tls_.ca_file.c_str(), nullptr);
      if (ok != 1) throw HttpError("loading CA " + tls_.ca_file + ": " + ssl_errors());
    }
  }
  if (!tls_.cert_pem.empty()) {
    std::unique_ptr<BIO, decltype(&BIO_free)> cb(BIO_new_mem_buf(tls_.cert_pem.data(), static_cast<int>(tls_.cert_pem.size())),
                                                 BIO_free);
    std::unique_ptr<X509, decltype(&X509_free)> cert(PEM_read_bio_X509(cb.get(), nullptr, nullptr, nullptr), X509_free);
    const std::string& kp = tls_.key_pem.empty() ? tls_.cert_pem : tls_.key_pem;
    std::unique_ptr<BIO, decltype(&BIO_free)> kb(BIO_new_mem_buf(kp.data(), static_cast<int>(kp.size())), BIO_free);
    std::unique_ptr<EVP_PKEY, decltype(&EVP_PKEY_free)> key(PEM_read_bio_PrivateKey(kb.get(), nullptr, nullptr, nullptr),
                                                            EVP_PKEY_free);
    if (!cert || !key || SSL_CTX_use_certificate(ctx, cert.get()) != 1 || SSL_CTX_use_PrivateKey(ctx, key.get()) != 1)
      throw HttpError("client-certificate-data: " + ssl_errors());
  } else if (!tls_.cert_file.empty()) {
    if (SSL_CTX_use_certificate_chain_file(ctx, tls_.cert_file.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(ctx, tls_.key_file.empty() ? tls_.cert_file.c_str() : tls_.key_file.c_str(),
                                    SSL_FILETYPE_PEM) != 1)
      throw HttpError("client certificate: " + ssl_errors());
  }
}

HttpClient::~HttpClient() = default;

std::unique_ptr<HttpClient::Conn> HttpClient::connect_(int timeout_ms) {
  auto c = std::make_unique<Conn>();
  if (url_.scheme == "unix") {
    c->fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (c->fd < 0) throw HttpError("socket: " + std::string(strerror(errno)));
    sockaddr_un sa{};
    sa.sun_family = AF_UNIX;
    if (url_.unix_path.size() >= sizeof sa.sun_path) throw HttpError("unix path too long");
    std::memcpy(sa.sun_path, url_.unix_path.c_str(), url_.unix_path.size() + 1);
    if (::connect(c->fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0)
      throw HttpError("connect " + url_.str() + ": " + strerror(errno));
    return c;
  }
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string port = std::to_string(url_.port);
  int rc = ::getaddrinfo(url_.host.c_str(), port.c_str(), &hints, &res);
  if (rc != 0) throw HttpError("getaddrinfo " + url_.host + ": " + gai_strerror(rc));
  std::string last_err = "no address";
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    int fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    // non-blocking connect with timeout
    int flags = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, flags | O_NONBLOCK);
    int r = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (r != 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      r = ::poll(&p, 1, timeout_ms);
      int err = 0;
      socklen_t len = sizeof err;
      if (r == 1 && getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len) == 0 && err == 0) {
        r = 0;
      } else {
        last_err = r == 0 ? "connect timeout" : strerror(err ? err : errno);
        r = -1;
      }
    } else if (r != 0) {
      last_err = strerror(errno);
    }
    if (r == 0) {
      fcntl(fd, F_SETFL, flags);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      c->fd = fd;
      break;
    }
    ::close(fd);
  }
  freeaddrinfo(res);
  if (c->fd < 0) throw HttpError("connect " + url_.str() + ": " + last_err);
  if (ssl_ctx_) {
    c->ssl = SSL_new(static_cast<SSL_CTX*>(ssl_ctx_.get()));
    if (!c->ssl) throw HttpError("SSL_new: " + ssl_errors());
    SSL_set_fd(c->ssl, c->fd);
    in6_addr a6{};
    in_addr a4{};
    bool is_ip = inet_pton(AF_INET, url_.host.c_str(), &a4) == 1 || inet_pton(AF_INET6, url_.host.c_str(), &a6) == 1;
    if (!is_ip) SSL_set_tlsext_host_name(c->ssl, url_.host.c_str());  // SNI
    if (!tls_.insecure) {
      X509_VERIFY_PARAM* vp = SSL_get0_param(c->ssl);
      if (is_ip) X509_VERIFY_PARAM_set1_ip_asc(vp, url_.host.c_str());
      else X509_VERIFY_PARAM_set1_host(vp, url_.host.c_str(), 0);
    }
    // blocking handshake bounded by the socket timeout
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    setsockopt(c->fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(c->fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    if (SSL_connect(c->ssl) != 1) {
      long vr = SSL_get_verify_result(c->ssl);
      std::string why = vr != X509_V_OK ? X509_verify_cert_error_string(vr) : ssl_errors();
      throw HttpError("TLS handshake with " + url_.str() + ": " + why);
    }
    timeval zero{0, 0};
    setsockopt(c->fd, SOL_SOCKET, SO_RCVTIMEO, &zero, sizeof zero);
    setsockopt(c->fd, SOL_SOCKET, SO_SNDTIMEO, &zero, sizeof zero);
  }
  return c;
}

std::unique_ptr<HttpClient::Conn> HttpClient::take_() {
  std::lock_guard<std::mutex> g(mu_);
  if (idle_.empty()) return nullptr;
  auto c = std::move(idle_.back());
  idle_.pop_back();
  return c;
}

void HttpClient::give_(std::unique_ptr<Conn> c) {
  std::lock_guard<std::mutex> g(mu_);
  if (idle_.size() < 16) idle_.push_back(std::move(c));
}

bool HttpClient::send_request_(Conn& c, const std::string& method, const std::string& path,
                               const std::string& body, const std::string& content_type,
                               const std::string& accept, const std::string& extra_headers,
                               const std::string* bearer) {
  std::string req;
  req.reserve(256 + body.size());
  req += method + " " + path + " HTTP/1.1\r\n";
  req += "Host: " + (url_.scheme == "unix" ? std::string("localhost") : url_.host) + "\r\n";
  req += "User-Agent: gpupool-manager/0.1\r\n";
  req += "Accept: " + accept + "\r\n";
  req += auth_headers_(method, path, body, bearer);
  req += extra_headers;
  if (!body.empty() || method == "POST" || method == "PUT" || method == "PATCH") {
    req += "Content-Type: " + content_type + "\r\n";
    req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  }
  req += "\r\n";
  req += body;
  return c.send_all(req);
}

namespace {

std::string lower(std::string s) {
  for (auto& ch : s) ch = static_cast<char>(tolower(static_cast<unsigned char>(ch)));
  return s;
}

// Parse status line + headers from c.rbuf (reading more as needed). Returns false on failure.
template <class ConnT>
bool read_head(ConnT& c, HttpResponse& r, int timeout_ms, std::string* err,
               const std::atomic<bool>* stop = nullptr, int poll_ms = 200) {
  size_t end;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while ((end = c.rbuf.find("\r\n\r\n")) == std::string::npos) {
    if (stop && stop->load()) {
      *err = "stopped";
      return false;
    }
    if (c.rbuf.size() > (1 << 20)) {
      *err = "header too large";
      return false;
    }
    int left = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(
                                    deadline - std::chrono::steady_clock::now())
                                    .count());
    if (left <= 0) {
      *err = "timeout reading response head";
      return false;
    }
    // with a stop flag, wait in poll_ms slices so a long-poll whose answer is still pending
    // (the server holds the head until something changes) can be abandoned promptly
    ssize_t n = c.fill(stop ? std::min(left, poll_ms) : left);
    if (n == 0) {
      *err = "connection closed";
      return false;
    }
    if (n == -2) {
      if (stop) continue;  // slice elapsed: re-check stop and the overall deadline
      *err = "timeout reading response head";
      return false;
    }
    if (n < 0) {
      *err = std::string("recv: ") + strerror(errno);
      return false;
    }
  }
  std::string head = c.rbuf.substr(0, end);
  c.rbuf.erase(0, end + 4);
  std::istringstream is(head);
  std::string line;
  std::getline(is, line);
  if (line.size() < 12 || line.compare(0, 5, "HTTP/") != 0) {
    *err = "bad status line";
    return false;
  }
  r.status = std::atoi(line.c_str() + 9);
  while (std::getline(is, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    auto colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string v = line.substr(colon + 1);
    size_t a = v.find_first_not_of(" \t");
    v = a == std::string::npos ? "" : v.substr(a);
    r.headers[lower(line.substr(0, colon))] = v;
  }
  return true;
}

}  // namespace

HttpResponse HttpClient::request(const std::string& method, const std::string& path,
                                 const std::string& body, const std::string& content_type,
                                 const std::string& accept, int timeout_ms, const std::string& extra_headers) {
  if (timeout_ms < 0) timeout_ms = timeout_ms_;
  const std::string used = tokens_ ? tokens_->token() : std::string();
  HttpResponse r = request_once_(method, path, body, content_type, accept, timeout_ms, extra_headers, &used);
  // a rotated credential: the file already holds the new one (or will within the kubelet's
  // refresh) — re-read it and send once more, instead of failing until the periodic reload
  if (r.status == 401 && reload_after_401_(used)) {
    const std::string fresh = tokens_->token();
    r = request_once_(method, path, body, content_type, accept, timeout_ms, extra_headers, &fresh);
  }
  return r;
}

HttpResponse HttpClient::request_once_(const std::string& method, const std::string& path,
                                       const std::string& body, const std::string& content_type,
                                       const std::string& accept, int timeout_ms,
                                       const std::string& extra_headers, const std::string* bearer) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    std::unique_ptr<Conn> c = take_();
    bool reused = c != nullptr;
    if (!c) c = connect_(timeout_ms);
    if (!send_request_(*c, method, path, body, content_type, accept, extra_headers, bearer)) {
      if (reused) continue;
      throw HttpError("send failed: " + std::string(strerror(errno)));
    }
    HttpResponse r;
    std::string err;
    if (!read_head(*c, r, timeout_ms, &err)) {
      if (reused && (err == "connection closed" || err.rfind("recv", 0) == 0)) continue;
      throw HttpError(method + " " + path + ": " + err);
    }
    bool keep = true;
    auto conn_hdr = r.headers.find("connection");
    if (conn_hdr != r.headers.end() && lower(conn_hdr->second) == "close") keep = false;
    auto te = r.headers.find("transfer-encoding");
    auto cl = r.headers.find("content-length");
    if (te != r.headers.end() && lower(te->second).find("chunked") != std::string::npos) {
      ChunkedDecoder dec;
      std::string pending = std::move(c->rbuf);
      c->rbuf.clear();
      for (;;) {
        if (!dec.feed(pending, r.body)) throw HttpError("bad chunked encoding");
        pending.clear();
        if (dec.done()) break;
        ssize_t n = c->fill(timeout_ms);
        if (n <= 0) throw HttpError("connection lost reading chunked body");
        pending = std::move(c->rbuf);
        c->rbuf.clear();
      }
    } else if (cl != r.headers.end()) {
      size_t want = std::stoull(cl->second);
      while (c->rbuf.size() < want) {
        ssize_t n = c->fill(timeout_ms);
        if (n <= 0) throw HttpError("connection lost reading body");
      }
      r.body = c->rbuf.substr(0, want);
      c->rbuf.erase(0, want);
    } else if (r.status != 204 && r.status != 304 && method != "HEAD") {
      for (;;) {
        ssize_t n = c->fill(timeout_ms);
        if (n == 0) break;
        if (n < 0) throw HttpError("connection lost reading body");
      }
      r.body = std::move(c->rbuf);
      keep = false;
    }
    if (keep) give_(std::move(c));
    return r;
  }
  throw HttpError(method + " " + path + ": retries exhausted");
}

int HttpClient::stream_lines(const std::string& path,
                             const std::function<bool(std::string_view)>& on_line,
                             const std::atomic<bool>* stop, std::string* err_body, int poll_ms) {
  std::string body401;
  const std::string used = tokens_ ? tokens_->token() : std::string();
  int status = stream_lines_once_(path, on_line, stop, &body401, poll_ms, &used);
  if (status == 401 && reload_after_401_(used)) {
    body401.clear();
    const std::string fresh = tokens_->token();
    status = stream_lines_once_(path, on_line, stop, &body401, poll_ms, &fresh);
  }
  if (status >= 400 && err_body) *err_body = body401;
  return status;
}

int HttpClient::stream_lines_once_(const std::string& path,
                                   const std::function<bool(std::string_view)>& on_line,
                                   const std::atomic<bool>* stop, std::string* err_body, int poll_ms,
                                   const std::string* bearer) {
  auto c = connect_(timeout_ms_);
  if (!send_request_(*c, "GET", path, "", "application/json", "application/json", "", bearer))
    throw HttpError("send failed");
  HttpResponse r;
  std::string err;
  if (!read_head(*c, r, timeout_ms_, &err, stop, poll_ms)) {
    if (stop && stop->load()) return 0;  // abandoned on request: not an error
    throw HttpError("GET " + path + ": " + err);
  }
  bool chunked = false;
  auto te = r.headers.find("transfer-encoding");
  if (te != r.headers.end() && lower(te->second).find("chunked") != std::string::npos) chunked = true;
  ChunkedDecoder dec;
  std::string payload, pending = std::move(c->rbuf);
  c->rbuf.clear();
  if (r.status >= 400) {
    // read the (short) error body fully
    for (int i = 0; i < 100; ++i) {
      if (chunked) {
        if (!dec.feed(pending, payload)) break;
        if (dec.done()) break;
      } else {
        payload += pending;
      }
      pending.clear();
      auto cl = r.headers.find("content-length");
      if (!chunked && cl != r.headers.end() && payload.size() >= std::stoull(cl->second)) break;
      ssize_t n = c->fill(timeout_ms_);
      if (n <= 0) break;
      pending = std::move(c->rbuf);
      c->rbuf.clear();
    }
    if (err_body) *err_body = payload;
    return r.status;
  }
  // A non-chunked body (long-poll answers) ends at Content-Length: the server keeps the
  // connection alive, so waiting for EOF would stall until its keep-alive timeout.
  int64_t remaining = -1;
  if (!chunked) {
    auto cl = r.headers.find("content-length");
    if (cl != r.headers.end()) remaining = static_cast<int64_t>(std::stoull(cl->second));
  }
  for (;;) {
    if (chunked) {
      if (!dec.feed(pending, payload)) throw HttpError("bad chunked encoding in stream");
    } else {
      payload += pending;
      if (remaining >= 0) remaining -= static_cast<int64_t>(pending.size());
    }
    pending.clear();
    size_t nl;
    while ((nl = payload.find('\n')) != std::string::npos) {
      std::string_view line(payload.data(), nl);
      if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
      bool cont = line.empty() ? true : on_line(line);
      payload.erase(0, nl + 1);
      if (!cont) return r.status;
    }
    if (chunked && dec.done()) return r.status;
    if (remaining == 0) {
      if (!payload.empty()) on_line(payload);  // last line without a trailing newline
      return r.status;
    }
    for (;;) {
      if (stop && stop->load()) return r.status;
      ssize_t n = c->fill(poll_ms);
      if (n == -2) continue;  // timeout: re-check stop
      if (n <= 0) return r.status;  // EOF / error: caller re-watches
      break;
    }
    pending = std::move(c->rbuf);
    c->rbuf.clear();
  }
}

// ------------------------------------------------------------------ server
HttpServer::~HttpServer() { stop(); }

void HttpServer::route(const std::string& path, Handler h) { routes_[path] = std::move(h); }

int HttpServer::listen(const std::string& addr) {
  std::string host = "0.0.0.0";
  int port = 0;
  auto colon = addr.rfind(':');
  if (colon == std::string::npos) {
    port = std::stoi(addr);
  } else {
    if (colon > 0) host = addr.substr(0, colon);
    port = std::stoi(addr.substr(colon + 1));
  }
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) throw HttpError("socket failed");
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host.c_str(), &sa.sin_addr) != 1) throw HttpError("bad listen host " + host);
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0)
    throw HttpError("bind " + addr + ": " + strerror(errno));
  if (::listen(lfd_, 64) != 0) throw HttpError("listen failed");
  socklen_t len = sizeof sa;
  getsockname(lfd_, reinterpret_cast<sockaddr*>(&sa), &len);
  th_ = std::thread([this] { loop_(); });
  return ntohs(sa.sin_port);
}

void HttpServer::stop() {
  if (stop_.exchange(true)) return;
  if (lfd_ >= 0) {
    ::shutdown(lfd_, SHUT_RDWR);
  }
  if (th_.joinable()) th_.join();
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
}

void HttpServer::loop_() {
  while (!stop_.load()) {
    pollfd p{lfd_, POLLIN, 0};
    int r = ::poll(&p, 1, 200);
    if (r <= 0) continue;
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    serve_(fd);  // handlers are fast (metrics/health); serve inline
    ::close(fd);
  }
}

void HttpServer::serve_(int fd) {
  std::string buf;
  char tmp[4096];
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(2);
  size_t hend;
  while ((hend = buf.find("\r\n\r\n")) == std::string::npos) {
    if (std::chrono::steady_clock::now() > deadline || buf.size() > 65536) return;
    pollfd p{fd, POLLIN, 0};
    if (::poll(&p, 1, 200) <= 0) continue;
    ssize_t n = ::recv(fd, tmp, sizeof tmp, 0);
    if (n <= 0) return;
    buf.append(tmp, static_cast<size_t>(n));
  }
  std::istringstream is(buf.substr(0, hend));
  std::string method, target;
  is >> method >> target;
  std::string body = buf.substr(hend + 4);
  auto q = target.find('?');
  std::string path = q == std::string::npos ? target : target.substr(0, q);
  Reply rep;
  auto it = routes_.find(path);
  if (it == routes_.end()) {
    rep.status = 404;
    rep.body = "not found\n";
  } else {
    try {
      rep = it->second(method, target, body);
    } catch (const std::exception& e) {
      rep.status = 500;
      rep.body = std::string("error: ") + e.what() + "\n";
    }
  }
  std::string out = "HTTP/1.1 " + std::to_string(rep.status) + " X\r\nContent-Type: " + rep.content_type +
                    "\r\nContent-Length: " + std::to_string(rep.body.size()) +
                    "\r\nConnection: close\r\n\r\n" + rep.body;
  size_t off = 0;
  while (off < out.size()) {
    ssize_t n = ::send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
    if (n <= 0) return;
    off += static_cast<size_t>(n);
  }
}

}  // namespace gpupool

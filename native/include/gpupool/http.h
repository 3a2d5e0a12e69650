// Blocking HTTP/1.1 client (TCP or unix socket, keep-alive pool, chunked decoding, line
// streaming for k8s watches) and a tiny HTTP server for /metrics and /healthz.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

namespace gpupool {

// TLS settings for https:// URLs (OpenSSL). ca_file empty -> system trust store.
struct TlsOptions {
  std::string ca_file;
  std::string cert_file;  // client certificate (kubeconfig client-certificate)
  std::string key_file;
  // in-memory PEM alternatives (kubeconfig *-data fields, already base64-decoded)
  std::string ca_pem, cert_pem, key_pem;
  bool insecure = false;  // skip peer verification (tests / --insecure-skip-tls-verify)
};

struct Url {
  std::string scheme;     // http | https | unix
  std::string host;       // tcp host
  int port = 80;
  std::string unix_path;  // for unix:///path/to.sock
  static Url parse(const std::string& s);  // throws std::invalid_argument
  std::string str() const;
};

struct HttpResponse {
  int status = 0;
  std::map<std::string, std::string> headers;  // lower-cased names
  std::string body;
};

class HttpError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// Incremental decoder for ``Transfer-Encoding: chunked`` bodies. Feed raw bytes; decoded payload
// bytes are appended to ``out``. ``done()`` after the terminating zero-size chunk.
class ChunkedDecoder {
 public:
  // Returns false on a protocol error (then the stream must be dropped).
  bool feed(std::string_view in, std::string& out);
  bool done() const { return state_ == State::Done; }

 private:
  enum class State { Size, SizeExt, SizeLF, Data, DataCR, DataLF, Trailer, TrailerLF, Done };
  State state_ = State::Size;
  uint64_t remaining_ = 0;
  int size_digits_ = 0;
  bool trailer_line_empty_ = true;
};

// A bearer credential that may rotate (projected ServiceAccount tokens, Workload Identity): a
// fixed string, or a file re-read at most every ``reload_after`` and at once after a 401 —
// client-go's behaviour. Thread-safe; shared by every client (and watch stream) that uses it.
class TokenSource {
 public:
  static std::shared_ptr<TokenSource> fixed(std::string token);
  static std::shared_ptr<TokenSource> file(std::string path,
                                           std::chrono::milliseconds reload_after = std::chrono::seconds(60));
  std::string token();  // current value (re-read from the file when due)
  bool reload();        // re-read now; true when the token changed
  uint64_t reloads() const { return reloads_.load(); }
  const std::string& path() const { return path_; }

 private:
  TokenSource() = default;
  void read_locked_();
  std::mutex mu_;
  std::string path_, token_;
  std::chrono::milliseconds reload_after_{60000};
  std::chrono::steady_clock::time_point read_at_{};
  std::atomic<uint64_t> reloads_{0};
};

// Extra header lines for one request, computed from it (the manager's per-request signature to
// a node agent): (method, target incl. query, body) -> "Name: value\r\n"...
using RequestSigner = std::function<std::string(const std::string& method, const std::string& target,
                                                const std::string& body)>;

class HttpClient {
 public:
  explicit HttpClient(Url url, std::string bearer_token = "", int timeout_ms = 30000,
                      TlsOptions tls = {});
  // bearer from a rotating source (nullptr: none); a 401 re-reads it and retries once
  HttpClient(Url url, std::shared_ptr<TokenSource> tokens, int timeout_ms = 30000, TlsOptions tls = {});
  void set_signer(RequestSigner s) { signer_ = std::move(s); }
  ~HttpClient();
  HttpClient(const HttpClient&) = delete;
  HttpClient& operator=(const HttpClient&) = delete;

  // ``extra_headers``: preformatted "Name: value\r\n" lines (e.g. the leader's fencing token)
  HttpResponse request(const std::string& method, const std::string& path,
                       const std::string& body = "",
                       const std::string& content_type = "application/json",
                       const std::string& accept = "application/json", int timeout_ms = -1,
                       const std::string& extra_headers = "");

  // Streams a GET response line by line (k8s watch / agent long-poll). ``on_line`` returns false
  // to stop. Returns the HTTP status; for status >= 400 ``err_body`` receives the body. Stops
  // early when ``stop`` becomes true (checked at least every ``poll_ms``).
  int stream_lines(const std::string& path, const std::function<bool(std::string_view)>& on_line,
                   const std::atomic<bool>* stop, std::string* err_body = nullptr,
                   int poll_ms = 200);

  const Url& url() const { return url_; }

 private:
  struct Conn;
  std::unique_ptr<Conn> connect_(int timeout_ms);
  std::unique_ptr<Conn> take_();
  void give_(std::unique_ptr<Conn> c);
  bool send_request_(Conn& c, const std::string& method, const std::string& path,
                     const std::string& body, const std::string& content_type,
                     const std::string& accept, const std::string& extra_headers = "",
                     const std::string* bearer = nullptr);

  // ``bearer``: the token to send (the one a 401 is judged against); nullptr = the current one
  HttpResponse request_once_(const std::string& method, const std::string& path, const std::string& body,
                             const std::string& content_type, const std::string& accept, int timeout_ms,
                             const std::string& extra_headers, const std::string* bearer);
  int stream_lines_once_(const std::string& path, const std::function<bool(std::string_view)>& on_line,
                         const std::atomic<bool>* stop, std::string* err_body, int poll_ms,
                         const std::string* bearer);
  std::string auth_headers_(const std::string& method, const std::string& path, const std::string& body,
                            const std::string* bearer);
  bool reload_after_401_(const std::string& used);
  Url url_;
  std::string token_;
  std::shared_ptr<TokenSource> tokens_;
  RequestSigner signer_;
  int timeout_ms_;
  TlsOptions tls_;
  std::shared_ptr<void> ssl_ctx_;  // SSL_CTX*, shared by all connections of this client
  std::mutex mu_;
  std::vector<std::unique_ptr<Conn>> idle_;
};

// Minimal threaded HTTP/1.1 server (Connection: close). For /metrics, /healthz, /readyz.
class HttpServer {
 public:
  struct Reply {
    int status = 200;
    std::string content_type = "text/plain; charset=utf-8";
    std::string body;
  };
  using Handler = std::function<Reply(const std::string& method, const std::string& path,
                                      const std::string& body)>;

  HttpServer() = default;
  ~HttpServer();
  void route(const std::string& path, Handler h);
  // addr like ":8080", "127.0.0.1:0"; returns bound port. Throws on failure.
  int listen(const std::string& addr);
  void stop();

 private:
  void loop_();
  void serve_(int fd);
  std::map<std::string, Handler> routes_;
  int lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread th_;
};

std::string url_encode(std::string_view s);
std::string url_decode(std::string_view s);  // %XX and '+' (query strings)
// RFC 4648 base64 (padding optional; whitespace and other non-alphabet bytes are skipped).
std::string base64_decode(std::string_view in);

}  // namespace gpupool

// HTTP/1.1 + HTTP/2 server and keep-alive client.
//
// Server: one thread per connection (blocking I/O, TCP_NODELAY) — latency-optimal for
// the handful of keep-alive connections the apiserver and kubelet probes open; an
// HTTP/1.1 request is served on the thread that read it, with no hand-off.  Over TLS the
// server also speaks HTTP/2 when the client selects "h2" by ALPN (the apiserver's Go
// webhook client does; axum-server's rustls acceptor offers h2 + http/1.1 the same way):
// the connection thread then runs an http2::Connection and every request stream is
// served on a pooled worker thread, so one connection carries concurrent requests.
// Replaces axum 0.6 (`/health`, `/mutate`, reference src/controller.rs:256-263,
// src/admission.rs:149-177).
//
// Client: per-endpoint pool of keep-alive connections (plain or TLS) plus streaming
// responses for WATCH.  Replaces hyper 0.14 inside kube-client / google-drive3.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "core/cancel.h"
#include "core/net.h"

namespace bgc::http {

class Headers {
 public:
  void add(std::string name, std::string value) { items_.emplace_back(std::move(name), std::move(value)); }
  void set(const std::string& name, std::string value);
  const std::string* get(const std::string& name) const;  // case-insensitive
  std::string get_or(const std::string& name, const std::string& dflt = "") const;
  bool has(const std::string& name) const { return get(name) != nullptr; }
  void remove(const std::string& name);
  const std::vector<std::pair<std::string, std::string>>& items() const { return items_; }

 private:
  std::vector<std::pair<std::string, std::string>> items_;
};

struct Request {
  std::string method;
  std::string target;  // raw request-target
  std::string path;    // decoded path component
  std::string query;   // raw query string (no '?')
  Headers headers;
  std::string body;
  std::string remote;
  // verified TLS client certificate (net::Stream::peer_identity): CN and O values
  std::string peer_cn;
  std::vector<std::string> peer_orgs;
  std::string query_param(const std::string& name, const std::string& dflt = "") const;
  bool has_query_param(const std::string& name) const;
  std::map<std::string, std::string> query_params() const;
};

struct Response {
  int status = 200;
  Headers headers;
  std::string body;
};

const char* status_text(int code);
std::string url_encode(const std::string& s, bool keep_slash = false);
std::string url_decode(const std::string& s);

struct Url {
  std::string scheme;  // http | https
  std::string host;
  uint16_t port = 0;
  std::string path;  // includes query if any; "" when absent
};
Url parse_url(const std::string& url);

// Buffered reader over a Stream (request/response parsing, chunked decoding).
class Reader {
 public:
  explicit Reader(net::Stream& s) : s_(s) {}
  // Returns false on EOF/error/timeout. `got_any` reports whether any byte arrived.
  bool read_line(std::string& line, int timeout_ms, size_t max_len = 1 << 16);
  bool read_exact(std::string& out, size_t n, int timeout_ms);
  // Reads whatever is available (at least 1 byte). Returns -1 error, 0 EOF, -2 timeout.
  ssize_t read_available(std::string& out, int timeout_ms);
  bool buffered() const { return pos_ < buf_.size() || s_.has_buffered(); }
  bool consumed_any() const { return consumed_any_; }
  // The last read from the socket waited out its timeout (as opposed to EOF or an error).
  bool timed_out() const { return last_ == -2; }

 private:
  ssize_t fill(int timeout_ms);
  net::Stream& s_;
  std::string buf_;
  size_t pos_ = 0;
  bool consumed_any_ = false;
  ssize_t last_ = 1;
};

// ---------------------------------------------------------------------------
// Server

// HTTP/1.1 response on the connection's stream; the HTTP/2 writer (http.cc) overrides
// every I/O method to emit HEADERS/DATA frames on its stream instead.
class ResponseWriter {
 public:
  ResponseWriter(net::Stream* s, bool keep_alive, const CancelToken& server_stop)
      : s_(s), keep_alive_(keep_alive), stop_(server_stop) {}
  virtual ~ResponseWriter() = default;
  virtual void send(int status, std::string_view body, const std::string& content_type = "text/plain; charset=utf-8",
                    const Headers* extra = nullptr);
  void send_json(int status, std::string_view body) { send(status, body, "application/json"); }
  // Streaming (chunked) responses for WATCH.
  virtual bool start_chunked(int status, const std::string& content_type);
  virtual bool write_chunk(const std::string& data);
  virtual void end_chunked();
  // Drops the connection without a response (fault injection: connection reset); over
  // HTTP/2 only the request's stream is reset.
  virtual void abort();
  bool sent() const { return sent_; }
  int status_code() const { return status_; }  // 0 until a response (or stream) has started
  bool keep_alive() const { return keep_alive_; }
  // True once the server is shutting down; streaming handlers should return.
  bool stopping() const { return stop_.cancelled(); }
  // Sleeps up to `d`; true (early) once the server is shutting down.
  bool wait_stopping(std::chrono::milliseconds d) const { return stop_.wait_for(d); }
  // Non-blocking peer liveness probe for long-lived streams.
  virtual bool peer_closed();
  // "HTTP/1.1" or "HTTP/2".
  virtual const char* protocol() const { return "HTTP/1.1"; }

 protected:
  net::Stream* s_;
  bool keep_alive_;
  const CancelToken& stop_;
  bool sent_ = false;
  bool chunked_ = false;
  int status_ = 0;
};

using Handler = std::function<void(Request&, ResponseWriter&)>;

struct ServerOptions {
  std::string addr = "0.0.0.0";
  uint16_t port = 0;
  std::shared_ptr<net::TlsContext> tls;  // null = plain HTTP
  size_t max_body = 64 << 20;
  int idle_timeout_ms = 90000;
  int header_timeout_ms = 10000;
  size_t max_connections = 4096;
  std::string name = "http";
  // TLS servers: offer HTTP/2 by ALPN (enables it on `tls`); HTTP/1.1 clients unaffected.
  bool http2 = true;
  // HTTP/2: exact paths whose handlers may run on the connection's reader thread when no
  // other stream of that connection is in flight (saves the hand-off to a worker thread).
  // Only for short handlers that answer with one send(); a response the peer's flow-control
  // window cannot take at once is finished on a worker.
  std::vector<std::string> h2_inline_paths;
};

class Server {
 public:
  explicit Server(ServerOptions opts);
  ~Server();
  void handle(const std::string& method, const std::string& path, Handler h);
  // Fallback for any path with this prefix (longest prefix wins).
  void handle_prefix(const std::string& prefix, Handler h);
  void start();  // binds and spawns the accept thread; throws on bind failure
  uint16_t port() const { return port_; }
  // Stops accepting, waits up to `grace` for in-flight requests, then force-closes.
  void stop(std::chrono::milliseconds grace = std::chrono::milliseconds(10000));
  size_t active_connections() const { return active_.load(); }
  // HTTP/2 streams whose handler ran on the connection's reader thread (h2_inline_paths)
  uint64_t h2_inline_served() const { return h2_inline_.load(); }

 private:
  void accept_loop();
  void serve_conn(int fd, std::string remote);
  void serve_h2(int fd, std::unique_ptr<net::Stream> s, const std::string& remote);
  bool dispatch(Request& req, ResponseWriter& w);
  void handle_request(Request& req, ResponseWriter& w);

  ServerOptions opts_;
  std::map<std::pair<std::string, std::string>, Handler> exact_;
  std::vector<std::pair<std::string, Handler>> prefix_;
  int listen_fd_ = -1;
  int wake_pipe_[2] = {-1, -1};
  uint16_t port_ = 0;
  std::thread accept_thread_;
  CancelToken stop_;
  std::atomic<size_t> active_{0};
  std::mutex conns_mu_;
  std::condition_variable conns_cv_;
  std::map<int, net::Stream*> conns_;
  bool started_ = false;
  std::atomic<int64_t> grace_ms_{10000};  // stop()'s grace, for draining HTTP/2 connections
  struct WorkerPool;  // HTTP/2 stream workers (cached threads)
  std::shared_ptr<WorkerPool> h2_workers_;
  std::atomic<uint64_t> h2_inline_{0};
};

// Process-wide readiness checks served on /readyz: each returns false (with a reason in
// *why) while its subsystem cannot do its job, e.g. a watch that has gone silent
// (kube::Watcher).  Registering a name twice replaces the check.
using ReadinessCheck = std::function<bool(std::string* why)>;
void add_readiness_check(const std::string& name, ReadinessCheck check);
// Runs every check; *report gets one "[+]name ok" / "[-]name failed: why" line per check.
bool readiness(std::string* report = nullptr);

// Attaches `/health` (-> "pong"), `/readyz` (200 when every readiness check passes, 503
// otherwise), `/metrics` and, only when metrics::debug_endpoints_enabled()
// (CONF_DEBUG_ENDPOINTS=true), GET/DELETE `/debug/samples/<name>`.
void add_standard_routes(Server& s);

// ---------------------------------------------------------------------------
// Client

struct ClientOptions {
  std::string base_url;                   // http(s)://host:port
  std::shared_ptr<net::TlsContext> tls;   // required for https (defaults to system roots)
  std::string tls_server_name;            // override verify host (defaults to URL host)
  int connect_timeout_ms = 5000;
  int timeout_ms = 30000;
  size_t max_idle = 256;
  Headers default_headers;
  // https: offer h2 by ALPN; when the server selects it, request() calls are multiplexed
  // as streams on one connection (stream() keeps its own HTTP/1.1 connections).  A
  // server that answers with HTTP/1.1 gets the keep-alive pool as before.
  bool http2 = false;
  // HTTP/2 connections request() streams are spread over (round robin); 1 = one
  // multiplexed connection, as Go's client (and so the apiserver) uses.
  size_t h2_connections = 1;
  // HTTP/2: no reader thread per connection; the callers waiting for responses read the
  // frames themselves (http2::Connection::set_caller_reads).
  bool h2_caller_reads = false;
};

class HttpError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Client;
}  // namespace bgc::http
namespace bgc::http2 {
class Connection;
}
namespace bgc::http {

// A response whose body is consumed incrementally (chunked/line-delimited).
class StreamingResponse {
 public:
  int status = 0;
  Headers headers;
  // Next '\n'-terminated line (without the newline). false on end/error/cancel.
  bool next_line(std::string& line, const CancelToken* cancel = nullptr, int poll_ms = 500);
  // Reads the whole remaining body (non-2xx error bodies).
  std::string read_all(int timeout_ms = 10000);
  void close();
  // Idle deadline: no body byte for `ms` ends the stream (next_line returns false and
  // idle_timed_out() turns true), so a peer or path that silently stops sending cannot hold
  // the reader forever.  0 (the default) = wait indefinitely.
  void set_idle_timeout(int ms) { idle_ms_ = ms; }
  bool idle_timed_out() const { return idle_timed_out_; }
  ~StreamingResponse();

 private:
  friend class Client;
  bool pull(const CancelToken* cancel, int poll_ms);
  // true (and the stream ends) once the idle deadline has passed
  bool idle_expired();
  std::unique_ptr<net::Stream> stream_;
  std::unique_ptr<Reader> reader_;
  bool chunked_ = false;
  int64_t remaining_ = -1;  // content-length mode
  bool done_ = false;
  std::string pending_;
  int idle_ms_ = 0;
  int64_t last_data_ns_ = 0;
  bool idle_timed_out_ = false;
};

class Client {
 public:
  explicit Client(ClientOptions opts);
  ~Client();
  Response request(const std::string& method, const std::string& path, const std::string& body = "",
                   const Headers* headers = nullptr, int timeout_ms = -1);
  std::unique_ptr<StreamingResponse> stream(const std::string& method, const std::string& path,
                                            const Headers* headers = nullptr, const std::string& body = "");
  const Url& url() const { return url_; }
  void set_default_header(const std::string& name, const std::string& value);
  void close_idle();

 private:
  std::unique_ptr<net::Stream> connect();
  std::unique_ptr<net::Stream> take_idle();
  void give_back(std::unique_ptr<net::Stream> s);
  std::string build_request(const std::string& method, const std::string& path, const std::string& body,
                            const Headers* headers);
  Headers merged_headers(const Headers* headers);
  std::shared_ptr<http2::Connection> h2_connection();
  // false: HTTP/2 not available for this request (fall back to HTTP/1.1)
  bool request_h2(const std::string& method, const std::string& path, const std::string& body,
                  const Headers* headers, int timeout_ms, Response* out);

  ClientOptions opts_;
  Url url_;
  std::mutex mu_;
  std::vector<std::unique_ptr<net::Stream>> idle_;
  std::mutex h2_mu_;
  std::vector<std::shared_ptr<http2::Connection>> h2_;
  size_t h2_next_ = 0;
  bool h2_refused_ = false;  // the server selected HTTP/1.1
};

// One-shot convenience (no pooling).
Response fetch(const std::string& method, const std::string& url, const std::string& body = "",
               const Headers* headers = nullptr, std::shared_ptr<net::TlsContext> tls = nullptr,
               int timeout_ms = 30000);

}  // namespace bgc::http

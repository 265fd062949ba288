#include "core/http.h"

#include <cerrno>

#include <openssl/crypto.h>

#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <arpa/inet.h>
#include <cctype>
#include <charconv>
#include <cstring>
#include <deque>

#include "core/http2.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/stall.h"
#include "core/trace.h"
#include "core/process.h"

namespace bgc::http {

static bool ieq(const std::string& a, const std::string& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i) {
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i]))) return false;
  }
  return true;
}

static std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

void Headers::set(const std::string& name, std::string value) {
  remove(name);
  add(name, std::move(value));
}

const std::string* Headers::get(const std::string& name) const {
  for (const auto& kv : items_) {
    if (ieq(kv.first, name)) return &kv.second;
  }
  return nullptr;
}

std::string Headers::get_or(const std::string& name, const std::string& dflt) const {
  const std::string* v = get(name);
  return v ? *v : dflt;
}

void Headers::remove(const std::string& name) {
  items_.erase(std::remove_if(items_.begin(), items_.end(), [&](auto& kv) { return ieq(kv.first, name); }),
               items_.end());
}

const char* status_text(int code) {
  switch (code) {
    case 100: return "Continue";
    case 200: return "OK";
    case 201: return "Created";
    case 202: return "Accepted";
    case 204: return "No Content";
    case 301: return "Moved Permanently";
    case 302: return "Found";
    case 304: return "Not Modified";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 406: return "Not Acceptable";
    case 408: return "Request Timeout";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Unknown";
  }
}

std::string url_encode(const std::string& s, bool keep_slash) {
  static const char kHex[] = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~' || (keep_slash && c == '/')) {
      out.push_back(static_cast<char>(c));
    } else {
      out.push_back('%');
      out.push_back(kHex[c >> 4]);
      out.push_back(kHex[c & 15]);
    }
  }
  return out;
}

std::string url_decode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      int v = 0;
      auto r = std::from_chars(s.data() + i + 1, s.data() + i + 3, v, 16);
      if (r.ec == std::errc() && r.ptr == s.data() + i + 3) {
        out.push_back(static_cast<char>(v));
        i += 2;
        continue;
      }
    }
    out.push_back(s[i] == '+' ? ' ' : s[i]);
  }
  return out;
}

std::map<std::string, std::string> Request::query_params() const {
  std::map<std::string, std::string> out;
  size_t start = 0;
  while (start < query.size()) {
    size_t amp = query.find('&', start);
    std::string kv = query.substr(start, amp == std::string::npos ? std::string::npos : amp - start);
    size_t eq = kv.find('=');
    if (!kv.empty()) {
      if (eq == std::string::npos) out[url_decode(kv)] = "";
      else out[url_decode(kv.substr(0, eq))] = url_decode(kv.substr(eq + 1));
    }
    if (amp == std::string::npos) break;
    start = amp + 1;
  }
  return out;
}

// Single-key lookups scan the raw query (no map): the last occurrence wins, as with
// query_params().  Keys are decoded only when they contain an escape.
static bool find_query_param(const std::string& query, const std::string& name, std::string* value) {
  bool found = false;
  size_t start = 0;
  while (start < query.size()) {
    size_t amp = query.find('&', start);
    size_t end = amp == std::string::npos ? query.size() : amp;
    size_t eq = query.find('=', start);
    if (eq == std::string::npos || eq > end) eq = end;
    std::string_view key(query.data() + start, eq - start);
    bool match = key.find_first_of("%+") == std::string_view::npos ? key == name
                                                                    : url_decode(std::string(key)) == name;
    if (match && end > start) {
      found = true;
      if (value) *value = eq < end ? url_decode(query.substr(eq + 1, end - eq - 1)) : "";
    }
    if (amp == std::string::npos) break;
    start = amp + 1;
  }
  return found;
}

std::string Request::query_param(const std::string& name, const std::string& dflt) const {
  std::string v;
  return find_query_param(query, name, &v) ? v : dflt;
}

bool Request::has_query_param(const std::string& name) const { return find_query_param(query, name, nullptr); }

Url parse_url(const std::string& url) {
  Url u;
  size_t p = url.find("://");
  if (p == std::string::npos) throw HttpError("invalid URL (no scheme): " + url);
  u.scheme = lower(url.substr(0, p));
  std::string rest = url.substr(p + 3);
  size_t slash = rest.find('/');
  std::string hostport = rest.substr(0, slash);
  u.path = slash == std::string::npos ? "" : rest.substr(slash);
  size_t at = hostport.rfind('@');
  if (at != std::string::npos) hostport = hostport.substr(at + 1);
  if (!hostport.empty() && hostport[0] == '[') {
    size_t rb = hostport.find(']');
    u.host = hostport.substr(1, rb - 1);
    if (rb + 1 < hostport.size() && hostport[rb + 1] == ':') u.port = static_cast<uint16_t>(std::stoi(hostport.substr(rb + 2)));
  } else {
    size_t colon = hostport.rfind(':');
    if (colon != std::string::npos) {
      u.host = hostport.substr(0, colon);
      u.port = static_cast<uint16_t>(std::stoi(hostport.substr(colon + 1)));
    } else {
      u.host = hostport;
    }
  }
  if (u.port == 0) u.port = u.scheme == "https" ? 443 : 80;
  if (u.scheme != "http" && u.scheme != "https") throw HttpError("unsupported scheme: " + u.scheme);
  return u;
}

// ---------------------------------------------------------------------------
// Reader

ssize_t Reader::fill(int timeout_ms) {
  if (pos_ > 0 && pos_ == buf_.size()) {
    buf_.clear();
    pos_ = 0;
  } else if (pos_ > (1 << 16)) {
    buf_.erase(0, pos_);
    pos_ = 0;
  }
  char tmp[16384];
  ssize_t r = s_.read_some(tmp, sizeof(tmp), timeout_ms);
  last_ = r;
  if (r > 0) {
    buf_.append(tmp, static_cast<size_t>(r));
    consumed_any_ = true;
  }
  return r;
}

bool Reader::read_line(std::string& line, int timeout_ms, size_t max_len) {
  while (true) {
    size_t nl = buf_.find('\n', pos_);
    if (nl != std::string::npos) {
      size_t end = nl;
      if (end > pos_ && buf_[end - 1] == '\r') --end;
      line.assign(buf_, pos_, end - pos_);
      pos_ = nl + 1;
      return true;
    }
    if (buf_.size() - pos_ > max_len) return false;
    ssize_t r = fill(timeout_ms);
    if (r <= 0) return false;
  }
}

bool Reader::read_exact(std::string& out, size_t n, int timeout_ms) {
  while (buf_.size() - pos_ < n) {
    ssize_t r = fill(timeout_ms);
    if (r <= 0) return false;
  }
  out.append(buf_, pos_, n);
  pos_ += n;
  return true;
}

ssize_t Reader::read_available(std::string& out, int timeout_ms) {
  if (pos_ < buf_.size()) {
    size_t n = buf_.size() - pos_;
    out.append(buf_, pos_, n);
    pos_ = buf_.size();
    return static_cast<ssize_t>(n);
  }
  ssize_t r = fill(timeout_ms);
  if (r <= 0) return r;
  size_t n = buf_.size() - pos_;
  out.append(buf_, pos_, n);
  pos_ = buf_.size();
  return static_cast<ssize_t>(n);
}

static bool parse_headers(Reader& r, Headers& h, int timeout_ms) {
  std::string line;
  for (int i = 0; i < 256; ++i) {
    if (!r.read_line(line, timeout_ms)) return false;
    if (line.empty()) return true;
    size_t c = line.find(':');
    if (c == std::string::npos) return false;
    std::string v = line.substr(c + 1);
    size_t a = v.find_first_not_of(" \t");
    v = a == std::string::npos ? "" : v.substr(a);
    while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.pop_back();
    h.add(line.substr(0, c), v);
  }
  return false;
}

static bool read_chunked(Reader& r, std::string& body, int timeout_ms, size_t max_body) {
  std::string line;
  while (true) {
    if (!r.read_line(line, timeout_ms)) return false;
    size_t semi = line.find(';');
    std::string hex = line.substr(0, semi);
    size_t n = 0;
    auto res = std::from_chars(hex.data(), hex.data() + hex.size(), n, 16);
    if (res.ec != std::errc()) return false;
    if (n == 0) {
      // trailers
      while (r.read_line(line, timeout_ms)) {
        if (line.empty()) return true;
      }
      return false;
    }
    if (body.size() + n > max_body) return false;
    if (!r.read_exact(body, n, timeout_ms)) return false;
    if (!r.read_line(line, timeout_ms)) return false;
  }
}

// ---------------------------------------------------------------------------
// Server

// Cached worker threads for HTTP/2 request streams: a stream is handed to an idle
// worker, or to a new one when none is idle; a worker exits after 30 s without work.
// Shared with the workers, so it outlives the Server if a worker is still winding down.
struct Server::WorkerPool {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  size_t idle = 0;

  static void run(const std::shared_ptr<WorkerPool>& self) {
    std::unique_lock<std::mutex> lk(self->mu);
    while (true) {
      ++self->idle;
      bool got = self->cv.wait_for(lk, std::chrono::seconds(30), [&] { return !self->q.empty(); });
      --self->idle;
      if (!got) break;
      auto job = std::move(self->q.front());
      self->q.pop_front();
      lk.unlock();
      job();
      job = nullptr;
      lk.lock();
    }
    lk.unlock();
    OPENSSL_thread_stop();  // handlers may have made TLS calls of their own (see below)
  }
  static void submit(const std::shared_ptr<WorkerPool>& self, std::function<void()> job) {
    bool spawn;
    {
      std::lock_guard<std::mutex> lk(self->mu);
      self->q.push_back(std::move(job));
      spawn = self->idle < self->q.size();
    }
    if (spawn) {
      std::thread([self] {
        set_thread_name("h2-worker");
        run(self);
      }).detach();
    }
    else self->cv.notify_one();
  }
};

void ResponseWriter::abort() {
  s_->shutdown();
  sent_ = true;
  keep_alive_ = false;
}

void ResponseWriter::send(int status, std::string_view body, const std::string& content_type,
                          const Headers* extra) {
  status_ = status;
  if (sent_) return;
  sent_ = true;
  std::string out;
  out.reserve(body.size() + 160);
  out.append("HTTP/1.1 ").append(std::to_string(status)).append(" ").append(status_text(status)).append("\r\n");
  if (!content_type.empty()) out.append("Content-Type: ").append(content_type).append("\r\n");
  out.append("Content-Length: ").append(std::to_string(body.size())).append("\r\n");
  if (extra) {
    for (auto& kv : extra->items()) out.append(kv.first).append(": ").append(kv.second).append("\r\n");
  }
  out.append(keep_alive_ ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
  out.append(body);
  s_->write_all(out);
}

bool ResponseWriter::start_chunked(int status, const std::string& content_type) {
  status_ = status;
  if (sent_) return false;
  sent_ = true;
  chunked_ = true;
  keep_alive_ = false;  // long-lived stream: close afterwards
  std::string out = "HTTP/1.1 " + std::to_string(status) + " " + status_text(status) + "\r\n";
  out += "Content-Type: " + content_type + "\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n";
  return s_->write_all(out);
}

bool ResponseWriter::write_chunk(const std::string& data) {
  if (data.empty()) return true;
  char hdr[32];
  int n = std::snprintf(hdr, sizeof(hdr), "%zx\r\n", data.size());
  std::string out;
  out.reserve(data.size() + 16);
  out.append(hdr, static_cast<size_t>(n)).append(data).append("\r\n");
  return s_->write_all(out);
}

void ResponseWriter::end_chunked() {
  if (chunked_) s_->write_all("0\r\n\r\n", 5);
}

bool ResponseWriter::peer_closed() {
  struct pollfd p {};
  p.fd = s_->fd();
  p.events = POLLIN | POLLRDHUP;
  int r = ::poll(&p, 1, 0);
  if (r <= 0) return false;
  if (p.revents & (POLLHUP | POLLERR | POLLRDHUP)) return true;
  if (p.revents & POLLIN) {
    char c;
    ssize_t n = ::recv(s_->fd(), &c, 1, MSG_PEEK | MSG_DONTWAIT);
    return n == 0;
  }
  return false;
}

Server::Server(ServerOptions opts) : opts_(std::move(opts)) {}

Server::~Server() {
  if (started_) stop(std::chrono::milliseconds(0));
}

void Server::handle(const std::string& method, const std::string& path, Handler h) {
  exact_[{method, path}] = std::move(h);
}

void Server::handle_prefix(const std::string& prefix, Handler h) {
  prefix_.emplace_back(prefix, std::move(h));
  std::stable_sort(prefix_.begin(), prefix_.end(),
                   [](const auto& a, const auto& b) { return a.first.size() > b.first.size(); });
}

void Server::start() {
  if (opts_.tls && opts_.http2) {
    opts_.tls->enable_h2();
    h2_workers_ = std::make_shared<WorkerPool>();
  }
  listen_fd_ = net::listen_tcp(opts_.addr, opts_.port, 1024, &port_);
  if (::pipe2(wake_pipe_, O_CLOEXEC) != 0) throw net::NetError("pipe2 failed");
  started_ = true;
  accept_thread_ = std::thread([this] { accept_loop(); });
}

void Server::accept_loop() {
  while (!stop_.cancelled()) {
    struct pollfd fds[2] = {};
    fds[0].fd = listen_fd_;
    fds[0].events = POLLIN;
    fds[1].fd = wake_pipe_[0];
    fds[1].events = POLLIN;
    int r = ::poll(fds, 2, 1000);
    if (r < 0 && errno != EINTR) break;
    if (r <= 0) continue;
    if (fds[1].revents) break;
    if (!(fds[0].revents & POLLIN)) continue;
    struct sockaddr_storage ss {};
    socklen_t len = sizeof(ss);
    int fd = ::accept4(listen_fd_, reinterpret_cast<sockaddr*>(&ss), &len, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, 1 /*TCP_NODELAY*/, &one, sizeof(one));
    char host[INET6_ADDRSTRLEN] = {0};
    if (ss.ss_family == AF_INET) {
      inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(&ss)->sin_addr, host, sizeof(host));
    } else {
      inet_ntop(AF_INET6, &reinterpret_cast<sockaddr_in6*>(&ss)->sin6_addr, host, sizeof(host));
    }
    if (active_.load() >= opts_.max_connections) {
      ::close(fd);
      continue;
    }
    active_.fetch_add(1);
    std::thread([this, fd, remote = std::string(host)] {
      set_thread_name(opts_.name.empty() ? "conn" : "conn:" + opts_.name);
      serve_conn(fd, remote);
      // OpenSSL keeps per-thread state (the thread's public/private DRBGs, its error queue)
      // that OPENSSL_thread_stop() releases at once (found by LeakSanitizer, tools/sanitize.sh
      // asan).  Also on a plain-HTTP server: a handler may have used TLS as a client (kube-lite's
      // webhook callouts).
      OPENSSL_thread_stop();
      // notify under the lock: once stop() observes active_==0 the Server (and the cv) may be destroyed
      std::lock_guard<std::mutex> lk(conns_mu_);
      active_.fetch_sub(1);
      conns_cv_.notify_all();
    }).detach();
  }
}

void Server::serve_conn(int fd, std::string remote) {
  std::unique_ptr<net::Stream> s;
  try {
    if (opts_.tls) {
      s = std::make_unique<net::TlsStream>(fd, opts_.tls->get(), true, "", false, opts_.header_timeout_ms);
    } else {
      s = std::make_unique<net::TcpStream>(fd);
    }
  } catch (const std::exception& e) {
    LOG_DEBUG(opts_.name) << "connection setup failed from " << remote << ": " << e.what();
    return;
  }
  {
    std::lock_guard<std::mutex> lk(conns_mu_);
    conns_[fd] = s.get();
  }
  std::string peer_cn;
  std::vector<std::string> peer_orgs;
  s->peer_identity(&peer_cn, &peer_orgs);
  if (opts_.tls && opts_.http2 && static_cast<net::TlsStream&>(*s).alpn() == "h2") {
    serve_h2(fd, std::move(s), remote);  // unregisters the stream before releasing it
    return;
  }
  Reader r(*s);
  while (!stop_.cancelled()) {
    Request req;
    req.remote = remote;
    req.peer_cn = peer_cn;
    req.peer_orgs = peer_orgs;
    std::string line;
    // wait for the request line, waking periodically to observe shutdown
    int idle = 0;
    bool got = false;
    while (!stop_.cancelled()) {
      if (r.read_line(line, 500)) {
        got = true;
        break;
      }
      // read_line false: timeout (no new bytes) or EOF/error. Distinguish by polling.
      struct pollfd p {};
      p.fd = fd;
      p.events = POLLIN;
      if (!r.buffered() && ::poll(&p, 1, 0) > 0) {
        char c;
        ssize_t n = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
        if (n <= 0) break;  // peer closed
        continue;
      }
      idle += 500;
      if (idle >= opts_.idle_timeout_ms) break;
    }
    if (!got) break;
    if (line.empty()) continue;  // tolerate stray CRLF between requests
    size_t sp1 = line.find(' ');
    size_t sp2 = line.rfind(' ');
    if (sp1 == std::string::npos || sp2 == sp1) break;
    req.method = line.substr(0, sp1);
    req.target = line.substr(sp1 + 1, sp2 - sp1 - 1);
    std::string version = line.substr(sp2 + 1);
    if (!parse_headers(r, req.headers, opts_.header_timeout_ms)) break;
    size_t q = req.target.find('?');
    req.path = url_decode(req.target.substr(0, q));
    req.query = q == std::string::npos ? "" : req.target.substr(q + 1);
    bool keep_alive = version == "HTTP/1.1";
    if (const std::string* c = req.headers.get("Connection")) {
      std::string lc = lower(*c);
      if (lc.find("close") != std::string::npos) keep_alive = false;
      if (lc.find("keep-alive") != std::string::npos) keep_alive = true;
    }
    if (const std::string* ex = req.headers.get("Expect")) {
      if (lower(*ex) == "100-continue") s->write_all("HTTP/1.1 100 Continue\r\n\r\n");
    }
    bool body_ok = true;
    if (const std::string* te = req.headers.get("Transfer-Encoding"); te && lower(*te).find("chunked") != std::string::npos) {
      body_ok = read_chunked(r, req.body, opts_.header_timeout_ms, opts_.max_body);
    } else if (const std::string* cl = req.headers.get("Content-Length")) {
      size_t n = 0;
      auto res = std::from_chars(cl->data(), cl->data() + cl->size(), n);
      if (res.ec != std::errc() || n > opts_.max_body) {
        ResponseWriter w(s.get(), false, stop_);
        w.send(413, "request body too large\n");
        break;
      }
      body_ok = r.read_exact(req.body, n, opts_.header_timeout_ms);
    }
    if (!body_ok) break;
    ResponseWriter w(s.get(), keep_alive && !stop_.cancelled(), stop_);
    handle_request(req, w);
    if (!w.keep_alive()) break;
  }
  {
    std::lock_guard<std::mutex> lk(conns_mu_);
    conns_.erase(fd);
  }
}

void Server::handle_request(Request& req, ResponseWriter& w) {
  try {
    if (!dispatch(req, w)) w.send(404, "404 page not found\n");
  } catch (const std::exception& e) {
    LOG_ERROR(opts_.name) << "handler error for " << req.method << " " << req.path << ": " << e.what();
    if (!w.sent()) w.send(500, std::string("internal error: ") + e.what() + "\n");
  }
  if (!w.sent()) w.send(500, "handler produced no response\n");
}

// ---------------------------------------------------------------------------
// HTTP/2 (ALPN "h2" over TLS)

namespace {

bool h2_forbidden_header(const std::string& lname) {
  // connection-specific fields are malformed in HTTP/2 (RFC 9113 section 8.2.2)
  return lname == "connection" || lname == "keep-alive" || lname == "transfer-encoding" || lname == "upgrade" ||
         lname == "proxy-connection";
}

class H2ResponseWriter final : public ResponseWriter {
 public:
  // `blocked_send`: set when the handler runs on the connection's reader thread, which
  // must never wait for a WINDOW_UPDATE it alone can read; a response that does not fit
  // the peer's window is handed to it (a worker finishes the send).
  using BlockedSend = std::function<void(hpack::HeaderList, std::string)>;
  H2ResponseWriter(std::shared_ptr<http2::Connection> c, std::shared_ptr<http2::Stream> st, const CancelToken& stop,
                   BlockedSend blocked_send = nullptr)
      : ResponseWriter(nullptr, true, stop), c_(std::move(c)), st_(std::move(st)), blocked_send_(std::move(blocked_send)) {}

  void send(int status, std::string_view body, const std::string& content_type, const Headers* extra) override {
    status_ = status;
    if (sent_) return;
    sent_ = true;
    hpack::HeaderList h = head(status, content_type, extra);
    h.emplace_back("content-length", std::to_string(body.size()));
    if (!blocked_send_) {
      c_->send_response(*st_, h, body);
    } else if (c_->try_send_response(*st_, h, body) == http2::Connection::SendResult::kWouldBlock) {
      blocked_send_(std::move(h), std::string(body));
    }
  }
  bool start_chunked(int status, const std::string& content_type) override {
    status_ = status;
    if (sent_) return false;
    if (blocked_send_) throw std::logic_error("streaming response from an inline HTTP/2 handler");
    sent_ = chunked_ = true;
    return c_->send_headers(*st_, head(status, content_type, nullptr), false);
  }
  bool write_chunk(const std::string& data) override { return data.empty() || c_->send_data(*st_, data, false); }
  void end_chunked() override {
    if (chunked_) c_->send_data(*st_, {}, true);
  }
  void abort() override {
    c_->reset_stream(*st_, http2::kInternalError);
    sent_ = true;
  }
  bool peer_closed() override { return c_->closed() || c_->locked([&] { return st_->reset; }); }
  const char* protocol() const override { return "HTTP/2"; }

 private:
  static hpack::HeaderList head(int status, const std::string& content_type, const Headers* extra) {
    hpack::HeaderList h;
    h.emplace_back(":status", std::to_string(status));
    if (!content_type.empty()) h.emplace_back("content-type", content_type);
    if (extra) {
      for (auto& kv : extra->items()) {
        std::string n = lower(kv.first);
        if (!h2_forbidden_header(n) && n != "content-length") h.emplace_back(std::move(n), kv.second);
      }
    }
    return h;
  }
  std::shared_ptr<http2::Connection> c_;
  std::shared_ptr<http2::Stream> st_;
  BlockedSend blocked_send_;
};

}  // namespace

void Server::serve_h2(int fd, std::unique_ptr<net::Stream> s, const std::string& remote) {
  static metrics::Counter& streams = metrics::Registry::global().counter(
      "bgc_http2_streams_total", "HTTP/2 request streams served (ALPN h2 over TLS)");
  // request complete on the reader thread -> handler returned (queueing + handler + write)
  static auto& server_time = metrics::Registry::global().samples("h2_server");
  struct Inflight {
    std::mutex mu;
    std::condition_variable cv;
    int n = 0;
  };
  auto inflight = std::make_shared<Inflight>();
  auto pool = h2_workers_;
  const size_t max_body = opts_.max_body;
  // one stream, start to finish: on a worker, or inline on the reader thread
  auto serve_stream = [this, inflight, pool, remote, max_body](const std::shared_ptr<http2::Connection>& c,
                                                                const std::shared_ptr<http2::Stream>& st, int64_t t0,
                                                                Request& req, bool ok, bool on_reader) {
    streams.inc();
    H2ResponseWriter::BlockedSend blocked;
    if (on_reader) {
      blocked = [inflight, pool, c, st](hpack::HeaderList h, std::string body) {
        {
          std::lock_guard<std::mutex> lk(inflight->mu);
          ++inflight->n;
        }
        WorkerPool::submit(pool, [inflight, c, st, h = std::move(h), body = std::move(body)] {
          c->send_response(*st, h, body);
          std::lock_guard<std::mutex> lk(inflight->mu);
          --inflight->n;
          inflight->cv.notify_all();
        });
      };
    }
    H2ResponseWriter h2w(c, st, stop_, std::move(blocked));
    ResponseWriter& w = h2w;
    if (ok) {
      if (req.method.empty() || req.target.empty()) w.send(400, "missing :method or :path\n");
      else if (req.body.size() > max_body) w.send(413, "request body too large\n");
      else handle_request(req, w);
    }
    server_time.add(static_cast<double>(metrics::now_ns() - t0) * 1e-9);
  };
  std::string peer_cn;
  std::vector<std::string> peer_orgs;
  s->peer_identity(&peer_cn, &peer_orgs);
  auto take_request = [remote, peer_cn, peer_orgs](const std::shared_ptr<http2::Connection>& c,
                                                  const std::shared_ptr<http2::Stream>& st, Request& req) {
    req.remote = remote;
    req.peer_cn = peer_cn;
    req.peer_orgs = peer_orgs;
    bool ok = c->locked([&] {
      for (auto& [k, v] : st->headers) {
        if (k == ":method") req.method = v;
        else if (k == ":path") req.target = v;
        else if (!k.empty() && k[0] != ':') req.headers.add(k, v);
      }
      req.body = std::move(st->data);
      return !st->reset;
    });
    size_t q = req.target.find('?');
    req.path = url_decode(req.target.substr(0, q));
    req.query = q == std::string::npos ? "" : req.target.substr(q + 1);
    return ok;
  };
  const bool any_inline = !opts_.h2_inline_paths.empty();
  auto conn = std::make_shared<http2::Connection>(
      std::move(s), http2::Connection::Role::kServer,
      [this, inflight, pool, serve_stream, take_request, any_inline](std::shared_ptr<http2::Connection> c,
                                                                     std::shared_ptr<http2::Stream> st) {
        const int64_t t0 = metrics::now_ns();
        bool idle;
        {
          std::lock_guard<std::mutex> lk(inflight->mu);
          idle = inflight->n == 0;
          ++inflight->n;
        }
        if (idle && any_inline) {
          auto req = std::make_shared<Request>();
          const bool ok = take_request(c, st, *req);
          const auto& paths = opts_.h2_inline_paths;
          if (std::find(paths.begin(), paths.end(), req->path) != paths.end()) {
            h2_inline_.fetch_add(1, std::memory_order_relaxed);
            serve_stream(c, st, t0, *req, ok, /*on_reader=*/true);
            std::lock_guard<std::mutex> lk(inflight->mu);
            --inflight->n;
            inflight->cv.notify_all();
            return;
          }
          WorkerPool::submit(pool, [inflight, serve_stream, t0, ok, c = std::move(c), st = std::move(st),
                                    req = std::move(req)] {
            serve_stream(c, st, t0, *req, ok, false);
            std::lock_guard<std::mutex> lk(inflight->mu);
            --inflight->n;
            inflight->cv.notify_all();
          });
          return;
        }
        WorkerPool::submit(pool, [inflight, serve_stream, take_request, t0, c = std::move(c), st = std::move(st)] {
          Request req;
          const bool ok = take_request(c, st, req);
          serve_stream(c, st, t0, req, ok, false);
          std::lock_guard<std::mutex> lk(inflight->mu);
          --inflight->n;
          inflight->cv.notify_all();
        });
      });
  conn->start();
  // Runs until the peer goes away, the server stops, or the connection idles out.
  uint64_t frames = conn->frames_received();
  int idle = 0;
  // (polled: waiting on the connection's condition variable would wake this thread on
  // every frame)
  while (!conn->closed()) {
    if (stop_.wait_for(std::chrono::milliseconds(250))) break;
    const uint64_t now = conn->frames_received();
    bool busy;
    {
      std::lock_guard<std::mutex> lk(inflight->mu);
      busy = inflight->n > 0;
    }
    idle = (now != frames || busy) ? 0 : idle + 250;
    frames = now;
    if (idle >= opts_.idle_timeout_ms) break;
  }
  if (stop_.cancelled() && !conn->closed()) {
    // graceful: GOAWAY, let the streams in flight finish (bounded by stop()'s grace)
    conn->drain();
    std::unique_lock<std::mutex> lk(inflight->mu);
    inflight->cv.wait_for(lk, std::chrono::milliseconds(grace_ms_.load()), [&] { return inflight->n == 0; });
  }
  conn->close();
  conn->join();  // no stream is dispatched after this
  {
    // handlers see their streams reset and return; the server must outlive them
    std::unique_lock<std::mutex> lk(inflight->mu);
    inflight->cv.wait(lk, [&] { return inflight->n == 0; });
  }
  std::lock_guard<std::mutex> lk(conns_mu_);
  conns_.erase(fd);
}

bool Server::dispatch(Request& req, ResponseWriter& w) {
  auto it = exact_.find({req.method, req.path});
  if (it != exact_.end()) {
    it->second(req, w);
    return true;
  }
  bool path_known = false;
  for (auto& kv : exact_) {
    if (kv.first.second == req.path) path_known = true;
  }
  for (auto& [prefix, h] : prefix_) {
    if (req.path.compare(0, prefix.size(), prefix) == 0) {
      h(req, w);
      return true;
    }
  }
  if (path_known) {
    w.send(405, "method not allowed\n");
    return true;
  }
  return false;
}

void Server::stop(std::chrono::milliseconds grace) {
  if (!started_) return;
  grace_ms_ = grace.count();
  stop_.cancel();
  if (wake_pipe_[1] >= 0) {
    char c = 1;
    (void)!::write(wake_pipe_[1], &c, 1);
  }
  if (accept_thread_.joinable()) accept_thread_.join();
  if (listen_fd_ >= 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
  }
  {
    std::unique_lock<std::mutex> lk(conns_mu_);
    conns_cv_.wait_for(lk, grace, [&] { return active_.load() == 0; });
    for (auto& kv : conns_) kv.second->shutdown();
    conns_cv_.wait_for(lk, std::chrono::milliseconds(2000), [&] { return active_.load() == 0; });
  }
  for (int& p : wake_pipe_) {
    if (p >= 0) ::close(p);
    p = -1;
  }
  started_ = false;
}

namespace {
std::mutex g_ready_mu;
std::vector<std::pair<std::string, ReadinessCheck>> g_ready_checks;
}  // namespace

void add_readiness_check(const std::string& name, ReadinessCheck check) {
  std::lock_guard<std::mutex> lk(g_ready_mu);
  for (auto& [n, c] : g_ready_checks) {
    if (n == name) {
      c = std::move(check);
      return;
    }
  }
  g_ready_checks.emplace_back(name, std::move(check));
}

bool readiness(std::string* report) {
  std::vector<std::pair<std::string, ReadinessCheck>> checks;
  {
    std::lock_guard<std::mutex> lk(g_ready_mu);
    checks = g_ready_checks;
  }
  bool ok = true;
  std::string out;
  for (const auto& [name, check] : checks) {
    std::string why;
    const bool pass = check(&why);
    ok = ok && pass;
    out += std::string(pass ? "[+]" : "[-]") + name + (pass ? " ok" : " failed: " + why) + "\n";
  }
  if (report) *report = out + (ok ? "readyz check passed\n" : "readyz check failed\n");
  return ok;
}

void add_standard_routes(Server& s) {
  // /health stays the reference's unconditional "pong" (liveness; controller.rs:256,
  // admission.rs:151); /readyz reports the registered readiness checks, in the
  // kube-apiserver's /readyz text format.
  s.handle("GET", "/health", [](Request&, ResponseWriter& w) { w.send(200, "pong"); });
  s.handle("GET", "/readyz", [](Request&, ResponseWriter& w) {
    std::string report;
    const bool ok = readiness(&report);
    w.send(ok ? 200 : 503, report);
  });
  s.handle("GET", "/metrics", [](Request&, ResponseWriter& w) {
    w.send(200, metrics::Registry::global().render(), "text/plain; version=0.0.4");
  });
  // Raw latency samples are a test/bench surface: off unless CONF_DEBUG_ENDPOINTS=true (the
  // reference serves only /mutate and /health, admission.rs:149-152).  A request never
  // creates a log: unknown names are 404.
  if (!metrics::debug_endpoints_enabled()) return;
  s.handle_prefix("/debug/samples/", [](Request& r, ResponseWriter& w) {
    std::string name = r.path.substr(std::strlen("/debug/samples/"));
    std::string body;
    if (r.method == "DELETE") body = metrics::Registry::global().clear_samples_json(name);
    else if (r.method == "GET") body = metrics::Registry::global().render_samples_json(name);
    else return w.send(405, "method not allowed\n");
    if (body.empty()) return w.send(404, "no such sample log\n");
    w.send(200, body, "application/json");
  });
  // Per-tenant stage marks (core/trace.h): POST <prefix> arms, GET reads, DELETE takes.
  s.handle("POST", "/debug/trace", [](Request& r, ResponseWriter& w) {
    trace::arm(r.body);
    w.send(200, "armed\n");
  });
  s.handle("GET", "/debug/trace", [](Request&, ResponseWriter& w) { w.send(200, trace::dump_json(false), "application/json"); });
  s.handle("DELETE", "/debug/trace", [](Request&, ResponseWriter& w) { w.send(200, trace::dump_json(true), "application/json"); });
  // Stalls the process's stall sampler kept (core/stall.h): GET reads, DELETE takes.
  s.handle("GET", "/debug/stalls", [](Request&, ResponseWriter& w) { w.send(200, stall::dump_json(false), "application/json"); });
  s.handle("DELETE", "/debug/stalls", [](Request&, ResponseWriter& w) { w.send(200, stall::dump_json(true), "application/json"); });
}

// ---------------------------------------------------------------------------
// Client

Client::~Client() = default;

Client::Client(ClientOptions opts) : opts_(std::move(opts)) {
  url_ = parse_url(opts_.base_url);
  if (url_.scheme == "https" && !opts_.tls) opts_.tls = net::TlsContext::client("", false);
}

void Client::set_default_header(const std::string& name, const std::string& value) {
  std::lock_guard<std::mutex> lk(mu_);
  opts_.default_headers.set(name, value);
}

void Client::close_idle() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    idle_.clear();
  }
  // multiplexed HTTP/2 connections too: the next request dials afresh (streams in flight
  // keep their connection alive until they end)
  std::lock_guard<std::mutex> lk(h2_mu_);
  h2_.clear();
}

std::unique_ptr<net::Stream> Client::connect() {
  int fd = net::connect_tcp(url_.host, url_.port, opts_.connect_timeout_ms);
  if (url_.scheme == "https") {
    std::string host = opts_.tls_server_name.empty() ? url_.host : opts_.tls_server_name;
    return std::make_unique<net::TlsStream>(fd, opts_.tls->get(), false, host, !opts_.tls->insecure(),
                                            opts_.connect_timeout_ms);
  }
  return std::make_unique<net::TcpStream>(fd);
}

std::unique_ptr<net::Stream> Client::take_idle() {
  std::lock_guard<std::mutex> lk(mu_);
  while (!idle_.empty()) {
    auto s = std::move(idle_.back());
    idle_.pop_back();
    // discard connections the server already closed
    struct pollfd p {};
    p.fd = s->fd();
    p.events = POLLIN;
    if (::poll(&p, 1, 0) > 0 && !s->has_buffered()) continue;
    return s;
  }
  return nullptr;
}

void Client::give_back(std::unique_ptr<net::Stream> s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (idle_.size() < opts_.max_idle) idle_.push_back(std::move(s));
}

std::string Client::build_request(const std::string& method, const std::string& path, const std::string& body,
                                  const Headers* headers) {
  std::string p = path.empty() ? "/" : path;
  std::string out;
  out.reserve(body.size() + 256);
  out.append(method).append(" ").append(p).append(" HTTP/1.1\r\n");
  out.append("Host: ").append(url_.host);
  if (!((url_.scheme == "http" && url_.port == 80) || (url_.scheme == "https" && url_.port == 443))) {
    out.append(":").append(std::to_string(url_.port));
  }
  out.append("\r\n");
  Headers merged = merged_headers(headers);
  for (auto& kv : merged.items()) out.append(kv.first).append(": ").append(kv.second).append("\r\n");
  if (!body.empty() || method == "POST" || method == "PUT" || method == "PATCH") {
    out.append("Content-Length: ").append(std::to_string(body.size())).append("\r\n");
  }
  out.append("\r\n").append(body);
  return out;
}

Headers Client::merged_headers(const Headers* headers) {
  Headers merged;
  {
    std::lock_guard<std::mutex> lk(mu_);
    merged = opts_.default_headers;
  }
  if (headers) {
    for (auto& kv : headers->items()) merged.set(kv.first, kv.second);
  }
  // client-go's convention: "<binary>/<version>" (an apiserver's audit log, and kube-lite's
  // default field manager and traces, name the component by it)
  static const std::string ua = std::string(program_invocation_short_name) + "/0.1";
  if (!merged.has("User-Agent")) merged.set("User-Agent", ua);
  return merged;
}

std::shared_ptr<http2::Connection> Client::h2_connection() {
  std::lock_guard<std::mutex> lk(h2_mu_);  // concurrent first requests share one handshake
  h2_.resize(std::max<size_t>(1, opts_.h2_connections));
  auto& slot = h2_[h2_next_++ % h2_.size()];
  if (slot && slot->usable() && (!opts_.h2_caller_reads || slot->poll_idle()) && slot->usable()) return slot;
  if (h2_refused_) return nullptr;
  int fd = net::connect_tcp(url_.host, url_.port, opts_.connect_timeout_ms);
  std::string host = opts_.tls_server_name.empty() ? url_.host : opts_.tls_server_name;
  auto ts = std::make_unique<net::TlsStream>(fd, opts_.tls->get(), false, host, !opts_.tls->insecure(),
                                             opts_.connect_timeout_ms, /*offer_h2=*/true);
  if (ts->alpn() != "h2") {
    h2_refused_ = true;
    give_back(std::move(ts));
    return nullptr;
  }
  slot = std::make_shared<http2::Connection>(std::move(ts), http2::Connection::Role::kClient);
  if (opts_.h2_caller_reads) slot->set_caller_reads();
  slot->start();
  return slot;
}

bool Client::request_h2(const std::string& method, const std::string& path, const std::string& body,
                        const Headers* headers, int timeout_ms, Response* out) {
  std::string authority = url_.host;
  if (!((url_.scheme == "http" && url_.port == 80) || (url_.scheme == "https" && url_.port == 443))) {
    authority += ":" + std::to_string(url_.port);
  }
  hpack::HeaderList h = {{":method", method}, {":scheme", url_.scheme}, {":authority", authority},
                         {":path", path.empty() ? "/" : path}};
  const Headers merged = merged_headers(headers);
  for (auto& kv : merged.items()) {
    std::string n = lower(kv.first);
    if (n != "host" && n != "content-length" && !h2_forbidden_header(n)) h.emplace_back(std::move(n), kv.second);
  }
  if (!body.empty() || method == "POST" || method == "PUT" || method == "PATCH") {
    h.emplace_back("content-length", std::to_string(body.size()));
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  for (int attempt = 0; attempt < 2; ++attempt) {
    auto c = h2_connection();
    if (!c) return false;
    auto st = c->open(h, body, true);
    if (!st) {
      if (c->usable()) return false;  // e.g. a header block beyond one frame: use HTTP/1.1
      continue;                       // the connection died or went away: a fresh one
    }
    c->wait_stream(*st, deadline, [&] { return st->remote_closed || st->reset; });
    bool done = false, refused = false, started = false;
    c->locked([&] {
      done = st->remote_closed && !st->reset;
      refused = st->reset && st->reset_code == http2::kRefusedStream;
      started = st->headers_received;
      if (done) {
        for (auto& [k, v] : st->headers) {
          if (k == ":status") out->status = std::atoi(v.c_str());
          else if (!k.empty() && k[0] != ':') out->headers.add(k, v);
        }
        out->body = std::move(st->data);
      }
      return 0;
    });
    if (done) return true;
    if (refused && !started) continue;  // RFC 9113 8.7: not processed, safe to retry
    if (!st->reset) c->reset_stream(*st, http2::kCancel);
    const bool timed_out = std::chrono::steady_clock::now() >= deadline;
    if (timed_out) close_idle();  // as over HTTP/1.1: the path may be dead
    throw HttpError(std::string(timed_out ? "timeout" : "stream reset") + " (HTTP/2): " + method + " " + path);
  }
  throw HttpError("request failed after retry (HTTP/2): " + method + " " + path);
}

Response Client::request(const std::string& method, const std::string& path, const std::string& body,
                         const Headers* headers, int timeout_ms) {
  int to = timeout_ms < 0 ? opts_.timeout_ms : timeout_ms;
  if (opts_.http2 && url_.scheme == "https") {
    Response resp;
    if (request_h2(method, path, body, headers, to, &resp)) return resp;
  }
  std::string wire = build_request(method, path, body, headers);
  for (int attempt = 0; attempt < 2; ++attempt) {
    // the retry dials afresh: when the server closed one pooled connection (its idle
    // timeout), it usually closed the ones opened with it too
    auto s = attempt == 0 ? take_idle() : nullptr;
    bool reused = s != nullptr;
    if (!s) s = connect();
    if (!s->write_all(wire)) {
      if (reused) continue;
      throw HttpError("write failed: " + method + " " + path);
    }
    Reader r(*s);
    std::string line;
    if (!r.read_line(line, to)) {
      if (r.timed_out()) {
        // No answer within the timeout: the path to the server may be dead (a wedged proxy,
        // a crashed host behind a stale NAT entry), and every pooled connection with it.
        // Drop them so the next request dials afresh; the request itself is not retried
        // (the server may have acted on it, and a retry would double the wait).
        close_idle();
        static auto& timeouts = metrics::Registry::global().counter(
            "bgc_http_client_timeouts_total", "Client requests that got no response within their timeout");
        timeouts.inc();
        throw HttpError("timeout (" + std::to_string(to) + " ms) waiting for the response: " + method + " " + path);
      }
      if (reused && !r.consumed_any()) continue;
      throw HttpError("no response (connection closed): " + method + " " + path);
    }
    Response resp;
    if (line.size() < 12 || line.compare(0, 5, "HTTP/") != 0) throw HttpError("malformed status line: " + line);
    resp.status = std::atoi(line.c_str() + 9);
    if (!parse_headers(r, resp.headers, to)) throw HttpError("malformed response headers");
    bool keep = line.compare(0, 8, "HTTP/1.1") == 0;
    if (const std::string* c = resp.headers.get("Connection")) {
      if (lower(*c).find("close") != std::string::npos) keep = false;
    }
    bool no_body = method == "HEAD" || resp.status == 204 || resp.status == 304 || resp.status / 100 == 1;
    if (!no_body) {
      if (const std::string* te = resp.headers.get("Transfer-Encoding");
          te && lower(*te).find("chunked") != std::string::npos) {
        if (!read_chunked(r, resp.body, to, size_t(1) << 31)) throw HttpError("truncated chunked body");
      } else if (const std::string* cl = resp.headers.get("Content-Length")) {
        size_t n = static_cast<size_t>(std::stoull(*cl));
        if (!r.read_exact(resp.body, n, to)) throw HttpError("truncated body");
      } else {
        // read until close
        while (true) {
          ssize_t n = r.read_available(resp.body, to);
          if (n <= 0) break;
        }
        keep = false;
      }
    }
    if (keep) give_back(std::move(s));
    return resp;
  }
  throw HttpError("request failed after retry: " + method + " " + path);
}

std::unique_ptr<StreamingResponse> Client::stream(const std::string& method, const std::string& path,
                                                  const Headers* headers, const std::string& body) {
  std::string wire = build_request(method, path, body, headers);
  auto s = connect();  // long-lived streams never share pooled connections
  if (!s->write_all(wire)) throw HttpError("write failed: " + path);
  auto sr = std::make_unique<StreamingResponse>();
  sr->reader_ = std::make_unique<Reader>(*s);
  std::string line;
  if (!sr->reader_->read_line(line, opts_.timeout_ms)) throw HttpError("no response to stream request: " + path);
  if (line.size() < 12 || line.compare(0, 5, "HTTP/") != 0) throw HttpError("malformed status line: " + line);
  sr->status = std::atoi(line.c_str() + 9);
  if (!parse_headers(*sr->reader_, sr->headers, opts_.timeout_ms)) throw HttpError("malformed response headers");
  if (const std::string* te = sr->headers.get("Transfer-Encoding"); te && lower(*te).find("chunked") != std::string::npos) {
    sr->chunked_ = true;
  } else if (const std::string* cl = sr->headers.get("Content-Length")) {
    sr->remaining_ = static_cast<int64_t>(std::stoll(*cl));
  }
  sr->stream_ = std::move(s);
  sr->last_data_ns_ = metrics::now_ns();
  return sr;
}

StreamingResponse::~StreamingResponse() { reader_.reset(); }

void StreamingResponse::close() {
  if (stream_) stream_->shutdown();
  done_ = true;
}

bool StreamingResponse::pull(const CancelToken* cancel, int poll_ms) {
  // Reads more body bytes into pending_. Returns false at end of body.
  while (!done_) {
    if (cancel && cancel->cancelled()) return false;
    if (chunked_) {
      std::string line;
      if (!reader_->read_line(line, poll_ms)) {
        if (reader_->consumed_any() || true) {
          // distinguish timeout from EOF via a zero-timeout probe of the socket
          struct pollfd p {};
          p.fd = stream_->fd();
          p.events = POLLIN;
          if (::poll(&p, 1, 0) > 0 && !reader_->buffered()) {
            char c;
            if (::recv(stream_->fd(), &c, 1, MSG_PEEK | MSG_DONTWAIT) <= 0) {
              done_ = true;
              return false;
            }
          }
        }
        if (idle_expired()) return false;
        continue;  // timeout: re-check cancel
      }
      last_data_ns_ = metrics::now_ns();
      size_t n = 0;
      size_t semi = line.find(';');
      std::string hex = line.substr(0, semi);
      auto res = std::from_chars(hex.data(), hex.data() + hex.size(), n, 16);
      if (res.ec != std::errc()) {
        done_ = true;
        return false;
      }
      if (n == 0) {
        done_ = true;
        return false;
      }
      std::string data;
      while (!reader_->read_exact(data, n, poll_ms)) {
        if (cancel && cancel->cancelled()) return false;
        struct pollfd p {};
        p.fd = stream_->fd();
        p.events = POLLIN;
        if (::poll(&p, 1, 0) > 0) {
          char c;
          if (::recv(stream_->fd(), &c, 1, MSG_PEEK | MSG_DONTWAIT) <= 0 && !reader_->buffered()) {
            done_ = true;
            return false;
          }
        }
        if (idle_expired()) return false;
      }
      pending_ += data;
      std::string crlf;
      reader_->read_line(crlf, 10000);
      last_data_ns_ = metrics::now_ns();
      return true;
    }
    if (remaining_ == 0) {
      done_ = true;
      return false;
    }
    std::string data;
    ssize_t r = reader_->read_available(data, poll_ms);
    if (r == -2) {
      if (idle_expired()) return false;
      continue;
    }
    if (r <= 0) {
      done_ = true;
      return false;
    }
    if (remaining_ > 0) {
      if (static_cast<int64_t>(data.size()) > remaining_) data.resize(static_cast<size_t>(remaining_));
      remaining_ -= static_cast<int64_t>(data.size());
    }
    pending_ += data;
    last_data_ns_ = metrics::now_ns();
    return true;
  }
  return false;
}

bool StreamingResponse::idle_expired() {
  if (idle_ms_ <= 0) return false;
  const int64_t now = metrics::now_ns();
  if (last_data_ns_ == 0) last_data_ns_ = now;
  if (now - last_data_ns_ < static_cast<int64_t>(idle_ms_) * 1000000) return false;
  idle_timed_out_ = true;
  done_ = true;
  return true;
}

bool StreamingResponse::next_line(std::string& line, const CancelToken* cancel, int poll_ms) {
  while (true) {
    size_t nl = pending_.find('\n');
    if (nl != std::string::npos) {
      line = pending_.substr(0, nl);
      pending_.erase(0, nl + 1);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      return true;
    }
    if (!pull(cancel, poll_ms)) {
      if (!pending_.empty()) {
        line.swap(pending_);
        pending_.clear();
        return true;
      }
      return false;
    }
  }
}

std::string StreamingResponse::read_all(int timeout_ms) {
  std::string out;
  std::string line;
  auto deadline = metrics::now_ns() + static_cast<int64_t>(timeout_ms) * 1000000;
  while (metrics::now_ns() < deadline && next_line(line, nullptr, 200)) {
    out += line;
    out += "\n";
  }
  return out;
}

Response fetch(const std::string& method, const std::string& url, const std::string& body, const Headers* headers,
               std::shared_ptr<net::TlsContext> tls, int timeout_ms) {
  Url u = parse_url(url);
  ClientOptions o;
  o.base_url = u.scheme + "://" + u.host + ":" + std::to_string(u.port);
  o.tls = std::move(tls);
  o.timeout_ms = timeout_ms;
  Client c(o);
  return c.request(method, u.path.empty() ? "/" : u.path, body, headers, timeout_ms);
}

}  // namespace bgc::http

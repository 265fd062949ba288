#include "core/net.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>
#include <chrono>

namespace bgc::net {

std::string ssl_errors() {
  std::string out;
  unsigned long e;
  while ((e = ERR_get_error()) != 0) {
    char buf[256];
    ERR_error_string_n(e, buf, sizeof(buf));
    if (!out.empty()) out += "; ";
    out += buf;
  }
  return out.empty() ? "unknown TLS error" : out;
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw NetError("cannot read file: " + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

void write_file(const std::string& path, const std::string& data) {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  if (!f) throw NetError("cannot write file: " + path);
  f << data;
}

static void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

static int poll_fd(int fd, short events, int timeout_ms) {
  struct pollfd p {};
  p.fd = fd;
  p.events = events;
  while (true) {
    int r = ::poll(&p, 1, timeout_ms);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return r;
    return p.revents;
  }
}

// ---------------------------------------------------------------------------

TcpStream::~TcpStream() {
  if (fd_ >= 0) ::close(fd_);
}

ssize_t TcpStream::read_some(char* buf, size_t n, int timeout_ms) {
  if (timeout_ms >= 0) {
    int r = poll_fd(fd_, POLLIN, timeout_ms);
    if (r == 0) return -2;
    if (r < 0) return -1;
  }
  while (true) {
    ssize_t r = ::recv(fd_, buf, n, 0);
    if (r < 0 && errno == EINTR) continue;
    return r < 0 ? -1 : r;
  }
}

bool TcpStream::write_all(const char* buf, size_t n) {
  while (n > 0) {
    ssize_t r = ::send(fd_, buf, n, MSG_NOSIGNAL);
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    buf += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

void TcpStream::shutdown() { ::shutdown(fd_, SHUT_RDWR); }

// ---------------------------------------------------------------------------

static std::shared_ptr<SSL_CTX> wrap_ctx(SSL_CTX* c) {
  return std::shared_ptr<SSL_CTX>(c, [](SSL_CTX* p) { SSL_CTX_free(p); });
}

static void load_cert_chain_pem(SSL_CTX* ctx, const std::string& cert_pem, const std::string& key_pem) {
  BIO* cb = BIO_new_mem_buf(cert_pem.data(), static_cast<int>(cert_pem.size()));
  X509* leaf = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr);
  if (!leaf) {
    BIO_free(cb);
    throw NetError("failed to parse certificate: " + ssl_errors());
  }
  if (SSL_CTX_use_certificate(ctx, leaf) != 1) {
    X509_free(leaf);
    BIO_free(cb);
    throw NetError("failed to use certificate: " + ssl_errors());
  }
  X509_free(leaf);
  // remaining certs in the bundle are the chain
  while (X509* extra = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr)) {
    SSL_CTX_add_extra_chain_cert(ctx, extra);
  }
  ERR_clear_error();
  BIO_free(cb);
  BIO* kb = BIO_new_mem_buf(key_pem.data(), static_cast<int>(key_pem.size()));
  EVP_PKEY* key = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
  BIO_free(kb);
  if (!key) throw NetError("failed to parse private key: " + ssl_errors());
  int ok = SSL_CTX_use_PrivateKey(ctx, key);
  EVP_PKEY_free(key);
  if (ok != 1 || SSL_CTX_check_private_key(ctx) != 1) {
    throw NetError("private key does not match certificate: " + ssl_errors());
  }
}

namespace {
// Read-ahead (BGC_TLS_READ_AHEAD=1): SSL_read pulls everything the socket holds into
// OpenSSL's buffer with one read(2), instead of one read for each record header and one
// for its body.  Every reader here calls SSL_read before it polls, and has_buffered()
// counts read-ahead bytes, so it is safe; but on the MI355X box it did not pay (no CPU
// or rate gain in an interleaved A/B, profiles/admission_h2_inline_r3/), so it is off.
void tune_ctx(SSL_CTX* c) {
  SSL_CTX_set_min_proto_version(c, TLS1_2_VERSION);
  SSL_CTX_set_mode(c, SSL_MODE_AUTO_RETRY);
  static const bool read_ahead = [] {
    const char* e = std::getenv("BGC_TLS_READ_AHEAD");
    return e && std::string(e) == "1";
  }();
  if (read_ahead) SSL_CTX_set_read_ahead(c, 1);
  // BGC_TLS13_CIPHERSUITES (A/B knob): the TLS 1.3 suites offered/accepted, e.g.
  // TLS_AES_128_GCM_SHA256 (OpenSSL's default list leads with AES-256-GCM)
  static const char* suites = std::getenv("BGC_TLS13_CIPHERSUITES");
  if (suites && *suites && SSL_CTX_set_ciphersuites(c, suites) != 1) ERR_clear_error();
}
}  // namespace

// Every certificate in a PEM bundle into the context's verification store; the count.
static int add_ca_pem(SSL_CTX* c, const std::string& ca_pem) {
  X509_STORE* store = SSL_CTX_get_cert_store(c);
  BIO* b = BIO_new_mem_buf(ca_pem.data(), static_cast<int>(ca_pem.size()));
  int added = 0;
  while (X509* x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr)) {
    X509_STORE_add_cert(store, x);
    X509_free(x);
    ++added;
  }
  BIO_free(b);
  ERR_clear_error();
  return added;
}

std::shared_ptr<TlsContext> TlsContext::server_from_pem(const std::string& cert_pem, const std::string& key_pem,
                                                        const std::string& client_ca_pem) {
  SSL_CTX* c = SSL_CTX_new(TLS_server_method());
  if (!c) throw NetError("SSL_CTX_new: " + ssl_errors());
  auto ctx = wrap_ctx(c);
  tune_ctx(c);
  load_cert_chain_pem(c, cert_pem, key_pem);
  if (!client_ca_pem.empty()) {
    // the kube-apiserver's --client-ca-file: a client certificate is requested and, when
    // one is sent, must verify; clients with bearer tokens send none
    if (!add_ca_pem(c, client_ca_pem)) throw NetError("no certificates found in the client CA bundle");
    SSL_CTX_set_verify(c, SSL_VERIFY_PEER | SSL_VERIFY_CLIENT_ONCE, nullptr);
    static const unsigned char kSid[] = "bgc-x509";
    SSL_CTX_set_session_id_context(c, kSid, sizeof(kSid) - 1);
  }
  auto t = std::make_shared<TlsContext>();
  t->ctx_ = ctx;
  t->client_ca_pem_ = client_ca_pem;
  t->server_ = true;
  return t;
}

std::shared_ptr<TlsContext> TlsContext::server_from_files(const std::string& cert_path, const std::string& key_path,
                                                          const std::string& client_ca_pem) {
  return server_from_pem(read_file(cert_path), read_file(key_path), client_ca_pem);
}

void TlsContext::reload_from_files(const std::string& cert_path, const std::string& key_path) {
  auto fresh = server_from_files(cert_path, key_path, client_ca_pem_);
  if (h2_) apply_alpn(fresh->ctx_.get());
  std::lock_guard<std::mutex> lk(mu_);
  ctx_ = fresh->ctx_;
}

namespace {
// ALPN wire format, in our order of preference.
constexpr unsigned char kAlpnH2[] = {2, 'h', '2', 8, 'h', 't', 't', 'p', '/', '1', '.', '1'};

int select_alpn(SSL*, const unsigned char** out, unsigned char* outlen, const unsigned char* in, unsigned int inlen,
                void*) {
  unsigned char* sel = nullptr;
  // first of OUR protocols that the client offered (h2 before http/1.1)
  if (SSL_select_next_proto(&sel, outlen, kAlpnH2, sizeof(kAlpnH2), in, inlen) == OPENSSL_NPN_NEGOTIATED) {
    *out = sel;
    return SSL_TLSEXT_ERR_OK;
  }
  return SSL_TLSEXT_ERR_NOACK;  // e.g. a client offering only "acme-tls/1": no ALPN, HTTP/1.1
}
}  // namespace

void TlsContext::apply_alpn(SSL_CTX* c) const {
  if (server_) SSL_CTX_set_alpn_select_cb(c, select_alpn, nullptr);
}

void TlsContext::enable_h2() {
  std::lock_guard<std::mutex> lk(mu_);
  h2_ = true;
  apply_alpn(ctx_.get());
}

std::shared_ptr<SSL_CTX> TlsContext::get() const {
  std::lock_guard<std::mutex> lk(mu_);
  return ctx_;
}

std::shared_ptr<TlsContext> TlsContext::client(const std::string& ca_pem, bool insecure,
                                               const std::string& client_cert_pem,
                                               const std::string& client_key_pem) {
  SSL_CTX* c = SSL_CTX_new(TLS_client_method());
  if (!c) throw NetError("SSL_CTX_new: " + ssl_errors());
  auto ctx = wrap_ctx(c);
  tune_ctx(c);
  // Session resumption keeps reconnect cost low for the webhook/apiserver clients.
  SSL_CTX_set_session_cache_mode(c, SSL_SESS_CACHE_CLIENT);
  if (!insecure) {
    if (ca_pem.empty()) {
      SSL_CTX_set_default_verify_paths(c);
    } else {
      if (!add_ca_pem(c, ca_pem)) throw NetError("no certificates found in CA bundle");
    }
    SSL_CTX_set_verify(c, SSL_VERIFY_PEER, nullptr);
  } else {
    SSL_CTX_set_verify(c, SSL_VERIFY_NONE, nullptr);
  }
  if (!client_cert_pem.empty()) load_cert_chain_pem(c, client_cert_pem, client_key_pem);
  auto t = std::make_shared<TlsContext>();
  t->ctx_ = ctx;
  t->server_ = false;
  t->insecure_ = insecure;
  return t;
}

TlsStream::TlsStream(int fd, std::shared_ptr<SSL_CTX> ctx, bool server, const std::string& verify_host,
                     bool verify_peer, int timeout_ms, bool offer_h2)
    : fd_(fd), ctx_(std::move(ctx)) {
  ssl_ = SSL_new(ctx_.get());
  if (!ssl_) {
    ::close(fd_);
    fd_ = -1;
    throw NetError("SSL_new: " + ssl_errors());
  }
  SSL_set_fd(ssl_, fd_);
  if (!server && offer_h2) SSL_set_alpn_protos(ssl_, kAlpnH2, sizeof(kAlpnH2));
  if (!server) {
    if (!verify_host.empty()) {
      bool is_ip = verify_host.find_first_not_of("0123456789.") == std::string::npos ||
                   verify_host.find(':') != std::string::npos;
      if (!is_ip) SSL_set_tlsext_host_name(ssl_, verify_host.c_str());
      if (verify_peer) {
        if (is_ip) {
          X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(ssl_), verify_host.c_str());
        } else {
          SSL_set1_host(ssl_, verify_host.c_str());
        }
      }
    }
  }
  // Blocking handshake bounded by timeout via SO_RCVTIMEO/SO_SNDTIMEO.
  struct timeval tv {};
  tv.tv_sec = timeout_ms / 1000;
  tv.tv_usec = (timeout_ms % 1000) * 1000;
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  int rc = server ? SSL_accept(ssl_) : SSL_connect(ssl_);
  struct timeval zero {};
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &zero, sizeof(zero));
  setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &zero, sizeof(zero));
  if (rc == 1) fcntl(fd_, F_SETFL, fcntl(fd_, F_GETFL, 0) | O_NONBLOCK);
  if (rc != 1) {
    std::string err = ssl_errors();
    long vr = SSL_get_verify_result(ssl_);
    if (vr != X509_V_OK) err += " (verify: " + std::string(X509_verify_cert_error_string(vr)) + ")";
    SSL_free(ssl_);
    ssl_ = nullptr;
    ::close(fd_);
    fd_ = -1;
    throw NetError("TLS handshake failed: " + err);
  }
}

TlsStream::~TlsStream() {
  if (ssl_) {
    SSL_shutdown(ssl_);
    SSL_free(ssl_);
    // SSL_shutdown on a connection that already failed queues an error on this thread;
    // left there, it would make the next SSL_get_error on another connection read
    // SSL_ERROR_SSL instead of WANT_READ
    ERR_clear_error();
  }
  if (fd_ >= 0) ::close(fd_);
}

bool TlsStream::has_buffered() const {
  std::lock_guard<std::mutex> lk(ssl_mu_);
  return ssl_ && SSL_has_pending(ssl_) == 1;  // decrypted or read-ahead (unprocessed) bytes
}

bool TlsStream::peer_identity(std::string* cn, std::vector<std::string>* orgs) const {
  std::lock_guard<std::mutex> lk(ssl_mu_);
  if (!ssl_) return false;
  X509* peer = SSL_get0_peer_certificate(ssl_);
  if (!peer || SSL_get_verify_result(ssl_) != X509_V_OK) return false;
  const X509_NAME* subj = X509_get_subject_name(peer);
  auto text = [](const X509_NAME_ENTRY* e) {
    const ASN1_STRING* d = X509_NAME_ENTRY_get_data(e);
    unsigned char* utf8 = nullptr;
    const int n = ASN1_STRING_to_UTF8(&utf8, d);
    std::string v = n > 0 ? std::string(reinterpret_cast<char*>(utf8), static_cast<size_t>(n)) : std::string();
    OPENSSL_free(utf8);
    return v;
  };
  std::string name;
  std::vector<std::string> groups;
  for (int i = 0, n = X509_NAME_entry_count(subj); i < n; ++i) {
    const X509_NAME_ENTRY* e = X509_NAME_get_entry(subj, i);
    const int nid = OBJ_obj2nid(X509_NAME_ENTRY_get_object(e));
    if (nid == NID_commonName) name = text(e);
    else if (nid == NID_organizationName) groups.push_back(text(e));
  }
  if (name.empty()) return false;
  if (cn) *cn = name;
  if (orgs) *orgs = groups;
  return true;
}

std::string TlsStream::alpn() const {
  const unsigned char* p = nullptr;
  unsigned int n = 0;
  std::lock_guard<std::mutex> lk(ssl_mu_);
  SSL_get0_alpn_selected(ssl_, &p, &n);
  return p ? std::string(reinterpret_cast<const char*>(p), n) : std::string();
}

// BGC_TLS_POLL_FIRST=1: when OpenSSL holds no buffered bytes, wait in poll() before the
// first SSL_read instead of after it fails: a reader that has consumed everything (a
// client waiting for its response, a watch stream between events) saves the EAGAIN
// recv() of every read.
static bool tls_poll_first() {
  static const bool on = [] {
    const char* e = std::getenv("BGC_TLS_POLL_FIRST");
    return e && std::string(e) == "1";
  }();
  return on;
}

ssize_t TlsStream::read_some(char* buf, size_t n, int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max(timeout_ms, 0));
  if (timeout_ms != 0 && tls_poll_first()) {
    bool pending;
    {
      std::lock_guard<std::mutex> lk(ssl_mu_);
      pending = SSL_has_pending(ssl_) == 1;
    }
    if (!pending) {
      const int pr = poll_fd(fd_, POLLIN, timeout_ms);
      if (pr == 0) return -2;
      if (pr < 0) return -1;
    }
  }
  while (true) {
    int r, err;
    {
      std::lock_guard<std::mutex> lk(ssl_mu_);
      ERR_clear_error();  // SSL_get_error reads this thread's queue first: start it empty
      r = SSL_read(ssl_, buf, static_cast<int>(n));
      if (r > 0) return r;
      err = SSL_get_error(ssl_, r);
      if (err != SSL_ERROR_WANT_READ && err != SSL_ERROR_WANT_WRITE) ERR_clear_error();
    }
    if (err == SSL_ERROR_ZERO_RETURN) return 0;
    if (err == SSL_ERROR_WANT_READ || err == SSL_ERROR_WANT_WRITE) {
      int wait = -1;
      if (timeout_ms >= 0) {
        wait = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(
                                    deadline - std::chrono::steady_clock::now()).count());
        if (wait < 0) return -2;
      }
      int pr = poll_fd(fd_, err == SSL_ERROR_WANT_READ ? POLLIN : POLLOUT, wait);
      if (pr == 0) return -2;
      if (pr < 0) return -1;
      continue;
    }
    if (err == SSL_ERROR_SYSCALL && errno == 0) return 0;  // unexpected EOF
    return -1;
  }
}

bool TlsStream::write_all(const char* buf, size_t n) {
  std::lock_guard<std::mutex> wl(write_mu_);
  while (n > 0) {
    int r, err;
    {
      std::lock_guard<std::mutex> lk(ssl_mu_);
      ERR_clear_error();
      r = SSL_write(ssl_, buf, static_cast<int>(n));
      if (r <= 0) {
        err = SSL_get_error(ssl_, r);
        if (err != SSL_ERROR_WANT_READ && err != SSL_ERROR_WANT_WRITE) ERR_clear_error();
      }
    }
    if (r > 0) {
      buf += r;
      n -= static_cast<size_t>(r);
      continue;
    }
    // retried with the same buffer, as a non-blocking SSL_write requires
    if (err == SSL_ERROR_WANT_WRITE || err == SSL_ERROR_WANT_READ) {
      if (poll_fd(fd_, err == SSL_ERROR_WANT_WRITE ? POLLOUT : POLLIN, 30000) <= 0) return false;
      continue;
    }
    return false;
  }
  return true;
}

void TlsStream::shutdown() { ::shutdown(fd_, SHUT_RDWR); }

// ---------------------------------------------------------------------------

namespace {
std::mutex g_keepalive_mu;
TcpKeepalive g_keepalive;
}  // namespace

void set_tcp_keepalive(TcpKeepalive k) {
  std::lock_guard<std::mutex> lk(g_keepalive_mu);
  g_keepalive = k;
}

TcpKeepalive tcp_keepalive() {
  std::lock_guard<std::mutex> lk(g_keepalive_mu);
  return g_keepalive;
}

bool apply_tcp_keepalive(int fd, const TcpKeepalive& k) {
  bool ok = true;
  if (k.idle_s > 0) {
    int one = 1;
    ok &= setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof(one)) == 0;
    ok &= setsockopt(fd, IPPROTO_TCP, TCP_KEEPIDLE, &k.idle_s, sizeof(k.idle_s)) == 0;
    const int intvl = std::max(1, k.interval_s), cnt = std::max(1, k.count);
    ok &= setsockopt(fd, IPPROTO_TCP, TCP_KEEPINTVL, &intvl, sizeof(intvl)) == 0;
    ok &= setsockopt(fd, IPPROTO_TCP, TCP_KEEPCNT, &cnt, sizeof(cnt)) == 0;
  }
  if (k.user_timeout_ms > 0) {
    const unsigned int ut = static_cast<unsigned int>(k.user_timeout_ms);
    ok &= setsockopt(fd, IPPROTO_TCP, TCP_USER_TIMEOUT, &ut, sizeof(ut)) == 0;
  }
  return ok;
}

int connect_tcp(const std::string& host_in, uint16_t port, int timeout_ms) {
  std::string host = host_in;
  if (host.size() > 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  struct addrinfo hints {};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  std::string ps = std::to_string(port);
  int gai = getaddrinfo(host.c_str(), ps.c_str(), &hints, &res);
  if (gai != 0) throw NetError("resolve " + host + ": " + gai_strerror(gai));
  std::string last_err = "no addresses";
  for (auto* ai = res; ai; ai = ai->ai_next) {
    int fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int flags = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, flags | O_NONBLOCK);
    int rc = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (rc < 0 && errno == EINPROGRESS) {
      int pr = poll_fd(fd, POLLOUT, timeout_ms);
      if (pr <= 0) {
        last_err = pr == 0 ? "connect timeout" : std::strerror(errno);
        ::close(fd);
        continue;
      }
      int soerr = 0;
      socklen_t len = sizeof(soerr);
      getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &len);
      if (soerr != 0) {
        last_err = std::strerror(soerr);
        ::close(fd);
        continue;
      }
    } else if (rc < 0) {
      last_err = std::strerror(errno);
      ::close(fd);
      continue;
    }
    fcntl(fd, F_SETFL, flags);
    set_nodelay(fd);
    apply_tcp_keepalive(fd, tcp_keepalive());
    freeaddrinfo(res);
    return fd;
  }
  freeaddrinfo(res);
  throw NetError("connect " + host + ":" + ps + ": " + last_err);
}

int listen_tcp(const std::string& addr, uint16_t port, int backlog, uint16_t* bound_port) {
  struct addrinfo hints {};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICHOST;
  struct addrinfo* res = nullptr;
  std::string ps = std::to_string(port);
  int gai = getaddrinfo(addr.empty() ? nullptr : addr.c_str(), ps.c_str(), &hints, &res);
  if (gai != 0) throw NetError("invalid listen address " + addr + ": " + gai_strerror(gai));
  int fd = ::socket(res->ai_family, res->ai_socktype | SOCK_CLOEXEC, res->ai_protocol);
  if (fd < 0) {
    freeaddrinfo(res);
    throw NetError(std::string("socket: ") + std::strerror(errno));
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (::bind(fd, res->ai_addr, res->ai_addrlen) < 0) {
    std::string e = std::strerror(errno);
    ::close(fd);
    freeaddrinfo(res);
    throw NetError("bind " + addr + ":" + ps + ": " + e);
  }
  freeaddrinfo(res);
  if (::listen(fd, backlog) < 0) {
    std::string e = std::strerror(errno);
    ::close(fd);
    throw NetError("listen: " + e);
  }
  if (bound_port) {
    struct sockaddr_storage ss {};
    socklen_t len = sizeof(ss);
    getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &len);
    if (ss.ss_family == AF_INET) *bound_port = ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
    else *bound_port = ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port);
  }
  return fd;
}


static sockaddr_un unix_addr(const std::string& path) {
  sockaddr_un sa{};
  sa.sun_family = AF_UNIX;
  if (path.size() >= sizeof(sa.sun_path)) throw NetError("unix socket path too long: " + path);
  std::memcpy(sa.sun_path, path.data(), path.size());
  return sa;
}

int connect_unix(const std::string& path, int timeout_ms) {
  sockaddr_un sa = unix_addr(path);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) throw NetError(std::string("socket: ") + std::strerror(errno));
    if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) return fd;
    int e = errno;
    ::close(fd);
    // The listener may be between unlink and bind (kubelet restart): retry until the deadline.
    if ((e == ENOENT || e == ECONNREFUSED || e == EAGAIN) && std::chrono::steady_clock::now() < deadline) {
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      continue;
    }
    throw NetError("connect " + path + ": " + std::strerror(e));
  }
}

int listen_unix(const std::string& path, int backlog) {
  sockaddr_un sa = unix_addr(path);
  ::unlink(path.c_str());
  int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) throw NetError(std::string("socket: ") + std::strerror(errno));
  if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(fd, backlog) != 0) {
    int e = errno;
    ::close(fd);
    throw NetError("listen " + path + ": " + std::strerror(e));
  }
  return fd;
}

}  // namespace bgc::net

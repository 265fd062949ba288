// Sockets and TLS streams (OpenSSL 3).
//
// Replaces hyper/rustls (clients) and axum-server's `tls_rustls` (webhook server with
// live certificate reload, reference src/admission.rs:104-126,141,174).
#pragma once

#include <openssl/ssl.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <sys/types.h>
#include <vector>

namespace bgc::net {

class NetError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Stream {
 public:
  virtual ~Stream() = default;
  // Returns bytes read, 0 on orderly EOF, -1 on error, -2 on timeout.
  virtual ssize_t read_some(char* buf, size_t n, int timeout_ms) = 0;
  virtual bool write_all(const char* buf, size_t n) = 0;
  // Unblocks readers from another thread.
  virtual void shutdown() = 0;
  virtual int fd() const = 0;
  virtual bool has_buffered() const { return false; }
  // A TLS server connection whose client presented a certificate that verified against
  // the server's client CA: its subject CN and O values (the Kubernetes x509
  // authenticator's username and groups).  false otherwise.
  virtual bool peer_identity(std::string* cn, std::vector<std::string>* orgs) const {
    (void)cn;
    (void)orgs;
    return false;
  }
  bool write_all(const std::string& s) { return write_all(s.data(), s.size()); }
};

class TcpStream : public Stream {
 public:
  explicit TcpStream(int fd) : fd_(fd) {}
  ~TcpStream() override;
  ssize_t read_some(char* buf, size_t n, int timeout_ms) override;
  bool write_all(const char* buf, size_t n) override;
  void shutdown() override;
  int fd() const override { return fd_; }

 private:
  int fd_;
};

// Shared SSL_CTX holder whose context can be swapped atomically (hot reload): new
// connections pick up the new certificate, established ones keep the old context.
class TlsContext {
 public:
  // client_ca_pem: also ask clients for a certificate and verify it against this CA
  // (optional: clients without one still connect; see TlsStream::peer_identity).
  static std::shared_ptr<TlsContext> server_from_files(const std::string& cert_path,
                                                       const std::string& key_path,
                                                       const std::string& client_ca_pem = "");
  static std::shared_ptr<TlsContext> server_from_pem(const std::string& cert_pem,
                                                     const std::string& key_pem,
                                                     const std::string& client_ca_pem = "");
  // ca_pem empty + insecure=false => system roots (with_native_roots).
  static std::shared_ptr<TlsContext> client(const std::string& ca_pem, bool insecure,
                                            const std::string& client_cert_pem = "",
                                            const std::string& client_key_pem = "");

  void reload_from_files(const std::string& cert_path, const std::string& key_path);
  std::shared_ptr<SSL_CTX> get() const;
  bool is_server() const { return server_; }
  bool insecure() const { return insecure_; }
  // ALPN (RFC 7301) for HTTP/2: a server context selects "h2" when the client offers it
  // and "http/1.1" otherwise.  Survives reloads.  (Clients choose per connection:
  // TlsStream's offer_h2.)
  void enable_h2();
  bool h2() const { return h2_.load(); }

 private:
  void apply_alpn(SSL_CTX* c) const;
  mutable std::mutex mu_;
  std::shared_ptr<SSL_CTX> ctx_;
  std::string client_ca_pem_;  // kept for reloads
  bool server_ = false;
  bool insecure_ = false;
  std::atomic<bool> h2_{false};
};

class TlsStream : public Stream {
 public:
  // Takes ownership of fd. Performs the handshake; throws NetError on failure.
  // offer_h2 (client): offer "h2" before "http/1.1" by ALPN on this connection only.
  TlsStream(int fd, std::shared_ptr<SSL_CTX> ctx, bool server, const std::string& verify_host,
            bool verify_peer, int timeout_ms, bool offer_h2 = false);
  ~TlsStream() override;
  ssize_t read_some(char* buf, size_t n, int timeout_ms) override;
  bool write_all(const char* buf, size_t n) override;
  void shutdown() override;
  int fd() const override { return fd_; }
  bool has_buffered() const override;
  bool peer_identity(std::string* cn, std::vector<std::string>* orgs) const override;
  // Protocol selected by ALPN during the handshake ("" when none was negotiated).
  std::string alpn() const;

 private:
  int fd_;
  std::shared_ptr<SSL_CTX> ctx_;
  SSL* ssl_ = nullptr;
  // After the handshake the socket is non-blocking and every SSL call runs under ssl_mu_,
  // waiting in poll() with the lock released: one thread may read while others write
  // (an HTTP/2 connection's reader thread and its stream writers share one SSL object,
  // which OpenSSL does not allow concurrently).  write_mu_ orders whole writes.
  mutable std::mutex ssl_mu_;
  std::mutex write_mu_;
};

// TCP liveness of outgoing connections (connect_tcp): kernel keepalive probes after
// `idle_s` without traffic, every `interval_s`, `count` unanswered probes closing the
// socket; and TCP_USER_TIMEOUT, the longest written data may stay unacknowledged before
// the kernel drops the connection.  A peer host that crashes or a NAT/conntrack entry that
// expires then fails the socket instead of leaving it open forever.  (A path that still
// answers probes but forwards nothing, e.g. a wedged proxy, is caught one level up by the
// watch idle deadline, kube::Watcher::Defaults::idle_timeout_ms.)  Go's net.Dialer under
// client-go starts probing after 15-30 s; these defaults are in that range.  idle_s = 0
// disables keepalive; user_timeout_ms = 0 keeps the kernel default.
struct TcpKeepalive {
  int idle_s = 30;
  int interval_s = 10;
  int count = 3;
  int user_timeout_ms = 60000;
};
void set_tcp_keepalive(TcpKeepalive k);  // process-wide, for connections opened afterwards
TcpKeepalive tcp_keepalive();
// Applies `k` to a connected socket (false if the kernel refused an option).
bool apply_tcp_keepalive(int fd, const TcpKeepalive& k);

// Resolves and connects (IPv4/IPv6) with the process's TcpKeepalive; throws NetError.
int connect_tcp(const std::string& host, uint16_t port, int timeout_ms);
// Listens; port 0 picks an ephemeral port (returned through bound_port).
int listen_tcp(const std::string& addr, uint16_t port, int backlog, uint16_t* bound_port);
// Unix-domain stream sockets (kubelet device-plugin gRPC).  listen_unix unlinks a stale
// socket file first; both throw NetError.
int connect_unix(const std::string& path, int timeout_ms);
int listen_unix(const std::string& path, int backlog);

std::string ssl_errors();
std::string read_file(const std::string& path);
void write_file(const std::string& path, const std::string& data);

}  // namespace bgc::net

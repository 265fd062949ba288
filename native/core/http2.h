// HTTP/2 (RFC 9113) over a plain stream socket + the gRPC wire protocol on top.
//
// Why this exists: the kubelet talks to device plugins only through gRPC on unix
// sockets (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1).  The image has no gRPC C++,
// protoc or nghttp2 headers, so the node agent carries its own small h2c stack:
//
//   Connection  one socket, one reader thread (or, for a client in caller-reads mode, the
//               waiting callers take turns reading); HPACK decoder state lives with the reader,
//               writes are serialised by a mutex (a frame, or a HEADERS+CONTINUATION
//               run, is written atomically).  Send-side flow control is honoured per
//               stream and per connection (senders block until WINDOW_UPDATE); the
//               receive side re-opens the window as soon as a DATA frame is buffered,
//               so a slow handler never stalls the peer.  PING/SETTINGS are answered on
//               the reader thread.  Server push is disabled.
//   grpc::Server   unary + server-streaming methods (all the device-plugin API needs).
//                  Each call runs on its own thread; a streaming handler learns about
//                  client cancellation (RST_STREAM, closed socket, server stop) through
//                  ServerCall::cancelled()/wait().
//   grpc::Channel  client for unary + server-streaming calls (plugin -> kubelet
//                  Registration, and the tests' own round trips).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "core/hpack.h"
#include "core/net.h"

namespace bgc::http2 {

enum FrameType : uint8_t {
  kData = 0, kHeaders = 1, kPriority = 2, kRstStream = 3, kSettings = 4,
  kPushPromise = 5, kPing = 6, kGoaway = 7, kWindowUpdate = 8, kContinuation = 9,
};
enum Flags : uint8_t { kEndStream = 0x1, kAck = 0x1, kEndHeaders = 0x4, kPadded = 0x8, kPriorityFlag = 0x20 };
enum ErrorCode : uint32_t {
  kNoError = 0, kProtocolError = 1, kInternalError = 2, kFlowControlError = 3, kStreamClosed = 5,
  kFrameSizeError = 6, kRefusedStream = 7, kCancel = 8, kCompressionError = 9,
};

constexpr const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr uint32_t kDefaultWindow = 65535;
constexpr uint32_t kOurWindow = 1u << 20;       // advertised receive window per stream
constexpr uint32_t kOurConnWindow = 64u << 20;  // ... and per connection: hundreds of concurrent
                                                // requests never wait for a WINDOW_UPDATE

class Connection;

// One HTTP/2 stream.  Fields are guarded by the owning connection's mutex.
struct Stream {
  uint32_t id = 0;
  hpack::HeaderList headers;   // request headers (server side) / response headers (client side)
  hpack::HeaderList trailers;
  bool headers_received = false;
  std::string data;            // received DATA payload not yet consumed
  bool remote_closed = false;  // END_STREAM seen
  bool local_closed = false;   // we sent END_STREAM
  bool reset = false;          // RST_STREAM either way, or the connection died
  uint32_t reset_code = 0;
  int64_t send_window = kDefaultWindow;
  bool dispatched = false;
  uint32_t recv_pending = 0;   // received DATA bytes not yet returned by WINDOW_UPDATE
  // Waiters for this stream alone (with the connection mutex): a client multiplexing
  // many requests wakes only the caller whose response arrived, not every caller.
  std::condition_variable cv;
};

class Connection : public std::enable_shared_from_this<Connection> {
 public:
  enum class Role { kClient, kServer };
  // Server side: invoked on the reader thread once a request stream is complete
  // (END_STREAM received).  Must not block: hand the stream to another thread.
  using RequestHandler = std::function<void(std::shared_ptr<Connection>, std::shared_ptr<Stream>)>;

  Connection(std::unique_ptr<net::Stream> io, Role role, RequestHandler on_request = {});
  ~Connection();
  Connection(const Connection&) = delete;
  Connection& operator=(const Connection&) = delete;

  // Sends the preface/SETTINGS and starts the reader thread (the object must be owned by
  // a shared_ptr: the reader keeps it alive until the socket closes).
  void start();
  // GOAWAY (best effort) + socket shutdown; the reader thread ends, all streams reset.
  void close(uint32_t code = kNoError);
  // Server: graceful drain.  Sends GOAWAY(NO_ERROR) naming the last stream accepted; the
  // streams in flight finish normally and any the peer opens afterwards are refused with
  // REFUSED_STREAM (which a client retries on a new connection).
  void drain();
  void join();
  bool closed() const { return closed_.load(); }
  // Client: new streams may still be opened (not closed, no GOAWAY, ids left).
  bool usable() const;

  // Client: allocates the next odd stream id and sends request HEADERS (+ body DATA).
  std::shared_ptr<Stream> open(const hpack::HeaderList& headers, std::string_view body, bool end_stream);

  bool send_headers(Stream& s, const hpack::HeaderList& headers, bool end_stream);
  // A complete response: HEADERS + DATA(END_STREAM) in one write when the body fits one
  // frame and the send windows, else send_headers + send_data.
  bool send_response(Stream& s, const hpack::HeaderList& headers, std::string_view body);
  // As send_response without ever waiting: kWouldBlock (nothing sent) when the body does
  // not fit one frame and the current send windows.
  enum class SendResult { kSent, kFailed, kWouldBlock };
  SendResult try_send_response(Stream& s, const hpack::HeaderList& headers, std::string_view body);

  // Blocks on flow control; false when the stream or connection died meanwhile.
  bool send_data(Stream& s, std::string_view data, bool end_stream);
  void reset_stream(Stream& s, uint32_t code);

  // Waits (connection mutex) until pred() holds, the connection closes, or the deadline
  // passes.  pred runs with the mutex held, so it may read Stream fields.
  template <class Pred>
  bool wait_until(std::chrono::steady_clock::time_point deadline, Pred pred) {
    std::unique_lock<std::mutex> lk(mu_);
    return cv_.wait_until(lk, deadline, [&] { return pred() || closed_.load(); }) && pred();
  }
  // As wait_until, on the stream's own condition variable (woken by that stream's frames,
  // its reset, and the connection closing).
  template <class Pred>
  bool wait_stream(Stream& s, std::chrono::steady_clock::time_point deadline, Pred pred) {
    std::unique_lock<std::mutex> lk(mu_);
    if (caller_reads_) return wait_reading(lk, s.cv, deadline, pred);
    return s.cv.wait_until(lk, deadline, [&] { return pred() || closed_.load(); }) && pred();
  }

  // Client, before start(): no reader thread.  A caller waiting for its stream reads the
  // connection's frames itself while no other caller does (one at a time; frames for other
  // streams wake their callers), and hands the reader role on when its own stream is done.
  // A response then costs one wake-up on this side (the caller's) instead of two (the
  // reader thread's, then the caller's), which is what matters on a saturated CPU set.
  void set_caller_reads() { caller_reads_ = true; }
  // Caller-reads client about to reuse an idle connection: processes the frames that
  // arrived while nobody waited (SETTINGS, PING, a GOAWAY, the peer closing); false if the
  // connection is closed.
  bool poll_idle();
  // Runs fn with the connection mutex held (to read/modify Stream fields).
  template <class Fn>
  auto locked(Fn fn) {
    std::lock_guard<std::mutex> lk(mu_);
    return fn();
  }
  void notify() { cv_.notify_all(); }

  uint64_t frames_received() const { return frames_in_.load(); }

 private:
  void reader_loop();
  enum class ReadResult { kFrame, kTimeout, kClosed };
  int fill(size_t n, int timeout_ms);
  ReadResult read_frame(int timeout_ms);  // reads and handles one frame (one reader at a time)
  void handle_frame(uint8_t type, uint8_t flags, uint32_t sid, const std::string& payload, uint32_t len);
  // caller-reads mode (mu_ held through lk): read one frame as the reader, up to deadline;
  // false when the connection closed or the deadline passed
  bool read_step_locked(std::unique_lock<std::mutex>& lk, std::chrono::steady_clock::time_point deadline);
  void hand_off_locked();
  template <class Pred>
  bool wait_reading(std::unique_lock<std::mutex>& lk, std::condition_variable& cv,
                    std::chrono::steady_clock::time_point deadline, Pred pred) {
    waiting_cvs_.push_back(&cv);
    bool ok = false;
    while (true) {
      if (pred()) {
        ok = true;
        break;
      }
      if (closed_) break;
      if (!reading_) {
        if (!read_step_locked(lk, deadline)) {
          ok = pred();
          break;
        }
        continue;
      }
      if (cv.wait_until(lk, deadline) == std::cv_status::timeout) {
        ok = pred();
        break;
      }
    }
    for (auto it = waiting_cvs_.begin(); it != waiting_cvs_.end(); ++it) {
      if (*it == &cv) {
        waiting_cvs_.erase(it);
        break;
      }
    }
    hand_off_locked();
    return ok;
  }
  bool write_frame(uint8_t type, uint8_t flags, uint32_t sid, std::string_view payload);
  bool write_frame_locked(uint8_t type, uint8_t flags, uint32_t sid, std::string_view payload);
  void on_headers(uint32_t sid, uint8_t flags, const std::string& block);
  void on_data(uint32_t sid, uint8_t flags, std::string_view payload, size_t flow_len);
  void on_settings(uint8_t flags, std::string_view payload);
  void on_window_update(uint32_t sid, std::string_view payload);
  void on_rst(uint32_t sid, std::string_view payload);
  void on_goaway(uint32_t last_stream);
  void fail_all();
  void goaway(uint32_t code, const std::string& why);
  std::shared_ptr<Stream> find(uint32_t sid);
  void maybe_forget(const std::shared_ptr<Stream>& s);  // mu_ held

  std::unique_ptr<net::Stream> io_;
  Role role_;
  RequestHandler on_request_;
  hpack::Decoder decoder_;
  std::mutex write_mu_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::condition_variable window_cv_;  // senders blocked on flow control (window changes only)
  std::map<uint32_t, std::shared_ptr<Stream>> streams_;
  uint32_t next_stream_id_ = 1;
  uint32_t last_peer_stream_ = 0;
  int64_t conn_send_window_ = kDefaultWindow;
  uint32_t peer_initial_window_ = kDefaultWindow;
  uint32_t peer_max_frame_ = 16384;
  bool goaway_received_ = false;
  bool goaway_sent_ = false;  // drain(): no new peer streams
  std::atomic<bool> closed_{false};
  std::atomic<uint64_t> frames_in_{0};
  std::thread reader_;
  // reader-thread-only state: connection-level DATA bytes not yet returned, and a header
  // block split over CONTINUATION frames
  uint64_t conn_recv_pending_ = 0;
  std::string hdr_block_;
  uint32_t hdr_sid_ = 0;
  uint8_t hdr_flags_ = 0;
  // read buffer
  std::string rbuf_;
  size_t rpos_ = 0;
  // caller-reads mode (set_caller_reads): whether a caller holds the reader role, and the
  // condition variables of the callers waiting (guarded by mu_)
  bool caller_reads_ = false;
  bool reading_ = false;
  std::vector<std::condition_variable*> waiting_cvs_;
};

}  // namespace bgc::http2

namespace bgc::grpc {

// https://grpc.github.io/grpc/core/md_doc_statuscodes.html
enum Code : int {
  kOk = 0, kCancelled = 1, kUnknown = 2, kInvalidArgument = 3, kDeadlineExceeded = 4, kNotFound = 5,
  kFailedPrecondition = 9, kUnimplemented = 12, kInternal = 13, kUnavailable = 14,
};

struct Status {
  int code = kOk;
  std::string message;
  bool ok() const { return code == kOk; }
  static Status Ok() { return {}; }
};

// 5-byte length prefix framing (compressed flag must be 0 — we never advertise an encoding).
std::string frame_message(std::string_view msg);
// Pops one complete message off `buf`; false when more bytes are needed.  Throws on a
// compressed message.
bool pop_message(std::string& buf, std::string* msg);

class ServerCall {
 public:
  ServerCall(std::shared_ptr<http2::Connection> conn, std::shared_ptr<http2::Stream> stream,
             std::atomic<bool>* server_stopping);
  const std::string& method() const { return method_; }
  const std::string& request() const { return request_; }
  const hpack::HeaderList& metadata() const;
  // Sends response headers on first use, then one length-prefixed message.
  bool send_message(std::string_view msg);
  void finish(const Status& st);
  bool cancelled() const;
  // Sleeps up to d, returning early (true) on cancellation.
  bool wait_cancelled(std::chrono::milliseconds d) const;

 private:
  friend class Server;
  std::shared_ptr<http2::Connection> conn_;
  std::shared_ptr<http2::Stream> stream_;
  std::atomic<bool>* stopping_;
  std::string method_;
  std::string request_;
  bool headers_sent_ = false;
  bool finished_ = false;
};

class Server {
 public:
  // A handler returns the call's status; streaming handlers send_message() repeatedly
  // before returning.  Unknown methods get UNIMPLEMENTED.
  using Handler = std::function<Status(ServerCall&)>;

  explicit Server(std::string unix_path);
  ~Server();
  void add(const std::string& method_path, Handler h);  // "/pkg.Service/Method"
  // Binds the unix socket (replacing a stale file) and starts accepting.
  void start();
  void stop();
  const std::string& path() const { return path_; }
  bool socket_present() const;  // the socket file still exists (kubelet restarts wipe the dir)
  uint64_t calls() const { return calls_.load(); }

 private:
  void accept_loop();
  void dispatch(std::shared_ptr<http2::Connection> c, std::shared_ptr<http2::Stream> s);
  void reap(bool all);
  std::string path_;
  std::map<std::string, Handler> handlers_;
  int listen_fd_ = -1;
  uint64_t inode_ = 0;
  std::atomic<bool> stopping_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::vector<std::shared_ptr<http2::Connection>> conns_;
  struct Worker {
    std::thread t;
    std::shared_ptr<std::atomic<bool>> done;
  };
  std::vector<Worker> workers_;
  std::atomic<uint64_t> calls_{0};
};

class Channel {
 public:
  // Connects lazily to a unix socket ("unix:///path" or a bare path).
  explicit Channel(std::string target, int connect_timeout_ms = 5000);
  ~Channel();
  Status unary(const std::string& method, std::string_view req, std::string* resp,
               std::chrono::milliseconds timeout = std::chrono::seconds(10));
  // Delivers each response message to on_msg until the stream ends, on_msg returns
  // false (the call is then cancelled), or `timeout` passes.
  Status server_stream(const std::string& method, std::string_view req,
                       const std::function<bool(const std::string&)>& on_msg,
                       std::chrono::milliseconds timeout = std::chrono::hours(24 * 365));
  void close();

 private:
  std::shared_ptr<http2::Connection> conn();
  Status call_status(http2::Stream& s, bool reset_seen);
  std::string path_;
  int connect_timeout_ms_;
  std::mutex mu_;
  std::shared_ptr<http2::Connection> conn_;
};

}  // namespace bgc::grpc

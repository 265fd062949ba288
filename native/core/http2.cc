#include "core/http2.h"

#include <openssl/crypto.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>

#include "core/log.h"

namespace bgc::http2 {
namespace {

uint32_t be32(const char* p) {
  return (uint32_t(static_cast<uint8_t>(p[0])) << 24) | (uint32_t(static_cast<uint8_t>(p[1])) << 16) |
         (uint32_t(static_cast<uint8_t>(p[2])) << 8) | uint32_t(static_cast<uint8_t>(p[3]));
}

void put32(std::string& out, uint32_t v) {
  out.push_back(static_cast<char>(v >> 24));
  out.push_back(static_cast<char>(v >> 16));
  out.push_back(static_cast<char>(v >> 8));
  out.push_back(static_cast<char>(v));
}

// Appends one frame (9-byte header + payload) to `out`, to coalesce several into one write.
void append_frame(std::string& out, uint8_t type, uint8_t flags, uint32_t sid, std::string_view payload) {
  const uint32_t len = static_cast<uint32_t>(payload.size());
  out.push_back(static_cast<char>(len >> 16));
  out.push_back(static_cast<char>(len >> 8));
  out.push_back(static_cast<char>(len));
  out.push_back(static_cast<char>(type));
  out.push_back(static_cast<char>(flags));
  put32(out, sid & 0x7fffffff);
  out.append(payload.data(), payload.size());
}

void put_setting(std::string& out, uint16_t id, uint32_t v) {
  out.push_back(static_cast<char>(id >> 8));
  out.push_back(static_cast<char>(id));
  put32(out, v);
}

// Strips PADDED (and, for HEADERS, PRIORITY) framing; false on a malformed frame.
bool strip_padding(uint8_t flags, bool headers, std::string_view& p) {
  size_t pad = 0;
  if (flags & kPadded) {
    if (p.empty()) return false;
    pad = static_cast<uint8_t>(p[0]);
    p.remove_prefix(1);
  }
  if (headers && (flags & kPriorityFlag)) {
    if (p.size() < 5) return false;
    p.remove_prefix(5);
  }
  if (pad > p.size()) return false;
  p.remove_suffix(pad);
  return true;
}

}  // namespace

Connection::Connection(std::unique_ptr<net::Stream> io, Role role, RequestHandler on_request)
    : io_(std::move(io)), role_(role), on_request_(std::move(on_request)) {}

Connection::~Connection() {
  close();
  join();
}

void Connection::start() {
  std::string hello;
  if (role_ == Role::kClient) hello.assign(kPreface, sizeof(kPreface) - 1);
  std::string settings;
  if (role_ == Role::kClient) put_setting(settings, 0x2, 0);      // ENABLE_PUSH = 0
  else put_setting(settings, 0x3, 1000);                           // MAX_CONCURRENT_STREAMS
  put_setting(settings, 0x4, kOurWindow);                          // INITIAL_WINDOW_SIZE
  std::string wu;
  put32(wu, kOurConnWindow - kDefaultWindow);  // connection window: 64 KiB -> 64 MiB
  {
    std::lock_guard<std::mutex> lk(write_mu_);
    bool ok = hello.empty() || io_->write_all(hello);
    ok = ok && write_frame_locked(kSettings, 0, 0, settings) && write_frame_locked(kWindowUpdate, 0, 0, wu);
    if (!ok) closed_ = true;
  }
  // The reader owns a reference for its whole run, so the Connection is never destroyed
  // under it; if that reference is the last one, the destructor runs at thread exit and
  // join() detaches instead of joining itself.
  if (caller_reads_) return;  // the callers waiting for responses read the frames
  reader_ = std::thread([self = shared_from_this()] {
    self->reader_loop();
    // OpenSSL's per-thread state (the error queue an SSL_read failure at close fills, the
    // DRBGs) is freed only by OPENSSL_thread_stop (LeakSanitizer, tools/sanitize.sh asan)
    OPENSSL_thread_stop();
  });
}

void Connection::close(uint32_t code) {
  bool was = closed_.exchange(true);
  if (!was) {
    std::string p;
    put32(p, locked([&] { return last_peer_stream_; }));
    put32(p, code);
    std::lock_guard<std::mutex> lk(write_mu_);
    write_frame_locked(kGoaway, 0, 0, p);
  }
  if (io_) io_->shutdown();
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& [id, st] : streams_) st->cv.notify_all();
  }
  window_cv_.notify_all();
  cv_.notify_all();
}

bool Connection::usable() const {
  std::lock_guard<std::mutex> lk(mu_);
  return !closed_ && !goaway_received_ && next_stream_id_ < 0x7fff0000u;
}

void Connection::join() {
  if (!reader_.joinable()) return;
  // The last reference can be dropped on the reader thread itself (a request dispatch
  // that outlived both the server's list and the handler): it cannot join itself.
  if (reader_.get_id() == std::this_thread::get_id()) reader_.detach();
  else reader_.join();
}

bool Connection::write_frame_locked(uint8_t type, uint8_t flags, uint32_t sid, std::string_view payload) {
  char hdr[9];
  const uint32_t len = static_cast<uint32_t>(payload.size());
  hdr[0] = static_cast<char>(len >> 16);
  hdr[1] = static_cast<char>(len >> 8);
  hdr[2] = static_cast<char>(len);
  hdr[3] = static_cast<char>(type);
  hdr[4] = static_cast<char>(flags);
  hdr[5] = static_cast<char>((sid >> 24) & 0x7f);
  hdr[6] = static_cast<char>(sid >> 16);
  hdr[7] = static_cast<char>(sid >> 8);
  hdr[8] = static_cast<char>(sid);
  if (payload.size() <= 4096) {  // one write() for small frames
    std::string buf(hdr, 9);
    buf.append(payload.data(), payload.size());
    return io_->write_all(buf.data(), buf.size());
  }
  return io_->write_all(hdr, 9) && io_->write_all(payload.data(), payload.size());
}

bool Connection::write_frame(uint8_t type, uint8_t flags, uint32_t sid, std::string_view payload) {
  std::lock_guard<std::mutex> lk(write_mu_);
  return write_frame_locked(type, flags, sid, payload);
}

std::shared_ptr<Stream> Connection::find(uint32_t sid) {
  auto it = streams_.find(sid);
  return it == streams_.end() ? nullptr : it->second;
}

void Connection::maybe_forget(const std::shared_ptr<Stream>& s) {
  if (s->reset || (s->remote_closed && s->local_closed)) streams_.erase(s->id);
}

std::shared_ptr<Stream> Connection::open(const hpack::HeaderList& headers, std::string_view body, bool end_stream) {
  auto s = std::make_shared<Stream>();
  const std::string block = hpack::encode(headers);
  bool body_sent = false;
  {
    std::lock_guard<std::mutex> wl(write_mu_);  // ids must hit the wire in increasing order
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (closed_ || goaway_received_) return nullptr;
      s->id = next_stream_id_;
      next_stream_id_ += 2;
      s->send_window = peer_initial_window_;
      if (block.size() > peer_max_frame_) return nullptr;  // never for gRPC request headers
      streams_[s->id] = s;
      // a small body goes out in the same write as the HEADERS frame
      const int64_t n = static_cast<int64_t>(body.size());
      if (!body.empty() && body.size() <= peer_max_frame_ && n <= conn_send_window_ && n <= s->send_window) {
        conn_send_window_ -= n;
        s->send_window -= n;
        body_sent = true;
      }
    }
    const bool headers_end = end_stream && body.empty();
    std::string out;
    out.reserve(block.size() + (body_sent ? body.size() + 18 : 9));
    append_frame(out, kHeaders, kEndHeaders | (headers_end ? kEndStream : 0), s->id, block);
    if (body_sent) append_frame(out, kData, end_stream ? kEndStream : 0, s->id, body);
    if (!io_->write_all(out)) return nullptr;
    if (headers_end || (body_sent && end_stream)) {
      std::lock_guard<std::mutex> lk(mu_);
      s->local_closed = true;
    }
  }
  if (!body.empty() && !body_sent && !send_data(*s, body, end_stream)) return nullptr;
  return s;
}

Connection::SendResult Connection::try_send_response(Stream& s, const hpack::HeaderList& headers,
                                                     std::string_view body) {
  const std::string block = hpack::encode(headers);
  std::lock_guard<std::mutex> wl(write_mu_);
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_ || s.reset || s.local_closed) return SendResult::kFailed;
    const int64_t n = static_cast<int64_t>(body.size());
    if (block.size() > peer_max_frame_ || body.size() > peer_max_frame_ || n > conn_send_window_ ||
        n > s.send_window) {
      return SendResult::kWouldBlock;
    }
    conn_send_window_ -= n;
    s.send_window -= n;
  }
  std::string out;
  out.reserve(block.size() + body.size() + 18);
  append_frame(out, kHeaders, kEndHeaders | (body.empty() ? kEndStream : 0), s.id, block);
  if (!body.empty()) append_frame(out, kData, kEndStream, s.id, body);
  if (!io_->write_all(out)) return SendResult::kFailed;
  std::lock_guard<std::mutex> lk(mu_);
  s.local_closed = true;
  if (auto sp = find(s.id)) maybe_forget(sp);
  return SendResult::kSent;
}

bool Connection::send_response(Stream& s, const hpack::HeaderList& headers, std::string_view body) {
  switch (try_send_response(s, headers, body)) {
    case SendResult::kSent: return true;
    case SendResult::kFailed: return false;
    case SendResult::kWouldBlock: break;
  }
  return send_headers(s, headers, body.empty()) && (body.empty() || send_data(s, body, true));
}

bool Connection::send_headers(Stream& s, const hpack::HeaderList& headers, bool end_stream) {
  const std::string block = hpack::encode(headers);
  std::lock_guard<std::mutex> wl(write_mu_);
  size_t max = 0;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_ || s.reset || s.local_closed) return false;
    max = peer_max_frame_;
  }
  std::string_view rest(block);
  std::string_view first = rest.substr(0, max);
  rest.remove_prefix(first.size());
  uint8_t flags = (end_stream ? kEndStream : 0) | (rest.empty() ? kEndHeaders : 0);
  if (!write_frame_locked(kHeaders, flags, s.id, first)) return false;
  while (!rest.empty()) {
    std::string_view part = rest.substr(0, max);
    rest.remove_prefix(part.size());
    if (!write_frame_locked(kContinuation, rest.empty() ? kEndHeaders : 0, s.id, part)) return false;
  }
  if (end_stream) {
    std::lock_guard<std::mutex> lk(mu_);
    s.local_closed = true;
    auto sp = find(s.id);
    if (sp) maybe_forget(sp);
  }
  return true;
}

bool Connection::send_data(Stream& s, std::string_view data, bool end_stream) {
  do {
    size_t n = 0;
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (!data.empty()) {
        auto can_send = [&] { return closed_ || s.reset || (conn_send_window_ > 0 && s.send_window > 0); };
        if (caller_reads_) wait_reading(lk, window_cv_, std::chrono::steady_clock::time_point::max(), can_send);
        else window_cv_.wait(lk, can_send);
      }
      if (closed_ || s.reset || s.local_closed) return false;
      n = std::min<size_t>({data.size(), static_cast<size_t>(std::max<int64_t>(0, conn_send_window_)),
                            static_cast<size_t>(std::max<int64_t>(0, s.send_window)), peer_max_frame_});
      conn_send_window_ -= static_cast<int64_t>(n);
      s.send_window -= static_cast<int64_t>(n);
    }
    const bool last = n == data.size();
    if (!write_frame(kData, (last && end_stream) ? kEndStream : 0, s.id, data.substr(0, n))) return false;
    data.remove_prefix(n);
    if (last && end_stream) {
      std::lock_guard<std::mutex> lk(mu_);
      s.local_closed = true;
      auto sp = find(s.id);
      if (sp) maybe_forget(sp);
    }
  } while (!data.empty());
  return true;
}

void Connection::reset_stream(Stream& s, uint32_t code) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (s.reset) return;
    s.reset = true;
    s.reset_code = code;
    streams_.erase(s.id);
  }
  std::string p;
  put32(p, code);
  write_frame(kRstStream, 0, s.id, p);
  s.cv.notify_all();
  window_cv_.notify_all();
  cv_.notify_all();
}

void Connection::goaway(uint32_t code, const std::string& why) {
  LOG_WARN("http2") << "connection error: " << why;
  close(code);
}

void Connection::fail_all() {
  std::map<uint32_t, std::shared_ptr<Stream>> dead;
  {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    for (auto& [id, s] : streams_) {
      s->reset = true;
      if (!s->reset_code) s->reset_code = kCancel;
    }
    dead.swap(streams_);
  }
  for (auto& [id, s] : dead) s->cv.notify_all();
  window_cv_.notify_all();
  cv_.notify_all();
}

// Ensures rbuf_ holds at least n unread bytes (from rpos_).  1: yes; 0: EOF or error;
// -2: timeout (what was read so far stays buffered for the next reader).
int Connection::fill(size_t n, int timeout_ms) {
  while (rbuf_.size() - rpos_ < n) {
    if (rpos_ == rbuf_.size()) {
      rbuf_.clear();
      rpos_ = 0;
    } else if (rpos_ >= 32 * 1024) {
      rbuf_.erase(0, rpos_);
      rpos_ = 0;
    }
    const size_t old = rbuf_.size();
    rbuf_.resize(old + 64 * 1024);
    const ssize_t r = io_->read_some(&rbuf_[old], 64 * 1024, timeout_ms);
    if (r <= 0) {
      rbuf_.resize(old);
      return r == -2 ? -2 : 0;
    }
    rbuf_.resize(old + static_cast<size_t>(r));
  }
  return 1;
}

Connection::ReadResult Connection::read_frame(int timeout_ms) {
  const int h = fill(9, timeout_ms);
  if (h != 1) return h == -2 ? ReadResult::kTimeout : ReadResult::kClosed;
  const char* hdr = rbuf_.data() + rpos_;
  const uint32_t len = (uint32_t(static_cast<uint8_t>(hdr[0])) << 16) |
                       (uint32_t(static_cast<uint8_t>(hdr[1])) << 8) | uint32_t(static_cast<uint8_t>(hdr[2]));
  if (len > 16384) {  // we never raise SETTINGS_MAX_FRAME_SIZE
    goaway(kFrameSizeError, "frame larger than 16384");
    return ReadResult::kClosed;
  }
  const int b = fill(9 + len, timeout_ms);
  if (b != 1) return b == -2 ? ReadResult::kTimeout : ReadResult::kClosed;
  hdr = rbuf_.data() + rpos_;
  const uint8_t type = static_cast<uint8_t>(hdr[3]);
  const uint8_t flags = static_cast<uint8_t>(hdr[4]);
  const uint32_t sid = be32(hdr + 5) & 0x7fffffff;
  std::string payload(hdr + 9, len);
  rpos_ += 9 + len;
  frames_in_.fetch_add(1, std::memory_order_relaxed);
  handle_frame(type, flags, sid, payload, len);
  return closed_ ? ReadResult::kClosed : ReadResult::kFrame;
}

void Connection::handle_frame(uint8_t type, uint8_t flags, uint32_t sid, const std::string& payload, uint32_t len) {
  if (hdr_sid_ && type != kContinuation) {
    goaway(kProtocolError, "header block interrupted");
    return;
  }
  std::string_view p(payload);
  switch (type) {
    case kData: {
      if (sid == 0 || !strip_padding(flags, false, p)) {
        goaway(kProtocolError, "bad DATA frame");
        break;
      }
      on_data(sid, flags, p, len);
      break;
    }
    case kHeaders: {
      if (sid == 0 || !strip_padding(flags, true, p)) {
        goaway(kProtocolError, "bad HEADERS frame");
        break;
      }
      hdr_block_.assign(p.data(), p.size());
      hdr_flags_ = flags;
      if (flags & kEndHeaders) {
        on_headers(sid, flags, hdr_block_);
      } else {
        hdr_sid_ = sid;
      }
      break;
    }
    case kContinuation: {
      if (!hdr_sid_ || sid != hdr_sid_) {
        goaway(kProtocolError, "unexpected CONTINUATION");
        break;
      }
      hdr_block_.append(p.data(), p.size());
      if (flags & kEndHeaders) {
        uint32_t s = hdr_sid_;
        hdr_sid_ = 0;
        on_headers(s, hdr_flags_, hdr_block_);
      }
      break;
    }
    case kSettings:
      if (sid != 0 || (!(flags & kAck) && len % 6 != 0)) {
        goaway(kProtocolError, "bad SETTINGS frame");
        break;
      }
      on_settings(flags, p);
      break;
    case kPing:
      if (len != 8) {
        goaway(kFrameSizeError, "bad PING frame");
        break;
      }
      if (!(flags & kAck)) write_frame(kPing, kAck, 0, p);
      break;
    case kWindowUpdate:
      if (len != 4) {
        goaway(kFrameSizeError, "bad WINDOW_UPDATE frame");
        break;
      }
      on_window_update(sid, p);
      break;
    case kRstStream:
      if (len != 4) {
        goaway(kFrameSizeError, "bad RST_STREAM frame");
        break;
      }
      on_rst(sid, p);
      break;
    case kGoaway: {
      if (len < 8) {
        goaway(kFrameSizeError, "bad GOAWAY frame");
        break;
      }
      on_goaway(be32(p.data()) & 0x7fffffff);
      break;
    }
    case kPushPromise:
      goaway(kProtocolError, "PUSH_PROMISE with push disabled");
      break;
    default:  // PRIORITY and unknown extension frames are ignored
      break;
  }
}

void Connection::reader_loop() {
  if (role_ == Role::kServer) {
    if (fill(sizeof(kPreface) - 1, -1) != 1 ||
        std::memcmp(rbuf_.data() + rpos_, kPreface, sizeof(kPreface) - 1) != 0) {
      fail_all();
      close(kProtocolError);
      return;
    }
    rpos_ += sizeof(kPreface) - 1;
  }
  while (!closed_ && read_frame(-1) == ReadResult::kFrame) {
  }
  fail_all();
  if (io_) io_->shutdown();
}

bool Connection::read_step_locked(std::unique_lock<std::mutex>& lk, std::chrono::steady_clock::time_point deadline) {
  const auto now = std::chrono::steady_clock::now();
  if (deadline <= now) return false;
  const auto left = std::chrono::ceil<std::chrono::milliseconds>(deadline - now);
  reading_ = true;
  lk.unlock();
  const ReadResult r = read_frame(static_cast<int>(std::min<int64_t>(left.count(), 1 << 30)));
  if (r == ReadResult::kClosed) {
    fail_all();
    if (io_) io_->shutdown();
  }
  lk.lock();
  reading_ = false;
  return r == ReadResult::kFrame || (r == ReadResult::kTimeout && std::chrono::steady_clock::now() < deadline);
}

void Connection::hand_off_locked() {
  // the reader role is free and callers still wait: wake one, it reads next
  if (!reading_ && !waiting_cvs_.empty()) waiting_cvs_.front()->notify_one();
}

bool Connection::poll_idle() {
  if (!caller_reads_) return !closed_;
  std::unique_lock<std::mutex> lk(mu_);
  if (reading_ || closed_) return !closed_;
  // frames that arrived while nobody waited: SETTINGS, PING, WINDOW_UPDATE, a GOAWAY or
  // the peer closing an idle connection
  reading_ = true;
  lk.unlock();
  ReadResult r;
  do {
    r = read_frame(0);
  } while (r == ReadResult::kFrame && !closed_);
  if (r == ReadResult::kClosed) {
    fail_all();
    if (io_) io_->shutdown();
  }
  lk.lock();
  reading_ = false;
  hand_off_locked();
  return !closed_;
}

void Connection::on_settings(uint8_t flags, std::string_view p) {
  if (flags & kAck) return;
  bool bad_window = false;
  // The peer enforces its new limits (e.g. a larger MAX_FRAME_SIZE) only after it has
  // read our ACK, so no frame sized by the new values may precede the ACK on the wire:
  // update and acknowledge under the write lock (order: write_mu_ -> mu_, as elsewhere).
  std::unique_lock<std::mutex> wl(write_mu_);
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i + 6 <= p.size(); i += 6) {
      const uint16_t id = static_cast<uint16_t>((static_cast<uint8_t>(p[i]) << 8) | static_cast<uint8_t>(p[i + 1]));
      const uint32_t v = be32(p.data() + i + 2);
      if (id == 0x4) {  // INITIAL_WINDOW_SIZE: shift every open stream's window by the delta
        if (v > 0x7fffffff) {
          bad_window = true;
          break;
        }
        const int64_t delta = int64_t(v) - int64_t(peer_initial_window_);
        peer_initial_window_ = v;
        for (auto& [sid, s] : streams_) s->send_window += delta;
      } else if (id == 0x5) {
        if (v >= 16384 && v <= 16777215) peer_max_frame_ = v;
      }
    }
  }
  if (bad_window) {
    wl.unlock();
    goaway(kFlowControlError, "INITIAL_WINDOW_SIZE too large");
    return;
  }
  write_frame_locked(kSettings, kAck, 0, {});
  wl.unlock();
  window_cv_.notify_all();
  cv_.notify_all();
}

void Connection::on_window_update(uint32_t sid, std::string_view p) {
  const uint32_t inc = be32(p.data()) & 0x7fffffff;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (sid == 0) {
      conn_send_window_ += inc;
    } else if (auto s = find(sid)) {
      s->send_window += inc;
    }
  }
  window_cv_.notify_all();
  cv_.notify_all();
}

void Connection::on_rst(uint32_t sid, std::string_view p) {
  std::shared_ptr<Stream> s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    s = find(sid);
    if (s) {
      s->reset = true;
      s->reset_code = be32(p.data());
      streams_.erase(sid);
    }
  }
  if (s) s->cv.notify_all();
  window_cv_.notify_all();
  cv_.notify_all();
}

void Connection::on_headers(uint32_t sid, uint8_t flags, const std::string& block) {
  hpack::HeaderList hl;
  std::string err;
  if (!decoder_.decode(block, &hl, &err)) {
    goaway(kCompressionError, "HPACK: " + err);
    return;
  }
  std::shared_ptr<Stream> dispatch, s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    s = find(sid);
    if (!s) {
      if (role_ == Role::kClient || (sid % 2) == 0 || sid <= last_peer_stream_) {
        // trailers for a stream we already forgot, or a bogus id: ignore (decoded for HPACK state)
        return;
      }
      if (goaway_sent_) {
        s = nullptr;  // draining: refused below (the peer may retry it elsewhere)
      } else {
        last_peer_stream_ = sid;
        s = std::make_shared<Stream>();
        s->id = sid;
        s->send_window = peer_initial_window_;
        streams_[sid] = s;
      }
    }
    if (s) {
      if (!s->headers_received) {
        s->headers = std::move(hl);
        s->headers_received = true;
      } else {
        for (auto& h : hl) s->trailers.push_back(std::move(h));
      }
      if (flags & kEndStream) {
        s->remote_closed = true;
        if (role_ == Role::kServer && !s->dispatched) {
          s->dispatched = true;
          dispatch = s;
        }
        maybe_forget(s);
      }
    }
  }
  if (!s) {
    std::string p;
    put32(p, kRefusedStream);
    write_frame(kRstStream, 0, sid, p);
    return;
  }
  s->cv.notify_all();
  cv_.notify_all();
  if (dispatch && on_request_) on_request_(shared_from_this(), dispatch);
}

void Connection::on_goaway(uint32_t last_stream) {
  // RFC 9113 6.8: our streams above last_stream were not processed and may be retried
  std::vector<std::shared_ptr<Stream>> refused;
  {
    std::lock_guard<std::mutex> lk(mu_);
    goaway_received_ = true;
    for (auto it = streams_.upper_bound(last_stream); it != streams_.end();) {
      if ((it->first % 2) == (role_ == Role::kClient ? 1u : 0u)) {
        it->second->reset = true;
        it->second->reset_code = kRefusedStream;
        refused.push_back(it->second);
        it = streams_.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& st : refused) st->cv.notify_all();
  window_cv_.notify_all();
  cv_.notify_all();
}

void Connection::drain() {
  uint32_t last;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (goaway_sent_ || closed_) return;
    goaway_sent_ = true;
    last = last_peer_stream_;
  }
  std::string p;
  put32(p, last);
  put32(p, kNoError);
  write_frame(kGoaway, 0, 0, p);
}

void Connection::on_data(uint32_t sid, uint8_t flags, std::string_view payload, size_t flow_len) {
  std::shared_ptr<Stream> dispatch, s;
  bool stream_open = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    s = find(sid);
    if (s && !s->remote_closed) {
      s->data.append(payload.data(), payload.size());
      if (flags & kEndStream) {
        s->remote_closed = true;
        if (role_ == Role::kServer && !s->dispatched) {
          s->dispatched = true;
          dispatch = s;
        }
        maybe_forget(s);
      } else {
        stream_open = true;
      }
    }
  }
  // Re-open the receive windows once half of one is used: data is buffered, not
  // back-pressured, and a request that fits in a window costs no WINDOW_UPDATE write.
  if (flow_len) {
    conn_recv_pending_ += flow_len;
    uint32_t stream_inc = 0;
    if (stream_open) {
      std::lock_guard<std::mutex> lk(mu_);
      s->recv_pending += static_cast<uint32_t>(flow_len);
      if (s->recv_pending >= kOurWindow / 2) {
        stream_inc = s->recv_pending;
        s->recv_pending = 0;
      }
    }
    std::string out;
    if (conn_recv_pending_ >= kOurConnWindow / 2) {
      std::string inc;
      put32(inc, static_cast<uint32_t>(conn_recv_pending_));
      append_frame(out, kWindowUpdate, 0, 0, inc);
      conn_recv_pending_ = 0;
    }
    if (stream_inc) {
      std::string inc;
      put32(inc, stream_inc);
      append_frame(out, kWindowUpdate, 0, sid, inc);
    }
    if (!out.empty()) {
      std::lock_guard<std::mutex> wl(write_mu_);
      io_->write_all(out);
    }
  }
  if (s) s->cv.notify_all();
  cv_.notify_all();
  if (dispatch && on_request_) on_request_(shared_from_this(), dispatch);
}

}  // namespace bgc::http2

// ===========================================================================
namespace bgc::grpc {

using http2::Connection;
using http2::Stream;

std::string frame_message(std::string_view msg) {
  std::string out;
  out.reserve(5 + msg.size());
  out.push_back(0);
  http2::put32(out, static_cast<uint32_t>(msg.size()));
  out.append(msg.data(), msg.size());
  return out;
}

bool pop_message(std::string& buf, std::string* msg) {
  if (buf.size() < 5) return false;
  if (buf[0] != 0) throw std::runtime_error("compressed gRPC messages are not supported");
  const uint32_t n = http2::be32(buf.data() + 1);
  if (buf.size() - 5 < n) return false;
  msg->assign(buf, 5, n);
  buf.erase(0, 5 + n);
  return true;
}

static const std::string* header(const hpack::HeaderList& hl, std::string_view name) {
  for (const auto& h : hl)
    if (h.first == name) return &h.second;
  return nullptr;
}

// grpc-message is percent-encoded (RFC 3986 unreserved + printable pass through).
static std::string percent_encode(std::string_view s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7e && c != '%') {
      out.push_back(static_cast<char>(c));
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    }
  }
  return out;
}

static std::string percent_decode(std::string_view s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && isxdigit(static_cast<unsigned char>(s[i + 1])) &&
        isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out.push_back(static_cast<char>(std::stoi(std::string(s.substr(i + 1, 2)), nullptr, 16)));
      i += 2;
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

// ---------------------------------------------------------------- ServerCall
ServerCall::ServerCall(std::shared_ptr<Connection> conn, std::shared_ptr<Stream> stream,
                       std::atomic<bool>* stopping)
    : conn_(std::move(conn)), stream_(std::move(stream)), stopping_(stopping) {}

const hpack::HeaderList& ServerCall::metadata() const { return stream_->headers; }

bool ServerCall::send_message(std::string_view msg) {
  if (finished_) return false;
  if (!headers_sent_) {
    if (!conn_->send_headers(*stream_, {{":status", "200"}, {"content-type", "application/grpc"}}, false)) return false;
    headers_sent_ = true;
  }
  return conn_->send_data(*stream_, frame_message(msg), false);
}

void ServerCall::finish(const Status& st) {
  if (finished_) return;
  finished_ = true;
  hpack::HeaderList tr;
  if (!headers_sent_) {  // trailers-only response
    tr.emplace_back(":status", "200");
    tr.emplace_back("content-type", "application/grpc");
  }
  tr.emplace_back("grpc-status", std::to_string(st.code));
  if (!st.message.empty()) tr.emplace_back("grpc-message", percent_encode(st.message));
  conn_->send_headers(*stream_, tr, true);
}

bool ServerCall::cancelled() const {
  if (stopping_ && stopping_->load()) return true;
  return conn_->locked([&] { return stream_->reset || conn_->closed(); });
}

bool ServerCall::wait_cancelled(std::chrono::milliseconds d) const {
  const auto deadline = std::chrono::steady_clock::now() + d;
  conn_->wait_until(deadline, [&] { return stream_->reset || (stopping_ && stopping_->load()); });
  return cancelled();
}

// ---------------------------------------------------------------- Server
Server::Server(std::string unix_path) : path_(std::move(unix_path)) {}

Server::~Server() { stop(); }

void Server::add(const std::string& method_path, Handler h) { handlers_[method_path] = std::move(h); }

void Server::start() {
  listen_fd_ = net::listen_unix(path_, 64);
  struct stat st {};
  if (::stat(path_.c_str(), &st) == 0) inode_ = st.st_ino;
  acceptor_ = std::thread([this] { accept_loop(); });
}

bool Server::socket_present() const {
  struct stat st {};
  return ::stat(path_.c_str(), &st) == 0 && st.st_ino == inode_;
}

void Server::accept_loop() {
  while (!stopping_) {
    int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      if (stopping_) break;
      if (errno == EMFILE || errno == ENFILE) {
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        continue;
      }
      break;
    }
    auto conn = std::make_shared<Connection>(
        std::make_unique<net::TcpStream>(fd), Connection::Role::kServer,
        [this](std::shared_ptr<Connection> c, std::shared_ptr<Stream> s) { dispatch(std::move(c), std::move(s)); });
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stopping_) break;
      conns_.erase(std::remove_if(conns_.begin(), conns_.end(),
                                  [](const std::shared_ptr<Connection>& c) { return c->closed(); }),
                   conns_.end());
      conns_.push_back(conn);
    }
    conn->start();
  }
}

void Server::reap(bool all) {
  std::vector<Worker> done;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = workers_.begin(); it != workers_.end();) {
      if (all || it->done->load()) {
        done.push_back(std::move(*it));
        it = workers_.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& w : done)
    if (w.t.joinable()) w.t.join();
}

void Server::dispatch(std::shared_ptr<Connection> c, std::shared_ptr<Stream> s) {
  reap(false);
  auto done = std::make_shared<std::atomic<bool>>(false);
  std::thread t([this, c, s, done] {
    calls_.fetch_add(1);
    ServerCall call(c, s, &stopping_);
    try {
      const std::string* path = header(s->headers, ":path");
      const std::string* ctype = header(s->headers, "content-type");
      call.method_ = path ? *path : "";
      if (!ctype || ctype->rfind("application/grpc", 0) != 0) {
        call.finish({kInternal, "content-type is not application/grpc"});
      } else {
        std::string body = c->locked([&] { return std::move(s->data); });
        std::string msg;
        if (!pop_message(body, &msg)) msg.clear();  // empty request (no DATA) = default message
        call.request_ = std::move(msg);
        auto it = handlers_.find(call.method_);
        if (it == handlers_.end()) {
          call.finish({kUnimplemented, "unknown method " + call.method_});
        } else {
          call.finish(it->second(call));
        }
      }
    } catch (const std::exception& e) {
      call.finish({kInternal, e.what()});
    }
    done->store(true);
  });
  std::lock_guard<std::mutex> lk(mu_);
  workers_.push_back({std::move(t), done});
}

void Server::stop() {
  if (stopping_.exchange(true)) return;
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
    ::close(listen_fd_);
  }
  if (acceptor_.joinable()) acceptor_.join();
  std::vector<std::shared_ptr<Connection>> conns;
  {
    std::lock_guard<std::mutex> lk(mu_);
    conns.swap(conns_);
  }
  // Closing first wakes handlers blocked on flow control or in wait_cancelled().
  for (auto& c : conns) c->close();
  reap(true);
  for (auto& c : conns) c->join();
  if (socket_present()) ::unlink(path_.c_str());
}

// ---------------------------------------------------------------- Channel
Channel::Channel(std::string target, int connect_timeout_ms) : connect_timeout_ms_(connect_timeout_ms) {
  path_ = target.rfind("unix://", 0) == 0 ? target.substr(7) : target;
}

Channel::~Channel() { close(); }

void Channel::close() {
  std::shared_ptr<Connection> c;
  {
    std::lock_guard<std::mutex> lk(mu_);
    c.swap(conn_);
  }
  if (c) {
    c->close();
    c->join();
  }
}

std::shared_ptr<Connection> Channel::conn() {
  std::lock_guard<std::mutex> lk(mu_);
  if (conn_ && !conn_->closed()) return conn_;
  if (conn_) {
    conn_->close();
    conn_->join();
  }
  int fd = net::connect_unix(path_, connect_timeout_ms_);
  conn_ = std::make_shared<Connection>(std::make_unique<net::TcpStream>(fd), Connection::Role::kClient);
  conn_->start();
  return conn_;
}

Status Channel::call_status(Stream& s, bool reset_seen) {
  if (reset_seen) return {kUnavailable, "stream reset (code " + std::to_string(s.reset_code) + ")"};
  const std::string* status = header(s.headers, ":status");
  if (!status || *status != "200") return {kUnknown, "HTTP status " + (status ? *status : std::string("?"))};
  const std::string* gs = header(s.trailers, "grpc-status");
  const std::string* gm = header(s.trailers, "grpc-message");
  if (!gs) {  // trailers-only response
    gs = header(s.headers, "grpc-status");
    gm = header(s.headers, "grpc-message");
  }
  if (!gs) return {kUnknown, "missing grpc-status"};
  return {std::atoi(gs->c_str()), gm ? percent_decode(*gm) : ""};
}

static hpack::HeaderList request_headers(const std::string& method) {
  return {{":method", "POST"},
          {":scheme", "http"},
          {":path", method},
          {":authority", "localhost"},
          {"content-type", "application/grpc"},
          {"te", "trailers"},
          {"user-agent", "bgc-grpc/1.0"}};
}

Status Channel::unary(const std::string& method, std::string_view req, std::string* resp,
                      std::chrono::milliseconds timeout) {
  std::string resp_body;
  Status st = server_stream(
      method, req,
      [&](const std::string& m) {
        resp_body = m;
        return true;
      },
      timeout);
  if (st.ok() && resp) *resp = std::move(resp_body);
  return st;
}

Status Channel::server_stream(const std::string& method, std::string_view req,
                              const std::function<bool(const std::string&)>& on_msg,
                              std::chrono::milliseconds timeout) {
  std::shared_ptr<Connection> c;
  try {
    c = conn();
  } catch (const std::exception& e) {
    return {kUnavailable, e.what()};
  }
  auto s = c->open(request_headers(method), frame_message(req), true);
  if (!s) return {kUnavailable, "connection closed"};
  const auto deadline = std::chrono::steady_clock::now() + timeout;
  std::string buf;
  while (true) {
    bool ended = false, reset = false;
    bool ok = c->wait_until(deadline, [&] { return !s->data.empty() || s->remote_closed || s->reset; });
    c->locked([&] {
      buf += s->data;
      s->data.clear();
      ended = s->remote_closed;
      reset = s->reset || (c->closed() && !s->remote_closed);
      return 0;
    });
    std::string msg;
    try {
      while (pop_message(buf, &msg)) {
        if (!on_msg(msg)) {
          c->reset_stream(*s, http2::kCancel);
          return {kCancelled, "cancelled by the client"};
        }
      }
    } catch (const std::exception& e) {
      c->reset_stream(*s, http2::kCancel);
      return {kInternal, e.what()};
    }
    if (reset) return call_status(*s, true);
    if (ended) return c->locked([&] { return call_status(*s, false); });
    if (!ok && std::chrono::steady_clock::now() >= deadline) {
      c->reset_stream(*s, http2::kCancel);
      return {kDeadlineExceeded, "deadline exceeded"};
    }
  }
}

}  // namespace bgc::grpc
